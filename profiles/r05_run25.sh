#!/bin/bash
# r05 run 25: c5 tile sizes with a smaller last tile (its resolve is the step's exposed tail):
# 16.8 Mpx (3 tiles: 16.8 + 16.8 + 15.4, the default), 20 Mpx (20 + 20 + 9), 22 Mpx (22 + 22 + 5)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run25}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for i in 1 2; do
  for T in 16777216 20000000 22000000; do
    timeout -k 10 200 python bench.py --config c5 --tile $T --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/c5_${T}_$i.json 2> $O/c5_${T}_$i.err
    python -c "import json;d=json.load(open('$O/c5_${T}_$i.json'));print('c5 $T',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
  done
done
