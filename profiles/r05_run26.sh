#!/bin/bash
# r05 run 26: c2 as one 49 Mpx launch (default) against two launches per scene (44 + 5 and
# 40 + 9 Mpx: the first launch's resolve stage runs beside the second's analyze), twice
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run26}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for i in 1 2; do
  for T in 49000000 44000000 40000000; do
    timeout -k 10 200 python bench.py --config c2 --tile $T --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/c2_${T}_$i.json 2> $O/c2_${T}_$i.err
    python -c "import json;d=json.load(open('$O/c2_${T}_$i.json'));print('c2 $T',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
  done
done
