#!/bin/bash
# r05 run 24: c4 at N = 1 with four tiles per rank (one 49 Mpx launch per scene) against the
# previous 32 tiles of 6.1 Mpx (--tile 6125056), twice, parity samples on
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run24}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then T="--tile 6125056"; else T=""; fi
    timeout -k 10 200 python bench.py --config c4 $T --no-cpu-baseline --e2e-steps 0 > $O/c4_${v}_$i.json 2> $O/c4_${v}_$i.err
    python -c "import json;d=json.load(open('$O/c4_${v}_$i.json'));print('c4 $v',d['value'],d['ms_per_step'],d['config']['tile_pixels'],d['config']['tiles'],d['roofline']['frac'],d['parity_sample']['mismatched_values'])"
  done
done
