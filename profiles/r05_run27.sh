#!/bin/bash
# r05 run 27: (1) c5 with the lazy resolve (LT_RESOLVE_FULL=0: the lazy DP with each ambiguous
# column decided exactly, instead of the exact-OPT DP over every column; measured slower on c2/c3
# in round 4, never on c5's 40-column low-line-cost series), (2) c3 at 3 waves per SIMD
# (LT_JIT_WAVES=3: no spills) — twice each against the default, parity samples on
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run27}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, env assignment or "", args
  env $2 timeout -k 10 200 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
for i in 1 2; do
  b c5_base_$i "" "--config c5"
  b c5_lazyres_$i LT_JIT_DEFINES=LT_RESOLVE_FULL=0 "--config c5"
  b c3_base_$i "" "--config c3"
  b c3_w3_$i LT_JIT_WAVES=3 "--config c3"
done
