#!/bin/bash
# r05 run 29: on the V12 product (6d4eff1), A/B of V13 (the int16 winner-pick loop branch-free:
# every lane takes every year, no exec-mask juggling per year, labels-only launches) and V14
# (pass A's closed-form segment sums branch-free: four slots per lane with zero selects), twice,
# parity samples on
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run29}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, override dir or "", args
  if [ -n "$2" ]; then export LT_JIT_OVERRIDE_DIR=$R/build/override/$2; else unset LT_JIT_OVERRIDE_DIR; fi
  timeout -k 10 170 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'],d['jit']['override'])"
}
for i in 1 2; do
  for C in c2 c3; do
    b ${C}_base_$i "" "--config $C"
    b ${C}_v13_$i v13 "--config $C"
    b ${C}_v14_$i v14 "--config $C"
  done
  b c5_base_$i "" "--config c5"
  b c5_v13_$i v13 "--config c5"
done
