#!/bin/bash
# Round-5 call 8: pass B of the certified labels path fits only the eqns pass A left undecided
# (lockstep slots). GPU suite, then c2 / c3 A/B against LT_PASSB_SLOTS=0 (same build otherwise).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
tail -1 $O/gpu_tests.txt
for c in c2 c3; do
  for v in slots noslots slots2; do
    if [ $v = noslots ]; then export LT_JIT_DEFINES=LT_PASSB_SLOTS=0; else unset LT_JIT_DEFINES; fi
    timeout -k 10 300 python bench.py --config $c --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/${c}_$v.json 2> $O/${c}_$v.err
    python -c "import json;d=json.load(open('$O/${c}_$v.json'));print('$c $v',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
  done
done
