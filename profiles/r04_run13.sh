#!/bin/bash
# Round-4 call 13: the resolve stage's lazy DP with exact decisions of the ambiguous columns only
# (default) vs the exact-OPT DP over every column (LT_RESOLVE_FULL=1, via LT_JIT_DEFINES), and the
# scene-specialised JIT kernels vs LT_JIT_SCENE=0; GPU tests first.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
set +e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
set -e
tail -3 $O/gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc $rc"; exit $rc; fi
run() {
  name=$1; C=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $C --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/${C}_$name.json 2> $O/${C}_$name.err
  python -c "import json;d=json.load(open('$O/${C}_$name.json'));print('$C $name',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
for i in 1 2; do
  for C in c2 c3; do
    run new_$i $C LT_X=1
    run full_$i $C LT_JIT_DEFINES=LT_RESOLVE_FULL=1
    run noscene_$i $C LT_JIT_SCENE=0
  done
done
for C in c5 c4; do
  run new $C LT_X=1
  run full $C LT_JIT_DEFINES=LT_RESOLVE_FULL=1
  run noscene $C LT_JIT_SCENE=0
done
