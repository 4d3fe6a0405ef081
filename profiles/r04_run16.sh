#!/bin/bash
# Round-4 call 16: c5 year-major rows stored LT_YEAR_STORE_LAG years late (0 / 1 / 2), so the
# fit steps' x-set loads do not wait for the stores just issued (in-order vmcnt); GPU tests of the
# c5-shaped paths first.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mosaic.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
tail -2 $O/gpu_tests.txt
run() {
  name=$1; C=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $C --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/${C}_$name.json 2> $O/${C}_$name.err
  python -c "import json;d=json.load(open('$O/${C}_$name.json'));print('$C $name',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
for i in 1 2; do
  run lag1_$i c5 LT_X=1
  run lag0_$i c5 LT_JIT_DEFINES=LT_YEAR_STORE_LAG=0
  run lag2_$i c5 LT_JIT_DEFINES=LT_YEAR_STORE_LAG=2
done
run lag1 c2 LT_X=1
