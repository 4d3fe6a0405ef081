#!/bin/bash
# Round-4 call 20: XCD-contiguous pixel chunks (LT_XCD_REMAP via LT_JIT_DEFINES) vs blockIdx order;
# GPU mosaic / parity tests with the remap first.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
LT_JIT_DEFINES=LT_XCD_REMAP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_mosaic.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_remap.txt 2>&1
tail -2 $O/gpu_tests_remap.txt
run() {
  name=$1; C=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $C --steps 8 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $O/${C}_$name.json 2> $O/${C}_$name.err
  python -c "import json;d=json.load(open('$O/${C}_$name.json'));print('$C $name',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
for i in 1 2; do
  for C in c5 c2 c3; do
    run base_$i $C LT_X=1
    run remap_$i $C LT_JIT_DEFINES=LT_XCD_REMAP=1
  done
done
