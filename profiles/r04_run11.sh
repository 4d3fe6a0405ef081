#!/bin/bash
# Round-4 call 11: GPU tests (certified labels path in the resolve stage), default c2/c3/c5 lines
# (JIT kernels specialised for the launch), the JIT analyze kernel at 5 waves per SIMD
# (LT_JIT_WAVES=5: 96 VGPRs, 35 spilled) vs 4, kernel-trace stats of the default c2 line.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
rc=0
timeout -k 10 1100 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || rc=$?
echo "gpu tests rc=$rc"; tail -2 $O/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
run() {
  name=$1; C=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $C --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/${C}_$name.json 2> $O/${C}_$name.err
  python -c "import json;d=json.load(open('$O/${C}_$name.json'));print('$C $name',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
for i in 1 2; do
  run w4_$i c2 LT_X=1
  run w5_$i c2 LT_JIT_WAVES=5
  run w4_$i c3 LT_X=1
  run w5_$i c3 LT_JIT_WAVES=5
done
run w4 c5 LT_X=1
run w5 c5 LT_JIT_WAVES=5
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --no-cpu-baseline --e2e-steps 0 --steps 10 > $O/kt.log 2>&1
echo "kernel trace ok"
