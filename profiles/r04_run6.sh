#!/bin/bash
# Round-4 call 6: GPU tests + c2/c3/c5 bench lines on the product build with the exact-integer
# despike; A/B of the certified labels path in the resolve stage (liblt_rcert_32 vs liblt_cur_32).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for C in c2 c3 c5; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --e2e-steps 0 > $O/bench_$C.json 2> $O/bench_$C.err
  python -c "import json;d=json.load(open('$O/bench_$C.json'));print('$C',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
done
for i in 1 2; do
  for L in cur rcert; do
    LT_HIP_LIB=$R/build/exp/liblt_${L}_32.so timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/c2_$L$i.json 2> $O/c2_$L$i.err
    python -c "import json;d=json.load(open('$O/c2_$L$i.json'));print('c2 $L',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
  done
done
