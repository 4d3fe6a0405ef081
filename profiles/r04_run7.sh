#!/bin/bash
# Round-4 call 7: GPU tests (JIT-fused index programs added), c2/c3/c5 bench lines at this build,
# the JIT attribution run ('(B1 - B2) * 2 / 2': the same values through a non-linear program) vs
# 'B1 - B2' and vs the index-raster path (LT_JIT_INDEX=0), resolve-certified A/B.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
rc=0
timeout -k 10 1100 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for C in c2 c3 c5; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --e2e-steps 0 > $O/bench_$C.json 2> $O/bench_$C.err
  python -c "import json;d=json.load(open('$O/bench_$C.json'));print('$C',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
done
timeout -k 10 400 python bench.py --index-eqn '(B1 - B2) * 2 / 2' --no-cpu-baseline --e2e-steps 0 > $O/bench_c2_jit.json 2> $O/bench_c2_jit.err
python -c "import json;d=json.load(open('$O/bench_c2_jit.json'));print('c2 jit',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['parity_sample']['mismatched_values'],d['config']['input'])"
LT_JIT_INDEX=0 timeout -k 10 400 python bench.py --index-eqn '(B1 - B2) * 2 / 2' --no-cpu-baseline --e2e-steps 0 > $O/bench_c2_raster.json 2> $O/bench_c2_raster.err
python -c "import json;d=json.load(open('$O/bench_c2_raster.json'));print('c2 raster',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['parity_sample']['mismatched_values'],d['config']['input'])"
for i in 1 2; do
  for L in cur rcert; do
    LT_HIP_LIB=$R/build/exp/liblt_${L}_32.so timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/c2_$L$i.json 2> $O/c2_$L$i.err
    python -c "import json;d=json.load(open('$O/c2_$L$i.json'));print('c2 $L',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
  done
done
