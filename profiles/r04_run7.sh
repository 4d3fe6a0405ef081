#!/bin/bash
# Round-4 call 7: GPU tests (JIT-fused index programs added), c2/c3/c5 bench lines at this build,
# the JIT attribution run ('(B1 - B2) * 2 / 2': the same values through a non-linear program) vs
# 'B1 - B2' and vs the index-raster path (LT_JIT_INDEX=0), the current analyze body (v_min/v_max bounds, no NaN selects in the year-major stores)
# against the committed one on c2 and c5 (build/exp/liblt_{n1,h1}_{32,48}.so).
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
  for L in h1 n1 rcert; do
    LT_HIP_LIB=$R/build/exp/liblt_${L}_32.so timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/c2_$L$i.json 2> $O/c2_$L$i.err
    python -c "import json;d=json.load(open('$O/c2_$L$i.json'));print('c2 $L',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
    [ $L = rcert ] && continue
    LT_HIP_LIB=$R/build/exp/liblt_${L}_48.so timeout -k 10 300 python bench.py --config c5 --steps 5 --no-cpu-baseline --e2e-steps 0 > $O/c5_$L$i.json 2> $O/c5_$L$i.err
    python -c "import json;d=json.load(open('$O/c5_$L$i.json'));print('c5 $L',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
  done
done
cd /tmp
# the resolve kernel's memory behaviour (c2 product build, one 16.8 Mpx launch)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SMEM \
  --output-format csv -d $O/pmc_res -o run -- python3 $R/bench.py --config c2 --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 --parity-sample 0 > $O/pmc_res.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d $O/pmc_res2 -o run -- python3 $R/bench.py --config c2 --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 --parity-sample 0 > $O/pmc_res2.log 2>&1
echo done
