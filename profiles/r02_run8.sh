#!/bin/bash
# GPU tests + c2/c5 bench lines after the straight-line small-segment fits; PMC of the new kernels.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
TAG=$2
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-steps 0 > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --e2e-steps 0 > $O/bench_c5.json \
  2> $O/bench_c5.err
echo "bench ok"
cd /tmp && export TMPDIR=/tmp
for MY in 32 48; do
  C=c2; [ $MY = 48 ] && C=c5
  LT_HIP_LIB=$R/profiles/build/exp_${TAG}_$MY.so timeout -s KILL 120 rocprofv3 --pmc \
    SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $O/pmc_$C -o run -- python3 $R/bench.py --config $C \
    --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 > $O/pmc_$C.log 2>&1
  echo "pmc $C ok"
done
