#!/bin/bash
# GPU tests after the one-pass trendline walk + GPU raster assembly; c5/c2 bench lines; PMC VALU
# counts of instruction-attribution experiment builds (profiles/build/exp_*.so, never product).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --e2e-steps 0 > $O/bench_c5.json \
  2> $O/bench_c5.err
timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-steps 0 > $O/bench_c2.json \
  2> $O/bench_c2.err
echo "bench ok"
cd /tmp && export TMPDIR=/tmp
for E in nofit nooffer notail noexit2; do
  LT_HIP_LIB=$R/profiles/build/exp_${E}_32.so timeout -s KILL 120 rocprofv3 --pmc \
    SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $O/exp_$E -o run -- python3 $R/bench.py --config c2 \
    --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 > $O/exp_$E.log 2>&1
  echo "exp $E ok"
done
