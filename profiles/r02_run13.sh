#!/bin/bash
# Re-entry check of HEAD: GPU tests, default bench line (cpu baseline + end-to-end), c3/c4/c5 lines,
# kernel-trace stats of the default line, one PMC instruction pass of a 16.8 Mpx c2 and c5 launch.
# Usage: bash profiles/r02_run13.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
echo "bench default ok"
for c in c5 c3 c4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --e2e-steps 0 > $O/bench_$c.json \
    2> $O/bench_$c.err
  echo "bench $c ok"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/kt_bench.json 2> $O/kt_bench.err
echo "kernel trace ok"
for C in c2 c5; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
  GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$C -o run -- python3 $R/bench.py --config $C \
  --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 > $O/pmc_$C.log 2>&1
echo "pmc $C ok"
done
