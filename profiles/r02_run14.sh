#!/bin/bash
# GPU tests, bench lines for c2/c3/c4/c5 (no cpu baseline), one PMC instruction pass of a 16.8 Mpx
# c2 and c3 launch. Usage: bash profiles/r02_run14.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
echo "tests ok"
for c in c2 c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --e2e-steps 0 > $O/bench_$c.json \
    2> $O/bench_$c.err
  echo "bench $c ok"
done
cd /tmp && export TMPDIR=/tmp
for C in c2 c3; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
  GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$C -o run -- python3 $R/bench.py --config $C \
  --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 > $O/pmc_$C.log 2>&1
echo "pmc $C ok"
done
