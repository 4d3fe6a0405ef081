#!/bin/bash
# GPU tests and bench lines (c2, c5, c3) after the zero-residual / same-base-tag lazy DP.
# Usage: bash profiles/r02_run10.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
echo "tests ok"
for c in c2 c5 c3; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --e2e-steps 0 > $O/bench_$c.json \
    2> $O/bench_$c.err
  echo "bench $c ok"
done
