#!/bin/bash
# Session-3 baseline on HEAD: GPU tests, the default bench line (cpu baseline + end-to-end), c5 and
# c3 lines. Usage: bash profiles/r02_run9.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err
echo "bench c2 ok"
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
echo "bench c5 ok"
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --e2e-steps 0 > $O/bench_c3.json 2> $O/bench_c3.err
echo "bench c3 ok"
