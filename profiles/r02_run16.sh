#!/bin/bash
# GPU tests + c3/c2 bench lines of the in-tree build (batched cloud-mask loads), and a c5 A/B of
# single-instance builds: per-year plane stores as built vs only the last year's (store cost).
# Usage: bash profiles/r02_run16.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
echo "tests ok"
for c in c3 c2; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --e2e-steps 0 > $O/bench_$c.json \
    2> $O/bench_$c.err
  echo "bench $c ok"
done
for T in base st1; do
  LT_HIP_LIB=$R/profiles/build/exp_${T}_48.so timeout -k 10 300 python bench.py --config c5 --steps 3 \
    --no-cpu-baseline --e2e-steps 0 > $O/ab_${T}_c5.json 2> $O/ab_${T}_c5.err
  echo "ab $T ok"
done
