#!/bin/bash
# GPU tests + c3 bench of the in-tree build (cloud-mask loads 8 in flight), and a c5 A/B of
# single-instance builds: as built, x-set factors computed inline (no table loads in the fits),
# and only the last year's planes stored. Usage: bash profiles/r02_run17.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --e2e-steps 0 > $O/bench_c3.json \
  2> $O/bench_c3.err
echo "bench c3 ok"
for T in base noxt st1; do
  LT_HIP_LIB=$R/profiles/build/exp_${T}_48.so timeout -k 10 300 python bench.py --config c5 --steps 3 \
    --no-cpu-baseline --e2e-steps 0 > $O/ab_${T}_c5.json 2> $O/ab_${T}_c5.err
  echo "ab $T ok"
done
