#!/bin/bash
# GPU tests + bench lines (c5, c2, c3) of the in-tree build with nontemporal plane stores, and the
# non-integer index cost (profiles/float_index.py). Usage: bash profiles/r02_run25.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
echo "tests ok"
for c in c5 c2 c3; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --e2e-steps 0 > $O/bench_$c.json \
    2> $O/bench_$c.err
  echo "bench $c ok"
done
timeout -k 10 600 python -u profiles/float_index.py $O/float_index.json > $O/float_index.log 2>&1
echo "float index ok"
