#!/bin/bash
# GPU tests + c2/c3/c5 lines of the in-tree build (DP window starts priced one at a time), and a
# same-box c2 A/B of nontemporal label/status stores (ntl) and of one start per deep-loop
# iteration (ex2) against it (base), with parity checks.
# Usage: bash profiles/r02_run28.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
echo "tests ok"
for c in c2 c3 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --e2e-steps 0 > $O/bench_$c.json \
    2> $O/bench_$c.err
  echo "bench $c ok"
done
for T in ntl ex2; do
  LT_HIP_LIB=$R/profiles/build/exp_${T}_32.so timeout -k 10 120 python3 profiles/ab_check.py 131072 11 30 \
    10 > $O/check_$T.log 2>&1
  echo "check $T ok"
done
for i in 1 2; do
for T in base ntl ex2; do
  LT_HIP_LIB=$R/profiles/build/exp_${T}_32.so timeout -k 10 300 python bench.py --config c2 --steps 3 \
    --no-cpu-baseline --e2e-steps 0 > $O/ab_${T}_c2_$i.json 2> $O/ab_${T}_c2_$i.err
  echo "ab $T $i ok"
done
done
