#!/bin/bash
# Same-box c5 A/B: u8 planes written per year by the analyze kernel (base) vs from year flags by
# year_flags_kernel (yf), alternated twice. Usage: bash profiles/r02_run21.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
for i in 1 2; do
for T in base yf; do
  LT_HIP_LIB=$R/profiles/build/exp_${T}_48.so timeout -k 10 300 python bench.py --config c5 --steps 3 \
    --no-cpu-baseline --e2e-steps 0 > $O/ab_${T}_c5_$i.json 2> $O/ab_${T}_c5_$i.err
  echo "ab $T $i ok"
done
done
