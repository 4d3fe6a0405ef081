#!/bin/bash
# Same-box c2 A/B of the DP's window pair: both starts priced then one exit test (base) vs start
# j-2 first with its own exit test, j-3 only if some lane goes on (ex1); parity check of each on a
# 131k-pixel c2 tile, then one PMC instruction pass each. Usage: bash profiles/r02_run27.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
for T in base ex1; do
  LT_HIP_LIB=$R/profiles/build/exp_${T}_32.so timeout -k 10 120 python3 profiles/ab_check.py 131072 11 30 10 \
    > $O/check_$T.log 2>&1
  echo "check $T ok"
done
for i in 1 2; do
for T in base ex1; do
  LT_HIP_LIB=$R/profiles/build/exp_${T}_32.so timeout -k 10 300 python bench.py --config c2 --steps 3 \
    --no-cpu-baseline --e2e-steps 0 > $O/ab_${T}_c2_$i.json 2> $O/ab_${T}_c2_$i.err
  echo "ab $T $i ok"
done
done
cd /tmp && export TMPDIR=/tmp
for T in base ex1; do
  LT_HIP_LIB=$R/profiles/build/exp_${T}_32.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU \
    SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$T -o run -- python3 \
    $R/bench.py --config c2 --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 \
    > $O/pmc_$T.log 2>&1
  echo "pmc $T ok"
done
