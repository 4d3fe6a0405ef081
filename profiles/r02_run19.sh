#!/bin/bash
# Final PMC passes of the current build (profiles/pmc_passes.sh: sq1, sq2, fetch, write) for one
# 16.8 Mpx launch of c2, c3 and c5, and the kernel-trace stats of the default bench line.
# Usage: bash profiles/r02_run19.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$1
cd $R
for C in c2 c3 c5; do
  timeout -k 10 600 bash profiles/pmc_passes.sh $O/pmc_$C --config $C --pixels 16777216 --steps 1 \
    --warmup 0 --e2e-steps 0
  python3 profiles/summarize_pmc.py $R/$O/pmc_$C $R/$O/pmc_$C.json 16777216 > /dev/null
  echo "pmc $C ok"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $R/$O/kt_bench.json \
  2> $R/$O/kt_bench.err
echo "kernel trace ok"
cd $R
for T in base nou8; do
  LT_HIP_LIB=$R/profiles/build/exp_${T}_48.so timeout -k 10 300 python bench.py --config c5 --steps 3 \
    --no-cpu-baseline --e2e-steps 0 > $O/ab_${T}_c5.json 2> $O/ab_${T}_c5.err
  echo "ab $T ok"
done
