#!/bin/bash
# A/B of single-instance builds (profiles/build/exp_<tag>_<MAXY>.so): c2 (MAXY 32) and c5
# (MAXY 48) bench lines and one PMC pass each. Usage: bash profiles/ab_libs.sh <outdir> <tag>...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1; shift
mkdir -p $O
for TAG in "$@"; do
  for MY in 32 48; do
    C=c2; [ $MY = 48 ] && C=c5
    L=$R/profiles/build/exp_${TAG}_$MY.so
    [ -f $L ] || continue
    (cd $R && LT_HIP_LIB=$L timeout -k 10 300 python bench.py --config $C --steps 5 \
      --no-cpu-baseline --e2e-steps 0 > $O/${TAG}_$C.json 2> $O/${TAG}_$C.err)
    (cd /tmp && export TMPDIR=/tmp && LT_HIP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc \
      SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
      --output-format csv -d $O/pmc_${TAG}_$C -o run -- python3 $R/bench.py --config $C \
      --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 \
      > $O/pmc_${TAG}_$C.log 2>&1)
    echo "$TAG $C ok"
  done
done
