#!/bin/bash
# One PMC pass (instruction counts, cycles) per single-instance build profiles/build/exp_<tag>_32.so
# on one 16.8 Mpx c2 launch. Usage: bash profiles/pmc_libs.sh <outdir> <tag>...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for TAG in "$@"; do
  LT_HIP_LIB=$R/profiles/build/exp_${TAG}_32.so timeout -s KILL 120 rocprofv3 --pmc \
    SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $O/pmc_$TAG -o run -- python3 $R/bench.py --config c2 \
    --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 > $O/pmc_$TAG.log 2>&1
  echo "$TAG ok"
done
