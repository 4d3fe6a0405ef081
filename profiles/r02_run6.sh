#!/bin/bash
# Per-phase PMC instruction counts: the analyze kernel cut after phase K (profiles/phases.sh
# builds) vs the full kernel, c2 (MAXY 32) and c5 (MAXY 48), one 16.8 Mpx launch each.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for MY in 32 48; do
  C=c2; [ $MY = 48 ] && C=c5
  for K in 0 1 2 3 full; do
    LT_HIP_LIB=$R/profiles/build/liblt_cut${MY}_$K.so timeout -s KILL 120 rocprofv3 --pmc \
      SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
      SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/cut${MY}_$K -o run -- \
      python3 $R/bench.py --config $C --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline \
      --e2e-steps 0 > $O/cut${MY}_$K.log 2>&1
    echo "cut $MY $K ok"
  done
done
