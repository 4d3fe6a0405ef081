#!/bin/bash
# c2 occupancy A/B (single-instance builds: 4 vs 5 waves/SIMD) and c5 per-phase PMC counts of the
# analyze kernel cut after each phase (profiles/phases.sh 48). Usage: bash profiles/r02_run15.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
for T in base w5; do
  LT_HIP_LIB=$R/profiles/build/exp_${T}_32.so timeout -k 10 300 python bench.py --config c2 --steps 5 \
    --no-cpu-baseline --e2e-steps 0 > $O/ab_${T}_c2.json 2> $O/ab_${T}_c2.err
  echo "ab $T ok"
done
cd /tmp && export TMPDIR=/tmp
for K in 0 1 2 3 full; do
  LT_HIP_LIB=$R/profiles/build/liblt_cut48_$K.so timeout -s KILL 120 rocprofv3 --pmc \
    SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/cut48_$K -o run -- \
    python3 $R/bench.py --config c5 --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline \
    --e2e-steps 0 > $O/cut48_$K.log 2>&1
  echo "cut 48 $K ok"
done
