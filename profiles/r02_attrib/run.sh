#!/bin/bash
# Attribution: c5 with and without its per-year trendline planes; per-phase PMC instruction counts
# of the analyze kernel (profiles/phases.sh cut builds) for c2 (MAXY 32) and c5 (MAXY 48); VMEM
# instruction counts of the full c5 kernel. Usage: bash profiles/r02_run11.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --e2e-steps 0 > $O/bench_c5.json 2> $O/bench_c5.err
timeout -k 10 300 python bench.py --config c5 --no-trendline --no-cpu-baseline --e2e-steps 0 \
  > $O/bench_c5_notl.json 2> $O/bench_c5_notl.err
echo "bench ok"
cd /tmp && export TMPDIR=/tmp
for MY in 32 48; do
  C=c2; [ $MY = 48 ] && C=c5
  for K in 0 1 2 3 full; do
    LT_HIP_LIB=$R/profiles/build/liblt_cut${MY}_$K.so timeout -s KILL 120 rocprofv3 --pmc \
      SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
      --output-format csv -d $O/cut_${C}_$K -o run -- python3 $R/bench.py --config $C \
      --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 > $O/cut_${C}_$K.log 2>&1
    echo "cut $C $K ok"
  done
done
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES \
  --output-format csv -d $O/vmem_c5 -o run -- python3 $R/bench.py --config c5 \
  --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 > $O/vmem_c5.log 2>&1
echo "vmem ok"
