#!/bin/bash
# A/B of the fused load stage's band layout (pixel-interleaved pairs: one 32-bit load per winner)
# against planar bands and the index raster path, plus c3 without the mask bit words and WB=16.
# Usage: bash profiles/r03_ab2.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
B="timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 --parity-sample 4096"
run() {  # name config lib fused layout
  LT_HIP_LIB=$3 LT_FUSED_INDEX=$4 LT_BAND_LAYOUT=$5 $B --config $2 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['parity_sample']['mismatched_values'])"
}
run c2_pair_pix c2 build/exp/c2_pair.so 1 pixel
run c2_pair_pla c2 build/exp/c2_pair.so 1 planar
run c2_pair_nf c2 build/exp/c2_pair.so 0 planar
run c2_wb16_pix c2 build/exp/c2_wb16.so 1 planar
run c5_pair_pix c5 build/exp/c5_pair.so 1 pixel
run c5_pair_nf c5 build/exp/c5_pair.so 0 planar
run c5_wb16 c5 build/exp/c5_wb16.so 1 planar
run c3_pair_novb_pix c3 build/exp/c3_pair_novb.so 1 pixel
run c3_karg_novb_pla c3 build/exp/c3_karg_novb.so 1 planar
run c3_karg_pla c3 build/exp/c3_karg.so 1 planar
run c3_wb16_novb c3 build/exp/c3_wb16_novb.so 1 planar
run c3_pair_novb_nf c3 build/exp/c3_pair_novb.so 0 planar
