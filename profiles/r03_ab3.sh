#!/bin/bash
# A/B: the fused load stage with the streamlined arithmetic (one bit-field extract per value for
# 'B1 - B2') against the index raster path; c3 with and without the mask bit words; then the c5
# phase cuts and the 4.2 Mpx job.
# Usage: bash profiles/r03_ab3.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
B="timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 --parity-sample 4096"
run() {  # name config lib fused layout
  LT_HIP_LIB=$3 LT_FUSED_INDEX=$4 LT_BAND_LAYOUT=$5 $B --config $2 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],(d['parity_sample'] or {}).get('mismatched_values'))"
}
run c2_fast_pix c2 build/exp/c2_fast.so 1 pixel
run c2_fast_nf c2 build/exp/c2_fast.so 0 planar
run c2_fast_pix2 c2 build/exp/c2_fast.so 1 pixel
run c5_fast_pix c5 build/exp/c5_fast.so 1 pixel
run c5_fast_nf c5 build/exp/c5_fast.so 0 planar
run c3_fast_novb_pix c3 build/exp/c3_fast_novb.so 1 pixel
run c3_fast_vb_pix c3 build/exp/c3_fast_vb.so 1 pixel
run c3_fast_novb_nf c3 build/exp/c3_fast_novb.so 0 planar
for K in 0 1 2 3; do
  run c5_cut$K c5 build/exp/liblt_cut48_$K.so 1 pixel || true
done
timeout -k 10 600 python profiles/job_scale.py 2048 2048 30 $O/job_4mpx.json > $O/job_4mpx.log 2>&1
python -c "import json;d=json.load(open('$O/job_4mpx.json'));print('job', d['times'], d['sample_mismatches'])"
