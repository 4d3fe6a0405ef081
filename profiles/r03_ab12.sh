#!/bin/bash
# A/B: winner-pick batch LT_WB = 8 (product) vs 16 (fewer load round trips per wave: 3 instead of 5
# batches for 40 years, 2 instead of 4 for 30), c5 and c2 instances.
# Usage: bash profiles/r03_ab12.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
B="timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 --parity-sample 4096"
run() {  # name config lib
  LT_HIP_LIB=build/exp/$3.so $B --config $2 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],(d['parity_sample'] or {}).get('mismatched_values'))"
}
run c5_wb8 c5 c5_wb8; run c5_wb16 c5 c5_wb16; run c5_wb8b c5 c5_wb8; run c5_wb16b c5 c5_wb16
run c2_wb8 c2 c2_wb8; run c2_wb16 c2 c2_wb16; run c2_wb8b c2 c2_wb8; run c2_wb16b c2 c2_wb16
