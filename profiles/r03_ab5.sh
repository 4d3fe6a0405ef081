#!/bin/bash
# A/B: uniform-row loads for unmasked scenes (+ the gapped x-set table), 3 waves per SIMD.
# Usage: bash profiles/r03_ab5.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
B="timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 --parity-sample 4096"
run() {  # name config lib
  LT_HIP_LIB=$3 $B --config $2 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],(d['parity_sample'] or {}).get('mismatched_values'))"
}
run c2_st0 c2 build/exp/c2_st0.so
run c2_uni c2 build/exp/c2_uni.so
run c2_uni_w3 c2 build/exp/c2_uni_w3.so
run c5_st0 c5 build/exp/c5_st0.so
run c5_uni c5 build/exp/c5_uni.so
run c2_st0b c2 build/exp/c2_st0.so
run c2_unib c2 build/exp/c2_uni.so
