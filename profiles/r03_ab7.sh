#!/bin/bash
# A/B: the c3 instance (MAXY 32, 4 rules, int16) at 4 waves/SIMD (128 VGPRs, 109 spilled) vs 3
# waves/SIMD (162 VGPRs, no spills). Usage: bash profiles/r03_ab7.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
B="timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 --parity-sample 4096"
for V in c3_w4 c3_w3 c3_w4 c3_w3; do
  LT_HIP_LIB=build/exp/$V.so $B --config c3 > $O/bench_$V.json 2> $O/bench_$V.err
  python -c "import json;d=json.load(open('$O/bench_$V.json'));print('$V',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],(d['parity_sample'] or {}).get('mismatched_values'))"
done
