#!/bin/bash
# A/B: the c3 launch (3 rules) on a 4-rule instance (99 spilled VGPRs) vs a 3-rule instance (66).
# Usage: bash profiles/r03_ab8.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
B="timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 --parity-sample 4096"
for V in c3_r4 c3_r3 c3_r4 c3_r3; do
  LT_HIP_LIB=build/exp/$V.so $B --config c3 > $O/bench_$V.json 2> $O/bench_$V.err
  python -c "import json;d=json.load(open('$O/bench_$V.json'));print('$V',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],(d['parity_sample'] or {}).get('mismatched_values'))"
done
