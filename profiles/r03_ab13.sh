#!/bin/bash
# A/B: nontemporal loads of the winners' band pairs (read once; keeps the x-set table L2-hot) vs
# plain loads, c5 and c2. Usage: bash profiles/r03_ab13.sh <outdir under gpurun_out>
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
run c5_base c5 c5_wb8; run c5_ntl c5 c5_ntl; run c5_base2 c5 c5_wb8; run c5_ntl2 c5 c5_ntl
run c2_base c2 c2_wb8; run c2_ntl c2 c2_ntl; run c2_base2 c2 c2_wb8; run c2_ntl2 c2 c2_ntl
