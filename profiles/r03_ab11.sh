#!/bin/bash
# A/B: the DP early exit tested against the largest start bound priced so far in the column (bmax)
# vs the current start's bound (base): c2, c3, c5; outputs must not change (parity sample 16k).
# Usage: bash profiles/r03_ab11.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
B="timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 --parity-sample 16384"
run() {  # name config lib
  LT_HIP_LIB=build/exp/$3.so $B --config $2 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],(d['parity_sample'] or {}).get('mismatched_values'))"
}
run c2_base c2 c2_ks30; run c2_bmax c2 c2_bmax; run c2_base2 c2 c2_ks30; run c2_bmax2 c2 c2_bmax
run c5_base c5 liblt_cut48_full; run c5_bmax c5 c5_bmax
run c3_base c3 c3_base; run c3_bmax c3 c3_bmax
