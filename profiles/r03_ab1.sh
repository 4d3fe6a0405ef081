#!/bin/bash
# A/B of the fused load stage and the kernarg-pointer kernel arguments (profiles/build_variant.sh
# builds in build/exp): c2 (MAXY 32, 1 rule), c5 (MAXY 48), c3 (MAXY 32, 4 rules, masked).
# Usage: bash profiles/r03_ab1.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
B="timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 --parity-sample 4096"
run() {  # name config lib fused
  LT_HIP_LIB=$3 LT_FUSED_INDEX=$4 $B --config $2 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['parity_sample']['mismatched_values'])"
}
run c2_lean_f c2 build/exp/c2_lean.so 1
run c2_karg_f c2 build/exp/c2_karg.so 1
run c2_karg_nf c2 build/exp/c2_karg.so 0
run c5_karg_f c5 build/exp/c5_karg.so 1
run c5_karg_nf c5 build/exp/c5_karg.so 0
run c3_karg_f c3 build/exp/c3_karg.so 1
run c3_vb_f c3 build/exp/c3_vb.so 1
run c3_novb_f c3 build/exp/c3_novb.so 1
