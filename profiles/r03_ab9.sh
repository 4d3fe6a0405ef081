#!/bin/bash
# A/B: the DP's screening half-width kScreen (lt_pixel.h) at 2^-30 (product) vs 2^-34 vs 2^-38, c2
# instance: speed, deferred pixels per tile, parity sample. Usage: bash profiles/r03_ab9.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
B="timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 --parity-sample 16384"
for V in c2_ks30 c2_ks34 c2_ks38 c2_ks30 c2_ks38; do
  LT_HIP_LIB=build/exp/$V.so $B --config c2 > $O/bench_$V.json 2> $O/bench_$V.err
  python -c "import json;d=json.load(open('$O/bench_$V.json'));print('$V',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage'],(d['parity_sample'] or {}).get('mismatched_values'))"
done
