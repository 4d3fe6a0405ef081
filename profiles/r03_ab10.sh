#!/bin/bash
# A/B: c5 with the unmasked raw rows (val_raw, winner) stored by the despike scan (c5_late) vs in
# the winner pick (liblt_cut48_full, the previous product body); then the kScreen A/B on c2
# (profiles/r03_ab9.sh). Usage: bash profiles/r03_ab10.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
B="timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 --parity-sample 16384"
for V in liblt_cut48_full c5_late liblt_cut48_full c5_late; do
  LT_HIP_LIB=build/exp/$V.so $B --config c5 > $O/bench_$V.json 2> $O/bench_$V.err
  python -c "import json;d=json.load(open('$O/bench_$V.json'));print('$V',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],(d['parity_sample'] or {}).get('mismatched_values'))"
done
bash profiles/r03_ab9.sh $1/ab9
