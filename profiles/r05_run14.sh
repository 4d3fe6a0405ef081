#!/bin/bash
# r05 run 14: (1) the LT_PASSB_SLOTS=0 c3 mismatches at lower analyze occupancy (LDS padding:
# co-resident waves interfering?); (2) c5: where the per-year stores' time goes — the plane stores
# redirected to the pixel's year-0 row (same instructions, ~1/Y of the bytes reach HBM), NT or not
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run14}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, defines
  LT_JIT_DEFINES=$2 timeout -k 10 300 python tools/debug_mismatch.py --config c3 --sample 100000 > $O/c3_$1.json 2> $O/c3_$1.err
  python -c "import json;d=json.load(open('$O/c3_$1.json'));print('$1',{k:v for k,v in d.items() if k!='examples'})"
}
dm slots0_pad40k LT_PASSB_SLOTS=0,LT_DEBUG_LDS_PAD=40960
dm slots0_pad16k LT_PASSB_SLOTS=0,LT_DEBUG_LDS_PAD=16384
b5() {  # name, defines
  LT_JIT_DEFINES=$2 timeout -k 10 300 python bench.py --config c5 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 --parity-sample 0 > $O/c5_$1.json 2> $O/c5_$1.err
  python -c "import json;d=json.load(open('$O/c5_$1.json'));print('c5 $1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'])"
}
b5 default ""
b5 sink_nt LT_AB_YEAR_SINK=1
b5 sink_l2 LT_AB_YEAR_SINK=2
b5 nostores LT_AB_NO_YEAR_STORES=1
b5 nostores2 LT_AB_NO_YEAR_STORES=2
