#!/bin/bash
# r05 run 16: (1) the LT_PASSB_SLOTS=0 c3 mismatches at 2 Mpx, hiprtc build vs every wait forced
# to zero (run 15's forcezero run at 49 Mpx printed nothing for 180 s); (2) the overlap probe incl.
# CU-masked analyze; (3) c5 as one launch per scene, XCD-aware block remap, plain plane stores;
# c2 with the remap; c3 / c4 at this build. (Second attempt: the forcezero run finished both
# steps at 2 Mpx but its isolation reruns ran past the step limit: now --no-rerun, 20k sample)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run16}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, override dir, pixels
  LT_JIT_OVERRIDE_DIR=$R/build/override/$2 LT_JIT_DEFINES=LT_PASSB_SLOTS=0 timeout -k 10 150 python tools/debug_mismatch.py --config c3 --sample 20000 --pixels $3 $4 > $O/c3_$1.json 2> $O/c3_$1.err
  python -c "import json;d=json.load(open('$O/c3_$1.json'));print('$1',{k:v for k,v in d.items() if k!='examples'})"
}
dm s0_override_2m s0 2000000 ""
timeout -k 10 170 python tools/overlap_probe.py > $O/overlap_probe.json 2> $O/overlap_probe.err
cat $O/overlap_probe.json
b() {  # name, defines, args
  LT_JIT_DEFINES=$2 timeout -k 10 170 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
b c5_whole "" "--config c5 --tile 49000000"
b c5 "" "--config c5"
b c5_xcd LT_XCD_REMAP=1 "--config c5"
b c5_plain LT_YEAR_NT=0 "--config c5"
b c2 "" "--config c2"
b c2_xcd LT_XCD_REMAP=1 "--config c2"
b c3 "" "--config c3"
b c4 "" "--config c4"
dm s0_forcezero_2m s0fz 2000000 --no-rerun
