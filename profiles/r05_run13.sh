#!/bin/bash
# r05 run 13: (1) HBM write rate of the per-year plane layout by store pattern (tools/store_pattern.hip);
# (2) the LT_PASSB_SLOTS=0 c3 nondeterminism: which stage (slot mask 1 / 2), stages serialised,
# and LDS poisoning (a read of a series slot the pixel did not write changes the result)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run13}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 build/bin/store_pattern > $O/store_pattern.json 2> $O/store_pattern.err
cat $O/store_pattern.err
dm() {  # name, defines, extra env
  env $3 LT_JIT_DEFINES=$2 timeout -k 10 300 python tools/debug_mismatch.py --config c3 --sample 100000 > $O/c3_$1.json 2> $O/c3_$1.err
  python -c "import json;d=json.load(open('$O/c3_$1.json'));print('$1',{k:v for k,v in d.items() if k!='examples'})"
}
dm poison_default LT_DEBUG_LDS_POISON=100
dm slots1 LT_PASSB_SLOTS=1
dm slots2 LT_PASSB_SLOTS=2
dm slots0_poison LT_PASSB_SLOTS=0,LT_DEBUG_LDS_POISON=100
dm slots0_sync LT_PASSB_SLOTS=0 LT_SYNC_LAUNCH=1
