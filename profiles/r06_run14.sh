#!/bin/bash
# r06 run 14: the LT_PASSB_SLOTS=0 c3 wrong-label variant at this build, 2 Mpx (full occupancy),
# code objects that differ from the variant's only in how much their s_waitcnt instructions wait
# (tools/co_patch.py --waitcnt: the counter field set to 0 in place, every address unchanged):
#   s6      the variant as hiprtc builds it (control on this box)
#   s6lgkm  every wait of lt_jit_analyze also waits for all LDS / scalar-memory accesses
#   s6vm    every wait of lt_jit_analyze also waits for all vector-memory accesses
# A stricter wait cannot change what correct code computes; a variant that turns bit-exact names
# the kind of access whose result was used too early.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run14}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, override dir, seconds
  LT_JIT_OVERRIDE_DIR=$R/build/override/$2 LT_JIT_DEFINES=LT_PASSB_SLOTS=0 timeout -k 10 $3 \
    python tools/debug_mismatch.py --config c3 --sample 20000 --pixels 2000000 --no-rerun \
    > $O/c3_$1.json 2> $O/c3_$1.err
  rc=$?
  echo "$1 rc=$rc"
  python -c "import json;d=json.load(open('$O/c3_$1.json'));print('$1',{k:v for k,v in d.items() if k not in ('examples','diff_first','diff_lane_hist')})" || true
  return $rc
}
dm s6 s6 240 && dm s6lgkm s6lgkm 240 && dm s6vm s6vm 300
