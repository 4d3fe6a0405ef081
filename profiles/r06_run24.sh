#!/bin/bash
# r06 run 24: the failing LT_PASSB_SLOTS=0 c3 code object with its VGPR allocation raised in place
# (co_patch.py --vgprs: 168 = 3 variant waves per SIMD, 248 = 2; identical code; both bit-exact
# alone in run 2), now beside small hold waves (4 VGPRs, tools/stagger.hip lt_hold) that fill the
# SIMDs' remaining wave slots: does the failure need 4 resident waves per SIMD of any kernel?
#   v168            control (3 waves per SIMD)
#   v168_small1024  + 1 small hold wave per SIMD (4 waves per SIMD)
#   v248_small2048  + 2 per SIMD (4 waves per SIMD)
#   v248_small1024  + 1 per SIMD (3 waves per SIMD)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run24}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, override, extra args, seconds
  LT_JIT_OVERRIDE_DIR=$R/build/override/$2 LT_JIT_DEFINES=LT_PASSB_SLOTS=0 timeout -k 10 $4 \
    python tools/debug_mismatch.py --config c3 --sample 20000 --pixels 2000000 --no-rerun $3 \
    > $O/c3_$1.json 2> $O/c3_$1.err
  rc=$?
  echo "$1 rc=$rc"
  python -c "import json;d=json.load(open('$O/c3_$1.json'));print('$1',{k:v for k,v in d.items() if k not in ('examples','diff_first','diff_lane_hist')})" || true
  return $rc
}
dm v168 s0old_v168 "" 240 && dm v168_small1024 s0old_v168 "--hold 1024,40,0" 240 && \
dm v248_small2048 s0old_v248 "--hold 2048,40,0" 240 && dm v248_small1024 s0old_v248 "--hold 1024,40,0" 240
