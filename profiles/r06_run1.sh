#!/bin/bash
# r06 run 1: the LT_PASSB_SLOTS=0 c3 wrong-label variant (DESIGN.md § Wrong-result variants,
# VERDICT r05 item 1), three code objects of the same source at 2 Mpx (full occupancy), each run
# once, stdout and stderr kept:
#   s0   the variant as hiprtc builds it (control on this box)
#   s0p  byte-identical code, private segment declared 2048 B/lane instead of 320 / 368
#        (tools/co_patch.py): an access past the declared scratch slot would land in padding
#   s0fz every wait forced to zero (-mllvm -amdgpu-waitcnt-forcezero)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run1}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, override dir, seconds
  LT_JIT_OVERRIDE_DIR=$R/build/override/$2 LT_JIT_DEFINES=LT_PASSB_SLOTS=0 timeout -k 10 $3 \
    python tools/debug_mismatch.py --config c3 --sample 20000 --pixels 2000000 --no-rerun \
    > $O/c3_$1.json 2> $O/c3_$1.err
  rc=$?
  echo "$1 rc=$rc"
  tail -c 1500 $O/c3_$1.err
  python -c "import json;d=json.load(open('$O/c3_$1.json'));print('$1',{k:v for k,v in d.items() if k not in ('examples','diff_first')})" || true
  return $rc
}
dm s0 s0 200 && dm s0p s0p 200 && dm s0fz s0fz 400
