#!/bin/bash
# r06 run 2: the LT_PASSB_SLOTS=0 c3 variant at 2 Mpx, once each:
#   s0v168 / s0v248  byte-identical code, the analyze kernel's VGPR allocation raised to 168 / 248
#                    (tools/co_patch.py --vgprs): 3 / 2 waves per SIMD with LDS and scratch as is
#   s0chk            the variant + LT_DEBUG_FIT_CHECK: a lane whose applied x-set table entry is not
#                    its own x-set's (f.m != m or f.rc != 0) sets status bit 256 in pass B
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run2}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, override dir, defines
  LT_JIT_OVERRIDE_DIR=$R/build/override/$2 LT_JIT_DEFINES=$3 timeout -k 10 200 \
    python tools/debug_mismatch.py --config c3 --sample 20000 --pixels 2000000 --no-rerun \
    > $O/c3_$1.json 2> $O/c3_$1.err
  rc=$?
  echo "$1 rc=$rc"
  python -c "import json;d=json.load(open('$O/c3_$1.json'));print('$1',{k:v for k,v in d.items() if k not in ('examples','diff_first','diff_lane_hist')}); print([(e['pixel'],e['fields'],e['got'].get('status')) for e in d['examples']])" || true
  return $rc
}
dm s0v168 s0v168 LT_PASSB_SLOTS=0 && dm s0v248 s0v248 LT_PASSB_SLOTS=0 && dm s0chk s0chk LT_PASSB_SLOTS=0,LT_DEBUG_FIT_CHECK=1
