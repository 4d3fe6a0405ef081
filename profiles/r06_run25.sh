#!/bin/bash
# r06 run 25: the failing code object's analyze kernel with its allocation raised by one granule
# (136 VGPRs, 3 waves per SIMD) and its AGPR split moved (co_patch.py --vgprs / --accum, identical
# code): does the failure follow the 128-VGPR allocation, or an allocation without AGPRs?
#   s0old         control (128 VGPRs, accum_offset 128: no AGPRs)
#   v136a128      136 VGPRs, accum_offset 128 (8 AGPRs)
#   v136a136      136 VGPRs, accum_offset 136 (no AGPRs)
#   v136a136_s    the same + 1 small hold wave per SIMD (4 waves per SIMD)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run25}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, override, extra args, seconds
  LT_JIT_OVERRIDE_DIR=$R/build/override/$2 LT_JIT_DEFINES=LT_PASSB_SLOTS=0 timeout -k 10 $4 \
    python tools/debug_mismatch.py --config c3 --sample 20000 --pixels 2000000 --no-rerun $3 \
    > $O/c3_$1.json 2> $O/c3_$1.err
  rc=$?
  echo "$1 rc=$rc"
  python -c "import json;d=json.load(open('$O/c3_$1.json'));print('$1',d['step2_differs_from_step1_pixels'],d['mismatching_pixels'],d['step_wall_ms'],d['hold_where'])" || true
  return $rc
}
dm s0old s0old "" 240 && dm v136a128 s0old_v136a128 "" 240 && dm v136a136 s0old_v136a136 "" 240 && \
dm v136a136_s s0old_v136a136 "--hold 1024,40,0" 240
