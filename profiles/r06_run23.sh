#!/bin/bash
# r06 run 23 (run 22 again, the step timed on its own stream: did it run beside the hold waves?): the failing LT_PASSB_SLOTS=0 c3 code object beside hold waves (tools/stagger.hip
# lt_hold, debug_mismatch.py --hold) that keep one slot per SIMD for the whole step, so the variant
# runs 3 waves per SIMD with its own code and allocation:
#   big1024    1,024 hold waves of the variant's size (128 VGPRs): the register file stays full
#   small1024  1,024 hold waves of 4 VGPRs: 3 variant waves per SIMD, 120 VGPRs of the file free
#   big2048    2,048 big hold waves: 2 variant waves per SIMD
# each reports where its hold waves ran (waves per SIMD over the SIMDs they used)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run23}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, extra args, seconds
  LT_JIT_OVERRIDE_DIR=$R/build/override/s0old LT_JIT_DEFINES=LT_PASSB_SLOTS=0 timeout -k 10 $3 \
    python tools/debug_mismatch.py --config c3 --sample 20000 --pixels 2000000 --no-rerun $2 \
    > $O/c3_$1.json 2> $O/c3_$1.err
  rc=$?
  echo "$1 rc=$rc"
  python -c "import json;d=json.load(open('$O/c3_$1.json'));print('$1',{k:v for k,v in d.items() if k not in ('examples','diff_first','diff_lane_hist')})" || true
  return $rc
}
dm big1024 "--hold 1024,40,1" 240 && dm small1024 "--hold 1024,40,0" 240 && \
dm big2048 "--hold 2048,40,1" 240
