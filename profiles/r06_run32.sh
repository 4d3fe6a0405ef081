#!/bin/bash
# r06 run 32: the failing c3 code object (128 VGPRs) at 1 wave per SIMD beside 3 guard waves
# (tools/reg_guard.hip, every register 0xA5A5_00kk) per SIMD, and at 2 beside 2: is another wave
# of the variant needed, and do the wrong values carry the guards' pattern? The mismatch examples
# are kept whole (their bits are checked on the host).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run32}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, env, extra args, seconds
  env $2 timeout -k 10 $4 \
    python tools/debug_mismatch.py --config c3 --sample 20000 --pixels 2000000 --no-rerun $3 \
    > $O/$1.json 2> $O/$1.err
  rc=$?
  echo "$1 rc=$rc"
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',d['step2_differs_from_step1_pixels'],d['mismatching_pixels'],d['step_wall_ms'],json.dumps(d['guard_found'])[:600])" || true
  return $rc
}
S0="LT_JIT_OVERRIDE_DIR=$R/build/override/s0old LT_JIT_DEFINES=LT_PASSB_SLOTS=0"
dm g3072_s0old "$S0" "--guard 3072,60" 240 && dm g2048_s0old_b "$S0" "--guard 2048,60" 240
