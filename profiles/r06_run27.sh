#!/bin/bash
# r06 run 27: does a wave of the failing c3 code object write past its 128-VGPR allocation?
# Guard waves (tools/reg_guard.hip: 128 VGPRs each, every register filled with 0xA5A5_00kk, held for
# the whole step in SALU-only code, then checked) run beside the step (debug_mismatch.py --guard);
# a changed register in a guard is a write from another wave into its allocation.
#   g1024_s0old   failing object (128 VGPRs), 1 guard per SIMD
#   g2048_s0old   failing object, 2 guards per SIMD
#   g2048_v136    the same code at 136 VGPRs (bit-exact), 2 guards per SIMD
#   g2048_prod    the product c3 instance (128 VGPRs), 2 guards per SIMD
#   g2048_none    the guards beside a step of the c2 product (control for the guard itself)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run27}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, env, config, extra args, seconds
  env $2 timeout -k 10 $5 \
    python tools/debug_mismatch.py --config $3 --sample 20000 --pixels 2000000 --no-rerun $4 \
    > $O/$1.json 2> $O/$1.err
  rc=$?
  echo "$1 rc=$rc"
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',d['step2_differs_from_step1_pixels'],d['mismatching_pixels'],d['step_wall_ms'],json.dumps(d['guard_found'])[:1500])" || true
  return $rc
}
S0="LT_JIT_OVERRIDE_DIR=$R/build/override/s0old LT_JIT_DEFINES=LT_PASSB_SLOTS=0"
V136="LT_JIT_OVERRIDE_DIR=$R/build/override/s0old_v136a136 LT_JIT_DEFINES=LT_PASSB_SLOTS=0"
dm g1024_s0old "$S0" c3 "--guard 1024,40" 240 && dm g2048_s0old "$S0" c3 "--guard 2048,40" 240 && \
dm g2048_v136 "$V136" c3 "--guard 2048,40" 240 && dm g2048_prod "LT_NONE=1" c3 "--guard 2048,40" 240 && \
dm g2048_none "LT_NONE=1" c2 "--guard 2048,40" 240
