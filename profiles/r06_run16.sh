#!/bin/bash
# r06 run 16: does the failing LT_PASSB_SLOTS=0 c3 code object (build/override/s0old, run 15) read
# registers it never wrote? Before each of its two launches every SIMD's register file (512 VGPR /
# AGPR, SGPRs) is filled with a pattern (tools/reg_poison.hip via debug_mismatch.py --poison): code
# that reads only what it wrote cannot tell the patterns apart; code that reads a register before
# writing it in its first generation of waves gets the pattern there instead of a previous
# kernel's leftovers. Last: the product build with the same poisons (control: must stay 0).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run16}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, override dir ('' = product), poison, seconds
  if [ -n "$2" ]; then export LT_JIT_OVERRIDE_DIR=$R/build/override/$2 LT_JIT_DEFINES=LT_PASSB_SLOTS=0
  else unset LT_JIT_OVERRIDE_DIR LT_JIT_DEFINES; fi
  P=""; [ -n "$3" ] && P="--poison $3"
  timeout -k 10 $4 python tools/debug_mismatch.py --config c3 --sample 20000 --pixels 2000000 --no-rerun $P \
    > $O/c3_$1.json 2> $O/c3_$1.err
  rc=$?
  echo "$1 rc=$rc"
  python -c "import json;d=json.load(open('$O/c3_$1.json'));print('$1',{k:v for k,v in d.items() if k not in ('examples','diff_first','diff_lane_hist','jit')})" || true
  return $rc
}
dm s0old s0old "" 240 && dm s0old_p0 s0old 0 240 && dm s0old_pnan s0old 7ff80000 240 && \
dm s0old_pff s0old ffffffff 240 && dm s0old_p0ff s0old 0,ffffffff 240 && \
dm product_pff "" ffffffff 240 && dm product_p0ff "" 0,ffffffff 240
