#!/bin/bash
# r06 run 21: does the failing LT_PASSB_SLOTS=0 c3 code object (rebuilt from the round-5 sources,
# tools/co_audit.py: profiles/r06_audit) need its first generation of waves to start together?
# A blocker kernel (tools/stagger.hip) holds every wave slot (4,096 waves of the variant's size)
# for START ms after its own start and then frees them over SPREAD ms; the debug_mismatch step is
# queued behind it on another stream, so its waves take the slots in the order they are freed.
#   s0old        control, no blocker
#   st_sync      blocker, every slot freed at once (a synchronised first generation again)
#   st_0.3       slots freed over 0.3 ms (about three wave lifetimes of this launch)
#   st_1         slots freed over 1 ms
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run21}
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
dm s0old "" 240 && dm st_sync "--stagger 20,0" 240 && dm st_0.3 "--stagger 20,0.3" 240 && \
dm st_1 "--stagger 20,1" 240
