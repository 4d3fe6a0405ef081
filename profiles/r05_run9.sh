#!/bin/bash
# r05 run 9: isolate the c3 parity mismatches of the LT_PASSB_SLOTS=0 JIT variant (tools/debug_mismatch.py)
set -e
OUT=${1:-gpurun_out/r05_run9}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
LT_JIT_DEFINES=LT_PASSB_SLOTS=0 timeout -k 10 300 python tools/debug_mismatch.py --config c3 --sample 100000 > $OUT/c3_noslots.json 2> $OUT/c3_noslots.err
timeout -k 10 300 python tools/debug_mismatch.py --config c3 --sample 100000 > $OUT/c3_slots.json 2> $OUT/c3_slots.err
