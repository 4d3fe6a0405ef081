#!/bin/bash
# r05 run 11: the c3 LT_PASSB_SLOTS=0 mismatches with the stages serialised (LT_SYNC_LAUNCH=1)
set -e
OUT=${1:-gpurun_out/r05_run11}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
LT_SYNC_LAUNCH=1 LT_JIT_DEFINES=LT_PASSB_SLOTS=0 timeout -k 10 300 python tools/debug_mismatch.py --config c3 --sample 100000 > $OUT/c3_slots0_sync.json 2> $OUT/c3_slots0_sync.err
LT_JIT_DEFINES=LT_PASSB_SLOTS=0 timeout -k 10 300 python tools/debug_mismatch.py --config c3 --sample 100000 > $OUT/c3_slots0.json 2> $OUT/c3_slots0.err
