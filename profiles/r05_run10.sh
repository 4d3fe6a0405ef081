#!/bin/bash
# r05 run 10: which stage's Pass B variant gives the c3 mismatches, and are they deterministic
set -e
OUT=${1:-gpurun_out/r05_run10}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for v in 0 1 2; do
  LT_JIT_DEFINES=LT_PASSB_SLOTS=$v timeout -k 10 300 python tools/debug_mismatch.py --config c3 --sample 100000 > $OUT/c3_slots$v.json 2> $OUT/c3_slots$v.err
done
