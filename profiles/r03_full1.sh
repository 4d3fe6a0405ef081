#!/bin/bash
# Whole-scene parity at the round-3 build: every pixel of bench's c2 and c3 scenes (labels only,
# the fields bench.py requests: the certified labels path, fused load stage, mask bit planes).
# Usage: bash profiles/r03_full1.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
for C in c2 c3; do
  timeout -k 10 540 python -u tests/full_scene_check.py --config $C --labels-only \
    --out $O/full_${C}_labels_only.json > $O/full_$C.log 2>&1
  tail -2 $O/full_$C.log
done
