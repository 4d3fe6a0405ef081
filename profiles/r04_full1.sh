#!/bin/bash
# Round-4 whole-scene parity at the final build: every pixel of bench's c2 and c3 scenes
# (labels only, the certified JIT path bench times) against the oracle.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
for C in c2 c3; do
  timeout -k 10 560 python -u tests/full_scene_check.py --config $C --labels-only \
    --out $O/full_${C}_labels_only.json > $O/full_$C.log 2>&1
  tail -2 $O/full_$C.log
done
