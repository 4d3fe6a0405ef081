#!/bin/bash
# Whole-scene parity of the round-2 final build, labels-only (the certified path, as bench.py runs
# c2/c3): every pixel of bench's c2 and c3 scenes against the oracle. Usage: bash profiles/r02_run30.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
for C in c2 c3; do
  timeout -k 10 540 python -u tests/full_scene_check.py --config $C --labels-only \
    --out $O/full_${C}_labels.json > $O/full_${C}_labels.log 2>&1
  echo "$C labels-only ok"
done
