#!/bin/bash
# Whole-scene parity of the certified labels-only path: every pixel of bench's c2 scene (49 Mpx,
# label rasters only, as bench.py requests them) re-analysed by the oracle.
# Usage: bash profiles/r02_run23.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
timeout -k 10 1000 python -u tests/full_scene_check.py --config c2 --labels-only \
  --out $O/full_c2_labels.json > $O/full_c2_labels.log 2>&1
echo "c2 labels-only ok"
