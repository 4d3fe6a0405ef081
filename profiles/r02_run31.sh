#!/bin/bash
# Whole-scene parity of the round-2 final build on bench's c5 scene (40 years, line_cost 1, every
# trendline plane), in two halves. Usage: bash profiles/r02_run31.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
timeout -k 10 520 python -u tests/full_scene_check.py --config c5 --first 0 --last 24500000 \
  --out $O/full_c5_first.json > $O/full_c5_first.log 2>&1
echo "c5 first half ok"
timeout -k 10 520 python -u tests/full_scene_check.py --config c5 --first 24500000 \
  --out $O/full_c5_second.json > $O/full_c5_second.log 2>&1
echo "c5 second half ok"
