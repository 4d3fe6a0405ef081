#!/bin/bash
# Round-4 whole-scene parity at the final build: every pixel of bench's c5 scene (all fifteen
# fields), in two halves.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 560 python -u tests/full_scene_check.py --config c5 --first 0 --last 24500000 \
  --out $O/full_c5_first_half.json > $O/full_c5a.log 2>&1
tail -2 $O/full_c5a.log
timeout -k 10 560 python -u tests/full_scene_check.py --config c5 --first 24500000 --last 49000000 \
  --out $O/full_c5_second_half.json > $O/full_c5b.log 2>&1
tail -2 $O/full_c5b.log
