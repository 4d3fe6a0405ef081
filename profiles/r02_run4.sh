#!/bin/bash
# Phase stamps of the analyze kernel (c2, c3, c5), then the first half of the c5 whole-scene check.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$1
mkdir -p $R/$O
cd $R
timeout -k 10 300 python -u profiles/stamps.py c2 c3 c5 > $R/$O/stamps.json 2> $R/$O/stamps.err
echo "stamps ok"
timeout -k 10 800 python -u tests/full_scene_check.py --config c5 --first 0 --last 24500000 \
  --threads 16 --out $R/$O/full_c5_first_half.json > $R/$O/full_c5_first.log 2>&1
echo "c5 first half ok"
