#!/bin/bash
# GPU tests (incl. non-integer / large-offset series, two scenes on two streams) and a 4 Mpx range
# of the c5 whole-scene check (all trendline planes). Usage: bash profiles/r02_run3.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$1
mkdir -p $R/$O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $R/$O/gpu_tests.log 2>&1
echo "tests ok"
timeout -k 10 600 python -u tests/full_scene_check.py --config c5 --first 0 --last 4194304 \
  --threads 16 --out $R/$O/full_c5_0_4M.json > $R/$O/full_c5.log 2>&1
echo "c5 range ok"
