#!/bin/bash
# Profile the current build on the GPU box (from the repo root):
#   kernel trace + stats of the default bench line, then the PMC passes of one c2 tile.
# Usage: bash profiles/collect.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 > $OUT/bench_default.json 2> $OUT/bench_default.err
echo "kernel trace ok"
cd $R
timeout -k 10 600 bash profiles/pmc_passes.sh ${1}/pmc --pixels 16777216 --steps 1 --warmup 0
python3 profiles/summarize_pmc.py $OUT/pmc $OUT/pmc_c2.json 16777216 > /dev/null
echo "pmc ok"
