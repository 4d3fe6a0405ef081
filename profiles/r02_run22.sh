#!/bin/bash
# Local job runner at scale: a 2048 x 2048 (4.2 Mpx) 30-year labels-only job and a 1024 x 1024
# job with every trendline raster. Usage: bash profiles/r02_run22.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
timeout -k 10 900 python -u profiles/job_scale.py 2048 2048 30 $O/job_4mpx.json > $O/job_4mpx.log 2>&1
echo "job 4mpx ok"
timeout -k 10 600 python -u profiles/job_scale.py 1024 1024 30 $O/job_1mpx_trend.json --trendline \
  > $O/job_1mpx_trend.log 2>&1
echo "job 1mpx trendline ok"
