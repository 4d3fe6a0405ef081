#!/bin/bash
# r06 run 6: the whole local job (tools/job_bench.py) on a 7000 x 7000 x 30-acquisition LZW
# GeoTIFF stack generated on the box: setup / parse / analysis / output timed, 20k pixels checked
# against the oracle
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run6}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python tools/job_bench.py --rows 7000 --cols 7000 --years 30 $JB_ARGS > $O/job_c2.json 2> $O/job_c2.err
rc=$?; tail -60 $O/job_c2.err; cat $O/job_c2.json; exit $rc
