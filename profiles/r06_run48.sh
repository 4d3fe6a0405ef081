#!/bin/bash
# r06 run 48: with the rasters uploaded during parse, the GPU job tests and the c2-size job with a 20k-pixel oracle
# check (eight rasters decoded at once)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run48}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_job.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/job_bench.py --rows 7000 --cols 7000 --years 30 --check 20000 > $O/job_c2.json 2> $O/job_c2.err
rc=$?
python -c "import json;d=json.load(open('$O/job_c2.json'));print('c2',d['seconds'],d['job_s'],d['parse_decoded_gb_per_s'],d['check']['mismatches'])" || tail -5 $O/job_c2.err
exit $rc
