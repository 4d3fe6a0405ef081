#!/bin/bash
# r06 run 46: cProfile of the c2-size job's analysis step (tools/job_bench.py --profile analyze)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run46}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/job_bench.py --rows 7000 --cols 7000 --years 30 --check 0 --profile analyze > $O/job_c2.json 2> $O/job_c2.err
rc=$?
python -c "import json;d=json.load(open('$O/job_c2.json'));print('c2',d['seconds'],d['job_s'],d['analyze_parts_s'])" || true
grep -A30 "Ordered by" $O/job_c2.err | head -34
exit $rc
