#!/bin/bash
# r06 run 47: after the host-side changes of the last commits (lazy load-kernel compile, LZW
# decoder, job pipeline): final check A (GPU suite, smoke, default bench line, kernel trace), then
# the c2-size job with a 20k-pixel oracle check
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=${1:-gpurun_out/r06_run47}
cd $R
bash profiles/r06_final.sh $O A || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/job_bench.py --rows 7000 --cols 7000 --years 30 --check 20000 > $R/$O/job_c2.json 2> $R/$O/job_c2.err
rc=$?
python -c "import json;d=json.load(open('$R/$O/job_c2.json'));print('job c2',d['seconds'],d['job_s'],d['parse_decoded_gb_per_s'],d['analyze_parts_s'],d['check']['mismatches'])" || tail -5 $R/$O/job_c2.err
exit $rc
