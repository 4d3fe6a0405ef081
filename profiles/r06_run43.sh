#!/bin/bash
# r06 run 43: the c2-size job's parse with 2, 4 (default), 8 and 16 rasters decoded at once
# (LT_INGEST_FILES; the host's 16 threads split among them), one box
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run43}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
jb() {  # name, files, check
  LT_INGEST_FILES=$2 timeout -k 10 400 python tools/job_bench.py --rows 7000 --cols 7000 --years 30 --check $3 > $O/job_$1.json 2> $O/job_$1.err
  rc=$?
  python -c "import json;d=json.load(open('$O/job_$1.json'));print('$1',d['seconds'],d['job_s'],d['parse_decoded_gb_per_s'],d.get('check',{}).get('mismatches'))" || tail -5 $O/job_$1.err
  return $rc
}
jb f4 4 0 && jb f8 8 0 && jb f16 16 0 && jb f2 2 0 && jb f4b 4 0
