#!/bin/bash
# r06 run 29: the c2-size job with rasters decoded in place into the stack (ingest_stack raster order), GPU job tests first
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run29}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_job.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
jb() {  # name, upload, check
  LT_JOB_UPLOAD=$2 timeout -k 10 400 python tools/job_bench.py --rows 7000 --cols 7000 --years 30 --check $3 > $O/job_$1.json 2> $O/job_$1.err
  rc=$?; grep -E "^(setup|parse|analyze|output)" $O/job_$1.err
  python -c "import json;d=json.load(open('$O/job_$1.json'));print('$1',d['seconds'],d['job_s'],d['analyze_parts_s'],d.get('check',{}).get('mismatches'))" || true
  return $rc
}
jb inplace whole 20000 && jb inplace2 whole 0
