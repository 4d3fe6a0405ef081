#!/bin/bash
# r06 run 31 (output() joins the grid writer): the c2-size job with the grid CSV written beside parse and the raster order made lazily (GPU job tests first)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run31}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_job.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
jb() {  # name, mmap, check
  LT_TIFF_MMAP=$2 timeout -k 10 400 python tools/job_bench.py --rows 7000 --cols 7000 --years 30 --check $3 > $O/job_$1.json 2> $O/job_$1.err
  rc=$?
  python -c "import json;d=json.load(open('$O/job_$1.json'));print('$1',d['seconds'],d['job_s'],d['parse_decoded_gb_per_s'],d['analyze_parts_s'],d.get('check',{}).get('mismatches'))" || true
  return $rc
}
jb a 1 20000 && jb b 1 0
