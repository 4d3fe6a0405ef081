#!/bin/bash
# r06 run 36 (run 34 with rasters written on a thread while the next is assembled; GPU job tests first): the job with every per-year trendline raster (8 keys per acquisition date, as the
# reference's output_reducer writes them) at 4000 x 4000 px x 30 dates, and the labels-only job at
# the same size, tools/job_bench.py with a 5k-pixel oracle check each
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run36}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_job.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
jb() {  # name, args
  timeout -k 10 500 python tools/job_bench.py --rows 4000 --cols 4000 --years 30 --check 5000 $2 > $O/job_$1.json 2> $O/job_$1.err
  rc=$?; grep -E "^(setup|parse|analyze|output)" $O/job_$1.err
  python -c "import json;d=json.load(open('$O/job_$1.json'));print('$1',d['seconds'],d['job_s'],d['output_rasters'],round(d['output_bytes']/1e9,2),d['analyze_parts_s'],d.get('check',{}).get('mismatches'))" || { tail -20 $O/job_$1.err; }
  return $rc
}
jb trendline "--trendline" && jb labels ""
