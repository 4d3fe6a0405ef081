#!/bin/bash
# r06 run 51: the trendline jobs with the four-byte LZW bit writer (5k-pixel oracle check each)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run51}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
jb() {  # name, args
  timeout -k 10 600 python tools/job_bench.py --years 30 --check 5000 --trendline $2 > $O/job_$1.json 2> $O/job_$1.err
  rc=$?
  python -c "import json;d=json.load(open('$O/job_$1.json'));print('$1',d['seconds'],d['job_s'],d['output_rasters'],round(d['output_bytes']/1e9,2),d['analyze_parts_s'],sum(d['check']['mismatches'].values()))" || tail -8 $O/job_$1.err
  return $rc
}
jb tl16 "--rows 4000 --cols 4000" && jb tl49 "--rows 7000 --cols 7000"
