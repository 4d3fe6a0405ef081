#!/bin/bash
# r06 run 42: the stack's and the trendline's host planes on huge-page-advised anonymous memory
# (ingest.host_empty, LT_HOST_HUGEPAGES=1, the new default) vs np.empty (=0), alternating on one box:
# the c2-size labels job and the 4000 x 4000 trendline job; GPU job tests first
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run42}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_job.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
jb() {  # name, hugepages, args
  LT_HOST_HUGEPAGES=$2 timeout -k 10 400 python tools/job_bench.py $3 > $O/job_$1.json 2> $O/job_$1.err
  rc=$?
  python -c "import json;d=json.load(open('$O/job_$1.json'));print('$1',d['seconds'],d['job_s'],d['parse_decoded_gb_per_s'],d['analyze_parts_s'],d.get('check',{}).get('mismatches'))" || tail -5 $O/job_$1.err
  return $rc
}
C2="--rows 7000 --cols 7000 --years 30"
TL="--rows 4000 --cols 4000 --years 30 --trendline"
jb c2_huge 1 "$C2 --check 20000" && jb c2_small 0 "$C2 --check 0" && jb c2_huge2 1 "$C2 --check 0" && \
jb tl_huge 1 "$TL --check 5000" && jb tl_small 0 "$TL --check 0"
