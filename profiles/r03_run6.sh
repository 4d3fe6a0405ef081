#!/bin/bash
# Build check of HEAD after the session restart: GPU tests, smoke, default bench line
# (with cpu baseline), bench c3 / c5 lines, kernel-trace stats of the default line.
# Usage: bash profiles/r03_run6.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1
echo "smoke ok"
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
cat $O/bench_default.json
for C in c3 c5; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --e2e-steps 0 > $O/bench_$C.json 2> $O/bench_$C.err
  python -c "import json;d=json.load(open('$O/bench_$C.json'));print('$C',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['parity_sample']['mismatched_values'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c2 -- python3 bench.py --no-cpu-baseline --e2e-steps 0 --steps 10 > $O/prof.log 2>&1
echo "prof ok"
