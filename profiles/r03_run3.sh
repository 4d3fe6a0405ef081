#!/bin/bash
# Round-3 fused load stage check: GPU tests, smoke, the default bench line (with the
# parity sample gate), c3/c5 bench lines, kernel-trace stats of the default line.
# Usage: bash profiles/r03_run1.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
# test failures (rc 1) do not stop the script; a fault, abort or time limit does
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1
echo "smoke ok"
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err
echo "bench c2 ok"; cat $O/bench_c2.json
for C in c3 c5; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --e2e-steps 0 > $O/bench_$C.json 2> $O/bench_$C.err
  echo "bench $C ok"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/kt_c2.json 2> $O/kt_c2.err
echo "kernel trace ok"
