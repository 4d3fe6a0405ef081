#!/bin/bash
# Final check of the round-2 build: GPU tests, the PMC passes of one 16.8 Mpx c2/c3/c5 launch
# (their summaries replace profiles/r02_pmc_*.json on the box before the bench lines, so the lines'
# roofline uses this build's counts), smoke(), the default bench line (cpu baseline + end-to-end),
# c3/c4/c5 lines, kernel-trace stats of the default line. Usage: bash profiles/r02_run29.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$1
mkdir -p $R/$O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $R/$O/gpu_tests.log 2>&1
echo "tests ok"
for C in c2 c3 c5; do
  timeout -k 10 400 bash profiles/pmc_passes.sh $O/pmc_$C --config $C --pixels 16777216 --steps 1 \
    --warmup 0 --e2e-steps 0
  python3 profiles/summarize_pmc.py $R/$O/pmc_$C $R/$O/pmc_$C.json 16777216 > /dev/null
  cp $R/$O/pmc_$C.json $R/profiles/r02_pmc_$C.json
  echo "pmc $C ok"
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > $R/$O/smoke.log 2>&1
echo "smoke ok"
timeout -k 10 400 python bench.py > $R/$O/bench_c2.json 2> $R/$O/bench_c2.err
echo "bench default ok"
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --e2e-steps 0 > $R/$O/bench_$c.json \
    2> $R/$O/bench_$c.err
  echo "bench $c ok"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $R/$O/kt_bench.json \
  2> $R/$O/kt_bench.err
echo "kernel trace ok"
