#!/bin/bash
# Round-end check of the current build: smoke(), the default bench line (cpu baseline + end-to-end,
# as the driver runs it), c4 and c5 lines, kernel-trace stats of the default line, and the PMC
# passes of one 16.8 Mpx c5 launch (its stores changed). Usage: bash profiles/r02_run26.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$1
mkdir -p $R/$O
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > $R/$O/smoke.log 2>&1
echo "smoke ok"
timeout -k 10 400 python bench.py > $R/$O/bench_default.json 2> $R/$O/bench_default.err
echo "bench default ok"
for c in c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --e2e-steps 0 > $R/$O/bench_$c.json \
    2> $R/$O/bench_$c.err
  echo "bench $c ok"
done
timeout -k 10 600 bash profiles/pmc_passes.sh $O/pmc_c5 --config c5 --pixels 16777216 --steps 1 \
  --warmup 0 --e2e-steps 0
python3 profiles/summarize_pmc.py $R/$O/pmc_c5 $R/$O/pmc_c5.json 16777216 > /dev/null
echo "pmc c5 ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $R/$O/kt_bench.json \
  2> $R/$O/kt_bench.err
echo "kernel trace ok"
