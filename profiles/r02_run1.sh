#!/bin/bash
# Round-2 first GPU call: GPU tests, the default bench line, kernel-trace stats of c3 and c5, and
# PMC passes of one 16.8 Mpx launch of c2, c3 and c5. Usage: bash profiles/r02_run1.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$1
mkdir -p $R/$O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $R/$O/gpu_tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python bench.py > $R/$O/bench_c2.json 2> $R/$O/bench_c2.err
echo "bench ok"
for c in c3 c5; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $R/$O/kt_$c -o run -- python3 $R/bench.py --config $c --steps 3 \
    --warmup 1 --no-cpu-baseline > $R/$O/bench_$c.json 2> $R/$O/bench_$c.err)
  echo "kt $c ok"
done
for c in c2 c3 c5; do
  timeout -k 10 600 bash profiles/pmc_passes.sh $O/pmc_$c --config $c --pixels 16777216 \
    --steps 1 --warmup 0
  python3 profiles/summarize_pmc.py $R/$O/pmc_$c $R/$O/pmc_$c.json 16777216 > /dev/null
  echo "pmc $c ok"
done
