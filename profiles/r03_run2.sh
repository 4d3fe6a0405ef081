#!/bin/bash
# Load-stage priority A/B on c2: kernel trace of the default line with the load stream at high
# priority (LT_LOAD_PRIORITY=-1) against the default stream priority.
# Usage: bash profiles/r03_run2.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for P in 0 -1; do
  LT_LOAD_PRIORITY=$P timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_p$P -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/c2_p$P.json 2> $O/c2_p$P.err
  echo "prio $P ok"
done
for P in 0 -1; do
  LT_LOAD_PRIORITY=$P timeout -k 10 300 python3 $R/bench.py --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/c2_bench_p$P.json 2> $O/c2_bench_p$P.err
  echo "bench prio $P ok"
done
