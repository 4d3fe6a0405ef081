#!/bin/bash
# Kernel-trace stats of the c3, c4 and c5 bench lines at the round-2 final build.
# Usage: bash profiles/r02_run32.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in c3 c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$C -o run -- \
    python3 $R/bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 \
    > $O/kt_$C.json 2> $O/kt_$C.err
  echo "kernel trace $C ok"
done
