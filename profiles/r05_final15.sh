#!/bin/bash
# Round-5 final check D, kernel trace: rocprofv3 --kernel-trace --stats of the default bench
# command with the libraries rebuilt in the re-created container (build 3aaa67174cf7b4f3)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_final15}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py > $O/c2_bench_under_rocprof.json 2> $O/kt.err
find $O/kt -name '*kernel_stats.csv' | head -3
