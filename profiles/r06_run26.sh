#!/bin/bash
# r06 run 26: binary64 results in the last register pair of a 128-VGPR allocation
# (tools/vgpr_edge.hip: v[126:127] vs v[120:121], same allocation, 4 waves per SIMD)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run26}
mkdir -p $O
cd $R
timeout -k 10 120 build/bin/vgpr_edge 262144 1000 > $O/vgpr_edge.jsonl 2> $O/vgpr_edge.err
rc=$?; cat $O/vgpr_edge.jsonl; echo "rc=$rc"; exit $rc
