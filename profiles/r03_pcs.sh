#!/bin/bash
# Which PC sampling configurations rocprofv3 offers on this GPU (listing only).
# Usage: bash profiles/r03_pcs.sh <outdir under gpurun_out>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/list.txt 2>&1
grep -i -B2 -A12 "pc.sampl\|pc_sampl" $O/list.txt | head -80
