#!/bin/bash
# Instruction-cache PMC of the analyze kernel (one 16.8 Mpx launch, c2 and c5).
# Usage: bash profiles/r02_run18.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in c2 c5; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
    SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/ic1_$C -o run -- python3 $R/bench.py \
    --config $C --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 > $O/ic1_$C.log 2>&1
  echo "ic1 $C ok"
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES \
    SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE --output-format csv -d $O/ic2_$C -o run -- python3 \
    $R/bench.py --config $C --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 \
    > $O/ic2_$C.log 2>&1
  echo "ic2 $C ok"
done
