#!/bin/bash
# GPU tests of the current product build (fused load stage, kernarg arguments), then r03_ab3.sh.
# Usage: bash profiles/r03_run4.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash profiles/r03_ab3.sh $1/ab3
