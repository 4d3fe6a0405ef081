#!/bin/bash
# Round-4 call 22: which fminb / fmaxb use breaks c3-bench (bisect through LT_SRC_DIR header sets)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
T="tests/test_gpu_mosaic.py::test_bench_path_full_size_sampled_vs_oracle"
for v in ${VARIANTS:-vA vB}; do
  rc=0
  LT_SRC_DIR=$R/build/ab/$v/csrc timeout -k 10 300 python -u -m pytest "$T" -m gpu -x -q --timeout 240 --timeout-method thread -k c3-bench > $O/t_$v.txt 2>&1 || rc=$?
  echo "$v rc=$rc"; tail -1 $O/t_$v.txt
  if [ $rc -gt 1 ]; then exit $rc; fi
done
