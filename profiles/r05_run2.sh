#!/bin/bash
# Round-5 call 2: the JIT lifecycle GPU tests (embedded headers, fallback, async compile, module
# cap) and the select-pattern VALU kinds.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 120 build/bin/valu_peak 20000 cmp_cnd2_vcc,cmp_cnd4_vcc,cmp_gap_cnd_vcc,cmp64_cnd2,cmp_cndmask_vcc,cndmask_vcc_valu > $O/valu_peak2.json
echo valu_peak done
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 300 --timeout-method thread > $O/gpu_jit_tests.txt 2>&1
tail -3 $O/gpu_jit_tests.txt
