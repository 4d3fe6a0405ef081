#!/bin/bash
# r06 run 20: the label exchange's device path on one GPU (tests/test_gpu_exchange.py: narrowed
# planes packed on the send stream, received and widened on the receive stream, a loopback
# transport in place of RCCL), then the 2-rank rehearsal (staged gloo path, byte views)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run20}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_exchange.py -m gpu -v --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -4 $O/tests.txt
bash profiles/r06_rehearsal.sh ${1:-gpurun_out/r06_run20}/rehearsal
