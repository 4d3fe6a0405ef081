#!/bin/bash
# r05 run 12 (session 2 re-entry): GPU suite at HEAD, the c2 bench, and the c3 mismatch isolation
# of the default pass B (slots in both stages) against LT_PASSB_SLOTS=0 (lost with session 1's
# gpurun_out)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run12}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python bench.py > $O/c2_bench.json 2> $O/c2_bench.err
python -c "import json;d=json.load(open('$O/c2_bench.json'));print('c2',d['value'],d['ms_per_step'],d['parity_sample']['mismatched_values'])"
timeout -k 10 300 python tools/debug_mismatch.py --config c3 --sample 100000 > $O/c3_default.json 2> $O/c3_default.err
head -c 400 $O/c3_default.json; echo
LT_JIT_DEFINES=LT_PASSB_SLOTS=0 timeout -k 10 300 python tools/debug_mismatch.py --config c3 --sample 100000 > $O/c3_slots0.json 2> $O/c3_slots0.err
head -c 1500 $O/c3_slots0.json; echo
