#!/bin/bash
# r05 run 17: GPU suite (JIT programs now also against the CPU checkers alone), the c5 per-year
# row stores with L2-dropping cache policies (sc1 / sc0 sc1 / nt sc1 via inline asm) against the
# compiler's nt stores, and 2-rank gloo rehearsals of bench's N > 1 path (runner.finish)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run17}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
b() {  # name, defines, args
  LT_JIT_DEFINES=$2 timeout -k 10 170 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
b c5 "" "--config c5"
b c5_sc1 LT_YEAR_STORE_MODE=1 "--config c5"
b c5_sc0sc1 LT_YEAR_STORE_MODE=2 "--config c5"
b c5_ntsc1 LT_YEAR_STORE_MODE=3 "--config c5"
b c5_again "" "--config c5"
timeout -k 10 700 bash profiles/r04_rehearsal.sh ${1:-gpurun_out/r05_run17}/rehearsal
