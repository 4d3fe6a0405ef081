#!/bin/bash
# r05 run 32: pipelined steps at N = 1 (runner.step overlap: a step's last resolve / expand runs
# beside the next step's first analyze) — the GPU test of the pipelined path against a joined
# step, then bench with (default) and without (--no-overlap) pipelining, c2 / c3 / c5, twice
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run32}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_mosaic.py -k pipelined -x -v --timeout 300 --timeout-method thread > $O/test_pipelined.txt 2>&1 || { tail -30 $O/test_pipelined.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/test_pipelined.txt
b() {  # name, args
  timeout -k 10 170 python bench.py $2 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'],d['config'].get('steps_pipelined'))"
}
for i in 1 2; do
  for C in c2 c3 c5; do
    b ${C}_pipe_$i "--config $C"
    b ${C}_join_$i "--config $C --no-overlap"
  done
done
