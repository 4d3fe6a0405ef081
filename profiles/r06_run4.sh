#!/bin/bash
# r06 run 4: pipelined steps after the ADVICE r05 fix (per-tile waits on the last writer of a
# tile's planes, two output banks for one-tile runners): the pipelined-step GPU tests incl. inputs
# changed between steps, then c2 / c3 bench lines (pipelined headline + joined_steps)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run4}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mosaic.py -k pipelined > $O/tests.txt 2>&1
rc=$?; tail -8 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
b() {  # name, args
  timeout -k 10 300 python bench.py $2 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err || return 1
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['kernel_ms_joined'],d['joined_steps'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
b c2 "--config c2" && b c3 "--config c3" && b c5 "--config c5"
