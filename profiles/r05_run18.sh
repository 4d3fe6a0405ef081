#!/bin/bash
# r05 run 18: c2 / c3 phase cuts of the JIT analyze kernel at this build (timing-only,
# LT_JIT_STOP_AFTER=k: the kernel ends after phase k), and c5 with 2 and 4 tiles per scene
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run18}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, defines, args
  LT_JIT_DEFINES=$2 timeout -k 10 170 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 --parity-sample 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'])"
}
for C in c2 c3; do
  for k in 0 1 2 3; do
    b ${C}_cut$k LT_JIT_STOP_AFTER=$k "--config $C"
  done
  b ${C}_full "" "--config $C"
done
b c5_t4 "" "--config c5 --tile 12250000"
b c5_t2 "" "--config c5 --tile 24500000"
b c5_t3 "" "--config c5"
