#!/bin/bash
# Round-4 call 18: first-round wave stagger (LT_STAGGER_TICKS x 0..3 of the 100 MHz clock, via
# LT_JIT_DEFINES) against waves kept in step (stores of all waves at once, arithmetic at once).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
run() {
  name=$1; C=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $C --steps 8 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $O/${C}_$name.json 2> $O/${C}_$name.err
  python -c "import json;d=json.load(open('$O/${C}_$name.json'));print('$C $name',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
for i in 1 2; do
  run base_$i c5 LT_X=1
  run st2500_$i c5 LT_JIT_DEFINES=LT_STAGGER_TICKS=2500,LT_STAGGER_WAVES=4096
  run st5000_$i c5 LT_JIT_DEFINES=LT_STAGGER_TICKS=5000,LT_STAGGER_WAVES=4096
  run st10000_$i c5 LT_JIT_DEFINES=LT_STAGGER_TICKS=10000,LT_STAGGER_WAVES=4096
done
run base c2 LT_X=1
run st2500 c2 LT_JIT_DEFINES=LT_STAGGER_TICKS=2500,LT_STAGGER_WAVES=4096
