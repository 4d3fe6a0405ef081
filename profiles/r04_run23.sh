#!/bin/bash
# Round-4 call 23: pixels per launch (tile) for the labels-only configs: 16.8 Mpx (default, 3
# launches per 49 Mpx scene) vs 24.5 Mpx (2) vs 49 Mpx (1).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
run() {
  name=$1; C=$2; shift 2
  timeout -k 10 400 python bench.py --config $C --steps 8 --warmup 2 --no-cpu-baseline --e2e-steps 0 "$@" > $O/${C}_$name.json 2> $O/${C}_$name.err
  python -c "import json;d=json.load(open('$O/${C}_$name.json'));print('$C $name',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'],d['config']['tiles'])"
}
for i in 1 2; do
  for C in c2 c3; do
    run t16_$i $C
    run t24_$i $C --tile 24500000
    run t49_$i $C --tile 49000000
  done
done
