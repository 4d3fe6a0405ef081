#!/bin/bash
# Round-4 call 12: JIT kernels specialised for the scene too (LT_SPEC_SCENE: year table, winner
# per year, observation order / distances as constants) vs LT_JIT_SCENE=0, c2 / c3 / c5 / c4.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
run() {
  name=$1; C=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $C --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/${C}_$name.json 2> $O/${C}_$name.err
  python -c "import json;d=json.load(open('$O/${C}_$name.json'));print('$C $name',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
for i in 1 2; do
  for C in c2 c3; do
    run scene_$i $C LT_X=1
    run noscene_$i $C LT_JIT_SCENE=0
  done
done
run scene c5 LT_X=1
run noscene c5 LT_JIT_SCENE=0
run scene c4 LT_X=1
run noscene c4 LT_JIT_SCENE=0
