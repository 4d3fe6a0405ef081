#!/bin/bash
# Round-4 call 25: which half of the despike change costs c5 (vE: the step test alone; vF: the
# unconditional reads alone), against the whole change and the previous headers.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
run() {
  name=$1; C=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $C --steps 8 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $O/${C}_$name.json 2> $O/${C}_$name.err
  python -c "import json;d=json.load(open('$O/${C}_$name.json'));print('$C $name',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['parity_sample']['mismatched_values'])"
}
for i in 1 2; do
  run new_$i c5 LT_X=1
  run old_$i c5 LT_SRC_DIR=$R/build/ab/old/csrc
  run vE_$i c5 LT_SRC_DIR=$R/build/ab/vE/csrc
  run vF_$i c5 LT_SRC_DIR=$R/build/ab/vF/csrc
done
for C in c2 c3; do
  run vE $C LT_SRC_DIR=$R/build/ab/vE/csrc
  run vF $C LT_SRC_DIR=$R/build/ab/vF/csrc
done
