#!/bin/bash
# Round-4 call 15: attribution of the JIT kernels (timing-only variants through LT_JIT_DEFINES,
# wrong outputs): phase cuts (LT_JIT_STOP_AFTER 0..3) for c5 and c2; c5 without the year-major
# stores / the winner-pick rows / the emulated fits.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
run() {
  name=$1; C=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $C --steps 6 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $O/${C}_$name.json 2> $O/${C}_$name.err || true
  python -c "import json;d=json.load(open('$O/${C}_$name.json'));print('$C $name',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
run full c5 LT_X=1
for k in 0 1 2 3; do run stop$k c5 LT_JIT_DEFINES=LT_JIT_STOP_AFTER=$k; done
run nostore1 c5 LT_JIT_DEFINES=LT_AB_NO_YEAR_STORES=1
run nostore2 c5 LT_JIT_DEFINES=LT_AB_NO_YEAR_STORES=2
run nofit c5 LT_JIT_DEFINES=LT_AB_NO_FITS=1
run nofit_nostore2 c5 LT_JIT_DEFINES=LT_AB_NO_FITS=1,LT_AB_NO_YEAR_STORES=2
run full c2 LT_X=1
for k in 0 1 2 3; do run stop$k c2 LT_JIT_DEFINES=LT_JIT_STOP_AFTER=$k; done
