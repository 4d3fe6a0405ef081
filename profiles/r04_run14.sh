#!/bin/bash
# Round-4 call 14: three deferred-list sets (default) vs two (LT_DEFER_SETS=2); resolve groups of
# 64 / 32 / 16 pixels (LT_RESOLVE_GROUP via LT_JIT_DEFINES); the lazy+exact resolve DP at group 16;
# then a kernel trace of the default c2 bench.
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
    run s3g64_$i $C LT_X=1
    run s2g64_$i $C LT_DEFER_SETS=2
    run s3g32_$i $C LT_JIT_DEFINES=LT_RESOLVE_GROUP=32
    run s3g16_$i $C LT_JIT_DEFINES=LT_RESOLVE_GROUP=16
  done
done
run s3g16lazy c2 LT_JIT_DEFINES=LT_RESOLVE_GROUP=16,LT_RESOLVE_FULL=0
for C in c5 c4; do
  run s3g64 $C LT_X=1
  run s2g64 $C LT_DEFER_SETS=2
  run s3g16 $C LT_JIT_DEFINES=LT_RESOLVE_GROUP=16
done
mkdir -p $O/kt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/kt.log 2>&1
echo kt ok
