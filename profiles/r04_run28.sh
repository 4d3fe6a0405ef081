#!/bin/bash
# Round-4 call 28: 24-bit multiplies in the analyze stage's lazy DP only (not the resolve's exact
# DP) — GPU suite, new vs previous headers on c2 / c5 (twice) and c3, PMC passes at this build.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || rc=$?
echo "gpu tests rc=$rc"; tail -2 $O/gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
run() {
  name=$1; C=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $C --steps 8 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $O/${C}_$name.json 2> $O/${C}_$name.err
  python -c "import json;d=json.load(open('$O/${C}_$name.json'));print('$C $name',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
for i in 1 2; do
  for C in c2 c5; do
    run new_$i $C LT_X=1
    run old_$i $C LT_SRC_DIR=$R/build/ab/old/csrc
  done
done
run new c3 LT_X=1
run old c3 LT_SRC_DIR=$R/build/ab/old/csrc
for C in c2 c3 c5; do
  bash $R/profiles/pmc_passes.sh $1/pmc/$C --config $C --pixels 16777216 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0
  python3 $R/profiles/summarize_pmc.py $O/pmc/$C $O/r04_pmc_$C.json 16777216 > /dev/null
  echo "pmc $C ok"
done
