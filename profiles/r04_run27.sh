#!/bin/bash
# Round-4 call 27: m * Sxx - Sx^2 with 24-bit multiplies (v_mul_u32_u24) instead of v_mul_lo_u32 —
# GPU suite, the JIT kernels from the new headers vs the previous commit's
# (LT_SRC_DIR=build/ab/old/csrc), then PMC passes of c2 / c3 / c5 at this build.
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
for C in c2 c3 c5; do
  run new $C LT_X=1
  run old $C LT_SRC_DIR=$R/build/ab/old/csrc
done
run new2 c2 LT_X=1
run old2 c2 LT_SRC_DIR=$R/build/ab/old/csrc
for C in c2 c3 c5; do
  bash $R/profiles/pmc_passes.sh $1/pmc/$C --config $C --pixels 16777216 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0
  python3 $R/profiles/summarize_pmc.py $O/pmc/$C $O/r04_pmc_$C.json 16777216 > /dev/null
  echo "pmc $C ok"
done
