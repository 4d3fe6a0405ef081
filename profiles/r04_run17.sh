#!/bin/bash
# Round-4 call 17: GPU tests, PMC passes of c2 / c3 / c5 at this build (JIT kernels), the default
# bench line.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || rc=$?
echo "gpu tests rc=$rc"; tail -2 $O/gpu_tests.txt
if [ $rc -gt 1 ]; then exit $rc; fi
for C in c2 c3 c5; do
  bash $R/profiles/pmc_passes.sh $1/pmc/$C --config $C --pixels 16777216 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0
  python3 $R/profiles/summarize_pmc.py $O/pmc/$C $O/r04_pmc_$C.json 16777216 > /dev/null
  echo "pmc $C ok"
done
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
python -c "import json;d=json.load(open('$O/bench_default.json'));print('c2',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['parity_sample']['mismatched_values'])"
