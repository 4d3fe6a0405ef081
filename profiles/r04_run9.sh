#!/bin/bash
# Round-4 call 9: GPU tests (JIT fixes), c2 JIT attribution, and the specialisation A/B: the c2
# instance compiled for bench's exact c2 configuration (build/exp/liblt_spec_32.so: 30 years, no
# mask, labels only, one GD rule, line_cost 10 as constants) vs the same source unspecialised.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
rc=0
timeout -k 10 1100 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for i in 1 2; do
  for L in nospec spec; do
    LT_HIP_LIB=$R/build/exp/liblt_${L}_32.so timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/c2_$L$i.json 2> $O/c2_$L$i.err
    python -c "import json;d=json.load(open('$O/c2_$L$i.json'));print('c2 $L',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
  done
  timeout -k 10 400 python bench.py --steps 10 --index-eqn '(B1 - B2) * 2 / 2' --no-cpu-baseline --e2e-steps 0 > $O/c2_jit$i.json 2> $O/c2_jit$i.err
  python -c "import json;d=json.load(open('$O/c2_jit$i.json'));print('c2 jit',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
done
