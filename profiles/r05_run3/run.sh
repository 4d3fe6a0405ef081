#!/bin/bash
# Round-5 call 3: the JIT lifecycle GPU tests (fixed key hashing), and the e32-select A/B on the
# bench kernels: the hiprtc module (default), the same source through hipcc (control) and that
# build with every v_cndmask_b32_e32 on VCC rewritten to its e64 form (tools/jit_asm.py).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 300 --timeout-method thread > $O/gpu_jit_tests.txt 2>&1
tail -1 $O/gpu_jit_tests.txt
for c in c2 c3 c5; do
  for v in default none e64; do
    if [ $v = default ]; then unset LT_JIT_OVERRIDE_DIR; else export LT_JIT_OVERRIDE_DIR=$R/build/override/$v; fi
    timeout -k 10 300 python bench.py --config $c --steps 5 --no-cpu-baseline --e2e-steps 0 > $O/${c}_$v.json 2> $O/${c}_$v.err
    python -c "import json;d=json.load(open('$O/${c}_$v.json'));print('$c $v',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['parity_sample']['mismatched_values'],d['jit'])"
  done
done
