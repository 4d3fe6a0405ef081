#!/bin/bash
# r06 run 40: more LLVM scheduler switches for the c2 module (tools/jit_variant.py --opt), loaded in
# place of the JIT compile, one box, default first and last, max-ilp again
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run40}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, env
  env $2 timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['parity_sample']['mismatched_values'],d['jit']['override'])"
}
b default LT_NONE=1 && b maxilp LT_JIT_OVERRIDE_DIR=$R/build/override/c2_max-ilp || exit 1
for v in build/override/c2x_*; do b $(basename $v) LT_JIT_OVERRIDE_DIR=$R/$v || exit 1; done
b default2 LT_NONE=1 && b maxilp2 LT_JIT_OVERRIDE_DIR=$R/build/override/c2_max-ilp
