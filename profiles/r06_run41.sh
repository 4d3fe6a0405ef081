#!/bin/bash
# r06 run 41: the c5 module under LLVM's max-ilp / max-memory-clause schedulers (store-bound
# launch), loaded in place of the JIT compile, one box, default first and last
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run41}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, env
  env $2 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['parity_sample']['mismatched_values'],d['jit']['override'])"
}
b default LT_NONE=1 && b maxilp LT_JIT_OVERRIDE_DIR=$R/build/override/c5_max-ilp && \
b maxmem LT_JIT_OVERRIDE_DIR=$R/build/override/c5_max-memory-clause && b default2 LT_NONE=1
