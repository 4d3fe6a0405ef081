#!/bin/bash
# Round-4 call 10: c2 load-stage / kernel-variant A/B at this build:
#   jit      the default: 'B1 - B2' in JIT kernels specialised for the launch (lt_jit.h Spec)
#   jitnospec LT_JIT_SPEC=0: JIT kernels with only the program inlined
#   lin      LT_JIT_LINEAR=0: the precompiled kernel's linear form (round-3 path)
#   spec / nospec: precompiled probe builds with / without the c2 constants (build/exp)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
run() {
  name=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/c2_$name.json 2> $O/c2_$name.err
  python -c "import json;d=json.load(open('$O/c2_$name.json'));print('$name',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
for i in 1 2; do
  run jit$i LT_X=1
  run jitnospec$i LT_JIT_SPEC=0
  run lin$i LT_JIT_LINEAR=0
  run spec$i LT_JIT_LINEAR=0 LT_HIP_LIB=$R/build/exp/liblt_spec_32.so
  run nospec$i LT_JIT_LINEAR=0 LT_HIP_LIB=$R/build/exp/liblt_nospec_32.so
done
for C in c3 c5; do
  timeout -k 10 400 python bench.py --config $C --no-cpu-baseline --e2e-steps 0 > $O/$C.json 2> $O/$C.err
  python -c "import json;d=json.load(open('$O/$C.json'));print('$C jit',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
  LT_JIT_LINEAR=0 timeout -k 10 400 python bench.py --config $C --no-cpu-baseline --e2e-steps 0 > $O/${C}_lin.json 2> $O/${C}_lin.err
  python -c "import json;d=json.load(open('$O/${C}_lin.json'));print('$C lin',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
done
