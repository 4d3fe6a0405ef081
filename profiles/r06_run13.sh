#!/bin/bash
# r06 run 13: tiles of whole waves as a JIT constant (LT_SPEC_FULL: every lane live), same-box A/B
# against LT_JIT_FULL=0 on c2 / c3 / c5
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run13}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, env, args
  env $2 timeout -k 10 300 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['joined_steps']['value'],d['parity_sample']['mismatched_values'])"
}
b c2 LT_JIT_FULL=1 "--config c2"; b c2_f0 LT_JIT_FULL=0 "--config c2"; b c3 LT_JIT_FULL=1 "--config c3"; b c3_f0 LT_JIT_FULL=0 "--config c3"; b c5 LT_JIT_FULL=1 "--config c5"; b c5_f0 LT_JIT_FULL=0 "--config c5"; b c2b LT_JIT_FULL=1 "--config c2"
