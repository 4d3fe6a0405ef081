#!/bin/bash
# r06 run 10: c2 / c5 with the output-field specialisation keeping winner / val_raw as run-time
# pointers (LT_JIT_FIELDS_OR=300: c3 2224 vs 2157 Mpx/s with them compile-time null, run 9)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run10}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, env, args
  env $2 timeout -k 10 300 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['joined_steps']['value'],d['parity_sample']['mismatched_values'])"
}
b c2_wv LT_JIT_FIELDS_OR=300 "--config c2"; b c2_f1 LT_JIT_FIELDS=1 "--config c2"; b c5_wv LT_JIT_FIELDS_OR=300 "--config c5"; b c5_f1 LT_JIT_FIELDS=1 "--config c5"; b c3_wv LT_JIT_FIELDS_OR=300 "--config c3"; b c2_wvb LT_JIT_FIELDS_OR=300 "--config c2"
