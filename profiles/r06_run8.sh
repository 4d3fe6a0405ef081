#!/bin/bash
# r06 run 8: c3 with the output-field specialisation but some dropped planes kept as runtime
# pointers (LT_JIT_FIELDS_OR): initial_val (RuleState1::init live again) / winner + val_raw (the
# winner pick's general store loop kept) — which drop slows the c3 instance (run 7: -2.8 %)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run8}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, env, args
  env $2 timeout -k 10 300 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['joined_steps']['value'],d['parity_sample']['mismatched_values'])"
}
b c3_f1 LT_JIT_FIELDS=1 "--config c3" && b c3_f0 LT_JIT_FIELDS=0 "--config c3" && b c3_init LT_JIT_FIELDS_OR=80 "--config c3" && b c3_wv LT_JIT_FIELDS_OR=300 "--config c3" && b c3_ny LT_JIT_FIELDS_OR=2 "--config c3" && b c3_f1b LT_JIT_FIELDS=1 "--config c3" && b c3_f0b LT_JIT_FIELDS=0 "--config c3"
