#!/bin/bash
# r06 run 9: (1) tools/scratch_probe: every resident wave's private memory its own? (light kernel
# at 8 waves per SIMD, 128-VGPR kernel at 4); (2) the rest of run 8 (c3 output-field variants,
# the LT_JIT_FIELDS_OR=80 variant gave 124 parity mismatches: kept out)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run9}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 build/bin/scratch_probe 1048576 200 4 > $O/scratch_probe.json 2> $O/scratch_probe.err
rc=$?; cat $O/scratch_probe.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 build/bin/scratch_probe 4194304 50 2 > $O/scratch_probe_4m.json 2>> $O/scratch_probe.err
rc=$?; cat $O/scratch_probe_4m.json; [ $rc -eq 0 ] || exit $rc
b() {  # name, env, args
  env $2 timeout -k 10 300 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['joined_steps']['value'],d['parity_sample']['mismatched_values'])"
}
b c3_wv LT_JIT_FIELDS_OR=300 "--config c3"; b c3_ny LT_JIT_FIELDS_OR=2 "--config c3"; b c3_f1 LT_JIT_FIELDS=1 "--config c3"; b c3_f0 LT_JIT_FIELDS=0 "--config c3"
