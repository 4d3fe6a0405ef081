#!/bin/bash
# r06 run 5: JIT analyze kernel with several waves per workgroup (LT_JIT_WPB: 64 * wpb consecutive
# pixels per workgroup, each wave its own LDS slice), A/B on one box: c5 (the per-year plane
# stores: a workgroup's row pieces leave side by side) and c2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run5}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, wpb, args
  LT_JIT_WPB=$2 timeout -k 10 300 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['joined_steps']['value'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
b c5_w1 1 "--config c5" && b c5_w4 4 "--config c5" && b c5_w2 2 "--config c5" && b c2_w1 1 "--config c2" && b c2_w4 4 "--config c2" && b c5_w1b 1 "--config c5" && b c5_w4b 4 "--config c5"
