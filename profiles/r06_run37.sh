#!/bin/bash
# r06 run 37: c5 and c3 bench lines at the last commit (kernels at build 75d052c3d92fece0), one box,
# twice each: the c5 >= 1450 Mpx/s question across boxes
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run37}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, args
  timeout -k 10 300 python bench.py $2 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['frac'],d['parity_sample']['mismatched_values'])"
}
b c5 "--config c5" && b c3 "--config c3" && b c5b "--config c5" && b c3b "--config c3"
