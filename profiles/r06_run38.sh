#!/bin/bash
# r06 run 38: the default line at the driver's step count (c2, 20 timed steps) and c4, at the last
# commit
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run38}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --steps 20 --warmup 2 > $O/c2_20.json 2> $O/c2_20.err || { tail -5 $O/c2_20.err; exit 1; }
python -c "import json;d=json.load(open('$O/c2_20.json'));print('c2_20',round(d['value'],1),d['ms_per_step'],d['roofline']['frac'],d['parity_sample']['mismatched_values'],d['joined_steps']['value'],d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --e2e-steps 0 > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
python -c "import json;d=json.load(open('$O/c4.json'));print('c4',round(d['value'],1),d['ms_per_step'],d['roofline']['frac'],d['parity_sample']['mismatched_values'])"
