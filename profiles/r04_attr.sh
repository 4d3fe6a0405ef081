#!/bin/bash
# Round-4 closing attribution: c2 with a non-linear index program (division) through the JIT
# kernels vs 'B1 - B2', same box.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $O/c2_b1mb2.json 2> $O/c2_b1mb2.err
timeout -k 10 400 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --e2e-steps 0 --index-eqn '(B1 - B2) * 2 / 2' > $O/c2_div.json 2> $O/c2_div.err
python -c "
import json
for n in ['b1mb2','div']:
    d=json.load(open('$O/c2_'+n+'.json')); print(n, d['value'], d['config']['input'], d['parity_sample']['mismatched_values'])"
