#!/bin/bash
# Round-4 closing check of the committed tree (build a8903609c4af3398 rebuilt after the revert):
# GPU suite, smoke, the default bench line.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/c2_bench.json 2> $O/c2_bench.err
python -c "import json;d=json.load(open('$O/c2_bench.json'));print('c2',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['pmc_matches_build'],d['parity_sample']['mismatched_values'],d['end_to_end']['value'],d['cpu_baseline']['value'])"
