#!/bin/bash
# Round-5 final check D: the default bench line with this build's committed PMC summaries
# (roofline achieved / frac / traffic from profiles/r05_pmc_c2.json).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
python -c "from land_trendr_amd._abi import build_hash; print('build', build_hash())" | tee $O/build.txt
timeout -k 10 300 python bench.py > $O/c2_bench.json 2> $O/c2_bench.err
python -c "import json;d=json.load(open('$O/c2_bench.json'));r=d['roofline'];print('c2',d['value'],d['ms_per_step'],r['achieved'],r['peak'],r['frac'],r.get('frac_at_kernel_occupancy'),r['pmc_matches_build'],r['traffic'],d['parity_sample']['mismatched_values'])"
