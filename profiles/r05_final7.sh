#!/bin/bash
# Round-5 re-validation C + D at the committed build: c5 whole-scene parity (all 15 fields, two
# halves), then the default bench line with this build's committed PMC summaries.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
python -c "from land_trendr_amd._abi import build_hash; print('build', build_hash())" | tee $O/build.txt
timeout -k 10 170 python bench.py > $O/c2_bench.json 2> $O/c2_bench.err
python -c "import json;d=json.load(open('$O/c2_bench.json'));r=d['roofline'];print('c2',d['value'],d['ms_per_step'],r['achieved'],r['peak'],r['frac'],r.get('frac_at_kernel_occupancy'),r['pmc_matches_build'],r['traffic'],d['parity_sample']['mismatched_values'])"
timeout -k 10 560 python -u tests/full_scene_check.py --config c5 --last 24500000 --out $O/r05_full_scene_parity_c5_first_half.json > $O/full_c5a.log 2>&1
tail -1 $O/full_c5a.log
timeout -k 10 560 python -u tests/full_scene_check.py --config c5 --first 24500000 --out $O/r05_full_scene_parity_c5_second_half.json > $O/full_c5b.log 2>&1
tail -1 $O/full_c5b.log
