#!/bin/bash
# Round-5 final check D at the committed build, libraries rebuilt in a re-created container (the
# .so files the driver's round-end GPU tiers load): build identity, GPU suite, smoke, the default
# bench line, the 2-rank gloo rehearsal of bench's N > 1 path, then c5 whole-scene parity (all 15
# fields, two halves). Usage: bash profiles/r05_final14.sh <outdir under gpurun_out> A|B
# (A: identity, suite, smoke, line, rehearsal; B: c5 whole-scene parity — one gpurun call each)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
python -c "from land_trendr_amd._abi import build_hash; print('build', build_hash())" | tee $O/build.txt
if [ "$2" = A ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 170 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
tail -1 $O/smoke.txt
timeout -k 10 170 python bench.py > $O/c2_bench.json 2> $O/c2_bench.err
python -c "import json;d=json.load(open('$O/c2_bench.json'));r=d['roofline'];print('c2',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['pmc_matches_build'],d['parity_sample']['mismatched_values'])"
timeout -k 10 400 bash profiles/r04_rehearsal.sh $1/rehearsal
fi
if [ "$2" = B ]; then
for C in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $C > $O/${C}_bench.json 2> $O/${C}_bench.err
  python -c "import json;d=json.load(open('$O/${C}_bench.json'));r=d['roofline'];print('$C',d['value'],d['ms_per_step'],r['frac'],r['pmc_matches_build'],d['parity_sample']['mismatched_values'])"
done
timeout -k 10 560 python -u tests/full_scene_check.py --config c5 --last 24500000 --out $O/r05_full_scene_parity_c5_first_half.json > $O/full_c5a.log 2>&1
tail -1 $O/full_c5a.log
timeout -k 10 560 python -u tests/full_scene_check.py --config c5 --first 24500000 --out $O/r05_full_scene_parity_c5_second_half.json > $O/full_c5b.log 2>&1
tail -1 $O/full_c5b.log
fi
