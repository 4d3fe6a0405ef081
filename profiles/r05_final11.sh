#!/bin/bash
# Round-5 final check A' at the committed build (pipelined steps): GPU suite, smoke, the default
# bench line (with this build's committed PMC), its rocprofv3 kernel-trace stats (the same
# command), and the c3 / c4 / c5 lines
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
python -c "from land_trendr_amd._abi import build_hash; print('build', build_hash())" | tee $O/build.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 170 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
tail -1 $O/smoke.txt
timeout -k 10 170 python bench.py > $O/c2_bench.json 2> $O/c2_bench.err
python -c "import json;d=json.load(open('$O/c2_bench.json'));r=d['roofline'];print('c2',d['value'],d['ms_per_step'],r['kernel_ms'],r['kernel_ms_joined'],r['frac'],r['frac_joined'],r['pmc_matches_build'],d['parity_sample']['mismatched_values'],d['end_to_end']['value'],d['n_gt_1_tiling']['ratio_to_value'],d['cpu_baseline']['value'])"
cd /tmp
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py > $O/kt.log 2>&1
echo "kernel trace ok"
cd $R
for C in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $C > $O/${C}_bench.json 2> $O/${C}_bench.err
  python -c "import json;d=json.load(open('$O/${C}_bench.json'));r=d['roofline'];print('$C',d['value'],d['ms_per_step'],r['frac'],r['frac_joined'],r['pmc_matches_build'],d['parity_sample']['mismatched_values'])"
done
