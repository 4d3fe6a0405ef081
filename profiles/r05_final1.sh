#!/bin/bash
# Round-5 final check A at the committed build: GPU suite, smoke, the default bench line, its
# rocprofv3 kernel-trace stats (the same command), and PMC passes of c2 / c3 / c5 at this build
# (profiles/pmc_passes.sh stamps the build hash at collection).
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
python -c "import json;d=json.load(open('$O/c2_bench.json'));print('c2',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['pmc_matches_build'],d['parity_sample']['mismatched_values'],d['end_to_end']['value'],d['cpu_baseline']['value'])"
cd /tmp
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py > $O/kt.log 2>&1
echo "kernel trace ok"
cd $R
for C in c2 c3 c5; do
  bash $R/profiles/pmc_passes.sh $1/pmc/$C --config $C --pixels 16777216 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0 --tiled-steps 0
  python3 $R/profiles/summarize_pmc.py $O/pmc/$C $O/r05_pmc_$C.json 16777216 > /dev/null
  echo "pmc $C ok"
done
