#!/bin/bash
# Round-6 final checks at the committed build (one gpurun call per part):
#   A  build identity, the GPU suite, smoke, the default bench line (c2), and the rocprofv3 kernel
#      trace of the same default command
#   P  PMC passes (profiles/pmc_passes.sh, build stamped) of the launches bench.py times: c2 and c3
#      one 49 Mpx launch each, c5 its 16.8 Mpx tiles of the 49 Mpx scene
#   B  c3 / c4 / c5 bench lines; run-to-run determinism of bench's exact c2 and c3 launches
#      (tools/debug_mismatch.py)
#   F  whole-scene parity of bench's exact c2 and c3 launches (every pixel against the oracle)
#   C  c5 whole-scene parity, all 15 fields, in two halves
# Usage: bash profiles/r06_final.sh <outdir under gpurun_out> A|P|B|F|C
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
python -c "from land_trendr_amd._abi import build_hash; print('build', build_hash())" | tee $O/build_$2.txt
if [ "$2" = A ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 170 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
tail -1 $O/smoke.txt
timeout -k 10 200 python bench.py > $O/c2_bench.json 2> $O/c2_bench.err
python -c "import json;d=json.load(open('$O/c2_bench.json'));r=d['roofline'];print('c2',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['pmc_matches_build'],d['parity_sample']['mismatched_values'],d['joined_steps']['value'],d['end_to_end']['value'],d['cpu_baseline']['value'])"
cd /tmp
timeout -k 10 220 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py > $O/c2_bench_under_rocprof.json 2> $O/kt.err
echo "kernel trace ok"
cd $R
fi
if [ "$2" = P ]; then
for C in c2 c3; do
  bash $R/profiles/pmc_passes.sh $1/pmc/$C --config $C --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0 --tiled-steps 0 --no-overlap
  python3 $R/profiles/summarize_pmc.py $O/pmc/$C $O/r06_pmc_$C.json 49000000 > /dev/null
  echo "pmc $C ok"
done
bash $R/profiles/pmc_passes.sh $1/pmc/c5 --config c5 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0 --tiled-steps 0 --no-overlap
python3 $R/profiles/summarize_pmc.py $O/pmc/c5 $O/r06_pmc_c5.json 16333333 > /dev/null
echo "pmc c5 ok"
fi
if [ "$2" = B ]; then
for C in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $C > $O/${C}_bench.json 2> $O/${C}_bench.err
  python -c "import json;d=json.load(open('$O/${C}_bench.json'));r=d['roofline'];print('$C',d['value'],d['ms_per_step'],r['frac'],r['pmc_matches_build'],d['parity_sample']['mismatched_values'])"
done
for C in c2 c3; do
  timeout -k 10 200 python tools/debug_mismatch.py --config $C --sample 200000 --no-rerun > $O/determinism_$C.json 2> $O/determinism_$C.err
  python -c "import json;d=json.load(open('$O/determinism_$C.json'));print('$C',{k:v for k,v in d.items() if k not in ('examples','diff_hist64','diff_first','diff_lane_hist')})"
done
fi
if [ "$2" = F ]; then
for C in c2 c3; do
  timeout -k 10 560 python -u tests/full_scene_check.py --config $C --labels-only --whole --bench-fields --out $O/r06_full_scene_parity_${C}_whole.json > $O/full_$C.log 2>&1
  tail -1 $O/full_$C.log
done
fi
if [ "$2" = C ]; then
timeout -k 10 560 python -u tests/full_scene_check.py --config c5 --last 24500000 --out $O/r06_full_scene_parity_c5_first_half.json > $O/full_c5a.log 2>&1
tail -1 $O/full_c5a.log
timeout -k 10 560 python -u tests/full_scene_check.py --config c5 --first 24500000 --out $O/r06_full_scene_parity_c5_second_half.json > $O/full_c5b.log 2>&1
tail -1 $O/full_c5b.log
fi
