#!/bin/bash
# Round-4 first GPU call: GPU tests (incl. bench's exact c2 / c3 labels-only instances at full
# size), the VALU issue-peak microbenchmark, the default bench line, PMC passes of c2 at this
# build, kernel-trace stats of the default line, and the 2-rank gloo rehearsals.
# Usage: bash profiles/r04_run1.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 120 ./build/bin/valu_peak 4000 > $O/valu_peak.json 2> $O/valu_peak.err
echo "valu_peak ok"
python -c "
import json;d=json.load(open('$O/valu_peak.json'))
for r in d['results']: print(r['kind'], r['waves_per_simd'], round(r['cycles_per_valu_simd'],3), round(r['g_valu_per_s_chip'],1), round(r['implied_clock_ghz'],3))"
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
python -c "import json;d=json.load(open('$O/bench_default.json'));print('c2',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['parity_sample']['mismatched_values'])"
bash $R/profiles/pmc_passes.sh $1/pmc/c2 --config c2 --pixels 16777216 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0
python3 $R/profiles/summarize_pmc.py $O/pmc/c2 $O/r04_pmc_c2.json 16777216 > /dev/null
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --no-cpu-baseline --e2e-steps 0 --steps 10 > $O/kt.log 2>&1
echo "kernel trace ok"
cd $R
bash $R/profiles/r04_rehearsal.sh $1/rehearsal
