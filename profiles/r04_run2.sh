#!/bin/bash
# Round-4 second call: VALU issue-peak microbenchmark (one generation of co-resident waves, SCC
# clobber fixed), GPU tests (the multi-rank GPU job over gloo with host-staged label slabs),
# resolve stream priority A/B on c2 (low = the new default vs normal), kernel trace of the
# default line, 2-rank gloo rehearsals with the exchange check.
# Usage: bash profiles/r04_run2.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 ./build/bin/valu_peak 20000 > $O/valu_peak.json 2> $O/valu_peak.err
python -c "
import json;d=json.load(open('$O/valu_peak.json'))
for r in d['results']: print(r['kind'], r['waves_per_simd'], 'cyc/instr/SIMD', round(r['cycles_per_valu_simd'],3), 'G/s', round(r['g_valu_per_s_chip'],1), 'clk', round(r['implied_clock_ghz'],3))"
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for i in 1 2; do
  for P in low normal; do
    LT_RESOLVE_PRIORITY=$P timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/bench_c2_$P$i.json 2> $O/bench_c2_$P$i.err
    python -c "import json;d=json.load(open('$O/bench_c2_$P$i.json'));print('c2 $P',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage'],d['parity_sample']['mismatched_values'])"
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --no-cpu-baseline --e2e-steps 0 --steps 10 > $O/kt.log 2>&1
echo "kernel trace ok"
cd $R
bash $R/profiles/r04_rehearsal.sh $1/rehearsal
python -c "
import json
for c in ('c2','c4'):
    d=json.load(open('$O/rehearsal/'+c+'_n2_gloo_rehearsal_1gpu.json')); print(c, d['exchange_check'])"
