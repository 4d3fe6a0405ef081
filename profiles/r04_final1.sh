#!/bin/bash
# Round-4 final call 1: GPU suite, smoke, the default bench line (cpu_baseline, end to end), the
# c3 / c4 / c5 lines, the kernel trace of the default line, the 2-rank gloo rehearsals.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || rc=$?
echo "gpu tests rc=$rc"; tail -2 $O/gpu_tests.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
echo "smoke ok"; tail -2 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/c2_bench.json 2> $O/c2_bench.err
python -c "import json;d=json.load(open('$O/c2_bench.json'));print('c2',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['pmc_matches_build'],d['parity_sample']['mismatched_values'],d['end_to_end']['value'],d['cpu_baseline']['value'])"
for C in c3 c4 c5; do
  timeout -k 10 400 python bench.py --config $C --no-cpu-baseline --e2e-steps 0 > $O/${C}_bench.json 2> $O/${C}_bench.err
  python -c "import json;d=json.load(open('$O/${C}_bench.json'));print('$C',d['value'],d['ms_per_step'],d['roofline']['frac'],d['parity_sample']['mismatched_values'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --no-cpu-baseline --e2e-steps 0 --steps 10 > $O/kt.log 2>&1
echo "kernel trace ok"
cd $R
bash $R/profiles/r04_rehearsal.sh $1/rehearsal
