#!/bin/bash
# Round-5 first GPU call: the extended VALU class table, the GPU suite with
# bench's exact whole-scene launches (item 1), the default bench line, and whole-scene parity of
# bench's exact c2 / c3 launches (one 49 Mpx tile, bench's fields). The JIT code objects are
# written under the output directory so their ISA can be read back.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
export LT_JIT_CACHE=$O/jit
timeout -k 10 180 build/bin/valu_peak 20000 > $O/valu_peak.json
echo valu_peak done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
tail -1 $O/gpu_tests.txt
timeout -k 10 400 python bench.py > $O/c2_bench.json 2> $O/c2_bench.err
python -c "import json;d=json.load(open('$O/c2_bench.json'));print('c2',d['value'],d['ms_per_step'],d['roofline']['frac'],d['parity_sample']['mismatched_values'],d['resolve_stage'])"
timeout -k 10 560 python -u tests/full_scene_check.py --config c2 --labels-only --whole --bench-fields --out $O/full_c2_whole.json > $O/full_c2.log 2>&1
tail -1 $O/full_c2.log
timeout -k 10 560 python -u tests/full_scene_check.py --config c3 --labels-only --whole --bench-fields --out $O/full_c3_whole.json > $O/full_c3.log 2>&1
tail -1 $O/full_c3.log
