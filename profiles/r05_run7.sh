#!/bin/bash
# Round-5 call 7: per-tile completion events for the label exchange (lt_analyze_tiles_ev), bench's
# N > 1 tiling rate at N = 1, the data-movement overlap probe, 2-rank gloo rehearsals.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
tail -1 $O/gpu_tests.txt
timeout -k 10 400 python bench.py > $O/c2_bench.json 2> $O/c2_bench.err
python -c "import json;d=json.load(open('$O/c2_bench.json'));print('c2',d['value'],d['ms_per_step'],d['parity_sample']['mismatched_values'],d['n_gt_1_tiling'],d['jit'])"
timeout -k 10 300 python tools/overlap_probe.py > $O/overlap_probe.json 2> $O/overlap_probe.err
cat $O/overlap_probe.json
timeout -k 10 700 bash profiles/r04_rehearsal.sh $1/rehearsal
