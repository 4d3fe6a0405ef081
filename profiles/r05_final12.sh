#!/bin/bash
# Round-5 final check B' at the committed build: whole-scene parity of bench's exact c2 / c3
# launches (one 49 Mpx launch, bench's labels-only fields, every pixel against the oracle), the
# run-to-run determinism check of the same launches (tools/debug_mismatch.py)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
python -c "from land_trendr_amd._abi import build_hash; print('build', build_hash())" | tee $O/build.txt
for C in c2 c3; do
  timeout -k 10 560 python -u tests/full_scene_check.py --config $C --labels-only --whole --bench-fields --out $O/r05_full_scene_parity_${C}_whole.json > $O/full_$C.log 2>&1
  tail -1 $O/full_$C.log
  timeout -k 10 170 python tools/debug_mismatch.py --config $C --sample 200000 --no-rerun > $O/determinism_$C.json 2> $O/determinism_$C.err
  python -c "import json;d=json.load(open('$O/determinism_$C.json'));print('$C',{k:v for k,v in d.items() if k!='examples'})"
done
