#!/bin/bash
# r06 run 52: the determinism guard at the session's last commit: bench's exact c2 and c3 49 Mpx
# launches run twice and compared bit for bit, 200k sampled pixels against the oracle
# (tools/debug_mismatch.py, the product code objects)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run52}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for C in c2 c3; do
  timeout -k 10 300 python tools/debug_mismatch.py --config $C --sample 200000 --no-rerun > $O/determinism_$C.json 2> $O/determinism_$C.err || { tail -5 $O/determinism_$C.err; exit 1; }
  python -c "import json;d=json.load(open('$O/determinism_$C.json'));print('$C',d['step2_differs_from_step1_pixels'],d['mismatching_pixels'],d['sampled'],d['jit'])"
done
