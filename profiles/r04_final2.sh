#!/bin/bash
# Round-4 final call 2: PMC passes of c2 / c3 / c5 at the final build (one 16.8 Mpx launch each),
# summarised with the build hash.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
for C in c2 c3 c5; do
  bash $R/profiles/pmc_passes.sh $1/pmc/$C --config $C --pixels 16777216 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0
  python3 $R/profiles/summarize_pmc.py $O/pmc/$C $O/r04_pmc_$C.json 16777216 > /dev/null
  echo "pmc $C ok"
done
