#!/bin/bash
# bench lines of c2 and c5 at several tile sizes (pixels per launch). Usage: bash tile_sweep.sh <out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
for C in c5 c2; do
  for T in 16777216 8388608 5505024 4194304; do
    timeout -k 10 300 python bench.py --config $C --tile $T --steps 5 --no-cpu-baseline \
      --e2e-steps 0 > $O/${C}_$T.json 2> $O/${C}_$T.err
    echo "$C $T ok"
  done
done
