#!/bin/bash
# Round-5 final check C' at the committed build: 2-rank gloo rehearsals of bench's N > 1 path on
# one GPU (pipelined steps: per-tile completion events left to finish()), then c5 whole-scene
# parity (all 15 fields, two halves)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
python -c "from land_trendr_amd._abi import build_hash; print('build', build_hash())" | tee $O/build.txt
timeout -k 10 400 bash profiles/r04_rehearsal.sh $1/rehearsal
timeout -k 10 560 python -u tests/full_scene_check.py --config c5 --last 24500000 --out $O/r05_full_scene_parity_c5_first_half.json > $O/full_c5a.log 2>&1
tail -1 $O/full_c5a.log
timeout -k 10 560 python -u tests/full_scene_check.py --config c5 --first 24500000 --out $O/r05_full_scene_parity_c5_second_half.json > $O/full_c5b.log 2>&1
tail -1 $O/full_c5b.log
