#!/bin/bash
# c3 A/B (same box, twice), c5 A/B of nontemporal plane stores (exp_nt_48 vs exp_yf_48),
# c3 A/B (same box, twice): the in-tree build vs mask bytes of a year loaded 4 at a time
# (profiles/build/exp_mb4_all.so); then whole-scene parity of the certified labels-only path on
# bench's c3 scene (masks, FD/GD/LD rules with filters). Usage: bash profiles/r02_run24.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c3 --steps 3 --no-cpu-baseline --e2e-steps 0 \
    > $O/ab_base_c3_$i.json 2> $O/ab_base_c3_$i.err
  LT_HIP_LIB=$R/profiles/build/exp_mb4_all.so timeout -k 10 300 python bench.py --config c3 \
    --steps 3 --no-cpu-baseline --e2e-steps 0 > $O/ab_mb4_c3_$i.json 2> $O/ab_mb4_c3_$i.err
  echo "ab $i ok"
done
for i in 1 2; do
for T in yf nt; do
  LT_HIP_LIB=$R/profiles/build/exp_${T}_48.so timeout -k 10 300 python bench.py --config c5 --steps 3 \
    --no-cpu-baseline --e2e-steps 0 > $O/ab_${T}_c5_$i.json 2> $O/ab_${T}_c5_$i.err
  echo "ab c5 $T $i ok"
done
done
timeout -k 10 900 python -u tests/full_scene_check.py --config c3 --labels-only \
  --out $O/full_c3_labels.json > $O/full_c3_labels.log 2>&1
echo "c3 labels-only ok"
