#!/bin/bash
# r05 run 31: A/B against the product (build 66502c3a) of V16 (the lazy DP's per-start ballots of
# single compares + the LDS start loop's counter in an SGPR; run 30), V17 (V16 + OPTa[i]'s
# exactness as a bit-field-extract mask anded into Emax: 3 VALU instead of 6 per start) and V18b
# (V17 + 16-bit year-offset slots beside int16 series of <= 32 years: one LDS address per point),
# twice, parity samples on
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run31}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, override dir or "", args
  if [ -n "$2" ]; then export LT_JIT_OVERRIDE_DIR=$R/build/override/$2; else unset LT_JIT_OVERRIDE_DIR; fi
  timeout -k 10 170 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'],d['jit']['override'])"
}
for i in 1 2; do
  for C in c2 c3 c5; do
    b ${C}_base_$i "" "--config $C"
    for V in v16 v17 v18b; do
      b ${C}_${V}_$i $V "--config $C"
    done
  done
done
