#!/bin/bash
# r05 run 30: the JIT modules compiled with other AMDGPU machine-scheduler settings (override code
# objects of the product's c2 / c3 sources, tools/jit_variant.py --opt): max-ilp, max-memory-clause,
# the AMDGPU register-pressure trackers, no unclustered high-RP reschedule; and V15 (the lazy DP's
# per-start ballots taken of single compares, masked by ballots taken once per column / per DP:
# no VGPR 0/1 round trip per test), V16 (V15 + the LDS start loop's counter in an SGPR); A/B
# against the product build, twice, parity samples on
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run30}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, override dir or "", args
  if [ -n "$2" ]; then export LT_JIT_OVERRIDE_DIR=$R/build/override/$2; else unset LT_JIT_OVERRIDE_DIR; fi
  timeout -k 10 170 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'],d['jit']['override'])"
}
for i in 1 2; do
  for C in c2 c3; do
    b ${C}_base_$i "" "--config $C"
    for V in maxilp memclause trk nounc; do
      b ${C}_${V}_$i s_$V "--config $C"
    done
    b ${C}_v15_$i v15 "--config $C"
    b ${C}_v16_$i v16 "--config $C"
  done
  b c5_base_$i "" "--config c5"
  b c5_v15_$i v15 "--config c5"
  b c5_v16_$i v16 "--config c5"
done
