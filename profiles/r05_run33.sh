#!/bin/bash
# r05 run 33: A/B against the product (build 3aaa6717) of pass B's per-slot values made
# branch-free (pbsel: x1 / xq loaded once before the slots; pbsel2: loaded in each slot), c2 and
# c3, twice, parity samples on. Overrides built by tools/jit_variant.py --hdr-root from a header copy.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run33}
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
    for V in pbsel pbsel2; do
      b ${C}_${V}_$i $V "--config $C"
    done
  done
done
