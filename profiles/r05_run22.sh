#!/bin/bash
# r05 run 22: the cost of v_mad_u64_u32 (the compiler's int32 a*a + s in the DP's sums) against
# v_mad_u32_u24 and v_mul_lo_u32 (tools/valu_peak.hip kinds), and variant V8 (V1 + the DP's
# Sxx += x*x as one v_mad_u32_u24) A/B against V1 and the product, twice, parity samples on
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run22}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 build/bin/valu_peak 20000 mad_u64_u32,mad_u32_u24,mul_lo_u32,add_u32,fma_f64 > $O/valu_peak_mul.json
python -c "
import json;d=json.load(open('$O/valu_peak_mul.json'))
for r in d['results']:
    if r['waves_per_simd'] in (4,8): print(r['kind'], r['waves_per_simd'], round(r['cycles_per_valu_simd_nominal'],2))"
b() {  # name, override dir or "", args
  if [ -n "$2" ]; then export LT_JIT_OVERRIDE_DIR=$R/build/override/$2; else unset LT_JIT_OVERRIDE_DIR; fi
  timeout -k 10 170 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'],d['jit']['override'])"
}
for i in 1 2; do
  for C in c2 c3; do
    b ${C}_base_$i "" "--config $C"
    b ${C}_v1_$i v1 "--config $C"
    b ${C}_v8_$i v8 "--config $C"
  done
done
