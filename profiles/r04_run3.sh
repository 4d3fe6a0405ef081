#!/bin/bash
# Round-4 call 3: VALU peak microbenchmark with VOP1 moves and VCC selects; c2 phase cuts of the
# analyze kernel (PMC instruction counts and timing per cut build, build/exp/liblt_cut32_<K>.so);
# A/B of the resolve kernel at 4 waves per SIMD (build/exp/liblt_res4_32.so vs liblt_cut32_full).
# Usage: bash profiles/r04_run3.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 ./build/bin/valu_peak 20000 > $O/valu_peak.json 2> $O/valu_peak.err
python -c "
import json;d=json.load(open('$O/valu_peak.json'))
for r in d['results']:
  if r['waves_per_simd'] in (4, 8): print(r['kind'], r['waves_per_simd'], 'G/s', round(r['g_valu_per_s_chip'],1), 'cyc', round(r['cycles_per_valu_simd_nominal'],3))"
for L in cut32_0 cut32_1 cut32_2 cut32_3 cut32_full res4_32; do
  LT_HIP_LIB=$R/build/exp/liblt_$L.so timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 --parity-sample 0 > $O/bench_$L.json 2> $O/bench_$L.err
  python -c "import json;d=json.load(open('$O/bench_$L.json'));print('$L',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'])"
done
LT_HIP_LIB=$R/build/exp/liblt_res4_32.so timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 > $O/bench_res4_parity.json 2> $O/bench_res4_parity.err
python -c "import json;d=json.load(open('$O/bench_res4_parity.json'));print('res4 parity',d['value'],d['parity_sample']['mismatched_values'])"
cd /tmp
for L in cut32_0 cut32_1 cut32_2 cut32_3 cut32_full; do
  LT_HIP_LIB=$R/build/exp/liblt_$L.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT \
    --output-format csv -d $O/pmc_$L -o run -- python3 $R/bench.py --config c2 --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 --parity-sample 0 > $O/pmc_$L.log 2>&1
  echo "pmc $L ok"
done
