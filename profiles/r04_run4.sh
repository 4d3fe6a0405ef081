#!/bin/bash
# Round-4 call 4: the division-free DP exit / tracking tests (build/exp/liblt_fastx_32.so, c2
# instance) against the product build: timing, parity sample, PMC instruction counts.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
for i in 1 2; do
  for L in base fastx; do
    LIB=$R/build/exp/liblt_${L}_32.so
    LT_HIP_LIB=$LIB timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/bench_$L$i.json 2> $O/bench_$L$i.err
    python -c "import json;d=json.load(open('$O/bench_$L$i.json'));print('$L',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['resolve_stage']['deferred_pixels_last_tile'],d['parity_sample']['mismatched_values'])"
  done
done
cd /tmp
for L in fastx; do
  LT_HIP_LIB=$R/build/exp/liblt_${L}_32.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT \
    --output-format csv -d $O/pmc_$L -o run -- python3 $R/bench.py --config c2 --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 --parity-sample 0 > $O/pmc_$L.log 2>&1
  echo "pmc $L ok"
done
