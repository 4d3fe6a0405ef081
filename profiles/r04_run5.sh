#!/bin/bash
# Round-4 call 5: exact-integer despike for int16 series (build/exp/liblt_idsp*_32.so) against the
# committed body (liblt_base*_32.so): c2 (1 rule) and c3 (4-rule instance) timing + parity sample,
# PMC instruction counts of the c2 instance.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
for i in 1 2; do
  for L in base idsp; do
    LT_HIP_LIB=$R/build/exp/liblt_${L}_32.so timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --e2e-steps 0 > $O/c2_$L$i.json 2> $O/c2_$L$i.err
    python -c "import json;d=json.load(open('$O/c2_$L$i.json'));print('c2 $L',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['resolve_stage']['deferred_pixels_last_tile'],d['parity_sample']['mismatched_values'])"
    LT_HIP_LIB=$R/build/exp/liblt_${L}4_32.so timeout -k 10 300 python bench.py --config c3 --steps 5 --no-cpu-baseline --e2e-steps 0 > $O/c3_$L$i.json 2> $O/c3_$L$i.err
    python -c "import json;d=json.load(open('$O/c3_$L$i.json'));print('c3 $L',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['resolve_stage']['deferred_pixels_last_tile'],d['parity_sample']['mismatched_values'])"
  done
done
cd /tmp
for L in idsp; do
  LT_HIP_LIB=$R/build/exp/liblt_${L}_32.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT \
    --output-format csv -d $O/pmc_$L -o run -- python3 $R/bench.py --config c2 --pixels 16777216 --steps 1 --warmup 0 --no-cpu-baseline --e2e-steps 0 --parity-sample 0 > $O/pmc_$L.log 2>&1
  echo "pmc $L ok"
done
