#!/bin/bash
# c5 attribution (timing-only variants, wrong outputs): product instance vs no year-major f64
# stores vs no per-year stores at all. Per 16.8 Mpx launch: VALU per wave, VALU issue, cycles,
# bytes read/written (rocprofv3 --pmc, one pass per block); then bench lines.
# Usage: bash profiles/r03_ab6.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="--config c5 --pixels 16777216 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0 --no-cpu-baseline"
for V in c5_prod c5_noys c5_nost; do
  export LT_HIP_LIB=$R/build/exp/$V.so
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/$V/sq -o run -- python3 $R/bench.py $A > $O/$V.sq.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$V/write -o run -- python3 $R/bench.py $A > $O/$V.w.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$V/fetch -o run -- python3 $R/bench.py $A > $O/$V.f.log 2>&1
  python3 $R/profiles/summarize_pmc.py $O/$V $O/$V.json 16777216 > /dev/null
  python3 -c "import json;a=json.load(open('$O/$V.json'))['analyze'];w=a['SQ_WAVES'];print('$V', 'valu/wave %.0f salu/wave %.0f valu_issue %.3f gui_cyc %.3g write_B/px %.0f read_B/px %.0f' % (a['SQ_INSTS_VALU']/w, a['SQ_INSTS_SALU']/w, a['SQ_INSTS_VALU']*4/(1024*a['GRBM_GUI_ACTIVE']/8), a['GRBM_GUI_ACTIVE']/8, a['hbm_write_bytes']/16777216, a['hbm_read_bytes']/16777216))"
done
unset LT_HIP_LIB
cd $R
B="timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 --parity-sample 0"
for V in c5_prod c5_noys c5_nost; do
  LT_HIP_LIB=build/exp/$V.so $B --config c5 > $O/bench_$V.json 2> $O/bench_$V.err
  python -c "import json;d=json.load(open('$O/bench_$V.json'));print('$V',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])"
done
