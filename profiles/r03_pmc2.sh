#!/bin/bash
# PMC of the c5 analyze launch cut after each phase (profiles/stop_probe.h builds) and of the full
# kernel: VALU / SALU instructions, wave cycles, and bytes written, per 16.8 Mpx launch.
# Usage: bash profiles/r03_pmc2.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="--config c5 --pixels 16777216 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0 --no-cpu-baseline"
for V in liblt_cut48_0 liblt_cut48_1 liblt_cut48_2 liblt_cut48_3 c5_st0; do
  export LT_HIP_LIB=$R/build/exp/$V.so
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/$V/sq -o run -- python3 $R/bench.py $A > $O/$V.sq.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$V/write -o run -- python3 $R/bench.py $A > $O/$V.w.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$V/fetch -o run -- python3 $R/bench.py $A > $O/$V.f.log 2>&1
  python3 $R/profiles/summarize_pmc.py $O/$V $O/$V.json 16777216 > /dev/null
  python3 -c "import json;a=json.load(open('$O/$V.json'))['analyze'];w=a['SQ_WAVES'];print('$V', 'valu/wave %.0f salu/wave %.0f valu_issue %.3f gui_cyc %.3g write_B/px %.0f read_B/px %.0f' % (a['SQ_INSTS_VALU']/w, a['SQ_INSTS_SALU']/w, a['SQ_INSTS_VALU']*4/(1024*a['GRBM_GUI_ACTIVE']/8), a['GRBM_GUI_ACTIVE']/8, a['hbm_write_bytes']/16777216, a['hbm_read_bytes']/16777216))"
done
