#!/bin/bash
# PMC summaries of the product build for c2 / c3 / c5 (one 16.8 Mpx launch each; the bench
# roofline's inputs, profiles/r03_pmc_<config>.json). Usage: bash profiles/r03_pmc_all.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$1
for C in c2 c3 c5; do
  bash $R/profiles/pmc_passes.sh $O/$C --config $C --pixels 16777216 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0
  python3 $R/profiles/summarize_pmc.py $R/$O/$C $R/$O/r03_pmc_$C.json 16777216 > /dev/null
  python3 -c "import json;a=json.load(open('$R/$O/r03_pmc_$C.json'))['analyze'];w=a['SQ_WAVES'];print('$C', 'valu/wave %.0f salu/wave %.0f valu_issue %.3f write_B/px %.0f read_B/px %.0f' % (a['SQ_INSTS_VALU']/w, a['SQ_INSTS_SALU']/w, a['SQ_INSTS_VALU']*4/(1024*a['GRBM_GUI_ACTIVE']/8), a['hbm_write_bytes']/16777216, a['hbm_read_bytes']/16777216))"
done
