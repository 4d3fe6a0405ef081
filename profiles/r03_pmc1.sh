#!/bin/bash
# PMC of the c2 analyze launch (one 16.8 Mpx tile), fused load stage (pixel-interleaved bands)
# against the index raster path, same library (build/exp/c2_pair.so).
# Usage: bash profiles/r03_pmc1.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export LT_HIP_LIB=$R/build/exp/c2_pair.so
LT_FUSED_INDEX=1 LT_BAND_LAYOUT=pixel timeout -k 10 500 bash profiles/pmc_passes.sh $1/fused --pixels 16777216 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0
python3 profiles/summarize_pmc.py $R/$1/fused $R/$1/fused.json 16777216 > /dev/null
LT_FUSED_INDEX=0 LT_BAND_LAYOUT=planar timeout -k 10 500 bash profiles/pmc_passes.sh $1/raster --pixels 16777216 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0
python3 profiles/summarize_pmc.py $R/$1/raster $R/$1/raster.json 16777216 > /dev/null
python3 - $R/$1 <<'PY'
import json, sys
a = json.load(open(sys.argv[1] + '/fused.json'))['analyze']
b = json.load(open(sys.argv[1] + '/raster.json'))['analyze']
for k in sorted(a):
    if isinstance(a[k], (int, float)) and k in b:
        print('%-24s fused %14.4g  raster %14.4g  ratio %.3f' % (k, a[k], b[k], a[k] / b[k] if b[k] else 0))
PY
