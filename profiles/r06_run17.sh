#!/bin/bash
# r06 run 17: c5 tilings with pipelined steps (each tile whole waves, so every launch is the
# LT_SPEC_FULL module): default 3 tiles (2 x 16,777,216 + 15,445,568), 2 tiles (24,500,032 +
# 24,499,968), 4 tiles (3 x 12,250,048 + 12,249,856); product first, then again, same box
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run17}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, args
  timeout -k 10 300 python bench.py $2 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  rc=$?
  python -c "import json;d=json.load(open('$O/$1.json'));c=d['config'];print('$1',round(d['value'],1),d['ms_per_step'],c['tiles'],c['tile_pixels'],d['roofline']['kernel_ms'],d['joined_steps']['value'],d['parity_sample']['mismatched_values'],d['jit']['tiles_fallback_timed'])" || true
  return $rc
}
b c5 "--config c5" && b c5_t2 "--config c5 --tile 24500032" && b c5_t4 "--config c5 --tile 12250048" && \
b c5_again "--config c5" && b c5_t2_again "--config c5 --tile 24500032"
