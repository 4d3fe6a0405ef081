#!/bin/bash
# r06 run 18: tile sizes with pipelined steps (run 17: c5 in 4 tiles 1456 vs 1405-1425 Mpx/s in
# 3). Every tile whole waves (the LT_SPEC_FULL module): c5 in 4, 5, 7, 8 tiles; c2 / c3 in 4 tiles
# against their one 49 Mpx launch; same box
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run18}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
b() {  # name, args
  timeout -k 10 300 python bench.py $2 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  rc=$?
  python -c "import json;d=json.load(open('$O/$1.json'));c=d['config'];print('$1',round(d['value'],1),d['ms_per_step'],c['tiles'],c['tile_pixels'],d['roofline']['kernel_ms'],d['joined_steps']['value'],d['parity_sample']['mismatched_values'],d['jit']['tiles_fallback_timed'])" || true
  return $rc
}
b c5_t4 "--config c5 --tile 12250048" && b c5_t5 "--config c5 --tile 9800000" && \
b c5_t7 "--config c5 --tile 7000000" && b c5_t8 "--config c5 --tile 6125056" && \
b c5_t3 "--config c5" && b c5_t4b "--config c5 --tile 12250048" && \
b c2_t1 "--config c2" && b c2_t4 "--config c2 --tile 12250048" && \
b c3_t1 "--config c3" && b c3_t4 "--config c3 --tile 12250048"
