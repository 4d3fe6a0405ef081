#!/bin/bash
# r06 run 15.
# (1) The LT_PASSB_SLOTS=0 c3 variant no longer fails at this build (run 14: its control 0 of 2 Mpx
#     differing). The round-6 code object that did fail (build/override/s0, built 2026-10-18 20:32
#     from the same kernel ABI: KernelArgs, lt_tile_in / lt_tile_out unchanged) is loaded in its
#     place, as is and with its s_waitcnt made stricter (tools/co_patch.py --waitcnt):
#       s0old      the failing code object (control)
#       s0oldlgkm  every wait of lt_jit_analyze also waits for all LDS / scalar-memory accesses
#       s0oldvm    every wait of lt_jit_analyze also waits for all vector-memory accesses
# (2) The resolve kernel at 3 waves per SIMD (__launch_bounds__(64, 3): 167 VGPRs, no spills;
#     the product's (64, 4) spills 35) — c2 / c3 bench, same box, product first.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run15}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, override dir, seconds
  LT_JIT_OVERRIDE_DIR=$R/build/override/$2 LT_JIT_DEFINES=LT_PASSB_SLOTS=0 timeout -k 10 $3 \
    python tools/debug_mismatch.py --config c3 --sample 20000 --pixels 2000000 --no-rerun \
    > $O/c3_$1.json 2> $O/c3_$1.err
  rc=$?
  echo "$1 rc=$rc"
  python -c "import json;d=json.load(open('$O/c3_$1.json'));print('$1',{k:v for k,v in d.items() if k not in ('examples','diff_first','diff_lane_hist')})" || true
  return $rc
}
b() {  # name, env, args
  env $2 timeout -k 10 300 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  rc=$?
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['joined_steps']['value'],d['resolve_stage'],d['parity_sample']['mismatched_values'],d['jit'])" || true
  return $rc
}
dm s0old s0old 240 && dm s0oldlgkm s0oldlgkm 240 && dm s0oldvm s0oldvm 300 && \
b c2 "LT_NONE=1" "--config c2" && b c2_rw3 "LT_JIT_OVERRIDE_DIR=$R/build/override/rw3" "--config c2" && \
b c3 "LT_NONE=1" "--config c3" && b c3_rw3 "LT_JIT_OVERRIDE_DIR=$R/build/override/rw3" "--config c3"
