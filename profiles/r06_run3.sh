#!/bin/bash
# r06 run 3: the LT_PASSB_SLOTS=0 c3 variant at 2 Mpx, once each:
#   re      the variant's hiprtc assembly (-save-temps) reassembled as is (control of this path)
#   resync  the same assembly with `s_waitcnt vmcnt(0) lgkmcnt(0)` after every memory instruction
#           (a correct forcezero: hiprtc's -amdgpu-waitcnt-forcezero also puts a wait inside the
#           s_getpc_b64 / s_add_u32 pc-relative pairs, so its constant-table addresses are off)
#   s0lds10k  the variant's code object with 10240 B of LDS per workgroup instead of 6464: still
#           16 waves per CU (VGPR-bound), a different LDS layout per CU
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run3}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, override dir, defines
  LT_JIT_OVERRIDE_DIR=$R/build/override/$2 LT_JIT_DEFINES=$3 timeout -k 10 240 \
    python tools/debug_mismatch.py --config c3 --sample 20000 --pixels 2000000 --no-rerun \
    > $O/c3_$1.json 2> $O/c3_$1.err
  rc=$?
  echo "$1 rc=$rc"
  python -c "import json;d=json.load(open('$O/c3_$1.json'));print('$1',{k:v for k,v in d.items() if k not in ('examples','diff_first','diff_lane_hist')}); print([(e['pixel'],e['fields'],e['got'].get('status')) for e in d['examples']])" || true
  return $rc
}
dm re re LT_PASSB_SLOTS=0 && dm resync resync LT_PASSB_SLOTS=0 && dm s0lds10k s0lds10k LT_PASSB_SLOTS=0
