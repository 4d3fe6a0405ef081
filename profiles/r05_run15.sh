#!/bin/bash
# r05 run 15: (1) the LT_PASSB_SLOTS=0 c3 mismatches with the JIT module compiled with every
# wait forced to zero (-mllvm -amdgpu-waitcnt-forcezero; tools/jit_variant.py) against the same
# hiprtc build without it; (2) the overlap probe incl. CU-masked analyze; (3) c5 as one launch per
# scene; c3 / c4 at this build
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run15}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
dm() {  # name, override dir
  LT_JIT_OVERRIDE_DIR=$R/build/override/$2 LT_JIT_DEFINES=LT_PASSB_SLOTS=0 timeout -k 10 300 python tools/debug_mismatch.py --config c3 --sample 100000 > $O/c3_$1.json 2> $O/c3_$1.err
  python -c "import json;d=json.load(open('$O/c3_$1.json'));print('$1',{k:v for k,v in d.items() if k!='examples'})"
}
dm s0_override s0
dm s0_forcezero s0fz
timeout -k 10 300 python tools/overlap_probe.py > $O/overlap_probe.json 2> $O/overlap_probe.err
cat $O/overlap_probe.json
b() {  # name, args
  timeout -k 10 300 python bench.py $2 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
b c5_whole "--config c5 --tile 49000000"
b c5 "--config c5"
b c3 "--config c3"
b c4 "--config c4"
