#!/bin/bash
# A/B timing of kernel build variants (build/dev/*.so, built on the CPU side with
# -DLT_DEV_ONE_CONFIG: c2 kernel instances only) on the c2 bench. Usage: bash profiles/ab.sh [bench args]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/ab
for so in $R/${AB_DIR:-build/dev}/*.so; do
  n=$(basename $so .so)
  LT_HIP_LIB=$so timeout -k 10 120 python3 $R/bench.py --no-cpu-baseline --steps 2 "$@" \
    > $R/gpurun_out/ab/$n.json 2> $R/gpurun_out/ab/$n.err
  LT_HIP_LIB=$so timeout -k 10 120 python3 $R/profiles/ab_check.py 131072 11 ${AB_YEARS:-30} ${AB_LC:-10} || true
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'], d['resolve_stage']['ms_per_launch'], d['status_numeric_pixels'])" $R/gpurun_out/ab/$n.json $n
done
