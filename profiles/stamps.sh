#!/bin/bash
# Profiling build of liblt_hip.so with the analyze stage's phase probe (profiles/stamp_probe.h).
# Built here (CPU) into profiles/build/; run on the box with profiles/stamps.py.
set -e
R=$(cd $(dirname $0)/.. && pwd)
mkdir -p $R/profiles/build
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -fPIC -shared \
  -Wno-unused-result -DLT_ANALYZE_PROBE=StampProbe -include $R/profiles/stamp_probe.h \
  -o $R/profiles/build/liblt_hip_stamps.so $R/land_trendr_amd/csrc/lt_abi.hip -lhiprtc "$@"
