#!/bin/bash
# Builds of the analyze kernel cut after phase K (profiles/stop_probe.h), one MAXY instance each
# (LT_DEV_ONE_CONFIG), for per-phase PMC instruction counts: profiles/build/liblt_cut<MAXY>_<K>.so
# (K = 0..3) and liblt_cut<MAXY>_full.so. Usage: bash profiles/phases.sh 32 48
set -e
R=$(cd $(dirname $0)/.. && pwd)
mkdir -p $R/profiles/build
F="-x hip --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -fPIC -shared -Wno-unused-result"
for MY in "$@"; do
  for K in 0 1 2 3; do
    /opt/rocm/bin/hipcc $F -DLT_DEV_ONE_CONFIG=$MY "-DLT_ANALYZE_PROBE=StopProbe<$K>" \
      -include $R/profiles/stop_probe.h -o $R/profiles/build/liblt_cut${MY}_$K.so \
      $R/land_trendr_amd/csrc/lt_abi.hip -lhiprtc &
  done
  /opt/rocm/bin/hipcc $F -DLT_DEV_ONE_CONFIG=$MY -o $R/profiles/build/liblt_cut${MY}_full.so \
    $R/land_trendr_amd/csrc/lt_abi.hip -lhiprtc &
  wait
done
