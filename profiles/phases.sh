#!/bin/bash
# Builds of the analyze kernel cut after phase K (profiles/stop_probe.h), one MAXY instance each,
# for per-phase PMC instruction counts: build/exp/liblt_cut<MAXY>_<K>.so (K = 0..3) and
# liblt_cut<MAXY>_full.so. Usage: bash profiles/phases.sh 32 48
set -e
R=$(cd $(dirname $0)/.. && pwd)
for MY in "$@"; do
  for K in 0 1 2 3; do
    bash $R/profiles/build_variant.sh liblt_cut${MY}_$K $MY "StopProbe<$K>" $R/profiles/stop_probe.h
  done
  bash $R/profiles/build_variant.sh liblt_cut${MY}_full $MY
done
