#!/bin/bash
# Profiling build with the analyze stage's phase probe (profiles/stamp_probe.h): cycle stamps per
# phase of the MAXY = ${1:-32} instance. Run on the box with profiles/stamps.py.
set -e
R=$(cd $(dirname $0)/.. && pwd)
bash $R/profiles/build_variant.sh liblt_hip_stamps ${1:-32} StampProbe $R/profiles/stamp_probe.h
