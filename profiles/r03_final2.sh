#!/bin/bash
# Round-3 final build check (nontemporal band loads): GPU tests, smoke, default bench line (cpu
# baseline, end to end), c3 / c5 / c4 lines, kernel-trace stats of the default line, then the
# 2-rank gloo rehearsals (profiles/r03_rehearsal.sh).
# Usage: bash profiles/r03_final2.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/profiles/r03_final.sh $1
bash $R/profiles/r03_rehearsal.sh $1/rehearsal
