#!/bin/bash
# PMC passes for the engine's kernels (one rocprofv3 run per counter group; MI355X_MICROARCH.md
# rocprofv3 PMC slots: <= 8 SQ, <= 2 GRBM, FETCH_SIZE and WRITE_SIZE in separate passes).
# Usage (on the GPU box, from the repo root): bash profiles/pmc_passes.sh <outdir> [bench args]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="$@"
# the build the counters belong to, with this environment (summarize_pmc.py reads it)
python3 -c "import sys; sys.path.insert(0, '$R'); from land_trendr_amd._abi import build_hash; print(build_hash())" > $OUT/_build.txt
run() {
  name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
    python3 $R/bench.py $ARGS --no-cpu-baseline > $OUT/$name.log 2>&1
  echo "pass $name ok"
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT
run sq2 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
run fetch FETCH_SIZE
run write WRITE_SIZE
