#!/bin/bash
# Round-2 GPU call: every GPU test (incl. the bench-path mosaic tests), the default bench line,
# c4 (196 Mpx mosaic) on one GPU, and a 2-rank gloo rehearsal of the c4 exchange on one GPU.
# Usage: bash profiles/r02_run2.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$1
mkdir -p $R/$O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $R/$O/gpu_tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python bench.py > $R/$O/bench_c2.json 2> $R/$O/bench_c2.err
echo "bench c2 ok"
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $R/$O/bench_c4.json \
  2> $R/$O/bench_c4.err
echo "bench c4 ok"
LT_BENCH_DEVICE=0 LT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py \
  --gpus 2 --config c4 --pixels 4000000 --steps 2 --warmup 1 --no-cpu-baseline \
  > $R/$O/bench_c4_n2_gloo.json 2> $R/$O/bench_c4_n2_gloo.err
echo "n2 rehearsal ok"
