#!/bin/bash
# 2-rank gloo rehearsals of bench.py's N>1 path on one GPU at the round-3 build (both ranks on
# cuda:0; label tiles sent point-to-point to rank 0; every rank's parity sample): c4 (one mosaic,
# tiles round-robin) and c2 (one scene per rank). The driver's N>1 runs use RCCL instead.
# Usage: bash profiles/r03_rehearsal.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
P=29541
for C in c4 c2; do
  LT_BENCH_DEVICE=0 LT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $P bench.py \
    --gpus 2 --config $C --pixels 4000000 --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 \
    > $O/bench_${C}_n2_gloo.json 2> $O/bench_${C}_n2_gloo.err
  grep '^{' $O/bench_${C}_n2_gloo.json > $O/${C}_line.json  # gloo logs share stdout
  python -c "import json;d=json.load(open('$O/${C}_line.json'));print('$C n2',d['value'],d['n_gpus'],d['config']['parallelism'],d['parity_sample']['mismatched_values'])"
  P=$((P + 1))
done
