#!/bin/bash
# 2-rank gloo rehearsals of bench.py's N>1 path on one GPU (both ranks on cuda:0; label tiles
# sent point-to-point to rank 0; every rank's parity sample): c2 (one scene per rank, the shape of
# the driver's weak-scaling runs) and c4 (one mosaic, tiles round-robin). The driver's N>1 runs
# use RCCL instead. The line is the LAST stdout line starting with '{"metric"' (gloo and
# torch.distributed.run write their own lines to the same stdout; r03_rehearsal.sh's grep '^{'
# picked up one of those).
# Usage: bash profiles/r04_rehearsal.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
P=29541
for C in c2 c4; do
  LT_BENCH_DEVICE=0 LT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $P bench.py \
    --gpus 2 --config $C --pixels 4000000 --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 \
    > $O/bench_${C}_n2_gloo.out 2> $O/bench_${C}_n2_gloo.err
  python - "$O/bench_${C}_n2_gloo.out" "$O/${C}_n2_gloo_rehearsal_1gpu.json" "$C" <<'PY'
import json, sys
lines = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')]
d = json.loads(lines[-1])
json.dump(d, open(sys.argv[2], 'w'))
print(sys.argv[3], 'n2', d['value'], d['n_gpus'], d['config']['parallelism'],
      'parity mismatches', d['parity_sample']['mismatched_values'], 'of',
      d['parity_sample']['pixels'], 'px')
PY
  P=$((P + 1))
done
