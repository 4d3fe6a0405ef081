#!/bin/bash
# 2-rank gloo rehearsals of bench.py's N>1 paths on one GPU (both ranks on cuda:0): c2 one scene
# per rank (weak) and c2 --strong (ONE scene, tiles round-robin: the north_star shape), each with
# an end-to-end step in the default N > 1 label mode ('own': every rank copies its own label
# planes to its host, no gather). The driver's N > 1 runs use RCCL. The line is the LAST stdout
# line starting with '{"metric"'.
# Usage: bash profiles/r06_rehearsal.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
P=29561
run() {  # name, args
  LT_BENCH_DEVICE=0 LT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $P bench.py \
    --gpus 2 $2 --pixels 4000000 --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 1 \
    > $O/bench_$1.out 2> $O/bench_$1.err
  python - "$O/bench_$1.out" "$O/$1.json" "$1" <<'PY'
import json, sys
lines = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')]
d = json.loads(lines[-1])
json.dump(d, open(sys.argv[2], 'w'))
print(sys.argv[3], d['value'], d['scaling'], d['config']['parallelism'], 'tiles', d['config']['tiles'],
      'parity mismatches', d['parity_sample']['mismatched_values'], 'of', d['parity_sample']['pixels'],
      'px; exchange', d['exchange_check'], '; e2e', d['end_to_end'] and (d['end_to_end']['value'], d['end_to_end']['labels']))
PY
  P=$((P + 1))
}
run c2_n2_weak "--config c2"
run c2_n2_strong "--config c2 --strong"
