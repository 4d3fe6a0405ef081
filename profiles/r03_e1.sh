set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/e1; mkdir -p $O
B="timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --e2e-steps 0"
$B --config c5 > $O/c5_prod.json 2> $O/c5_prod.err; echo c5 prod; tail -c 400 $O/c5_prod.json
for v in base48 noys48 nost48; do
  LT_HIP_LIB=build/exp/$v.so $B --config c5 > $O/c5_$v.json 2> $O/c5_$v.err; echo $v
done
$B > $O/c2_prod.json 2> $O/c2_prod.err; echo c2 prod
LT_LOAD_PRIORITY=-1 $B > $O/c2_prio.json 2> $O/c2_prio.err; echo c2 prio
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/e1/*.json')):
    d=json.load(open(f)); print(f, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['load_stage']['ms_per_launch_overlapped'], d['resolve_stage'])
PY
