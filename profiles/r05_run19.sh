#!/bin/bash
# r05 run 19: VALU / SALU instructions per wave by phase (PMC of the JIT analyze kernel cut after
# each phase, LT_JIT_STOP_AFTER=k, one 16.8 Mpx c2 / c3 launch each; timing-only builds), and c5
# without the winner pick's winner-row stores (timing-only: what a separate fill launch would save)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r05_run19}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for C in c2 c3; do
  for k in 0 1 2 3 full; do
    if [ $k = full ]; then unset LT_JIT_DEFINES; else export LT_JIT_DEFINES=LT_JIT_STOP_AFTER=$k; fi
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/${C}_$k -o run -- python3 $R/bench.py --config $C --pixels 16777216 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0 --tiled-steps 0 --no-cpu-baseline > $O/${C}_$k.log 2>&1
    python3 - $O/${C}_$k <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); disp = set()
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'lt_jit_analyze' in r['Kernel_Name']:
            tot[r['Counter_Name']] += float(r['Counter_Value']); disp.add(r['Dispatch_Id'])
n = max(1, len(disp)); w = tot['SQ_WAVES'] / n
print(sys.argv[1].split('/')[-1], 'launches', len(disp), 'waves/launch %.0f' % w,
      'GRBM_GUI_ACTIVE/launch %.0f' % (tot['GRBM_GUI_ACTIVE'] / n),
      ' '.join('%s/wave=%.0f' % (k[9:], v / n / w) for k, v in sorted(tot.items())
               if k.startswith('SQ_INSTS') and w))
PY
  done
done
cd $R
for v in base nowinner; do
  if [ $v = nowinner ]; then export LT_JIT_DEFINES=LT_AB_NO_WINNER_STORE=1; else unset LT_JIT_DEFINES; fi
  timeout -k 10 170 python bench.py --config c5 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 --parity-sample 0 > $O/c5_$v.json 2> $O/c5_$v.err
  python -c "import json;d=json.load(open('$O/c5_$v.json'));print('c5 $v',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'])"
done
