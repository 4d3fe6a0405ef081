#!/bin/bash
# r06 run 19: one-tile pipelined steps at world 1 with their own label rasters per bank (runner
# _flip_bank + LabelExchange.rebind). Before, the label slabs were shared by the two banks, so a
# step's analyze waited for the previous step's resolve (kernel trace of r06_fa: analyze starts
# 53 us after the resolve ends, every step). (1) the pipelined-steps GPU tests; (2) c2 / c3 bench,
# the product's resolve (4 waves per SIMD, grid 4096) and the no-spill resolve at 3 and
# 2 waves per SIMD (grids 3072 / 2048; override code objects, the latter by co_patch --vgprs 248); (3) the default
# c2 command under rocprofv3 --kernel-trace: does the resolve now run beside the next analyze?
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run19}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_mosaic.py -m gpu -q -x --timeout 300 --timeout-method thread -k pipelined > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
b() {  # name, env, args
  env $2 timeout -k 10 300 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  rc=$?
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['joined_steps']['value'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])" || true
  return $rc
}
b c2 "LT_NONE=1" "--config c2" && b c2_rw3 "LT_JIT_OVERRIDE_DIR=$R/build/override/rw3" "--config c2" && \
b c3 "LT_NONE=1" "--config c3" && b c3_rw3 "LT_JIT_OVERRIDE_DIR=$R/build/override/rw3" "--config c3" && \
b c2_rw2 "LT_JIT_OVERRIDE_DIR=$R/build/override/rw3v248" "--config c2" && \
b c3_rw2 "LT_JIT_OVERRIDE_DIR=$R/build/override/rw3v248" "--config c3" && \
b c2_again "LT_NONE=1" "--config c2" || exit 1
cd /tmp
timeout -k 10 220 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/c2_under_rocprof.json 2> $O/kt.err
echo "kernel trace rc=$?"
cd $R
python - <<PY
import csv, glob
f = glob.glob('$O/kt/**/run_kernel_trace.csv', recursive=True) + glob.glob('$O/kt/run_kernel_trace.csv')
rows = list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
ks = [r for r in rows if r['Kernel_Name'] in ('lt_jit_analyze', 'lt_jit_resolve')]
t0 = int(ks[0]['Start_Timestamp'])
for r in ks[:16]:
    print('%s %9.3f %9.3f' % (r['Kernel_Name'][7:], (int(r['Start_Timestamp']) - t0) / 1e6, (int(r['End_Timestamp']) - t0) / 1e6))
PY
