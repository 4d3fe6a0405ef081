#!/bin/bash
# Build check (index kernels read pixel-interleaved bands in place: lt_index_kernel4i): GPU tests,
# smoke, default bench line (load_stage.alone, r03 PMC roofline), c5 phase-cut PMC (SQ counters of
# the kernel cut after each phase, profiles/phases.sh 48), then the c5 whole-scene parity.
# Usage: bash profiles/r03_run9.sh <outdir under gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1
echo "smoke ok"
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
python -c "import json;d=json.load(open('$O/bench_default.json'));print('c2',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['load_stage']['alone'],d['parity_sample']['mismatched_values'])"
cd /tmp
A="--config c5 --pixels 16777216 --steps 1 --warmup 0 --parity-sample 0 --e2e-steps 0 --no-cpu-baseline"
for V in liblt_cut48_0 liblt_cut48_1 liblt_cut48_2 liblt_cut48_3 liblt_cut48_full; do
  export LT_HIP_LIB=$R/build/exp/$V.so
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/cut/$V/sq -o run -- python3 $R/bench.py $A > $O/$V.sq.log 2>&1
  python3 $R/profiles/summarize_pmc.py $O/cut/$V $O/$V.json 16777216 > /dev/null
  python3 -c "import json;a=json.load(open('$O/$V.json'))['analyze'];w=a['SQ_WAVES'];print('$V', 'valu/wave %.0f salu/wave %.0f lds/wave %.0f valu_issue %.3f gui_ms %.2f' % (a['SQ_INSTS_VALU']/w, a['SQ_INSTS_SALU']/w, a['SQ_INSTS_LDS']/w, a['SQ_INSTS_VALU']*4/(1024*a['GRBM_GUI_ACTIVE']/8), a['GRBM_GUI_ACTIVE']/8/2.4e6))"
done
unset LT_HIP_LIB
cd $R
bash profiles/r03_full2.sh $1/full2
