#!/bin/bash
# r06 run 12: the int16 band pair as one nontemporal 32-bit load in the JIT kernels
# (LT_SPEC_BAND_PAIR): GPU tests of the JIT / bench paths, then c2 / c3 / c5 lines, c2 twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run12}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_jit.py tests/test_gpu_index.py tests/test_gpu_mosaic.py > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
b() {  # name, env, args
  env $2 timeout -k 10 300 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['joined_steps']['value'],d['parity_sample']['mismatched_values'])"
}
b c2 LT_JIT_FIELDS=1 "--config c2"; b c3 LT_JIT_FIELDS=1 "--config c3"; b c5 LT_JIT_FIELDS=1 "--config c5"; b c2b LT_JIT_FIELDS=1 "--config c2"
