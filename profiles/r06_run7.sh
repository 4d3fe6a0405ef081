#!/bin/bash
# r06 run 7: JIT kernels specialised for the launch's output planes (LT_SPEC_FIELDS; c3 instance
# 37 -> 12 spilled VGPRs): GPU tests of the JIT / bench / job paths, then same-box A/B of bench
# c2 / c3 / c5 against LT_JIT_FIELDS=0, then the job bench with the new defaults
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/r06_run7}
mkdir -p $O
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_jit.py tests/test_gpu_mosaic.py tests/test_gpu_job.py > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
b() {  # name, env, args
  env $2 timeout -k 10 300 python bench.py $3 --steps 5 --no-cpu-baseline --e2e-steps 0 --tiled-steps 0 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['joined_steps']['value'],d['resolve_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
}
b c3_f1 LT_JIT_FIELDS=1 "--config c3" && b c3_f0 LT_JIT_FIELDS=0 "--config c3" && b c2_f1 LT_JIT_FIELDS=1 "--config c2" && b c2_f0 LT_JIT_FIELDS=0 "--config c2" && b c5_f1 LT_JIT_FIELDS=1 "--config c5" && b c5_f0 LT_JIT_FIELDS=0 "--config c5" && b c3_f1b LT_JIT_FIELDS=1 "--config c3" && b c2_f1b LT_JIT_FIELDS=1 "--config c2" || exit 1
timeout -k 10 600 python tools/job_bench.py --rows 7000 --cols 7000 --years 30 --diag > $O/job_c2.json 2> $O/job_c2.err
rc=$?; grep -E "^(setup|parse|analyze|output)" $O/job_c2.err; python -c "import json;d=json.load(open('$O/job_c2.json'));print(d['seconds'],d['job_s'],d['parse_decoded_gb_per_s'],d['diag'],d['check']['mismatches'])"; exit $rc
