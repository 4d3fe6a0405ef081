#!/bin/bash
# Round-5 call 5: the trendline expand kernel with one thread per (pixel, 8-year chunk); c5 A/B against the
# year-major loop, a kernel trace, the compact-trendline tests, and the v_rcp_f64 accuracy check.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_trendline.py -x -v --timeout 240 --timeout-method thread > $O/gpu_tl_tests.txt 2>&1
tail -1 $O/gpu_tl_tests.txt
for v in split year_major; do
  case $v in split) E="LT_TL_SPLIT=1";; year_major) E="LT_TL_SPLIT=0";; esac
  env $E timeout -k 10 300 python bench.py --config c5 --steps 5 --no-cpu-baseline --e2e-steps 0 > $O/c5_$v.json 2> $O/c5_$v.err
  python -c "import json;d=json.load(open('$O/c5_$v.json'));print('c5 $v',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['expand_stage']['ms_per_launch'],d['parity_sample']['mismatched_values'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_c5 -o c5 -- python bench.py --config c5 --steps 3 --no-cpu-baseline --e2e-steps 0 --parity-sample 0 > $O/prof_c5.log 2>&1
echo prof done
