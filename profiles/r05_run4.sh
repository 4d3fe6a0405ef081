#!/bin/bash
# Round-5 call 4: the compact trendline (lt_fast.h tl_split + trendline_expand_kernel) — its
# GPU tests, the whole GPU suite, c5 bench A/B (split default, LT_TL_SPLIT=0, expand stream
# priorities) and a kernel trace of the split c5 bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_trendline.py -x -v --timeout 240 --timeout-method thread > $O/gpu_tl_tests.txt 2>&1
tail -1 $O/gpu_tl_tests.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
tail -1 $O/gpu_tests.txt
for v in split year_major xhigh xlow; do
  case $v in
    split) E="";; year_major) E="LT_TL_SPLIT=0";; xhigh) E="LT_EXPAND_PRIORITY=high";; xlow) E="LT_EXPAND_PRIORITY=low";;
  esac
  env $E timeout -k 10 300 python bench.py --config c5 --steps 5 --no-cpu-baseline --e2e-steps 0 > $O/c5_$v.json 2> $O/c5_$v.err
  python -c "import json;d=json.load(open('$O/c5_$v.json'));print('c5 $v',round(d['value'],1),d['ms_per_step'],d['roofline']['kernel_ms'],d['resolve_stage']['ms_per_launch'],d['expand_stage'],d['parity_sample']['mismatched_values'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 -- python bench.py --config c5 --steps 3 --no-cpu-baseline --e2e-steps 0 --parity-sample 0 > $O/prof_c5.log 2>&1
echo prof done
