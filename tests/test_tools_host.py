"""CPU smoke tests of the diagnostics in tools/ that run without a GPU: the deferral diagnostic
(tools/defer_diag.py: the kernels' host build of the lazy DP + the reference's binary64 DP, used
for DESIGN.md § 2. resolve) on a small c2 scene."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_defer_diag_classifies_the_deferred_columns():
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, 'tools', 'defer_diag.py'),
                                   '--config', 'c2', '--pixels', '1500', '--examples', '2'],
                                  cwd=ROOT, timeout=300)
    d = json.loads(out)
    st = d['stats']
    assert st['pixels'] == 1500 and st['columns'] > 1500 * 20
    # about one pixel in a hundred defers (the GPU: 1.17 % of the c2 scene); every ambiguous
    # column on a deferred path is classified as an exact or a near tie
    assert 0 < st['deferred'] < 60
    kinds = d['ambiguous_columns_on_deferred_paths']
    assert sum(kinds.values()) == st.get('exact_tie_columns', 0) + st.get('near_tie_columns', 0)
    assert sum(kinds.values()) >= st['deferred']
