"""A/B variant parity check (used by profiles/ab.sh): one c2-shaped tile (30 years, 1 obs/yr, GD
rule, line_cost 10) through the library LT_HIP_LIB names, bit-compared with the oracle."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
from golden_io import _bits_equal  # noqa: E402
from land_trendr_amd.engine import get_engine  # noqa: E402
from land_trendr_amd.scene import build_scene, parse_date  # noqa: E402
from land_trendr_amd.settings import compile_params  # noqa: E402
from land_trendr_amd.synth import make_scene  # noqa: E402
from oracle import oracle  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 17
years = int(sys.argv[3]) if len(sys.argv) > 3 else 30
lc = float(sys.argv[4]) if len(sys.argv) > 4 else 10.0
sc = make_scene(n, n_years=years, seed=int(sys.argv[2]) if len(sys.argv) > 2 else 11)
meta = build_scene(sc.dates, parse_date('2014-07-01'))
params, _ = compile_params(lc, [{'name': 'gd', 'val': 1, 'change_type': 'GD'}])
eng = get_engine(0)
exp = oracle.analyze_tile(meta, params, sc.values.numpy(), None, n_threads=16)
for fields in (None, ('status', 'n_years', 'matched', 'class_val', 'onset_year', 'duration',
                      'magnitude', 'initial_val')):
    out = (eng.analyze_tile(meta, params, sc.values.to(eng.device), None) if fields is None else
           eng.analyze_tile(meta, params, sc.values.to(eng.device), None, fields))
    torch.cuda.synchronize()
    got = {k: t.cpu().numpy() for k, t in out.items()}
    bad = {}
    for k, a in got.items():
        e = exp[k][:a.shape[0]] if a.ndim == 2 else exp[k]
        if k in ('onset_year', 'duration', 'class_val', 'magnitude', 'initial_val'):
            m = exp['matched'][:a.shape[0]].astype(bool)
            a, e = np.where(m, a, 0), np.where(m, e, 0)
        ok = _bits_equal(a, e) if a.dtype.kind == 'f' else (a == e)
        if not ok.all():
            bad[k] = int((~ok).sum())
    print('parity', n, 'px', 'all fields' if fields is None else 'labels only',
          'OK' if not bad else bad)
