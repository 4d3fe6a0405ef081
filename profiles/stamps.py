"""Phase breakdown of the analyze kernel from the profiling build (profiles/stamps.sh): one
16.8 Mpx tile of a bench config through the runner path, the per-phase shader cycles summed over
waves. Usage (GPU box): python profiles/stamps.py c2 [c5 ...] > gpurun_out/stamps.json"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ['LT_HIP_LIB'] = os.path.join(ROOT, 'profiles', 'build', 'liblt_hip_stamps.so')
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from land_trendr_amd import _abi  # noqa: E402
from land_trendr_amd.distributed import Mosaic  # noqa: E402
from land_trendr_amd.engine import get_engine  # noqa: E402
from land_trendr_amd.index_eqn import IndexProgram  # noqa: E402
from land_trendr_amd.runner import MosaicRunner  # noqa: E402
from land_trendr_amd.settings import compile_params  # noqa: E402
from land_trendr_amd.synth import mosaic_inputs  # noqa: E402

PHASES = ['winner', 'despike', 'dp', 'fits_walk_offers', 'label_writes']


def main(cfgs):
    lib = _abi.load_lib()
    lib.lt_diag_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    res = {}
    for name in cfgs:
        c = bench.CONFIGS[name]
        eng = get_engine(0)
        m = Mosaic([1 << 24], 1 << 24, 1, 0, 'by_scene')
        items = mosaic_inputs(m, c['years'], c['k'][0], c['k'][1], c['mask'], c['seed'],
                              eng.device, bench.TARGET)
        params, _ = compile_params(c['line_cost'], c['rules'], c['mode'])
        fn = eng.compile_index(IndexProgram('B1 - B2', band_dtype='int16'))
        fields = ['status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude']
        if c['trendline']:
            fields += bench.TRENDLINE_FIELDS
        r = MosaicRunner(eng, m, params, items, fields, fn)
        r.step()
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 8)()
        lib.lt_diag_stamps(buf, 1)  # reset after the warm-up pass
        r.step()
        torch.cuda.synchronize()
        lib.lt_diag_stamps(buf, 1)
        tot = sum(buf[k] for k in range(5))
        res[name] = {'waves': buf[7], 'cycles_per_wave': {p: round(buf[k] / max(1, buf[7]))
                                                          for k, p in enumerate(PHASES)},
                     'fraction': {p: round(buf[k] / tot, 4) for k, p in enumerate(PHASES)}}
        print(name, json.dumps(res[name]), file=sys.stderr, flush=True)
        del r, items
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == '__main__':
    main(sys.argv[1:] or ['c2'])
