"""A CPU stand-in for the HIP engine (land_trendr_amd/engine.Engine) in the multi-process gloo
tests: index_tile evaluates the IndexProgram with numpy (oracle/index_oracle.py), analyze_tiles
runs oracle/lt_oracle.c into the given outputs. Test infrastructure only: on a GPU job the same
runner / job code drives liblt_hip.so."""
import numpy as np
import torch


class OracleEngine:
    device = torch.device('cpu')

    def compile_index(self, program):
        from land_trendr_amd.engine import IndexFn
        return IndexFn(None, program)

    def index_tile(self, fn, bands, out=None, stream=None):
        from oracle import index_oracle
        b = bands.numpy()
        v = torch.from_numpy(np.ascontiguousarray(
            index_oracle.evaluate(fn.program, np.moveaxis(b, 1, 0))))
        if out is None:
            return v
        out.copy_(v)
        return out

    def analyze_tiles(self, scene, params, tiles, fields, outs=None, ready=None):
        from oracle import oracle
        from land_trendr_amd.engine import valid_bytes
        for (vals, valid), o in zip(tiles, outs):
            want = oracle.analyze_tile(scene, params, vals.numpy().astype(np.float64),
                                       None if valid is None else
                                       valid_bytes(valid, scene.n_obs).numpy())
            for f in fields:
                o[f].copy_(torch.from_numpy(want[f][..., :o[f].shape[-1]]))
        return outs
