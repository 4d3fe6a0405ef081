"""TEST INFRASTRUCTURE — CPU oracle of the load stage (index_eqn), never on the product path.

Evaluates a land_trendr_amd.index_eqn.IndexProgram with numpy on host arrays, node by node as
numpy 1.x ran the reference's `eval` (utils.py:476-482): both operands cast to the node's result
dtype, the numpy ufunc in that dtype (integer wrap, floor division with x // 0 = 0), then the store
into the output type with the rules index_eqn.py documents (GDAL's conversion: identity, integer
saturation, float -> floor(x + 0.5) then saturation, NaN -> 0; parity-unpinned without GDAL).
The numpy arithmetic is independent of the generated HIP source it checks.
"""
import numpy as np

from land_trendr_amd import _abi


def _as(x, t):
    if isinstance(x, np.ndarray):
        return x.astype(t, copy=False) if x.dtype == t else x.astype(t, casting='unsafe')
    return np.asarray(x).astype(t, casting='unsafe')  # a scalar cast like numpy's value cast


def evaluate(program, bands):
    """bands: [NB, ...] array of band planes (program.bands order, program.band_dtype).
    Returns the index in program.out_dtype."""
    st = []
    with np.errstate(all='ignore'):
        for op, t, v in program.ops:
            t = np.dtype(t)
            if op == _abi.LT_OP_BAND:
                st.append(np.asarray(bands[v], dtype=program.band_dtype))
            elif op in (_abi.LT_OP_CONST_I, _abi.LT_OP_CONST_F):
                st.append(v)
            elif op == _abi.LT_OP_NEG:
                st.append(np.negative(_as(st.pop(), t)))
            else:
                b = _as(st.pop(), t)
                a = _as(st.pop(), t)
                if op == _abi.LT_OP_ADD:
                    r = np.add(a, b, dtype=t)
                elif op == _abi.LT_OP_SUB:
                    r = np.subtract(a, b, dtype=t)
                elif op == _abi.LT_OP_MUL:
                    r = np.multiply(a, b, dtype=t)
                elif op == _abi.LT_OP_DIV and t.kind == 'f':
                    r = np.true_divide(a, b, dtype=t)
                else:
                    r = np.floor_divide(a, b, dtype=t)
                st.append(r)
        assert len(st) == 1
        r = st[0]
        if not isinstance(r, np.ndarray):
            r = np.full(np.shape(bands[0]), r)
        return store(r, program.out_dtype)


def store(r, out):
    out = np.dtype(out)
    if r.dtype == out:
        return r.copy()
    if out.kind == 'f':
        return r.astype(out)
    info = np.iinfo(out)
    if r.dtype.kind == 'f':
        x = np.floor(r.astype(np.float64) + 0.5)
        x = np.where(np.isnan(r), 0.0, np.clip(x, info.min, info.max))
        return x.astype(out)
    x = np.clip(r.astype(np.int64) if r.dtype != np.uint64 else r, info.min, info.max)
    return x.astype(out)
