"""settings.json `index_eqn` (README.md:47, :75) compiled for the GPU load stage.

The reference evaluates the equation per raster with Python 2 `eval` on numpy band arrays
(`rast_algebra`, utils.py:447-484; band names from `parse_eqn_bands`, utils.py:219-225) and
writes the result with the input raster's band type (`array2raster`, utils.py:374-412, data_type
taken from the template at :396-397); `apply_grid` then reads it back as `float(val)`
(utils.py:357). Here the equation is parsed into a typed postfix program (no `eval`): the arithmetic
subset — band names B<n>, int and float literals, + - * / // and unary +/- with parentheses —
with numpy 1.x semantics as the reference ran them under Python 2:

  * dtypes follow numpy's legacy value-based promotion: array (+) array -> promote_types; array (+)
    Python scalar -> the scalar's min_scalar_type joins the promotion when its kind is not above
    the array's (int16 - 1 stays int16, int16 + 40000 becomes int32), else the scalar's own type
    (int16 * 0.5 -> float64);
  * integer results wrap (two's complement); `/` on integers is floor division (Python 2
    classic division), division by zero gives 0 (numpy's integer loops);
  * scalar-only subexpressions fold with Python 2 rules (int / int floors).

The store into the template type (GDAL's conversion, not available here) is: identity for the same
type, saturation for a narrower integer type, round-half-up (floor(x + 0.5)) then saturation for
float -> integer, NaN -> 0. Those three rules are parity-unpinned (no GDAL in this image); the
arithmetic is pinned by numpy itself (tests/test_index_eqn.py).

The program is compiled to a device kernel with hiprtc by the C++ side (lt_index_compile); the
kernel source is generated there from the program, never from the equation text.
"""
import ast
import re

import numpy as np

from . import _abi

# numpy dtype <-> LT_T_* element type codes (include/lt_abi.h)
DTYPES = {
    np.dtype(np.float64): _abi.LT_T_F64,
    np.dtype(np.int16): _abi.LT_T_I16,
    np.dtype(np.uint16): _abi.LT_T_U16,
    np.dtype(np.int32): _abi.LT_T_I32,
    np.dtype(np.float32): _abi.LT_T_F32,
    np.dtype(np.uint8): _abi.LT_T_U8,
    np.dtype(np.uint32): _abi.LT_T_U32,
    np.dtype(np.int8): _abi.LT_T_I8,
    np.dtype(np.int64): _abi.LT_T_I64,
}
CODES = {v: k for k, v in DTYPES.items()}

_BAND = re.compile(r'B(?P<band_num>\d+)')
_KIND_RANK = {'b': 0, 'u': 1, 'i': 1, 'f': 2}


def parse_eqn_bands(eqn):
    """Band numbers an equation references (utils.py:219-225): '(B2-B2)/(B3+B4)-B6' -> 2, 3, 4, 6.
    The reference returns them in set order; sorted here."""
    return sorted(int(d) for d in set(_BAND.findall(eqn)))


def multiple_replace(string, replacements):
    """utils.py:227-236: every key of `replacements` replaced in one regex pass."""
    pattern = re.compile('|'.join(replacements.keys()))
    return pattern.sub(lambda x: replacements[x.group()], string)


def _min_scalar_type(v, signed_array=False):
    """numpy's legacy min_scalar_type, with its 'small unsigned' rule: a non-negative integer
    that fits the signed type of its width promotes as that signed type next to a signed array
    (int8 array + 1000 -> int16, not int32)."""
    if isinstance(v, float):
        return np.min_scalar_type(v)
    order = ((np.int8, np.int16, np.int32, np.int64) if v < 0 or signed_array else
             (np.uint8, np.uint16, np.uint32, np.uint64))
    for t in order:
        info = np.iinfo(t)
        if info.min <= v <= info.max:
            return np.dtype(t)
    if v >= 0 and signed_array and v <= np.iinfo(np.uint64).max:
        return np.dtype(np.uint64)
    raise ValueError('index_eqn: integer literal %r out of range' % v)


def _scalar_default_type(v):
    return np.dtype(np.float64) if isinstance(v, float) else np.dtype(np.int64)  # Py2 int = C long


def result_dtype(a, b):
    """numpy 1.x (legacy) result type of an operation on a and b, each either a np.dtype (an
    array operand) or a Python int/float (a scalar operand)."""
    arrays = [x for x in (a, b) if isinstance(x, np.dtype)]
    scalars = [x for x in (a, b) if not isinstance(x, np.dtype)]
    if not scalars:
        return np.promote_types(a, b)
    t = arrays[0]
    s = scalars[0]
    s_kind = 'f' if isinstance(s, float) else 'i'
    if _KIND_RANK[s_kind] <= _KIND_RANK[t.kind]:
        return np.promote_types(t, _min_scalar_type(s, t.kind == 'i'))
    return np.promote_types(t, _scalar_default_type(s))


def _py2_binop(op, x, y):
    if isinstance(op, ast.Add):
        return x + y
    if isinstance(op, ast.Sub):
        return x - y
    if isinstance(op, ast.Mult):
        return x * y
    if isinstance(op, (ast.Div, ast.FloorDiv)):
        if isinstance(x, int) and isinstance(y, int):
            return x // y  # Python 2 classic division of ints floors; ZeroDivisionError as in Py2
        return x / y if isinstance(op, ast.Div) else float(np.floor(x / y))
    raise ValueError('index_eqn: unsupported operator %s' % type(op).__name__)


_OPS = {ast.Add: _abi.LT_OP_ADD, ast.Sub: _abi.LT_OP_SUB, ast.Mult: _abi.LT_OP_MUL,
        ast.Div: _abi.LT_OP_DIV, ast.FloorDiv: _abi.LT_OP_FLOORDIV}


class IndexProgram:
    """A validated, typed postfix program for one index_eqn.

    bands: the reference band numbers (1-based) the equation uses, in the order of the band planes
    the load kernel receives (plane s holds band bands[s]). ops: (op, dtype, ival, fval) tuples.
    """

    def __init__(self, eqn, band_dtype=np.int16, out_dtype=None, raster_count=None):
        self.eqn = eqn
        self.band_dtype = np.dtype(band_dtype)
        self.out_dtype = np.dtype(out_dtype) if out_dtype is not None else self.band_dtype
        if self.band_dtype not in DTYPES or self.out_dtype not in DTYPES:
            raise ValueError('index_eqn: unsupported raster type %s / %s' %
                             (self.band_dtype, self.out_dtype))
        bands = parse_eqn_bands(eqn)
        if not bands:
            raise ValueError('index_eqn: %r references no band' % eqn)
        # rast_algebra's own checks (utils.py:462-465), same messages
        if raster_count is not None and max(bands) > raster_count:
            raise Exception('Band %s not present in %s' % (max(bands), '<raster>'))
        if min(bands) <= 0:
            raise Exception('Invalid band "%s" - bands must be >= 1')
        self.bands = bands
        try:
            tree = ast.parse(eqn.strip(), mode='eval')
        except SyntaxError as e:
            raise ValueError('index_eqn: %s' % e)
        self.ops = []
        root = self._emit(tree.body)
        if not isinstance(root, np.dtype):  # a constant equation: numpy broadcasts it
            self.ops.append((_abi.LT_OP_CONST_F if isinstance(root, float) else _abi.LT_OP_CONST_I,
                             _scalar_default_type(root), root))
            root = _scalar_default_type(root)
        self.result_dtype = root
        if len(self.ops) > _abi.LT_MAX_PROG:
            raise ValueError('index_eqn: more than %d operations' % _abi.LT_MAX_PROG)
        if len(self.bands) > _abi.LT_MAX_BANDS:
            raise ValueError('index_eqn: more than %d bands' % _abi.LT_MAX_BANDS)

    # Returns the operand: a np.dtype for an array value (code emitted) or a Python scalar.
    def _emit(self, node):
        if isinstance(node, ast.Name):
            m = re.fullmatch(r'B(\d+)', node.id)
            if not m:
                raise ValueError('index_eqn: unknown name %r' % node.id)
            self.ops.append((_abi.LT_OP_BAND, self.band_dtype, self.bands.index(int(m.group(1)))))
            return self.band_dtype
        if isinstance(node, ast.Constant) and type(node.value) in (int, float):
            return node.value
        if isinstance(node, ast.UnaryOp) and isinstance(node.op, (ast.USub, ast.UAdd)):
            v = self._emit(node.operand)
            if not isinstance(v, np.dtype):
                return -v if isinstance(node.op, ast.USub) else +v
            if isinstance(node.op, ast.USub):
                self.ops.append((_abi.LT_OP_NEG, v, 0))
            return v
        if isinstance(node, ast.BinOp) and type(node.op) in _OPS:
            # evaluate both sides first (postfix), scalars become typed constants
            n0 = len(self.ops)
            a = self._emit(node.left)
            b = self._emit(node.right)
            if not isinstance(a, np.dtype) and not isinstance(b, np.dtype):
                return _py2_binop(node.op, a, b)
            t = result_dtype(a, b)
            if not isinstance(a, np.dtype):
                self.ops.insert(n0, self._const(a))  # before the right operand's code
            if not isinstance(b, np.dtype):
                self.ops.append(self._const(b))
            self.ops.append((_OPS[type(node.op)], t, 0))
            return t
        raise ValueError('index_eqn: unsupported expression %s' % ast.dump(node))

    @staticmethod
    def _const(v):
        if isinstance(v, float):
            return (_abi.LT_OP_CONST_F, np.dtype(np.float64), v)
        return (_abi.LT_OP_CONST_I, np.dtype(np.int64), v)

    def to_c(self):
        p = _abi.LtIndexProg()
        p.n_ops = len(self.ops)
        p.n_bands = len(self.bands)
        p.band_type = DTYPES[self.band_dtype]
        p.out_type = DTYPES[self.out_dtype]
        for k, (op, t, v) in enumerate(self.ops):
            p.ops[k].op = op
            p.ops[k].type = DTYPES[np.dtype(t)]
            if op == _abi.LT_OP_CONST_F:
                p.ops[k].fval = float(v)
            else:
                p.ops[k].ival = int(v)
        return p

    def __repr__(self):
        return 'IndexProgram(%r: %s -> %s)' % (self.eqn, self.result_dtype, self.out_dtype)
