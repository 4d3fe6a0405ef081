"""CPU-side checks of the boundary: the HIP library loads and exports every symbol that
include/lt_abi.h declares, the ctypes mirror matches the header's struct layouts, and the
host-side reference semantics (LabelRule validation, pick_winners date grouping) hold.
No compute call is made here (no GPU in this suite)."""
import ctypes
import datetime as dt
import os
import re
import subprocess

import numpy as np
import pytest

from land_trendr_amd import _abi
from land_trendr_amd.classes import LabelRule
from land_trendr_amd.scene import build_scene, parse_date
from land_trendr_amd.settings import compile_params

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'lt_abi.h')


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r'^\w[\w\s\*]*?\b(lt_\w+)\s*\(', src, re.M)))


def test_library_exports_every_declared_symbol():
    lib = _abi.load_lib()
    decl = declared_functions()
    assert set(decl) == set(_abi.EXPORTS), decl
    for name in decl:
        assert hasattr(lib, name), name
    assert lib.lt_abi_version() == _abi.LT_ABI_VERSION


def test_library_is_gfx950_code_object():
    blob = open(_abi.LIB_PATH, 'rb').read()
    assert b'amdgcn-amd-amdhsa--gfx950' in blob     # offload bundle entry of the fat binary
    assert b'gfx90a' not in blob and b'gfx942' not in blob


def test_struct_layouts_match_header():
    """Compile a tiny C program against the header and compare sizeof/offsetof with ctypes."""
    import tempfile
    checks = {
        'lt_rule': _abi.LtRule, 'lt_params': _abi.LtParams, 'lt_scene': _abi.LtScene,
        'lt_tile_in': _abi.LtTileIn, 'lt_tile_out': _abi.LtTileOut,
        'lt_label_in': _abi.LtLabelIn, 'lt_jit_stats': _abi.LtJitStats,
    }
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s"' % HEADER,
             'int main(void){']
    for cname, cls in checks.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in cls._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append('return 0;}')
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, 'l.c')
        open(c, 'w').write('\n'.join(lines))
        exe = os.path.join(d, 'l')
        subprocess.check_call(['gcc', '-o', exe, c])
        got = dict(l.split() for l in subprocess.check_output([exe], text=True).splitlines())
    for cname, cls in checks.items():
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(got['%s.%s' % (cname, f)]) == getattr(cls, f).offset, (cname, f)


# ---- LabelRule (classes_test.py:9-30 and classes.py:32-64) ----

def test_label_rule_create():
    lr = LabelRule({'name': 'greatest_fast_disturbance', 'val': 5, 'change_type': 'GD',
                    'duration': ['<', 4]})
    assert (lr.name, lr.val, lr.change_type, lr.duration) == (
        'greatest_fast_disturbance', 5, 'GD', ['<', 4])
    assert lr.onset_year is None and lr.pre_threshold is None


@pytest.mark.parametrize('opts', [
    {'name': 'g', 'val': 5, 'change_type': 'GD', 'duration': ['<', 4, 'BAD']},
    {'val': 5},
    {'name': 'g', 'val': 0},
    {'name': 'g', 'val': 5, 'change_type': 'XX'},
    {'name': 'g', 'val': 5, 'onset_year': ('>=', 1990)},
    {'name': 'g', 'val': 5, 'pre_threshold': ['>']},
])
def test_label_rule_invalid(opts):
    with pytest.raises(ValueError):
        LabelRule(opts)


def test_rule_compilation():
    p, rules = compile_params(2.5, [
        {'name': 'a', 'val': 3, 'change_type': 'FD', 'onset_year': ['>=', 1995],
         'duration': ['<', 4]},
        {'name': 'b', 'val': 7, 'change_type': None, 'onset_year': ['>', 1995],
         'pre_threshold': ['<', 100]},
        {'name': 'c', 'val': 1, 'change_type': 'LD', 'duration': []},
    ], 'documented')
    assert p.line_cost == 2.5 and p.n_rules == 3 and p.pre_threshold_mode == 1
    r = p.rules
    assert (r[0].change_type, r[0].onset_op, r[0].onset_val) == (1, _abi.LT_Q_GE, 1995.0)
    assert (r[0].duration_op, r[0].duration_val, r[0].class_val) == (_abi.LT_Q_LT, 4.0, 3)
    assert (r[1].change_type, r[1].onset_op, r[1].pre_op) == (0, _abi.LT_Q_OTHER, _abi.LT_Q_LT)
    assert (r[2].change_type, r[2].duration_op) == (3, _abi.LT_Q_UNSET)


def test_non_numeric_qualifiers_follow_python2_ordering():
    """The reference runs on Python 2, where a number compares below any str/list and above None
    (classes.py:190-211 compare the raw JSON value): '2000' is not 2000. Each such qualifier has
    a constant outcome; the compiled rules reproduce it (checked through the oracle's labels)."""
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    sc = make_scene(256, n_years=30, seed=9)
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    base = {'name': 'g', 'val': 1, 'change_type': 'GD'}
    cases = [  # (filter, same-as-unfiltered?)
        ({'onset_year': ['>=', '2000']}, False), ({'onset_year': ['<=', '2000']}, True),
        ({'onset_year': ['=', '1990']}, False), ({'onset_year': ['<=', None]}, False),
        ({'onset_year': ['>=', None]}, True), ({'duration': ['>', 'x']}, False),
        ({'duration': ['<', 'x']}, True), ({'duration': ['>', None]}, True),
        ({'duration': ['<', None]}, False), ({'onset_year': ['>=', [1]]}, False),
        ({'pre_threshold': ['>', 'x']}, False), ({'pre_threshold': ['<', 'x']}, True),
    ]
    params, _ = compile_params(10.0, [base] + [dict(base, name='r%d' % i, **f)
                                               for i, (f, _) in enumerate(cases)], 'documented')
    out = oracle.analyze_tile(meta, params, sc.values.numpy(), None)
    m = out['matched']
    assert m[0].sum() > 200
    for i, (f, same) in enumerate(cases):
        assert (m[i + 1] == m[0]).all() if same else not m[i + 1].any(), f


# ---- pick_winners' date half (utils.py:491-521) ----

def test_scene_grouping_and_distances():
    dates = ['2001-07-02', '2001-06-30', '1999-01-01', '2001-07-01', '1999-12-31']
    s = build_scene(dates, parse_date('2014-07-01'))
    assert list(s.years) == [1999, 2001]
    assert list(s.slot_begin) == [0, 2, 5]
    assert list(s.order) == [2, 4, 0, 1, 3]        # input order kept inside a year
    assert list(s.dist) == [181, 183, 1, 1, 0]
    assert list(s.feb29_bad) == [0, 0]


def test_scene_feb29_target():
    s = build_scene(['1996-03-01', '1997-03-01'], parse_date('2012-02-29'))
    assert list(s.feb29_bad) == [0, 1]
    assert s.dist[0] == 1


def test_parse_date_strict():
    assert parse_date('2014-07-01') == dt.datetime(2014, 7, 1)
    for bad in ['2014/07/01', '14-07-01', 'x', '2014-02-30']:
        with pytest.raises(ValueError):
            parse_date(bad)


def _c2_jit_source(flags=_abi.LT_JIT_SRC_SPEC | _abi.LT_JIT_SRC_SCENE):
    import sys
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import jit_isa
    return jit_isa, jit_isa.jit_source('c2', flags=flags)


def test_jit_source_is_host_only_and_self_contained():
    """lt_jit_source (ABI 7) gives, without a GPU, the module source a c2 launch compiles: the
    launch constants and the scene's tables as literals, the kernel headers included by their bare
    names (the copies embedded in the library), no path into the source tree."""
    _, src = _c2_jit_source()
    assert 'lt_jit_analyze' in src and 'lt_jit_resolve' in src
    assert '#define LT_SPEC_Y 30' in src and 'lt_spec_scene' in src
    assert '#include "lt_kernels_dev.h"' in src and '../' not in src
    _, generic = _c2_jit_source(0)
    assert 'LT_SPEC_Y' not in generic and 'lt_spec_scene' not in generic


def test_library_embeds_the_current_kernel_headers(tmp_path):
    """liblt_hip.so carries the JIT kernel headers it was built with (the JIT kernels
    must read the struct layouts of the library's host code): the embedded copies, regenerated
    from the headers on disk now, are byte for byte inside the library — a header edited without
    a rebuild fails here."""
    import __graft_entry__ as ge
    inc = ge.embed_headers(out=str(tmp_path / 'e.inc'))
    blob = open(_abi.LIB_PATH, 'rb').read()
    for rel in ge.JIT_HEADERS:
        text = open(os.path.join(ROOT, rel)).read().replace(
            '#include "../../include/lt_abi.h"', '#include "lt_abi.h"')
        assert text.encode() in blob, rel
    assert open(inc).read() == open(ge.EMBED_INC).read()


def test_jit_module_compiles_on_the_host():
    """The c2 JIT module compiles with hiprtc for gfx950 on this CPU-only host from the headers as
    they are embedded (the build check of the code the GPU compiles at run time)."""
    jit_isa, src = _c2_jit_source()
    code = jit_isa.hiprtc_compile(src)
    assert len(code) > 10000 and code[:4] == b'\x7fELF'
