"""lt_settings_compile (the C ABI's settings.json compiler for non-Python hosts) against the Python
host it restates: LabelRule validation and compilation (classes.py:32-64 + classes._qual),
parse_date's strptime grammar (utils.py:194-202) and index_eqn.IndexProgram (utils.py:219-225,
447-484). Same outputs byte for byte, same exception types. No GPU needed (a host function)."""
import ctypes
import json
import math

import numpy as np
import pytest

from land_trendr_amd import _abi
from land_trendr_amd.index_eqn import DTYPES, IndexProgram
from land_trendr_amd.scene import parse_date
from land_trendr_amd.settings import compile_params

BASE = {'index_eqn': 'B1 - B2', 'line_cost': 10, 'target_date': '2014-07-01',
        'label_rules': [{'name': 'greatest_disturbance', 'val': 1, 'change_type': 'GD'}]}


def c_compile(settings, mode=0, band_type=_abi.LT_T_I16, out_type=-1, raster_count=0):
    lib = _abi.load_lib()
    out = _abi.LtSettings()
    exc = ctypes.c_int32()
    err = ctypes.create_string_buffer(512)
    text = settings if isinstance(settings, str) else json.dumps(settings)
    rc = lib.lt_settings_compile(text.encode(), mode, band_type, out_type, raster_count,
                                 ctypes.byref(out), ctypes.byref(exc), err, 512)
    if rc != 0:
        raise _abi.EXC_TYPES.get(exc.value, Exception)(err.value.decode())
    return out


def py_compile(settings, mode='reference', band_dtype=np.int16, raster_count=None):
    s = json.loads(settings) if isinstance(settings, str) else settings
    params, _ = compile_params(s['line_cost'], s.get('label_rules', ()), mode)
    d = parse_date(s['target_date'])
    prog = (IndexProgram(s['index_eqn'], band_dtype=band_dtype, raster_count=raster_count)
            if 'index_eqn' in s else None)
    return params, d, prog


def same_bytes(a, b):
    return bytes(memoryview(a).cast('B')) == bytes(memoryview(b).cast('B'))


def check_same(settings, mode='reference', band_dtype=np.int16):
    params, d, prog = py_compile(settings, mode, band_dtype)
    c = c_compile(settings, 0 if mode == 'reference' else 1, DTYPES[np.dtype(band_dtype)])
    for r in range(_abi.LT_MAX_RULES):  # NaN payloads compare by bits
        assert same_bytes(c.params.rules[r], params.rules[r]), (settings, r)
    assert same_bytes(c.params, params), settings
    assert (c.target_year, c.target_month, c.target_day) == (d.year, d.month, d.day)
    if prog is not None:
        want = prog.to_c()
        assert same_bytes(c.index, want), (settings.get('index_eqn'), prog.ops)
        assert list(c.index_bands[:c.n_index_bands]) == prog.bands


RULE_CASES = [
    {'name': 'a', 'val': 3, 'change_type': 'FD', 'onset_year': ['>=', 1995], 'duration': ['<', 4]},
    {'name': 'b', 'val': 7, 'change_type': None, 'onset_year': ['>', 1995],
     'pre_threshold': ['<', 100]},
    {'name': 'c', 'val': 1, 'change_type': 'LD', 'duration': []},
    {'name': 'd', 'val': 2.7, 'change_type': 'GD', 'onset_year': ['=', 2000.5],
     'duration': ['>', True]},
    {'name': 'e', 'val': '5', 'change_type': 'GD', 'onset_year': ['>=', '2000']},
    {'name': 'f', 'val': 'x', 'onset_year': ['<=', None], 'duration': ['<', 'y'],
     'pre_threshold': ['>', [1]]},
    {'name': 'g', 'val': -4, 'onset_year': 0, 'duration': None, 'pre_threshold': ''},
    {'name': 'h', 'val': True, 'change_type': 'FD', 'onset_year': ['>=', -1e300]},
]


@pytest.mark.parametrize('mode', ['reference', 'documented'])
def test_rules_compile_like_labelrule(mode):
    for r in RULE_CASES:
        check_same(dict(BASE, label_rules=[r]), mode)
    check_same(dict(BASE, label_rules=RULE_CASES), mode)
    check_same(dict(BASE, label_rules=[], line_cost=0.5))


@pytest.mark.parametrize('rule', [
    {'name': 'g', 'val': 5, 'change_type': 'GD', 'duration': ['<', 4, 'BAD']},
    {'val': 5}, {'name': '', 'val': 5}, {'name': 'g', 'val': 0}, {'name': 'g', 'val': []},
    {'name': 'g', 'val': 5, 'change_type': 'XX'}, {'name': 'g', 'val': 5, 'change_type': 3},
    {'name': 'g', 'val': 5, 'onset_year': {'a': 1}}, {'name': 'g', 'val': 5, 'onset_year': 'x'},
    {'name': 'g', 'val': 5, 'pre_threshold': ['>']},
])
def test_invalid_rules_raise_value_error_like_labelrule(rule):
    with pytest.raises(ValueError) as want:
        py_compile(dict(BASE, label_rules=[rule]))
    with pytest.raises(ValueError) as got:
        c_compile(dict(BASE, label_rules=[rule]))
    assert str(got.value) == str(want.value)


@pytest.mark.parametrize('date,ok', [
    ('2014-07-01', True), ('2014-7-1', True), ('2014-12-31', True), ('2012-02-29', True),
    ('2014-07- 1', True), ('2014-02-29', False), ('2014-13-01', False), ('2014-00-10', False),
    ('14-07-01', False), ('2014-07-01 ', False), ('2014/07/01', False), ('2014-07-32', False),
    ('2014-07-001', False), ('20140-07-01', False), ('2014-011-01', False), ('', False),
])
def test_target_date_grammar_matches_strptime(date, ok):
    s = dict(BASE, target_date=date)
    if ok:
        check_same(s)
    else:
        with pytest.raises(ValueError):
            parse_date(date)
        with pytest.raises(ValueError):
            c_compile(s)


EQNS = ['B1 - B2', '(B4 - B3) / (B4 + B3)', '(B4-B3)*1.0/(B4+B3)', 'B1', '2 * B1 - 3',
        '-B1 + 40000', 'B1 // 2', 'B1 / 2', 'B1 * 0.5', '(B1 + B2) * (B3 - 1) / 7', 'B2 - -B1',
        '1 - B1', '2 * 3 - B1', 'B1 - (2 + 3)', 'B1 + 2 - B2', '+B3 * -2', 'B1 + 100000',
        'B1 * 1e300', 'B1 + 70000.5', '10 / 4 + B1', '10.0 / 4 + B1', '7 // 2 * B1', '-7 // 2 + B1',
        'B12 - B3', 'B1 - B1 + 0x10', 'B1 + 1_000', '.5 * B1', '1. + B2', 'B1*B1*B1*B1',
        '((((B1))))', 'B1 + 4294967296', 'B1 - 9223372036854775808', 'B1 + 3.4e38',
        'B1 + 65000.0', 'B1 + 64999.0', '  B1 - B2  ', '(B1 -\n B2)']


@pytest.mark.parametrize('band_dtype', [np.int16, np.uint16, np.float32, np.uint8, np.int32])
def test_index_programs_match_indexprogram(band_dtype):
    for e in EQNS:
        try:
            IndexProgram(e, band_dtype=band_dtype).to_c()
        except Exception as exc:  # the Python host rejects it: so must the C ABI
            with pytest.raises(type(exc)):
                c_compile(dict(BASE, index_eqn=e), band_type=DTYPES[np.dtype(band_dtype)])
            continue
        check_same(dict(BASE, index_eqn=e), band_dtype=band_dtype)


@pytest.mark.parametrize('eqn', ['B1 ** 2', 'B1 % 2', 'log(B1)', 'B1 < B2', 'C1 - B2', '1 - 2',
                                 'B1 +', 'B1 - B2)', '3j * B1', '012 + B1', 'B1 / (2 - 2)',
                                 'B0 - B1', 'B1\n- B2'])
def test_bad_equations_raise_like_indexprogram(eqn):
    try:
        IndexProgram(eqn, band_dtype=np.int16).to_c()
        ok = True
    except Exception as exc:
        ok = False
        want = type(exc)
    if ok:
        check_same(dict(BASE, index_eqn=eqn))
        return
    with pytest.raises(want):
        c_compile(dict(BASE, index_eqn=eqn))


@pytest.mark.parametrize('depth', [63, 200, 201, 5000, 100000])
@pytest.mark.parametrize('kind', ['paren', 'sign', 'sign_const'])
def test_deep_nesting_is_rejected_not_a_crash(kind, depth):
    """Nested parentheses / sign chains: the C ABI accepts what the Python host accepts and
    raises ValueError for the rest (the host's parser stops at 200 parentheses; long sign chains
    exceed its 64 operations, reference no band, or exhaust the interpreter: RecursionError /
    MemoryError there), instead of exhausting the native stack."""
    eqn = {'paren': '(' * depth + 'B1' + ')' * depth, 'sign': '-' * depth + 'B1',
           'sign_const': '-' * depth + '1 + B1'}[kind]
    try:
        IndexProgram(eqn, band_dtype=np.int16).to_c()
        host_ok = True
    except (Exception, RecursionError, MemoryError):
        host_ok = False
    if host_ok:
        check_same(dict(BASE, index_eqn=eqn))
    else:
        with pytest.raises(ValueError):
            c_compile(dict(BASE, index_eqn=eqn))


def test_settings_keys_and_json():
    with pytest.raises(KeyError):
        c_compile({'target_date': '2014-07-01'})
    with pytest.raises(KeyError):
        c_compile({'line_cost': 10})
    with pytest.raises(ValueError):
        c_compile('{"line_cost": 10, ')
    with pytest.raises(ValueError):
        c_compile(dict(BASE, label_rules=[{'name': 'x', 'val': 1}] * (_abi.LT_MAX_RULES + 1)))
    c = c_compile('{"line_cost": NaN, "target_date": "2014-07-01", "label_rules": []}')
    assert math.isnan(c.params.line_cost)
    c = c_compile('{"line_cost": 1, "line_cost": 2.5, "target_date": "2014-07-01"}')
    assert c.params.line_cost == 2.5 and c.index.n_ops == 0
    c = c_compile(dict(BASE, index_eqn='B3 - B7'), raster_count=7)
    assert list(c.index_bands[:2]) == [3, 7]
    with pytest.raises(Exception):
        c_compile(dict(BASE, index_eqn='B3 - B9'), raster_count=7)
