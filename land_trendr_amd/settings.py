"""settings.json semantics (README.md:46-85 of the reference) → the C ABI's lt_params.

Only the analysis keys matter on this path: index_eqn, line_cost, target_date, label_rules.
NODATA mirrors /root/reference/settings.py:16. The S3 bucket / key templates of that file belong
to the storage layer, which is out of scope.
"""
import json

from . import _abi
from .classes import LabelRule

NODATA = _abi.LT_NODATA


def compile_params(line_cost, label_rules=(), pre_threshold_mode='reference'):
    """line_cost + LabelRule list (or settings dicts) → LtParams.

    pre_threshold_mode 'reference' reproduces classes.py:207 (any pre_threshold filter raises
    AttributeError); 'documented' applies the filter the docstring describes (classes.py:26-29).
    """
    rules = [r if isinstance(r, LabelRule) else LabelRule(r) for r in label_rules]
    if len(rules) > _abi.LT_MAX_RULES:
        raise ValueError('at most %d label rules' % _abi.LT_MAX_RULES)
    if pre_threshold_mode not in ('reference', 'documented'):
        raise ValueError('pre_threshold_mode must be "reference" or "documented"')
    p = _abi.LtParams()
    p.line_cost = float(line_cost)
    p.n_rules = len(rules)
    p.pre_threshold_mode = (_abi.LT_PRE_REFERENCE if pre_threshold_mode == 'reference'
                            else _abi.LT_PRE_DOCUMENTED)
    for i, r in enumerate(rules):
        p.rules[i] = r.to_c()
    return p, rules


def load_settings(path_or_dict):
    """Read a settings.json (path, JSON text or dict) the way get_settings does (utils.py:241)."""
    if isinstance(path_or_dict, dict):
        return path_or_dict
    if path_or_dict.lstrip().startswith('{'):
        return json.loads(path_or_dict)
    with open(path_or_dict) as fh:
        return json.load(fh)
