"""Domain records of the reference (/root/reference/classes.py), same names and attributes.

LabelRule validates exactly like classes.py:32-64 and compiles to the C ABI's lt_rule.
TrendlinePoint / Trendline / Disturbance are the result records analyze() returns; their
mr_label_output() keys match classes.py:84-154 character for character. Trendline.match_rule
runs on the GPU (lt_analyze_tile's label stage via land_trendr_amd.utils), never on the CPU.
"""
from . import _abi


class LabelRule:
    """classes.py:1-64. options: name, val, change_type (FD/GD/LD/None), onset_year,
    duration, pre_threshold (each a 2-item list [qualifier, value] or falsy)."""

    def __init__(self, options):
        name = options.get('name')
        if not name:
            raise ValueError('name required')
        self.name = name

        val = options.get('val')
        if not val:
            raise ValueError('val required')
        self.val = val

        change_type = options.get('change_type')
        if change_type not in ['FD', 'GD', 'LD', None]:
            raise ValueError('Invalid change_type: %s' % change_type)
        self.change_type = change_type

        for param_name in ['onset_year', 'duration', 'pre_threshold']:
            param_val = options.get(param_name)
            if param_val:
                if type(param_val) != list or len(param_val) != 2:
                    raise ValueError('Parameter %s - invalid value: %s' % (
                        param_name, param_val))
                setattr(self, param_name, param_val)
            else:
                setattr(self, param_name, None)

    def to_c(self):
        """Compile to an LtRule (qualifiers the reference ignores become LT_Q_OTHER)."""
        r = _abi.LtRule()
        r.change_type = _abi.LT_CT[self.change_type]
        r.onset_op, r.onset_val = _qual(self.onset_year, {'=': _abi.LT_Q_EQ, '<=': _abi.LT_Q_LE,
                                                          '>=': _abi.LT_Q_GE})
        r.duration_op, r.duration_val = _qual(self.duration, {'>': _abi.LT_Q_GT,
                                                              '<': _abi.LT_Q_LT})
        r.pre_op, r.pre_val = _qual(self.pre_threshold, {'>': _abi.LT_Q_GT, '<': _abi.LT_Q_LT})
        try:
            r.class_val = int(self.val)
        except (TypeError, ValueError):
            r.class_val = _abi.LT_NODATA
        return r


def _qual(param, table):
    """[qualifier, value] -> (LT_Q_* op, float value). A value that is not a number compares the
    way Python 2 (the reference's interpreter) orders mixed types: any number is smaller than a
    str/list/dict (so '2000' is NOT 2000) and larger than None. Each qualifier then has a constant
    outcome, encoded with an op/value pair whose device comparison gives that same constant:
    never-filters -> LT_Q_OTHER; always-rejects -> '=' NaN (onset), '>' +inf (duration, pre)."""
    if not param:
        return _abi.LT_Q_UNSET, 0.0
    q, v = param
    op = table.get(q, _abi.LT_Q_OTHER)
    if op == _abi.LT_Q_OTHER:
        return op, 0.0
    if isinstance(v, (bool, int, float)):
        return op, float(v)
    # classes.py:190-211 drop the disturbance when `d <op'> v` holds, op' the negation of q
    num_lt_v = v is not None  # number < v (v a str/list/...), number > v (v None)
    rejects = {_abi.LT_Q_EQ: True,            # d != v: always true across types
               _abi.LT_Q_LE: not num_lt_v,    # d > v
               _abi.LT_Q_GE: num_lt_v,        # d < v
               _abi.LT_Q_GT: num_lt_v,        # d <= v
               _abi.LT_Q_LT: not num_lt_v}[op]  # d >= v
    if not rejects:
        return _abi.LT_Q_OTHER, 0.0
    if op in (_abi.LT_Q_EQ, _abi.LT_Q_LE, _abi.LT_Q_GE):  # onset_year (an int year)
        return _abi.LT_Q_EQ, float('nan')
    return _abi.LT_Q_GT, float('inf')  # duration / pre_threshold: nothing is > +inf


class TrendlinePoint:
    """classes.py:67-116."""

    def __init__(self, val_raw, val_fit, eqn_fit, eqn_right, index_date, index_day, spike,
                 vertex):
        self.val_raw = val_raw
        self.val_fit = val_fit
        self.eqn_fit = eqn_fit
        self.eqn_right = eqn_right
        self.index_date = index_date
        self.index_day = index_day
        self.spike = spike
        self.vertex = vertex

    def mr_label_output(self):
        d = {
            'val_raw': self.val_raw,
            'val_fit': self.val_fit,
            'eqn_fit_slope': self.eqn_fit[0],
            'eqn_fit_intercept': self.eqn_fit[1],
            'eqn_right_slope': self.eqn_right[0],
            'eqn_right_intercept': self.eqn_right[1],
            'spike': 1 if self.spike else 0,
            'vertex': 1 if self.vertex else 0,
        }
        date = self.index_date
        return dict(('%s-%s' % (date, k), v) for k, v in d.items())


class Trendline:
    """classes.py:119-232. match_rule evaluates on the GPU (utils.match_rules_gpu)."""

    def __init__(self, points):
        self.points = points

    def __str__(self):
        vertices = [p for p in self.points if p.vertex]
        return '\n'.join(' | '.join([v.index_date, str(v.val_fit)]) for v in vertices)

    def mr_label_output(self):
        out = {}
        for p in self.points:
            out.update(p.mr_label_output())
        return out

    def parse_disturbances(self):
        """classes.py:156-176: one Disturbance per segment between consecutive vertices (the
        first point counts as the first left vertex)."""
        from .scene import parse_date
        it = iter(self.points)
        left_vertex = next(it)
        for p in it:
            if not p.vertex:
                continue
            start_yr = parse_date(left_vertex.index_date).year
            end_yr = parse_date(p.index_date).year
            yield Disturbance(start_yr, left_vertex.val_fit, left_vertex.val_fit - p.val_fit,
                              end_yr - start_yr)
            left_vertex = p

    def match_rule(self, rule):
        """classes.py:178-232, computed by the GPU label stage."""
        from .utils import match_rules_gpu
        return match_rules_gpu(self, [rule])[0]


class Disturbance:
    """classes.py:235-244."""

    def __init__(self, onset_year, initial_val, magnitude, duration):
        self.onset_year = onset_year
        self.initial_val = initial_val
        self.magnitude = magnitude
        self.duration = duration

    def __repr__(self):
        return 'Disturbance(onset_year=%r, initial_val=%r, magnitude=%r, duration=%r)' % (
            self.onset_year, self.initial_val, self.magnitude, self.duration)
