"""A/B variant (attribution only, wrong outputs): the year-major output loop of lt_fast.h computes
everything but stores none of the five f64 per-year planes."""
import sys
p = sys.argv[1] + '/land_trendr_amd/csrc/lt_fast.h'
s = open(p).read()
n = 0
for f in ('val_fit', 'fit_m', 'fit_b', 'right_m', 'right_b'):
    old = 'if (out.%s) __builtin_nontemporal_store(' % f
    n += s.count(old)
    s = s.replace(old, 'if (false) __builtin_nontemporal_store(')
assert n == 5, n
open(p, 'w').write(s)
