"""A/B variant (attribution only, wrong outputs): no per-year plane stores at all (the five f64
planes of the year-major loop, and winner / val_raw of the winner pick)."""
import runpy
import sys
runpy.run_path(sys.argv[0].replace('no_stores.py', 'no_year_stores.py'))
p = sys.argv[1] + '/land_trendr_amd/csrc/lt_fast.h'
s = open(p).read()
for old in ('if (out.winner) __builtin_nontemporal_store(', 'if (out.val_raw) __builtin_nontemporal_store('):
    assert old in s, old
    s = s.replace(old, 'if (false) __builtin_nontemporal_store(')
s = s.replace('} else if (out.val_raw) {  // the other', '} else if (false) {  // the other')
open(p, 'w').write(s)
