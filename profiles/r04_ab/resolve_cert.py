# A/B patch (profiles/build_variant.sh LT_PATCH): the resolve stage (EXACT) takes the certified
# labels path too (closed-form vertex fits with intervals, emulated fits only around the rules'
# candidates) instead of one emulated fit per vertex number.
import sys
p = sys.argv[1] + '/land_trendr_amd/csrc/lt_fast.h'
s = open(p).read()
old = '} else if constexpr (!EXACT && RMAX <= LT_CERT_RULES) {'
assert old in s
open(p, 'w').write(s.replace(old, '} else if constexpr (RMAX <= LT_CERT_RULES) {'))
