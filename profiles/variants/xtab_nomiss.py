# TIMING-ONLY variant (profiles/build_variant.sh LT_PATCH; its outputs are wrong): the vertex fits
# never factor an x-set on the fly (lanes that miss the x-set table take slot 0), to measure what
# the table misses cost.
import sys
p = sys.argv[1] + '/land_trendr_amd/csrc/lt_fast.h'
s = open(p).read()
old = """  const int key = act ? xset_key(m, X) : 0;
  const bool miss = act && key < 0;
  lsq_xf f;
  if (act && !miss) f = xtab[key];
  if (__ballot(miss)) {
    if (miss) lsq_factor(m, X, f);
  }
  slope = 0.0;
  icpt = 0.0;
  int rc = 0;"""
new = """  const int key = act ? xset_key(m, X) : 0;
  lsq_xf f = xtab[key < 0 ? 0 : key];
  slope = 0.0;
  icpt = 0.0;
  int rc = 0;"""
assert old in s
open(p, 'w').write(s.replace(old, new))
