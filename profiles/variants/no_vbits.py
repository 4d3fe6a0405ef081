# A/B variant (profiles/build_variant.sh LT_PATCH): the masked winner scan loads each mask byte
# when it tests it (the mask bit words of lt_fast.h off).
import sys
p = sys.argv[1] + '/land_trendr_amd/csrc/lt_fast.h'
s = open(p).read()
old = 'in.obs_valid != nullptr && K <= 128;  // launch-uniform'
assert old in s
open(p, 'w').write(s.replace(old, 'in.obs_valid != nullptr && K <= 0;  // launch-uniform'))
