# A/B patch (profiles/build_variant.sh LT_PATCH): the resolve kernel built for 4 waves per SIMD
# (<= 128 VGPRs, like the analyze kernel) instead of the compiler's choice (170 VGPRs, 2 waves).
import sys
p = sys.argv[1] + '/land_trendr_amd/csrc/lt_kernels.h'
s = open(p).read()
old = '__global__ __launch_bounds__(64) void resolve_fast_kernel'
assert old in s
open(p, 'w').write(s.replace(old, '__global__ __launch_bounds__(64, 4) void resolve_fast_kernel'))
