# A/B patch (profiles/build_variant.sh LT_PATCH): the analyze body of an earlier commit, saved by
# the caller as /tmp/lt_fast_head.h (git show <commit>:land_trendr_amd/csrc/lt_fast.h) and, when
# present, /tmp/lt_pixel_head.h, in place of the current files, everything else as it is now.
import os
import shutil
import sys
shutil.copy('/tmp/lt_fast_head.h', sys.argv[1] + '/land_trendr_amd/csrc/lt_fast.h')
if os.path.exists('/tmp/lt_pixel_head.h'):
    shutil.copy('/tmp/lt_pixel_head.h', sys.argv[1] + '/land_trendr_amd/csrc/lt_pixel.h')
