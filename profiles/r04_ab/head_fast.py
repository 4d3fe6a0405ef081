# A/B patch (profiles/build_variant.sh LT_PATCH): the analyze body of an earlier commit, saved by
# the caller as /tmp/lt_fast_head.h (git show <commit>:land_trendr_amd/csrc/lt_fast.h), in place
# of the current lt_fast.h, everything else as it is now.
import shutil
import sys
shutil.copy('/tmp/lt_fast_head.h', sys.argv[1] + '/land_trendr_amd/csrc/lt_fast.h')
