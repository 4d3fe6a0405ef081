#!/bin/bash
# Library variants for profiling and A/B runs, built here (CPU) into build/exp/ (git-ignored; sent
# to the GPU box while it exists — delete it when the runs are done):
#   bash profiles/build_variant.sh <name> <maxy> [<probe type> <probe header>] [-- hipcc flags]
# links the product lt_abi.hip with profiles/lt_dispatch_probe.hip (one instance, MAXY = <maxy>,
# one rule) into build/exp/<name>.so; run with LT_HIP_LIB=build/exp/<name>.so.
# LT_PATCH=<script>: a copy of the sources is edited by `python3 <script> <copy root>` first (A/B
# variants of the kernel body; the product sources stay as they are).
set -e
R=$(cd $(dirname $0)/.. && pwd)
OUT=$R/build/exp
NAME=$1; MY=$2; shift 2
PROBE=lt::NoProbe; INC=()
if [ $# -ge 2 ] && [ "$1" != "--" ]; then PROBE=$1; INC=(-include $2); shift 2; fi
[ "$1" = "--" ] && shift
mkdir -p $OUT
if [ -n "$LT_PATCH" ]; then
  S=$(mktemp -d /tmp/ltvar.XXXX)
  mkdir -p $S/land_trendr_amd $S/profiles
  cp -r $R/include $S/ && cp -r $R/land_trendr_amd/csrc $S/land_trendr_amd/ && \
    cp $R/profiles/lt_dispatch_probe.hip $R/profiles/*.h $S/profiles/
  python3 $LT_PATCH $S
  R=$S
fi
F="-x hip --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -fPIC -Wno-unused-result"
/opt/rocm/bin/hipcc $F -c -o $OUT/$NAME.abi.o $R/land_trendr_amd/csrc/lt_abi.hip "$@" &
/opt/rocm/bin/hipcc $F -c -DLT_PROBE_MAXY=$MY "-DLT_PROBE=$PROBE" "${INC[@]}" \
  -o $OUT/$NAME.disp.o $R/profiles/lt_dispatch_probe.hip "$@" &
wait %1 && wait %2
/opt/rocm/bin/hipcc -shared -o $OUT/$NAME.so $OUT/$NAME.abi.o \
  $OUT/$NAME.disp.o -lhiprtc
rm -f $OUT/$NAME.abi.o $OUT/$NAME.disp.o
