#!/bin/bash
# Build a variant of the library for an A/B run into ablib/NAME.so (git-ignored,
# travels to the GPU box; bench.py loads it with TPF_LIB=ablib/NAME.so).
#   scripts/build_ab_lib.sh NAME [REV] [EXTRA flags...]
#   REV = a git revision (its committed sources) or "tree" (the working tree)
set -e
cd "$(dirname "$0")/.."
NAME=$1; REV=${2:-tree}; shift; shift || true
D=/tmp/tpf_ab_$NAME
rm -rf $D && mkdir -p $D ablib
if [ "$REV" = tree ]; then
  cp -r turbopfor-cpp_amd include $D/ && rm -rf $D/turbopfor-cpp_amd/build $D/turbopfor-cpp_amd/lib
else
  git archive $REV turbopfor-cpp_amd include | tar -x -C $D
fi
make -s -C $D/turbopfor-cpp_amd -j8 EXTRA="$*"
cp $D/turbopfor-cpp_amd/lib/libturbopfor_amd.so ablib/$NAME.so
echo "ablib/$NAME.so <- $REV $*"
