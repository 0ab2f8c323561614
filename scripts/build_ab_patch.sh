#!/bin/bash
# Build a patched copy of the working tree's library for an A/B run:
#   scripts/build_ab_patch.sh NAME 'python-expr-file-edits'
# The second argument is a Python snippet run in the copy's csrc/ with a
# helper sub(file, old, new) (exact, must match once); the library is built
# there and copied to ablib/NAME.so (git-ignored; bench.py loads it with
# TPF_LIB=ablib/NAME.so, e.g. LIBS="tree ablib/NAME.so" scripts/gpu.sh ab:WL).
set -e
cd "$(dirname "$0")/.."
NAME=$1; EDIT=$2
D=/tmp/tpf_abp_$NAME
rm -rf $D && mkdir -p $D ablib
cp -r turbopfor-cpp_amd include $D/ && rm -rf $D/turbopfor-cpp_amd/build $D/turbopfor-cpp_amd/lib
(cd $D/turbopfor-cpp_amd/csrc && python3 - "$EDIT" <<'PY'
import sys
def sub(f, old, new):
    s = open(f).read()
    assert s.count(old) == 1, (f, old[:60], s.count(old))
    open(f, 'w').write(s.replace(old, new))
exec(sys.argv[1])
PY
)
make -s -C $D/turbopfor-cpp_amd -j8 lib/libturbopfor_amd.so
cp $D/turbopfor-cpp_amd/lib/libturbopfor_amd.so ablib/$NAME.so
echo "ablib/$NAME.so <- tree + edit"
