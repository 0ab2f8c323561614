#!/bin/bash
# Builds the measurement tools that are NOT part of the library:
#   scripts/libdecvar.so  (decode work-dealing / store-policy variants, dec_variants.hip)
#   scripts/libdecgrp.so  (grouped-load decode A/B of round 4, dec_groups.hip)
# (the rejected single-pass encoders, enc_variants.hip, were removed in round 5:
#  git history)
set -e
cd "$(dirname "$0")/.."
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="--offload-arch=gfx950 -O3 -std=c++20 -shared -fPIC -munsafe-fp-atomics -I turbopfor-cpp_amd/csrc -I include"
make -s -C turbopfor-cpp_amd
$HIPCC $FLAGS -o scripts/libdecvar.so scripts/dec_variants.hip &
$HIPCC $FLAGS -o scripts/libdecgrp.so scripts/dec_groups.hip &
wait
