#!/bin/bash
# Builds the measurement tools that are NOT part of the library:
#   scripts/libdecvar.so  (decode work-dealing / store-policy variants, dec_variants.hip)
#   scripts/libencvar.so  (rejected single-pass encoders, enc_variants.hip; links the library
#                          for grid_cap and the run scan)
set -e
cd "$(dirname "$0")/.."
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="--offload-arch=gfx950 -O3 -std=c++20 -shared -fPIC -munsafe-fp-atomics -I turbopfor-cpp_amd/csrc -I include"
make -s -C turbopfor-cpp_amd
$HIPCC $FLAGS -o scripts/libdecvar.so scripts/dec_variants.hip &
$HIPCC $FLAGS -o scripts/libdecgrp.so scripts/dec_groups.hip &
$HIPCC $FLAGS -o scripts/libencvar.so scripts/enc_variants.hip -L turbopfor-cpp_amd/lib -lturbopfor_amd \
    -Wl,-rpath,'$ORIGIN/../turbopfor-cpp_amd/lib'
wait
