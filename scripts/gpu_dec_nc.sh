# Decode pipeline depth / occupancy variants (scripts/dec_variants.hip deals
# 20-25: NC blocks in flight at MINW waves/SIMD, product store policy) against
# the product kernel on full-size streams.  -> gpurun_out/$TAG_dec_nc.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-nc}
md5sum turbopfor-cpp_amd/lib/libturbopfor_amd.so
DEALS=${DEALS:-20,21,22,23,24,25} timeout -k 10 600 python scripts/dec_variants.py ${NB:-10000000} 3 ${STREAMS:-c2 bw1 bw4 bw16 bw32 c3} > gpurun_out/${T}_dec_nc.txt 2>&1 || { echo "variants rc=$?"; tail -20 gpurun_out/${T}_dec_nc.txt; exit 1; }
cat gpurun_out/${T}_dec_nc.txt
