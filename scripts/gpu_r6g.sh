# round 6: per-block aggregate rate per library build / wait policy (1..128 threads)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r6g}
LIBS="tree ablib/nap31.so" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=$T PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
TPF_PERBLOCK_WAIT=spin LIBS="tree" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=${T}spin PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
LIBS="tree" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=${T}b PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
