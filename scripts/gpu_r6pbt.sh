# round 6 end library: per-block aggregate calls/s at 1-128 threads, twice (latch harness, scripts/perblock_threads.cpp)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for i in 1 2; do
  LIBS="tree" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=r6endpbt$i PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
done
