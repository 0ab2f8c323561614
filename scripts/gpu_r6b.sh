# round 6: encoder tests + A/B of the lane-plane write pass against round 5, per-block thread scaling
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r6b}
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_enc256v32.py tests/test_gpu_edges.py tests/test_gpu_nstream.py tests/test_gpu_chained.py tests/test_gpu_dropin.py tests/test_gpu_fuzz.py > gpurun_out/${T}_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
LIBS="tree ablib/r5base.so" ROUNDS=2 TAG=$T bash scripts/gpu.sh ab:c3enc ab:c4 || exit 1
LIBS="tree" K=3000 THREADS="1 16 24 32 64 128" TAG=$T PBT_TIMEOUT=200 bash scripts/pbt_libs.sh
