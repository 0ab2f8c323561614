set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dropin.py > gpurun_out/r6a_dropin.log 2>&1 || { echo "dropin rc=$?"; tail -30 gpurun_out/r6a_dropin.log; exit 1; }
tail -1 gpurun_out/r6a_dropin.log
LIBS="tree ablib/r5base.so" K=3000 THREADS="1 16 24 32 64 128" TAG=r6a PBT_TIMEOUT=200 bash scripts/pbt_libs.sh
