# phase A (lane per block) check: chained / fuzz / decode tests, then c3chain A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_chained.py tests/test_gpu_fuzz.py tests/test_gpu_dec256v32.py > gpurun_out/r3b_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/r3b_tests.log; exit 1; }
tail -1 gpurun_out/r3b_tests.log
LIBS="tree ablib/w8k.so ablib/w12k.so ablib/base.so" WL=c3chain TAG=r3b ROUNDS=2 bash scripts/gpu_ab.sh
