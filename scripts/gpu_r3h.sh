set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chained.py tests/test_gpu_fuzz.py > gpurun_out/r3h_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/r3h_tests.log; exit 1; }
tail -1 gpurun_out/r3h_tests.log
LIBS="tree ablib/base.so tree ablib/base.so" bash scripts/gpu_phase_probe.sh
