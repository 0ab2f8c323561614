set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chained.py tests/test_gpu_fuzz.py > gpurun_out/r3c_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/r3c_tests.log; exit 1; }
tail -1 gpurun_out/r3c_tests.log
LIBS="tree ablib/base.so ablib/w8k.so ablib/stage16k.so tree" bash scripts/gpu_phase_probe.sh
