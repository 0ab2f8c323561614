set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dropin.py tests/test_gpu_chained.py tests/test_gpu_formats.py tests/test_gpu_fuzz.py tests/test_gpu_edges.py > gpurun_out/r3e_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/r3e_tests.log; exit 1; }
tail -1 gpurun_out/r3e_tests.log
LIBS="tree ablib/base.so tree" bash scripts/gpu_phase_probe.sh
LIBS="tree ablib/base.so" WL=c1 TAG=r3e ROUNDS=2 bash scripts/gpu_ab.sh
