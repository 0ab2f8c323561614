set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_formats.py tests/test_gpu_fuzz.py > gpurun_out/r3f_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/r3f_tests.log; exit 1; }
tail -1 gpurun_out/r3f_tests.log
LIBS="tree ablib/np3.so ablib/np4.so ablib/base.so" WL=c1 TAG=r3f ROUNDS=2 bash scripts/gpu_ab.sh
LIBS="tree ablib/skb.so ablib/skc.so ablib/skrp.so ablib/base.so" bash scripts/gpu_phase_probe.sh
