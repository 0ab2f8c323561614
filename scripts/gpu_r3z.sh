# windowed p4Dec32: branch-free plain unpack (tree) vs h32c (committed): format tests, C1 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_formats.py tests/test_gpu_fuzz.py tests/test_gpu_nstream.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3z_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r3z_tests.log; exit 1; }
tail -1 gpurun_out/r3z_tests.log
LIBS="tree ablib/h32c.so" WL=c1 ROUNDS=3 TAG=r3z bash scripts/gpu_ab.sh
