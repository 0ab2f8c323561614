# hot-path decode with non-temporal packed-stream loads (ablib/decpol11.so, TPF_DEC_POL=11) vs default loads: C2 and C3 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TPF_LIB=$R/ablib/decpol11.so timeout -k 10 300 python -u -m pytest tests/test_gpu_dec256v32.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3aa_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r3aa_tests.log; exit 1; }
tail -1 gpurun_out/r3aa_tests.log
LIBS="tree ablib/decpol11.so" WL=c2 ROUNDS=3 TAG=r3aa bash scripts/gpu_ab.sh || exit 1
LIBS="tree ablib/decpol11.so" WL=c3 ROUNDS=2 TAG=r3ab bash scripts/gpu_ab.sh
