# SGPR cap 80 on the encoder passes (ablib/sgpr80.so, TPF_SGPR_CAP=80; 82-96 SGPRs hold a wave slot per SIMD):
# encoder tests on the variant, C4 and C1 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TPF_LIB=$R/ablib/sgpr80.so timeout -k 10 300 python -u -m pytest tests/test_gpu_enc256v32.py tests/test_gpu_formats.py tests/test_gpu_nstream.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3ac_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r3ac_tests.log; exit 1; }
tail -1 gpurun_out/r3ac_tests.log
LIBS="tree ablib/sgpr80.so" WL=c4 ROUNDS=3 TAG=r3ac bash scripts/gpu_ab.sh || exit 1
LIBS="tree ablib/sgpr80.so" WL=c1 ROUNDS=2 TAG=r3ad bash scripts/gpu_ab.sh
