# generic encoder: 16-byte copy-out + 32-bit wave OR in the plan (p4Enc32 batches): format tests, C1 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_formats.py tests/test_gpu_fuzz.py tests/test_gpu_nstream.py tests/test_gpu_dropin.py tests/test_gpu_edges.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3v_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r3v_tests.log; exit 1; }
tail -1 gpurun_out/r3v_tests.log
LIBS="tree ablib/gencdw.so" WL=c1 ROUNDS=2 TAG=r3v bash scripts/gpu_ab.sh
