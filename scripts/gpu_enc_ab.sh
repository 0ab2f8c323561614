# Encoder A/B on one box: the tests that exercise the 256v32 encoder, then
# the rejected encoders of scripts/enc_variants.hip (built on the box) checked
# byte-exact and timed against the production two-pass encoder.  -> gpurun_out/$TAG_*
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-enc}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_enc256v32.py tests/test_gpu_edges.py tests/test_gpu_nstream.py tests/test_gpu_chained.py > gpurun_out/${T}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
scripts/build_variants.sh > gpurun_out/${T}_build.log 2>&1 || { echo "variant build failed"; tail -20 gpurun_out/${T}_build.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m variants tests/test_gpu_enc_variants.py > gpurun_out/${T}_variants.log 2>&1 || { echo "variants rc=$?"; tail -30 gpurun_out/${T}_variants.log; exit 1; }
timeout -k 10 300 python scripts/enc_ab.py > gpurun_out/${T}_ab.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/${T}_ab.txt; exit 1; }
cat gpurun_out/${T}_ab.txt
