# round 6: 64-bit chained phase A (two values per walk step) tests + phase times; per-block scaling with fixed naps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r6i}
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_chained64.py tests/test_gpu_formats.py tests/test_gpu_dropin.py tests/test_gpu_fuzz.py > gpurun_out/${T}_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for lib in tree ablib/r5base.so tree ablib/r5base.so; do
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  timeout -k 10 200 python scripts/chain64_phase_probe.py 10000000 10 >> gpurun_out/${T}_chain64.log 2>&1 || { echo "probe $lib rc=$?"; tail -5 gpurun_out/${T}_chain64.log; exit 1; }
  tail -1 gpurun_out/${T}_chain64.log
done
unset TPF_LIB
LIBS="tree" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=$T PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
LIBS="tree" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=${T}b PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
