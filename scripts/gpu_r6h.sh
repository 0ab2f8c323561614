# round 6: drop-in tests + per-block scaling (futex mailbox wait, adaptive nap), then the 64-bit chained phase ablations
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r6h}
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dropin.py > gpurun_out/${T}_dropin.log 2>&1 || { echo "dropin rc=$?"; tail -40 gpurun_out/${T}_dropin.log; exit 1; }
tail -1 gpurun_out/${T}_dropin.log
LIBS="tree" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=$T PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
LIBS="tree" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=${T}b PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
for lib in tree ablib/abl0.so ablib/ablpos.so ablib/ablwalk.so ablib/ablbase.so tree; do
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  timeout -k 10 200 python scripts/chain64_phase_probe.py 10000000 10 >> gpurun_out/${T}_chain64.log 2>&1 || { echo "probe $lib rc=$?"; tail -5 gpurun_out/${T}_chain64.log; exit 1; }
  tail -1 gpurun_out/${T}_chain64.log
done
