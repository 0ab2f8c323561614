# round 6: chained phase A (fast-path rewrite, read-ahead of the base sums and the region) vs r6final
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
O=gpurun_out/r6p_phaseA.txt; : > $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chained.py > gpurun_out/r6p_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r6p_tests.log; exit 1; }
tail -3 gpurun_out/r6p_tests.log
for rep in 1 2; do
  for lib in ablib/r6final.so tree; do
    if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$lib; fi
    timeout -k 10 200 python -u scripts/chain_phase_probe.py 10000000 >> $O 2>&1 || { echo "rc=$? $lib"; tail -5 $O; exit 1; }
  done
done
unset TPF_LIB
timeout -k 10 200 python -u scripts/chain64_phase_probe.py 10000000 >> $O 2>&1 || { echo "rc=$? c64"; tail -5 $O; exit 1; }
grep -v amdgpu.ids $O
