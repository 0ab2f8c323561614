# round 6: 64-bit phase A with a branch-free bitmap exception loop (every lane's bx <= 32) vs r6last; 64-bit chained tests
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
O=gpurun_out/r6v_phaseA64.txt; : > $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chained64.py > gpurun_out/r6v_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r6v_tests.log; exit 1; }
tail -2 gpurun_out/r6v_tests.log
for rep in 1 2; do
  for lib in ablib/r6last.so tree; do
    if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$lib; fi
    timeout -k 10 200 python -u scripts/chain64_phase_probe.py 10000000 >> $O 2>&1 || { echo "rc=$? c64 $lib"; tail -5 $O; exit 1; }
  done
done
grep -v amdgpu.ids $O
