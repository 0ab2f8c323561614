# round 6: chained phase-A occupancy variants (window 8 KB / 4 waves, 12 KB / 3 waves) vs the tree
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
O=gpurun_out/r6o_phaseA.txt; : > $O
for rep in 1 2; do
  for lib in tree ablib/dsum4w.so ablib/dsum3w.so; do
    if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$lib; fi
    timeout -k 10 200 python -u scripts/chain_phase_probe.py 10000000 >> $O 2>&1 || { echo "rc=$? $lib"; tail -5 $O; exit 1; }
  done
  for lib in tree ablib/d64w4.so; do
    if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$lib; fi
    timeout -k 10 200 python -u scripts/chain64_phase_probe.py 10000000 >> $O 2>&1 || { echo "rc=$? $lib"; tail -5 $O; exit 1; }
  done
done
cat $O
