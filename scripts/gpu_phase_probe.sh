# chain_phase_probe.py for each library in LIBS (tree = the working tree's)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for lib in ${LIBS:-tree}; do
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  timeout -k 10 200 python scripts/chain_phase_probe.py ${NB:-10000000} 2>>gpurun_out/phase_probe.err || { echo "$lib rc=$?"; tail -5 gpurun_out/phase_probe.err; exit 1; }
done
