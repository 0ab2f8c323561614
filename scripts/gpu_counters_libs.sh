# SQ counter pass of one kernel (KFILTER) for each library in LIBS (tree = working tree)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for lib in ${LIBS:-tree}; do
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  echo "== $lib"
  TAGC=$(basename $lib .so) bash scripts/gpu_counters.sh || exit 1
done
