# round 6: drop-in tests (128 callers, server lifetime), per-block scaling, encoder pass probes and the occ8 variant
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r6f}
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dropin.py > gpurun_out/${T}_dropin.log 2>&1 || { echo "dropin rc=$?"; tail -40 gpurun_out/${T}_dropin.log; exit 1; }
tail -1 gpurun_out/${T}_dropin.log
LIBS="tree" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=$T PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
for spec in "tree 0 c3" "tree 0 c4" "tree 1 c4" "tree 2 c4" "ablib/occ8.so 0 c3" "ablib/occ8.so 0 c4"; do
  set -- $spec; lib=$1; mode=$2; data=$3; n=$(basename $lib .so)
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_${n}_${mode}_${data}_prof -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 5 $mode $data > $R/gpurun_out/${T}_${n}_${mode}_${data}.log 2>&1) || { echo "prof $spec rc=$?"; tail -5 $R/gpurun_out/${T}_${n}_${mode}_${data}.log; exit 1; }
  python3 -c "
import csv,glob,sys
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if '_write' in r['Name'] or '_plan' in r['Name']:
            print(sys.argv[2], r['Name'][15:48], r['Calls'], round(float(r['AverageNs'])/1e6, 4), 'ms')
" $R/gpurun_out/${T}_${n}_${mode}_${data}_prof "$spec"
done
