# round 6: per-kernel times of the C3 D1 / C4 256v32 encoders for two library builds + SQ counters of the tree's
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r6c}
for lib in ${LIBS:-tree ablib/r5base.so}; do
  n=$(basename $lib .so)
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  for data in c3 c4; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_${n}_${data}_prof -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 5 0 $data > $R/gpurun_out/${T}_${n}_${data}.log 2>&1) || { echo "prof $n $data rc=$?"; tail -5 $R/gpurun_out/${T}_${n}_${data}.log; exit 1; }
    python3 -c "
import csv,glob,sys
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'enc' in r['Name'] or 'scan' in r['Name']:
            print(sys.argv[2], sys.argv[3], r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6, 4), 'ms')
" $R/gpurun_out/${T}_${n}_${data}_prof $n $data
  done
done
unset TPF_LIB
MODES=3 DATA=c3 TAG=${T}c3 bash scripts/gpu_enc_counters.sh || exit 1
