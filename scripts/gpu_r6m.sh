# round 6: encoder tests + C3 / C4 encoder kernel times, tree (exception ranks by ballot + mbcnt) vs HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r6m}
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_enc256v32.py tests/test_gpu_nstream.py tests/test_gpu_edges.py tests/test_gpu_formats.py > gpurun_out/${T}_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for round in 1 2; do
for lib in tree ablib/head.so; do
  n=$(basename $lib .so)
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  for data in c3 c4; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_${n}_${data}_${round}_prof -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 5 0 $data > $R/gpurun_out/${T}_${n}.log 2>&1) || { echo "prof $n rc=$?"; tail -5 $R/gpurun_out/${T}_${n}.log; exit 1; }
  python3 -c "
import csv,glob,sys
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if '_write' in r['Name']:
            print(sys.argv[2], r['Name'][15:48], r['Calls'], round(float(r['AverageNs'])/1e6, 4), 'ms')
" $R/gpurun_out/${T}_${n}_${data}_${round}_prof $n
  done
done
done
