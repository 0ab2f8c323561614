# round 6: drop-in tests on the final server loop, per-block scaling vs round 5 (latch harness),
# C3 D1 write-pass variants (4 value chunks in flight / 64-block D1 runs) against the tree
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r6k}
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dropin.py tests/test_gpu_enc256v32.py > gpurun_out/${T}_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for i in 1 2; do
  LIBS="tree" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=${T}auto$i PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
  LIBS="ablib/r5base.so" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=${T}r5$i PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
done
for round in 1 2; do
for lib in tree ablib/nc4.so ablib/run64.so; do
  n=$(basename $lib .so)
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_${n}_${round}_prof -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 5 0 c3 > $R/gpurun_out/${T}_${n}.log 2>&1) || { echo "prof $n rc=$?"; tail -5 $R/gpurun_out/${T}_${n}.log; exit 1; }
  python3 -c "
import csv,glob,sys
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if '_write' in r['Name'] or '_plan' in r['Name']:
            print(sys.argv[2], r['Name'][15:48], r['Calls'], round(float(r['AverageNs'])/1e6, 4), 'ms')
" $R/gpurun_out/${T}_${n}_${round}_prof $n
done
done
