# round 6: raw vbyte words stored as aligned dwords (one store + one OR per raw block) vs r6end
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for lib in rawdw; do
  TPF_LIB=$R/ablib/$lib.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_enc256v32.py tests/test_gpu_fuzz.py tests/test_gpu_edges.py tests/test_gpu_formats.py > gpurun_out/r6z4_tests_$lib.log 2>&1 || { echo "tests $lib rc=$?"; tail -30 gpurun_out/r6z4_tests_$lib.log; exit 1; }
  echo $lib; tail -1 gpurun_out/r6z4_tests_$lib.log
done
O=gpurun_out/r6z4_enc_ab.txt; : > $O
for rep in 1 2; do
for spec in "ablib/r6end.so 0 c3" "ablib/rawdw.so 0 c3" "ablib/r6end.so 0 c4" "ablib/rawdw.so 0 c4"; do
  set -- $spec; lib=$1; mode=$2; data=$3; tag=$(basename $lib .so)_${data}_$rep
  export TPF_LIB=$R/$lib
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6z4_${tag}_prof -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 5 $mode $data > $R/gpurun_out/r6z4_${tag}.log 2>&1) || { echo "prof $spec rc=$?"; tail -5 $R/gpurun_out/r6z4_${tag}.log; exit 1; }
  python3 -c "
import csv,glob,sys
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if '_write' in r['Name']:
            print(sys.argv[2], r['Name'][15:48], r['Calls'], round(float(r['AverageNs'])/1e6, 4), 'ms')
" $R/gpurun_out/r6z4_${tag}_prof "$spec" >> $O
done
done
unset TPF_LIB
cat $O
