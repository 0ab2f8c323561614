# 256v32 encoder write pass: dword copy-out (ablib/encdw.so, TPF_ENC_COPY_DW=1) vs
# 16-byte chunks: encoder tests on the variant, C4 A/B, per-pass times of both
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TPF_LIB=$R/ablib/encdw.so timeout -k 10 400 python -u -m pytest tests/test_gpu_enc256v32.py tests/test_gpu_nstream.py tests/test_gpu_edges.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3w_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r3w_tests.log; exit 1; }
tail -1 gpurun_out/r3w_tests.log
LIBS="tree ablib/encdw.so" WL=c4 ROUNDS=3 TAG=r3w bash scripts/gpu_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp
for lib in tree ablib/encdw.so; do
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  for p in 0 2; do
  d=$R/gpurun_out/r3w_enc_$(basename $lib .so)_$p
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 10 $p > $d.log 2>&1 || { echo "enc $lib rc=$?"; tail -5 $d.log; exit 1; }
  echo "== $lib probe $p"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_enc256v32' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e6, 4))
" $(find $d -name "*kernel_stats.csv")
  done
done
