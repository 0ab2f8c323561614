# plan pass with shifted suffix sums through LDS (ablib/sfx.so, TPF_PLAN_SUFFIX_LDS=1):
# encoder tests on the variant, C4 A/B, per-pass times
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TPF_LIB=$R/ablib/sfx.so timeout -k 10 300 python -u -m pytest tests/test_gpu_enc256v32.py tests/test_gpu_nstream.py tests/test_gpu_chained.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3ai_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r3ai_tests.log; exit 1; }
tail -1 gpurun_out/r3ai_tests.log
LIBS="tree ablib/sfx.so" WL=c4 ROUNDS=3 TAG=r3ai bash scripts/gpu_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp
for lib in tree ablib/sfx.so; do
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  d=$R/gpurun_out/r3ai_enc_$(basename $lib .so)
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 10 0 > $d.log 2>&1 || { echo "enc $lib rc=$?"; tail -5 $d.log; exit 1; }
  echo "== $lib"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_enc256v32' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e6, 4))
" $(find $d -name "*kernel_stats.csv")
done
