# full GPU suite on the working tree, C1 A/B (templated elements per lane vs the
# committed windowed decoder), per-pass encoder times for the tree and the
# previous encoder (rocprofv3 kernel stats)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/r3r_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r3r_tests.log; exit 1; }
tail -1 gpurun_out/r3r_tests.log
LIBS="tree ablib/h32pf.so" WL=c1 ROUNDS=2 TAG=r3r bash scripts/gpu_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp
for lib in tree ablib/h32aux0.so; do
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  d=$R/gpurun_out/r3r_enc_$(basename $lib .so)
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 10 0 > $d.log 2>&1 || { echo "enc $lib rc=$?"; tail -5 $d.log; exit 1; }
  echo "== $lib"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_enc256v32' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e6, 4))
" $(find $d -name "*kernel_stats.csv")
done
