# 256v32 encoder pipeline depth per pass (TPF_ENC_NC_PLAN / TPF_ENC_NC_WRITE
# build knobs): C4 A/B, then per-pass kernel times of each library
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
LIBS="tree ablib/encP2.so ablib/encP4.so ablib/encW2.so ablib/encW4.so" WL=c4 ROUNDS=2 TAG=r3u bash scripts/gpu_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp
for lib in tree ablib/encP4.so ablib/encW4.so; do
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  d=$R/gpurun_out/r3u_enc_$(basename $lib .so)
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 10 0 > $d.log 2>&1 || { echo "enc $lib rc=$?"; tail -5 $d.log; exit 1; }
  echo "== $lib"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_enc256v32' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e6, 4))
" $(find $d -name "*kernel_stats.csv")
done
