# round 6: C3 D1 write-pass ablation (timing only, outputs wrong): encnovb = no vbyte exception emission, encnobase = no base
# packing in vbyte blocks; tree = the end library; mode 2 = the write pass's data-movement probe
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
O=gpurun_out/r6y_enc_ablation.txt; : > $O
for rep in 1 2; do
for spec in "tree 0" "ablib/encnovb.so 0" "ablib/encnobase.so 0" "tree 2"; do
  set -- $spec; lib=$1; mode=$2; tag=$(basename $lib .so)_$mode_$rep
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6y_${tag}_prof -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 5 $mode c3 > $R/gpurun_out/r6y_${tag}.log 2>&1) || { echo "prof $spec rc=$?"; tail -5 $R/gpurun_out/r6y_${tag}.log; exit 1; }
  python3 -c "
import csv,glob,sys
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if '_write' in r['Name'] or '_plan' in r['Name']:
            print(sys.argv[2], r['Name'][15:48], r['Calls'], round(float(r['AverageNs'])/1e6, 4), 'ms')
" $R/gpurun_out/r6y_${tag}_prof "$spec" >> $O
done
done
unset TPF_LIB
cat $O
