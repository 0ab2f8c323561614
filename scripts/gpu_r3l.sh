# encoder pipeline depth A/B: per-kernel times (rocprofv3 --kernel-trace --stats)
# of the C4-mix 256v32 encode for each library in LIBS; PROBES: probe kinds
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for lib in ${LIBS}; do
  export TPF_LIB=$R/$lib
  for p in ${PROBES:-0}; do
    d=$R/gpurun_out/r3l_$(basename $lib .so)_$p
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 10 $p > $d.log 2>&1 || { echo "$lib probe $p rc=$?"; tail -5 $d.log; exit 1; }
    echo "== $lib probe $p"; grep -h "k_enc256v32" $(find $d -name "*kernel_stats.csv") | cut -d, -f1-4 | sed 's/(unsigned.*",/",/'
  done
done
