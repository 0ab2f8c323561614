set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for p in 0 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/encp_$p -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 10 $p > $R/gpurun_out/encp_$p.log 2>&1 || { echo "probe $p rc=$?"; tail -5 $R/gpurun_out/encp_$p.log; exit 1; }
  echo "== probe $p"; grep -h "k_enc256v32" $(find $R/gpurun_out/encp_$p -name "*kernel_stats.csv") | cut -d, -f1-4 | sed 's/(unsigned.*",/",/'
done
