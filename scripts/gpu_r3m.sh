# read-only load-shape ceilings (scripts/read_shape_probe.hip) and the encoder's
# per-pass times with its two data-movement probes, same box
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 120 ./scripts/read_shape_probe > gpurun_out/r3m_read_shapes.txt 2>&1 || { echo "probe rc=$?"; tail -5 gpurun_out/r3m_read_shapes.txt; exit 1; }
cat gpurun_out/r3m_read_shapes.txt
cd /tmp && export TMPDIR=/tmp
for p in 0 1 2; do
  d=$R/gpurun_out/r3m_enc_$p
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 10 $p > $d.log 2>&1 || { echo "probe $p rc=$?"; tail -5 $d.log; exit 1; }
  echo "== enc probe $p"; grep -h "k_enc256v32" $(find $d -name "*kernel_stats.csv") | cut -d, -f1-4 | sed 's/(unsigned.*",/",/'
done
