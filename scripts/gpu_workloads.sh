# Runs every bench workload once on one GPU (JSON lines -> gpurun_out/wl_*.json).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python bench.py --e2e --sweep > gpurun_out/wl_c2.json 2> gpurun_out/wl_c2.err || { echo "c2 rc=$?"; tail -5 gpurun_out/wl_c2.err; exit 1; }
cat gpurun_out/wl_c2.json
for w in c1 c3 c3chain c4; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/wl_$w.json 2> gpurun_out/wl_$w.err || { echo "$w rc=$?"; tail -5 gpurun_out/wl_$w.err; exit 1; }
  cat gpurun_out/wl_$w.json
done
