# Bench lines of every workload on one GPU (JSON -> gpurun_out/$TAG_bench_*.json):
# c2 with the end-to-end host legs, then c1 c3 c3chain c4 with their CPU baselines.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-wl}
timeout -k 10 400 python bench.py --e2e --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_bench_c2_e2e.json 2> gpurun_out/${T}_c2_e2e.err || { echo "c2 e2e rc=$?"; tail -5 gpurun_out/${T}_c2_e2e.err; exit 1; }
tail -1 gpurun_out/${T}_bench_c2_e2e.json
for w in ${WLS:-c1 c3 c3chain c4}; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 > gpurun_out/${T}_bench_$w.json 2> gpurun_out/${T}_$w.err || { echo "$w rc=$?"; tail -5 gpurun_out/${T}_$w.err; exit 1; }
  tail -1 gpurun_out/${T}_bench_$w.json
done
