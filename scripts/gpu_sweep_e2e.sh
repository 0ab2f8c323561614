# Full-size per-width decode sweep (10M blocks per bit width) and the
# end-to-end host-memory rates on the current tree.  -> gpurun_out/$TAG_*
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-sw}
timeout -k 10 600 python bench.py --workload sweep --steps 10 --warmup 2 > gpurun_out/${T}_sweep.json 2> gpurun_out/${T}_sweep.err || { echo "sweep rc=$?"; tail -20 gpurun_out/${T}_sweep.err; exit 1; }
grep "\[sweep\]" gpurun_out/${T}_sweep.err
timeout -k 10 400 python bench.py --e2e --no-cpu-baseline --no-probes --steps 10 --warmup 2 > gpurun_out/${T}_e2e.json 2> gpurun_out/${T}_e2e.err || { echo "e2e rc=$?"; tail -20 gpurun_out/${T}_e2e.err; exit 1; }
grep "\[e2e\]" gpurun_out/${T}_e2e.err
