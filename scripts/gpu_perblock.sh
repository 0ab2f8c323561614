# Per-block drop-in designs on the GPU: the drop-in tests (both designs,
# concurrent threads), the latency of both designs, and the end-to-end
# host-memory rates.  -> gpurun_out/$TAG_*
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-pb}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dropin.py > gpurun_out/${T}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 120 python scripts/perblock_latency.py 5000 > gpurun_out/${T}_latency.txt 2>&1 || { echo "latency rc=$?"; tail -20 gpurun_out/${T}_latency.txt; exit 1; }
cat gpurun_out/${T}_latency.txt
timeout -k 10 400 python bench.py --e2e --no-cpu-baseline --no-probes --steps 5 --warmup 1 > gpurun_out/${T}_e2e.json 2> gpurun_out/${T}_e2e.err || { echo "e2e rc=$?"; tail -20 gpurun_out/${T}_e2e.err; exit 1; }
grep "\[e2e\]" gpurun_out/${T}_e2e.err
