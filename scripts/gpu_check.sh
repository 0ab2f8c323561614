# GPU tests + smoke + default bench (+ optional extra bench args), one call.
# usage: TAG=r2_v1 bash scripts/gpu_check.sh   (-> gpurun_out/$TAG_*)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-chk}
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/${T}_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
