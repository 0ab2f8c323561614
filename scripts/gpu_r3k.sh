# round-3 snapshot: every GPU test, smoke, every bench workload (TAG=r3k)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/r3k_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r3k_tests.log; exit 1; }
tail -1 gpurun_out/r3k_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r3k_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/r3k_smoke.log; exit 1; }
tail -3 gpurun_out/r3k_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r3k_bench_default.json 2> gpurun_out/r3k_default.err || { echo "default rc=$?"; tail -5 gpurun_out/r3k_default.err; exit 1; }
tail -1 gpurun_out/r3k_bench_default.json
TAG=r3k WLS="c1 c3 c3chain c4 c5" bash scripts/gpu_workloads.sh
