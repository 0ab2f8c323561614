# round-3 final library, part A: every GPU test, smoke, default bench, every workload line
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/r3f1_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error" gpurun_out/r3f1_tests.log | tail -8; exit 1; }
tail -1 gpurun_out/r3f1_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r3f1_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/r3f1_smoke.log; exit 1; }
tail -3 gpurun_out/r3f1_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r3f1_bench_default.json 2> gpurun_out/r3f1_default.err || { echo "default rc=$?"; tail -5 gpurun_out/r3f1_default.err; exit 1; }
tail -1 gpurun_out/r3f1_bench_default.json | cut -c1-300
TAG=r3f1 WLS="c1 c3 c3chain c4 c5" bash scripts/gpu_workloads.sh 2>&1 | cut -c1-300
