# round-3 final library (second freeze): every GPU test, smoke, default bench, every
# workload line, rocprofv3 kernel stats (default bench, chained C3), FETCH/WRITE PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r3f2}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error" gpurun_out/${T}_tests.log | tail -8; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/${T}_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -2 gpurun_out/${T}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_default.err || { echo "default rc=$?"; tail -5 gpurun_out/${T}_default.err; exit 1; }
tail -1 gpurun_out/${T}_bench_default.json | cut -c1-200
TAG=$T WLS="c1 c3 c3chain c4 c5" bash scripts/gpu_workloads.sh 2>&1 | cut -c1-200 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_c3chain_prof -o run --output-format csv -- python3 $R/bench.py --workload c3chain --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${T}_bench_c3chain_under_rocprof.json 2> $R/gpurun_out/${T}_c3chain_prof.err || { echo "c3chain rocprof rc=$?"; tail -5 $R/gpurun_out/${T}_c3chain_prof.err; exit 1; }
TAG=$T bash $R/scripts/gpu_bench_profile.sh 2>&1 | cut -c1-300
cd $R
# afterwards (does not change the package): non-temporal packed-stream loads in the hot decode, C2 A/B
true  # (the nt-load A/B ran with r3f2)
