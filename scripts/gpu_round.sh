# One-call round check on a GPU box: GPU tests, smoke, every bench workload,
# then the rocprofv3 kernel-trace summary and FETCH/WRITE PMC passes of the
# default bench.  usage: TAG=r1 bash scripts/gpu_round.sh  (-> gpurun_out/)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash scripts/gpu_workloads.sh || exit 1
[ -n "$NOPROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stats -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/bench_prof.json 2>$R/gpurun_out/bench_prof.err || { echo "rocprof rc=$?"; tail -20 $R/gpurun_out/bench_prof.err; exit 1; }
cat $R/gpurun_out/bench_prof.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench_pmcf.json 2>&1 || { echo "pmc fetch rc=$?"; tail -20 $R/gpurun_out/bench_pmcf.json; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench_pmcw.json 2>&1 || { echo "pmc write rc=$?"; tail -20 $R/gpurun_out/bench_pmcw.json; exit 1; }
cd $R
python3 scripts/pmc_traffic.py gpurun_out/pmc_fetch/run_counter_collection.csv gpurun_out/pmc_write/run_counter_collection.csv 10000000 gpurun_out/pmc_traffic.json
find gpurun_out/prof_stats -name "*stats*.csv"
