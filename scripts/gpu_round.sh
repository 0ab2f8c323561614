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
rm -f $R/gpurun_out/pmc_traffic.json
for w in c2 c3 c1 c3chain c4; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_${w}_$c -o run --output-format csv -- python3 $R/bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench_pmc_${w}_$c.json 2>&1 || { echo "pmc $w $c rc=$?"; tail -20 $R/gpurun_out/bench_pmc_${w}_$c.json; exit 1; }
  done
  python3 $R/scripts/pmc_traffic.py $w $R/gpurun_out/pmc_${w}_FETCH_SIZE/run_counter_collection.csv $R/gpurun_out/pmc_${w}_WRITE_SIZE/run_counter_collection.csv 10000000 $R/gpurun_out/pmc_traffic.json || exit 1
done
cd $R
find gpurun_out/prof_stats -name "*stats*.csv"
