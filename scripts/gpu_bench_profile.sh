# Round profile set for the hot path (C2, default bench size):
#   smoke, bench --sweep, rocprofv3 --kernel-trace --stats, and separate
#   FETCH_SIZE / WRITE_SIZE PMC passes -> profiles/pmc_traffic.json.
# usage: TAG=r1 bash scripts/gpu_bench_profile.sh   (outputs under gpurun_out/)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r1}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --sweep > gpurun_out/bench_sweep.json 2> gpurun_out/bench_sweep.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_sweep.err; exit 1; }
cat gpurun_out/bench_sweep.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stats -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/bench_prof.json 2>$R/gpurun_out/bench_prof.err || { echo "rocprof rc=$?"; tail -20 $R/gpurun_out/bench_prof.err; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench_pmcf.json 2>&1 || { echo "pmc fetch rc=$?"; tail -20 $R/gpurun_out/bench_pmcf.json; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench_pmcw.json 2>&1 || { echo "pmc write rc=$?"; tail -20 $R/gpurun_out/bench_pmcw.json; exit 1; }
cd $R
python3 scripts/pmc_traffic.py c2 gpurun_out/pmc_fetch/run_counter_collection.csv gpurun_out/pmc_write/run_counter_collection.csv 10000000 gpurun_out/pmc_traffic.json
find gpurun_out/prof_stats -name "*.csv" | head
