set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --sweep > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json; cat gpurun_out/bench1.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/bench_prof.json 2>&1 || { echo "rocprof rc=$?"; tail -20 $R/gpurun_out/bench_prof.json; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc1f -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench_pmcf.json 2>&1 || { echo "pmc fetch rc=$?"; tail -20 $R/gpurun_out/bench_pmcf.json; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc1w -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench_pmcw.json 2>&1 || { echo "pmc write rc=$?"; tail -20 $R/gpurun_out/bench_pmcw.json; exit 1; }
find $R/gpurun_out -name "*.csv" | head -20
