# FETCH_SIZE / WRITE_SIZE passes of bench workloads (default: all five)
# into gpurun_out/pmc_traffic.json (merged with profiles/pmc_traffic.json);
# LABEL names the measurement (e.g. r2_v3), the entry also records the
# library's md5 so bench.py replays it only for that library.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
cd /tmp && export TMPDIR=/tmp
for w in ${WLS:-c2 c3 c3chain c4 c1}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_${w}_$c -o run --output-format csv -- python3 $R/bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench_pmc_${w}_$c.json 2>&1 || { echo "pmc $w $c rc=$?"; tail -20 $R/gpurun_out/bench_pmc_${w}_$c.json; exit 1; }
  done
  python3 $R/scripts/pmc_traffic.py $w $R/gpurun_out/pmc_${w}_FETCH_SIZE/run_counter_collection.csv $R/gpurun_out/pmc_${w}_WRITE_SIZE/run_counter_collection.csv 10000000 $R/gpurun_out/pmc_traffic.json ${LABEL:-unlabelled} || exit 1
  if [ $w = c4 ]; then
    python3 $R/scripts/pmc_traffic.py c4_64 $R/gpurun_out/pmc_${w}_FETCH_SIZE/run_counter_collection.csv $R/gpurun_out/pmc_${w}_WRITE_SIZE/run_counter_collection.csv 10000000 $R/gpurun_out/pmc_traffic.json ${LABEL:-unlabelled} || exit 1
  fi
done
