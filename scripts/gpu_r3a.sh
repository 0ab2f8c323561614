# Round 3 first check: GPU tests, then c2 / c3chain / c4 bench lines (no CPU baseline).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r3a}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for w in ${WLS:-c2 c3chain c4}; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_$w.json 2> gpurun_out/${T}_$w.err || { echo "$w rc=$?"; tail -5 gpurun_out/${T}_$w.err; exit 1; }
  tail -c 600 gpurun_out/${T}_$w.json; echo
done
