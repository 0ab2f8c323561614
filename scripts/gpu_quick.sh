# GPU tests + N bench runs of the default workload: RUNS=2 bash scripts/gpu_quick.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for i in $(seq ${RUNS:-2}); do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 ${BENCH_ARGS} > gpurun_out/q_$i.json 2> gpurun_out/q_$i.err || { echo "bench rc=$?"; tail -5 gpurun_out/q_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/q_$i.json'));print('run $i', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms_avg'], d['config'].get('verified'))"
done
