# A/B an environment knob of the decode kernel: ENVVAR=NAME VALUES="a b c" bash scripts/gpu_env_ab.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for round in 1 2; do
for v in $VALUES; do
  env $ENVVAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 ${BENCH_ARGS} > gpurun_out/env_$v.json 2> gpurun_out/env_$v.err || { echo "$v rc=$?"; tail -5 gpurun_out/env_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/env_$v.json'));print('round $round $ENVVAR=$v', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms_avg'], d['config']['verified'])"
done
done
