# Decode layout A/B (RunPlaneT ONE = one load per block in flight, rest of
# big blocks at staging): decode tests with ONE forced on, then each
# workload alternating TPF_DEC_ONE=0 / 1, ROUNDS times.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TPF_DEC_ONE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_dec256v32.py tests/test_gpu_chained.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/one_t.log 2>&1 || { tail -30 gpurun_out/one_t.log; exit 1; }
tail -1 gpurun_out/one_t.log
for i in $(seq ${ROUNDS:-2}); do for w in ${WLS:-c2 c3 c3chain}; do for one in 0 1; do
  TPF_DEC_ONE=$one timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/one_${w}_$one.json 2>/dev/null || { echo "$w $one failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/one_${w}_$one.json'));r=d['roofline'];print('$w one=$one', d['value'], r['kernel_ms_avg'], r.get('probe_GBps'), d['config']['verified'])"
done; done; done
