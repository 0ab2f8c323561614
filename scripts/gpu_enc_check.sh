# Encoder iteration on one GPU: encode/drop-in GPU tests, then bench c4
# (prints round trip, encode and decode rates).  RUNS=n repeats the bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_enc256v32.py tests/test_gpu_dropin.py tests/test_gpu_formats.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/enc_t.log 2>&1 || { tail -30 gpurun_out/enc_t.log; exit 1; }
tail -1 gpurun_out/enc_t.log
for i in $(seq ${RUNS:-1}); do
  timeout -k 10 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c4_$i.json 2> gpurun_out/c4_$i.err || { echo "c4 rc=$?"; tail -5 gpurun_out/c4_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c4_$i.json'));c=d['config'];r=c['roundtrip_256v64'];print('c4', d['value'], 'enc', c['enc256v32_G_int32_per_s'], 'dec', c['dec256v32_G_int32_per_s'], c['verified'], '| 64:', r['G_int64_per_s'], 'enc', r['enc_G_int64_per_s'], 'dec', r['dec_G_int64_per_s'], r['verified'])"
done
