# A/B of a saved library (abtmp/lib_a.so, TPF_LIB) against the current build:
# C4 (256v32 + 256v64 encode rates) and C1 (p4Enc32 batch) per library,
# alternating ROUNDS times; then the GPU tests on the current build.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for i in $(seq ${ROUNDS:-2}); do for lib in a cur; do
  if [ $lib = a ]; then export TPF_LIB=$R/abtmp/lib_a.so; else unset TPF_LIB; fi
  timeout -k 10 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_c4_$lib.json 2>/dev/null || { echo "c4 $lib failed"; exit 1; }
  timeout -k 10 200 python bench.py --workload c1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_c1_$lib.json 2>/dev/null || { echo "c1 $lib failed"; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/ab_c4_$lib.json'));c=d['config'];r=c['roundtrip_256v64']
e=json.load(open('gpurun_out/ab_c1_$lib.json'));
print('lib=$lib', 'enc32', c['enc256v32_G_int32_per_s'], 'enc64', r['enc_G_int64_per_s'], 'c1enc', e['config'].get('enc32_G_int32_per_s'), 'verified', c['verified'], r['verified'], e['config']['verified'])"
done; done
unset TPF_LIB
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/tests.log
