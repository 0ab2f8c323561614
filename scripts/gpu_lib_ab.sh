# A/B of the working-tree library against abtmp/base.so (scripts/build_base_lib.sh)
# on one box, alternating ROUNDS times: bench.py --workload $WL, key numbers per run.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
WL=${WL:-c4}
for i in $(seq ${ROUNDS:-2}); do
  for lib in base new; do
    if [ $lib = base ]; then export TPF_LIB=$R/abtmp/base.so; else unset TPF_LIB; fi
    timeout -k 10 200 python bench.py --workload $WL --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/ab_${lib}_$i.json 2> gpurun_out/ab_${lib}_$i.err || { echo "$lib rc=$?"; tail -5 gpurun_out/ab_${lib}_$i.err; exit 1; }
    python - gpurun_out/ab_${lib}_$i.json $lib <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); c = d['config']
extra = {k: v for k, v in c.items() if k.endswith('per_s')}
r = c.get('roundtrip_256v64')
if r:
    extra['64'] = (r['G_int64_per_s'], r['enc_G_int64_per_s'], r['dec_G_int64_per_s'], r['verified'])
print(sys.argv[2], d['value'], c.get('verified'), extra)
PY
  done
done
