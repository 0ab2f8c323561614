# A/B of the plan pass's histogram variants (TPF_ENC_PROBE 0 = kept C=16,
# 3 = C=32, 4 = C=16 + in-lane merge, 5 = C=8 + merge): C4 encode rate and
# full round-trip verification per variant, alternating ROUNDS times.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for i in $(seq ${ROUNDS:-2}); do for p in ${VARIANTS:-0 3 4 5}; do
  TPF_ENC_PROBE=$p timeout -k 10 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/eh_$p.json 2>/dev/null || { echo "variant $p failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/eh_$p.json'));c=d['config'];print('probe=$p', 'enc', c['enc256v32_G_int32_per_s'], 'rt', d['value'], 'verified', c['verified'])"
done; done
