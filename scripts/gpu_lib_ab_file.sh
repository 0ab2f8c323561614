# A/B of the working-tree library against another built library file
# (NEW=abtmp/x.so) on one box, alternating ROUNDS times: bench.py --workload $WL.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
WL=${WL:-c4}
for i in $(seq ${ROUNDS:-2}); do
  for lib in tree new; do
    if [ $lib = new ]; then export TPF_LIB=$R/$NEW; else unset TPF_LIB; fi
    timeout -k 10 200 python bench.py --workload $WL --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/abf_${lib}_$i.json 2> gpurun_out/abf_${lib}_$i.err || { echo "$lib rc=$?"; tail -5 gpurun_out/abf_${lib}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[2], d['value'], c.get('verified'), {k: v for k, v in c.items() if k.endswith('per_s')})" gpurun_out/abf_${lib}_$i.json $lib
  done
done
