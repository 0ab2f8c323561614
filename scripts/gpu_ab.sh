# A/B of library builds on one box: LIBS="tree ablib/x.so ..." WL=c3chain ROUNDS=2
# bash scripts/gpu_ab.sh -> one line per run (value, verified, per-pass rates).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
WL=${WL:-c3chain}; T=${TAG:-ab}
for i in $(seq ${ROUNDS:-2}); do
  for lib in ${LIBS:-tree}; do
    if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
    n=$(basename $lib .so)
    timeout -k 10 240 python bench.py --workload $WL --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-probes ${BARGS} > gpurun_out/${T}_${n}_$i.json 2> gpurun_out/${T}_${n}_$i.err || { echo "$n rc=$?"; tail -5 gpurun_out/${T}_${n}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; r=d['roofline']; print(sys.argv[2], d['value'], 'ms', r.get('kernel_ms_avg'), 'verified', c.get('verified'), {k: v for k, v in c.items() if k.endswith('per_s')})" gpurun_out/${T}_${n}_$i.json $n
  done
done
