# round 6 end library: repeatability on one box -- the default bench (C2) three times, the chained lists twice each
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
O=gpurun_out/r6x_repeat.txt; : > $O
for spec in c2 c2 c2 c3chain c3chain64 c3chain c3chain64; do
  timeout -k 10 300 python -u bench.py --workload $spec --no-cpu-baseline > gpurun_out/r6x_$spec.json 2> gpurun_out/r6x_$spec.err || { echo "bench $spec rc=$?"; tail -5 gpurun_out/r6x_$spec.err; exit 1; }
  tail -1 gpurun_out/r6x_$spec.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$spec', d['value'], d['unit'], 'frac', r['frac'], 'kernel_ms', r.get('kernel_ms_avg'), 'probe_frac', r.get('frac_of_probe'))" >> $O
done
cat $O
