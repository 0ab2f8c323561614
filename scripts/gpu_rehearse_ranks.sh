# Rehearsal of bench.py's multi-rank path on a one-GPU box (never a measured
# configuration): 2 ranks via torch.distributed.run, both on cuda:0, the
# collectives over gloo; c2, c3chain (the all-gather exchange step) and c4
# with small shards.  JSON lines -> gpurun_out/rank2_*.json
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for w in c2 c3chain c4; do
  TPF_BENCH_BACKEND=gloo TPF_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload $w --nblocks 1000000 --steps 5 --warmup 1 > gpurun_out/rank2_$w.json 2> gpurun_out/rank2_$w.err || { echo "$w rc=$?"; tail -20 gpurun_out/rank2_$w.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/rank2_$w.json').read().strip().splitlines()[-1]);print('$w', d['n_gpus'], d['value'], d['config']['verified'], d['config'].get('parallelism'))"
done
