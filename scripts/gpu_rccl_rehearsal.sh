# Multi-rank rehearsals on a one-GPU box (never measured configurations):
#  1. bench.py's own launcher (--gpus 2, no WORLD_SIZE): two ranks on cuda:0
#     (TPF_BENCH_SAME_GPU=1) with the collectives over gloo -- RCCL refuses
#     two ranks on one device ("Duplicate GPU detected", NCCL 2.26.6);
#  2. the RCCL path itself: torch.distributed.run with one rank, so
#     init_process_group("nccl", device_id=...), barrier, all_gather and
#     all_reduce run over RCCL on the real GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-rccl}
for w in ${WLS:-c2 c3chain}; do
  TPF_BENCH_SAME_GPU=1 TPF_BENCH_BACKEND=gloo timeout -k 10 240 python bench.py --gpus 2 --workload $w --nblocks 1000000 --steps 5 --warmup 1 --no-cpu-baseline --no-probes > gpurun_out/${T}_gloo2_$w.json 2> gpurun_out/${T}_gloo2_$w.err || { echo "gloo2 $w rc=$?"; tail -30 gpurun_out/${T}_gloo2_$w.err; exit 1; }
  tail -1 gpurun_out/${T}_gloo2_$w.json
  NCCL_DEBUG=WARN timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --workload $w --nblocks 1000000 --steps 5 --warmup 1 --no-cpu-baseline --no-probes > gpurun_out/${T}_rccl1_$w.json 2> gpurun_out/${T}_rccl1_$w.err || { echo "rccl1 $w rc=$?"; tail -30 gpurun_out/${T}_rccl1_$w.err; exit 1; }
  tail -1 gpurun_out/${T}_rccl1_$w.json
done
