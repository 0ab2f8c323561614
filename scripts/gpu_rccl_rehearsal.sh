# bench.py's own multi-rank launcher (--gpus 2, no WORLD_SIZE) on a one-GPU
# box with the RCCL backend: both ranks on cuda:0 (TPF_BENCH_SAME_GPU=1),
# init_process_group("nccl", device_id=...), barrier, all_gather and
# all_reduce over RCCL.  A rehearsal, never a measured configuration.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-rccl}
for w in ${WLS:-c2 c3chain}; do
  TPF_BENCH_SAME_GPU=1 NCCL_DEBUG=WARN timeout -k 10 240 python bench.py --gpus 2 --workload $w --nblocks 1000000 --steps 5 --warmup 1 --no-cpu-baseline --no-probes > gpurun_out/${T}_$w.json 2> gpurun_out/${T}_$w.err || { echo "$w rc=$?"; tail -30 gpurun_out/${T}_$w.err; exit 1; }
  tail -1 gpurun_out/${T}_$w.json
done
