# final library: multi-rank rehearsal on a one-GPU box (launcher --gpus 2 over gloo, RCCL at world size 1) and the
# full-size per-bit-width sweep
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TAG=r3f3_rehearsal WLS="c2 c3chain c5" bash scripts/gpu_rccl_rehearsal.sh 2>&1 | cut -c1-300 || exit 1
timeout -k 10 600 python bench.py --workload sweep --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r3f3_bench_sweep.json 2> gpurun_out/r3f3_sweep.txt || { echo "sweep rc=$?"; tail -5 gpurun_out/r3f3_sweep.txt; exit 1; }
grep "\[sweep\]" gpurun_out/r3f3_sweep.txt | tail -34
