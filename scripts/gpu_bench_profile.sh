# Round profile set for the hot path (C2, default bench size), one call:
#   rocprofv3 --kernel-trace --stats of the default bench, then separate
#   FETCH_SIZE / WRITE_SIZE PMC passes of every workload (gpu_pmc_steps.sh)
#   -> gpurun_out/pmc_traffic.json (copy to profiles/ to have bench replay it).
# usage: TAG=r2_final bash scripts/gpu_bench_profile.sh   (outputs under gpurun_out/)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${TAG:-prof}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof_stats -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/${T}_bench_c2_under_rocprof.json 2>$R/gpurun_out/${T}_bench_prof.err || { echo "rocprof rc=$?"; tail -20 $R/gpurun_out/${T}_bench_prof.err; exit 1; }
tail -1 $R/gpurun_out/${T}_bench_c2_under_rocprof.json
LABEL=$T bash $R/scripts/gpu_pmc_steps.sh
