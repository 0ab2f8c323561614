# round 6 final evidence, part 2: bench lines (with CPU baselines) and rocprofv3 kernel stats per workload
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r6end}
steps=""
for wl in ${WLS:-c2 c3 c3chain c3chain64}; do steps="$steps bench:$wl prof:$wl"; done
TAG=$T bash scripts/gpu.sh $steps
