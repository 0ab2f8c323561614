# round-3 final library, part B: rocprofv3 kernel stats of the default bench and
# of the chained C3 line, then FETCH/WRITE PMC passes of every workload
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3_f1_c3chain_prof -o run --output-format csv -- python3 $R/bench.py --workload c3chain --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/r3_f1_bench_c3chain_under_rocprof.json 2> $R/gpurun_out/r3_f1_c3chain_prof.err || { echo "c3chain rocprof rc=$?"; tail -5 $R/gpurun_out/r3_f1_c3chain_prof.err; exit 1; }
TAG=r3_f1 bash $R/scripts/gpu_bench_profile.sh
