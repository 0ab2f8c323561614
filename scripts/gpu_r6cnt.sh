# round 6 end library: SQ counters of both chained phase-A kernels (k_dsum256v32_lanes on c3chain, k_dsum128v64_lanes on c3chain64)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
C="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_ANY SQ_WAIT_ANY,SQ_LDS_BANK_CONFLICT,SQ_BUSY_CYCLES,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_WAVES,GRBM_GUI_ACTIVE"
COUNTERS="$C" BENCH_ARGS="--workload c3chain" KFILTER=k_dsum TAGC=r6endd32 bash scripts/gpu_counters.sh > gpurun_out/r6end_dsum32_counters.txt 2>&1 || { echo "c32 rc=$?"; tail -5 gpurun_out/r6end_dsum32_counters.txt; exit 1; }
COUNTERS="$C" BENCH_ARGS="--workload c3chain64" KFILTER=k_dsum TAGC=r6endd64 bash scripts/gpu_counters.sh > gpurun_out/r6end_dsum64_counters.txt 2>&1 || { echo "c64 rc=$?"; tail -5 gpurun_out/r6end_dsum64_counters.txt; exit 1; }
cat gpurun_out/r6end_dsum32_counters.txt gpurun_out/r6end_dsum64_counters.txt
