# phase A counters (k_dsum256v32_lanes) for the committed library and the tree
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export KFILTER=k_dsum256v32_lanes BENCH_ARGS="--workload c3chain" NB=10000000
export COUNTERS="SQ_ACTIVE_INST_ANY,SQ_BUSY_CYCLES,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_VALU,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES GRBM_GUI_ACTIVE,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_VALU,SQ_INSTS_BRANCH,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAVES"
LIBS="ablib/head.so ablib/stage.so tree" bash scripts/gpu_counters_libs.sh > gpurun_out/r3i_counters.txt 2>&1 || { tail -20 gpurun_out/r3i_counters.txt; exit 1; }
cat gpurun_out/r3i_counters.txt
