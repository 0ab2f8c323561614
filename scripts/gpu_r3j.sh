# phase B (k_dec256v32w<Prefix>) issue counters on the C3 chained list
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export KFILTER=k_dec256v32w BENCH_ARGS="--workload c3chain" NB=10000000
export COUNTERS="SQ_ACTIVE_INST_ANY,SQ_BUSY_CYCLES,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_VALU,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES GRBM_GUI_ACTIVE,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_VALU,SQ_INSTS_BRANCH,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAVES"
LIBS="ablib/head.so" bash scripts/gpu_counters_libs.sh > gpurun_out/r3j_counters.txt 2>&1 || { tail -20 gpurun_out/r3j_counters.txt; exit 1; }
cat gpurun_out/r3j_counters.txt | cut -c40-
