# SQ counters of the final library's 256v32 encoder passes and their probes (C4 workload, 2M blocks)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
C="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_ACTIVE_INST_ANY SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_INSTS_BRANCH,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_SCA"
KFILTER=k_enc256v32 TAGC=encf BENCH_ARGS="--workload c4" COUNTERS="$C" bash scripts/gpu_counters.sh > gpurun_out/r3f3_enc_counters.txt 2>&1 || { echo "counters rc=$?"; tail -5 gpurun_out/r3f3_enc_counters.txt; exit 1; }
cat gpurun_out/r3f3_enc_counters.txt | cut -c1-160
