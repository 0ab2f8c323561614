# round 6: chained phase A after the fast-path rewrite + read-ahead: ablation builds (TPF_DSUM_ABLATE 16 stage only,
# 1 no base sums, 2 no compressed vbyte, 4 no raw vbyte, 8 no positions, 6 neither vbyte form) and SQ counters incl. LDS stalls
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
O=gpurun_out/r6r_phaseA.txt; : > $O
for lib in tree ablib/abl16.so ablib/abl1.so ablib/abl2.so ablib/abl4.so ablib/abl8.so ablib/abl6.so tree ablib/r6final.so; do
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$lib; fi
  timeout -k 10 200 python -u scripts/chain_phase_probe.py 10000000 >> $O 2>&1 || { echo "rc=$? $lib"; tail -5 $O; exit 1; }
done
unset TPF_LIB
grep -v amdgpu.ids $O
COUNTERS="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_ANY SQ_WAIT_ANY,SQ_LDS_BANK_CONFLICT,SQ_BUSY_CYCLES,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_WAVES,GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS,SQ_LDS_UNALIGNED_STALL,SQ_LDS_ADDR_CONFLICT,SQ_INSTS_SMEM" BENCH_ARGS="--workload c3chain" KFILTER=k_dsum TAGC=r6rdsum bash scripts/gpu_counters.sh > gpurun_out/r6r_dsum_counters.txt 2>&1 || { echo "counters rc=$?"; tail -5 gpurun_out/r6r_dsum_counters.txt; exit 1; }
cat gpurun_out/r6r_dsum_counters.txt
