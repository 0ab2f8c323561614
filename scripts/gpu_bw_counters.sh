# Per-bit-width SQ counters of the hot-path decode (scripts/bw_counters.py
# under rocprofv3 --pmc, two passes within the per-block limits), reported
# per block by scripts/bw_counters_report.py -> gpurun_out/${TAG}_bw_counters.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
T=${TAG:-bwc}
NB=${NB:-2000000}
cd /tmp && export TMPDIR=/tmp
i=0
for c in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" "SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c -d $R/gpurun_out/${T}_p$i -o run --output-format csv -- python3 $R/scripts/bw_counters.py $NB > $R/gpurun_out/${T}_p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $R/gpurun_out/${T}_p$i.log; exit 1; }
done
ORDER=$(grep "^ORDER" $R/gpurun_out/${T}_p1.log | cut -d' ' -f2)
python3 $R/scripts/bw_counters_report.py $NB "$ORDER" $R/gpurun_out/${T}_p1/run_counter_collection.csv $R/gpurun_out/${T}_p2/run_counter_collection.csv > $R/gpurun_out/${T}_bw_counters.txt && cat $R/gpurun_out/${T}_bw_counters.txt
