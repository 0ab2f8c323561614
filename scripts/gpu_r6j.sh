# round 6: per-block scaling with the latch harness (auto / spin policy / round-5 library), the D1 write-pass probe,
# SQ counters of the 32-bit chained phase A (k_dsum256v32_lanes) on the final kernels
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r6j}
for i in 1 2; do
  LIBS="tree" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=${T}auto$i PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
  TPF_PERBLOCK_WAIT=spin LIBS="tree" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=${T}spin$i PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
  LIBS="ablib/r5base.so" K=3000 THREADS="1 16 24 32 48 64 96 128" TAG=${T}r5$i PBT_TIMEOUT=240 bash scripts/pbt_libs.sh || exit 1
done
for spec in "0 c3" "2 c3" "0 c4" "2 c4"; do
  set -- $spec; mode=$1; data=$2
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_enc_${mode}_${data}_prof -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 5 $mode $data > $R/gpurun_out/${T}_enc_${mode}_${data}.log 2>&1) || { echo "prof $spec rc=$?"; tail -5 $R/gpurun_out/${T}_enc_${mode}_${data}.log; exit 1; }
  python3 -c "
import csv,glob,sys
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if '_write' in r['Name'] or '_plan' in r['Name']:
            print(sys.argv[2], r['Name'][15:48], r['Calls'], round(float(r['AverageNs'])/1e6, 4), 'ms')
" $R/gpurun_out/${T}_enc_${mode}_${data}_prof "$spec"
done
COUNTERS="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_ANY SQ_WAIT_ANY,SQ_LDS_BANK_CONFLICT,SQ_BUSY_CYCLES,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_WAVES,GRBM_GUI_ACTIVE" BENCH_ARGS="--workload c3chain" KFILTER=k_dsum TAGC=${T}dsum bash scripts/gpu_counters.sh > gpurun_out/${T}_dsum_counters.txt 2>&1 || { echo "counters rc=$?"; tail -5 gpurun_out/${T}_dsum_counters.txt; exit 1; }
cat gpurun_out/${T}_dsum_counters.txt
