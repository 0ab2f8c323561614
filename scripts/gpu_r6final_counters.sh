# round 6 final evidence, part 3: SQ counters of the final encoders (C3 D1, C4, 256v64) and the write-pass probes
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r6final}
MODES=3 DATA=c3 TAG=${T}c3 bash scripts/gpu_enc_counters.sh || exit 1
MODES=3 DATA=c4 TAG=${T}c4 bash scripts/gpu_enc_counters.sh || exit 1
DATA=v64 MODES=3 TAG=${T}v64 bash scripts/gpu_enc_counters.sh || exit 1
for spec in "0 c3" "2 c3" "0 c4" "1 c4" "2 c4"; do
  set -- $spec; mode=$1; data=$2
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_encp_${mode}_${data}_prof -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 5 $mode $data > $R/gpurun_out/${T}_encp_${mode}_${data}.log 2>&1) || { echo "prof $spec rc=$?"; exit 1; }
  python3 -c "
import csv,glob,sys
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if '_write' in r['Name'] or '_plan' in r['Name']:
            print(sys.argv[2], r['Name'][15:48], r['Calls'], round(float(r['AverageNs'])/1e6, 4), 'ms')
" $R/gpurun_out/${T}_encp_${mode}_${data}_prof "$spec" | tee -a $R/gpurun_out/${T}_enc_probes.txt
done
