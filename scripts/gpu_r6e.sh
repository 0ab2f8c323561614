# round 6: 64-bit encoder tests + C4 A/B (256v32 and 256v64 encoders) and C3 D1 encode A/B per library build
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r6e}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_formats.py tests/test_gpu_chained64.py tests/test_gpu_enc256v32.py tests/test_gpu_edges.py tests/test_gpu_host_pageable.py > gpurun_out/${T}_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
LIBS="$LIBS" ROUNDS=2 TAG=$T bash scripts/gpu.sh ab:c4 ab:c3enc || exit 1
for lib in $LIBS; do
  n=$(basename $lib .so)
  if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_${n}_v64_prof -o run --output-format csv -- python3 $R/scripts/enc64_kernel_times.py 10000000 5 > $R/gpurun_out/${T}_${n}_v64.log 2>&1) || { echo "prof $n rc=$?"; tail -5 $R/gpurun_out/${T}_${n}_v64.log; exit 1; }
  python3 -c "
import csv,glob,sys
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if '_write' in r['Name'] or '_plan' in r['Name']:
            print(sys.argv[2], r['Name'][15:45], r['Calls'], round(float(r['AverageNs'])/1e6, 4), 'ms')
" $R/gpurun_out/${T}_${n}_v64_prof $n
done
