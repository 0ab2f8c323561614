# 256v64 decode output stores: sc1 nt via run descriptor (ablib/d64sc1.so) vs nt: format tests on the variant, C4 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TPF_LIB=$R/ablib/d64sc1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_formats.py tests/test_gpu_fuzz.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3x_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r3x_tests.log; exit 1; }
tail -1 gpurun_out/r3x_tests.log
for i in 1 2 3; do
  for lib in tree ablib/d64sc1.so; do
    if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
    n=$(basename $lib .so)
    timeout -k 10 240 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline --no-probes > gpurun_out/r3x_${n}_$i.json 2> gpurun_out/r3x_${n}_$i.err || { echo "$n rc=$?"; tail -5 gpurun_out/r3x_${n}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']['roundtrip_256v64']; print(sys.argv[2], c)" gpurun_out/r3x_${n}_$i.json $n
  done
done
