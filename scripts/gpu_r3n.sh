# windowed p4Dec32 decoder: generic-format GPU tests, then the C1 bench line
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_formats.py tests/test_gpu_fuzz.py tests/test_gpu_nstream.py tests/test_gpu_dropin.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3n_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error|error" gpurun_out/r3n_tests.log | head -20; tail -30 gpurun_out/r3n_tests.log; exit 1; }
tail -1 gpurun_out/r3n_tests.log
for i in 1 2; do
timeout -k 10 300 python bench.py --workload c1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3n_bench_c1_$i.json 2> gpurun_out/r3n_c1.err || { echo "c1 rc=$?"; tail -5 gpurun_out/r3n_c1.err; exit 1; }
tail -1 gpurun_out/r3n_bench_c1_$i.json | cut -c1-400
done
