# plan-pass VALU diet (ffbh-keyed histogram, hoisted bpermute lanes, ballot vbyte
# costs): encoder tests, C4 A/B against the previous encoder and cache-policy
# knobs, then SQ counters of the windowed p4Dec32 decoder
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_enc256v32.py tests/test_gpu_formats.py tests/test_gpu_dropin.py tests/test_gpu_nstream.py tests/test_gpu_chained.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3q_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r3q_tests.log; exit 1; }
tail -1 gpurun_out/r3q_tests.log
LIBS="tree ablib/h32aux0.so ablib/encnoffbh.so ablib/encA.so ablib/encB.so" WL=c4 ROUNDS=2 TAG=r3q bash scripts/gpu_ab.sh || exit 1
KFILTER=k_dec_h32w TAGC=c1w BENCH_ARGS="--workload c1" COUNTERS="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_ACTIVE_INST_ANY SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_INSTS_BRANCH,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_VALU,SQ_INSTS_SMEM,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_MISC FETCH_SIZE WRITE_SIZE" bash scripts/gpu_counters.sh > gpurun_out/r3q_c1_counters.txt 2>&1 || { echo "counters rc=$?"; tail -5 gpurun_out/r3q_c1_counters.txt; exit 1; }
cat gpurun_out/r3q_c1_counters.txt
