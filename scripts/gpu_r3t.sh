# full GPU suite (async, as the driver runs it), then the C1 A/B and per-pass encoder times of gpu_r3r.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/r3t_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "PASSED|FAILED|Error" gpurun_out/r3t_tests.log | tail -8; exit 1; }
tail -1 gpurun_out/r3t_tests.log
sed -n '/^LIBS=/,$p' scripts/gpu_r3r.sh > /tmp/r3r_tail.sh && bash /tmp/r3r_tail.sh
