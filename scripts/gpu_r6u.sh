# round 6: per-block drop-in tests after the seq_cst mailbox wait; the end-to-end (pinned host) rates of the last library
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dropin.py tests/test_gpu_host_pageable.py > gpurun_out/r6u_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r6u_tests.log; exit 1; }
tail -2 gpurun_out/r6u_tests.log
timeout -k 10 400 python -u bench.py --workload c2 --e2e > gpurun_out/r6u_bench_c2_e2e.json 2> gpurun_out/r6u_bench_c2_e2e.err || { echo "bench rc=$?"; tail -20 gpurun_out/r6u_bench_c2_e2e.err; exit 1; }
tail -1 gpurun_out/r6u_bench_c2_e2e.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['config'].get('e2e_host_pinned')))"
