set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread --deselect tests/test_gpu_edges.py::test_host_dec_rejects_bad_offsets_and_reports_corrupt_block > gpurun_out/iso1.log 2>&1 || { echo "iso1 rc=$?"; tail -30 gpurun_out/iso1.log; exit 1; }
tail -1 gpurun_out/iso1.log
AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_edges.py::test_host_dec_rejects_bad_offsets_and_reports_corrupt_block tests/test_gpu_enc256v32.py::test_full_size_c2_sample_vs_oracle > gpurun_out/iso2.log 2>&1 || { echo "iso2 rc=$?"; tail -40 gpurun_out/iso2.log; exit 1; }
tail -1 gpurun_out/iso2.log
