# round 6: C1 output-shape ceilings incl. 16-byte aligned chunks (scripts/c1_store_probe.hip, built on the box)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o gpurun_out/c1_store_probe scripts/c1_store_probe.hip > /dev/null 2>&1 || { echo "probe build failed"; exit 1; }
timeout -k 10 120 gpurun_out/c1_store_probe > gpurun_out/r6n_c1_store_probe.txt 2>&1 || { echo "probe rc=$?"; tail -5 gpurun_out/r6n_c1_store_probe.txt; exit 1; }
cat gpurun_out/r6n_c1_store_probe.txt
