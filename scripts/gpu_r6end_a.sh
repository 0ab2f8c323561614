# round 6 end library (64-bit bitmap loop), call A: GPU suite + smoke on the final library, per-block latency tails, PMC traffic of every workload
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TAG=r6end bash scripts/gpu_r6l.sh || exit 1
PY_TIMEOUT=200 PY_TAIL=12 TAG=r6end bash scripts/gpu.sh py:scripts/perblock_latency.py:20000 || exit 1
LABEL=r6end TAG=r6end bash scripts/gpu.sh pmc:c2 pmc:c1 pmc:c3 pmc:c3chain pmc:c3chain64 pmc:c3enc pmc:c4 pmc:c5
