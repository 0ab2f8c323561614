# round 6 final evidence, part 1: PMC traffic (FETCH_SIZE / WRITE_SIZE passes) of every workload on the final kernel sources
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
LABEL=${LABEL:-r6final} TAG=${TAG:-r6final} bash scripts/gpu.sh ${WLS:-pmc:c2 pmc:c1 pmc:c3 pmc:c3chain pmc:c3chain64 pmc:c3enc pmc:c4 pmc:c5}
