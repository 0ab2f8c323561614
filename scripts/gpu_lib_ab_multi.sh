# Library A/B (abtmp/base.so = HEAD vs the working tree) over several
# workloads on one box: WLS="c3chain c2 c1 c3" ROUNDS=2 bash scripts/gpu_lib_ab_multi.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
for w in ${WLS:-c3chain c2}; do
  echo "== $w"
  WL=$w bash scripts/gpu_lib_ab.sh || exit 1
done
