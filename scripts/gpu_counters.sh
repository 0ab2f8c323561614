# PMC counter passes for the bench kernels (one counter group per pass; no
# tracing domains combined with --pmc).  Prints the per-launch median of each
# counter for every kernel whose name matches KFILTER (default k_dec256v32).
# Usage: COUNTERS="A,B,C D" BENCH_ARGS="--workload c3chain" bash scripts/gpu_counters.sh
#   (space separates passes, comma separates counters inside one pass)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for c in ${COUNTERS:-FETCH_SIZE WRITE_SIZE}; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc ${c//,/ } -d $R/gpurun_out/pmc_${TAGC:-x}_$i -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --nblocks ${NB:-2000000} ${BENCH_ARGS} > $R/gpurun_out/pmc_${TAGC:-x}_$i.log 2>&1 || { echo "pmc $c rc=$?"; tail -5 $R/gpurun_out/pmc_${TAGC:-x}_$i.log; exit 1; }
  python3 - "$R/gpurun_out/pmc_${TAGC:-x}_$i/run_counter_collection.csv" "${KFILTER:-k_dec256v32}" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r['Kernel_Name']]
agg = collections.defaultdict(list)
for r in rows:
    k = r['Kernel_Name'].split('(')[0][-60:] + ' ' + r['Kernel_Name'].split('<')[1][:40] if '<' in r['Kernel_Name'] else r['Kernel_Name'][:60]
    agg[(k, r['Counter_Name'])].append(float(r['Counter_Value']))
for (k, c), v in sorted(agg.items()):
    print(f"{k:50s} {c:24s} median {sorted(v)[len(v)//2]:.5g}  (n={len(v)})")
PY
done
