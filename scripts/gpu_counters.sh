# PMC counter passes for the decode kernel (one counter group per pass; no
# tracing domains combined with --pmc).  Usage: COUNTERS="A B" bash scripts/gpu_counters.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for c in ${COUNTERS:-FETCH_SIZE WRITE_SIZE}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_$i -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --nblocks ${NB:-2000000} > $R/gpurun_out/pmc_$i.log 2>&1 || { echo "pmc $c rc=$?"; tail -5 $R/gpurun_out/pmc_$i.log; exit 1; }
  python3 - "$R/gpurun_out/pmc_$i/run_counter_collection.csv" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'k_dec256v32' in r['Kernel_Name']]
agg = collections.defaultdict(list)
for r in rows: agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in agg.items(): print(f"{k:28s} median {sorted(v)[len(v)//2]:.4g}  (n={len(v)})")
PY
done
