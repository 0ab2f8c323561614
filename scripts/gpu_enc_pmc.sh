# PMC passes over the 256v32 encoders (scripts/enc_kernel_times.py, C4 mix,
# 10M blocks, 3 launches): FETCH_SIZE and WRITE_SIZE per kernel for the
# two-pass encoder (probe mode 3) and one pipelined variant.  -> gpurun_out/encpmc_*
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
PIPE=$((16 + 512 + 1024 * 2 + (8 << 20)))
i=0
for spec in "3:FETCH_SIZE" "3:WRITE_SIZE" "$PIPE:FETCH_SIZE" "$PIPE:WRITE_SIZE"; do
  i=$((i+1)); mode=${spec%%:*}; ctr=${spec#*:}
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $R/gpurun_out/encpmc_$i -o run --output-format csv -- python3 $R/scripts/enc_kernel_times.py 10000000 3 $mode > $R/gpurun_out/encpmc_$i.log 2>&1 || { echo "pass $i ($spec) rc=$?"; tail -5 $R/gpurun_out/encpmc_$i.log; exit 1; }
  python3 - "$R/gpurun_out/encpmc_$i" "$spec" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    k = "plan" if "k_enc256v32_plan" in n else "write" if "k_enc256v32_write" in n else "pipe" if "k_enc256v32_pipe" in n else None
    if k: agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    v = sorted(v)
    print(f"{sys.argv[2].split(':')[0]:>10s} {k:6s} {c:22s} median/launch {v[len(v)//2]:.6g}  per block {v[len(v)//2]/1e7:.4g}  (n={len(v)})")
PY
done
