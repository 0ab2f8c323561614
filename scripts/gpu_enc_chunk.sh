# Encoder pass times vs chunk size (scripts/enc_chunk_probe.py) under
# rocprofv3 --kernel-trace --stats; prints each kernel's total time per
# 10M-block pass.  -> gpurun_out/encchunk_*
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-full chunk65536 chunk131072 chunk262144}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/encchunk_$m -o run --output-format csv -- python3 $R/scripts/enc_chunk_probe.py $m 3 > $R/gpurun_out/encchunk_$m.log 2>&1 || { echo "$m rc=$?"; tail -5 $R/gpurun_out/encchunk_$m.log; exit 1; }
  grep "one 10M" $R/gpurun_out/encchunk_$m.log
  python3 - "$R/gpurun_out/encchunk_$m" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = collections.defaultdict(float); cnt = collections.Counter()
for r in rows:
    n = r["Kernel_Name"]
    k = "plan" if "k_enc256v32_plan" in n else "write" if "k_enc256v32_write" in n else "scan" if "rocprim" in n or "hipcub" in n else None
    if k is None: continue
    tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6; cnt[k] += 1
# 4 passes of 10M blocks were run (3 warm + 1 timed)
for k in ("plan", "scan", "write"):
    print(f"  {k:6s} launches={cnt[k]:6d}  ms per 10M-block pass={tot[k]/4:.3f}")
PY
done
