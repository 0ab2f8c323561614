# SQ counters of the 256v32 encoders (scripts/enc_kernel_times.py under
# rocprofv3 --pmc, two passes within the per-block limits), per block, for
# each path in MODES (3 = two-pass, 4 = slot, 5 = slot without the fused
# scans) on DATA (c4 mix, c3 D1 list, or v64: the 256v64 encoder on C4's
# 64-bit leg).  -> gpurun_out/${TAG}_enc_counters.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
T=${TAG:-encc}
NB=${NB:-2000000}
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-3 4}; do
  i=0
  for c in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" "SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    if [ "${DATA:-c4}" = v64 ]; then prog="$R/scripts/enc64_kernel_times.py $NB 3"; else prog="$R/scripts/enc_kernel_times.py $NB 3 $m ${DATA:-c4}"; fi
    timeout -k 10 120 rocprofv3 --pmc $c -d $R/gpurun_out/${T}_m${m}_p$i -o run --output-format csv -- python3 $prog > $R/gpurun_out/${T}_m${m}_p$i.log 2>&1 || { echo "mode $m pass $i rc=$?"; tail -5 $R/gpurun_out/${T}_m${m}_p$i.log; exit 1; }
  done
done
python3 - $R/gpurun_out $T $NB ${MODES:-3 4} > $R/gpurun_out/${T}_enc_counters.txt <<'PY'
import csv, sys, collections, glob
d, T, nb, modes = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4:]
print(f"# 256v32 encoder SQ counters per block ({nb} blocks per launch; per-launch medians)")
for m in modes:
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{d}/{T}_m{m}_p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name']
            if 'k_enc' not in k:
                continue
            k = k.split('(')[0].replace('void tpf::dev::', '')[:40]
            agg[(k, r['Counter_Name'])].append(float(r['Counter_Value']))
    kern = sorted({k for k, _ in agg})
    for k in kern:
        vals = {c: sorted(v)[len(v) // 2] for (kk, c), v in agg.items() if kk == k}
        per = {c: v / nb for c, v in vals.items()}
        print(f"mode {m} {k}: " + " ".join(f"{c.replace('SQ_', '')}={per[c]:.1f}" for c in sorted(per)))
PY
cat $R/gpurun_out/${T}_enc_counters.txt
