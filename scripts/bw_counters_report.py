"""Per-block counter table from scripts/bw_counters.py runs under rocprofv3
--pmc: the decode launches (k_dec256v32w<None>) of each run, in dispatch
order, grouped REPS per bit width; each counter as a per-block median.
usage: python scripts/bw_counters_report.py NBLOCKS ORDER_LINE csv [csv ...]"""
import collections
import csv
import statistics
import sys

REPS = 3
nb = int(sys.argv[1])
order = [(int(x.split(":")[0]), float(x.split(":")[1])) for x in sys.argv[2].split(";")]
table = collections.defaultdict(dict)
for path in sys.argv[3:]:
    rows = [r for r in csv.DictReader(open(path))
            if "k_dec256v32w" in r["Kernel_Name"] and ("StartModeE0E" in r["Kernel_Name"] or "StartMode)0," in r["Kernel_Name"])]
    by_counter = collections.defaultdict(list)
    for r in rows:
        by_counter[r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    for cname, vals in by_counter.items():
        vals.sort()
        # one value per dispatch (sum over the per-agent/XCD rows of that dispatch)
        per = collections.OrderedDict()
        for d, v in vals:
            per[d] = per.get(d, 0.0) + v
        seq = list(per.values())
        if len(seq) != REPS * len(order):
            raise SystemExit(f"{path}: {cname}: {len(seq)} decode dispatches, expected {REPS * len(order)}")
        for i, (bw, _) in enumerate(order):
            table[bw][cname] = statistics.median(seq[REPS * i: REPS * (i + 1)]) / nb
names = sorted({c for v in table.values() for c in v})
print("bw  B/blk  " + "  ".join(f"{c[:22]:>22s}" for c in names))
for bw, bpb in order:
    print(f"{bw:2d} {bpb:6.1f}  " + "  ".join(f"{table[bw].get(c, float('nan')):22.2f}" for c in names))
