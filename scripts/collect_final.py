"""Collect a final-evidence call's bench lines and rocprofv3 kernel stats
from gpurun_out/ into profiles/ (tag r6final): <tag>_bench_<wl>.json,
<tag>_<wl>_under_rocprof.json and one <tag>_kernel_stats.txt with a section
per workload (every kernel: calls, average and total time).
usage: python scripts/collect_final.py TAG WL [WL ...]"""
import csv
import glob
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
O, P = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles")
tag, wls = sys.argv[1], sys.argv[2:]
stats = os.path.join(P, f"{tag}_kernel_stats.txt")
have = open(stats).read() if os.path.exists(stats) else (
    f"# {tag}: rocprofv3 --kernel-trace --stats of python bench.py --workload WL --steps 20 --warmup 5 --no-cpu-baseline\n"
    "# (scripts/gpu.sh prof:WL), one section per workload: kernel, calls, average ms, total ms.\n")
for wl in wls:
    for src, dst in ((f"{tag}_bench_{wl}.json", f"{tag}_bench_{wl}.json"), (f"{tag}_{wl}_under_rocprof.json", f"{tag}_{wl}_under_rocprof.json")):
        if os.path.exists(os.path.join(O, src)):
            shutil.copy(os.path.join(O, src), os.path.join(P, dst))
    rows = []
    for f in glob.glob(os.path.join(O, f"{tag}_{wl}_prof", "**", "*kernel_stats.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    if not rows or f"## {wl}\n" in have:
        continue
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    have += f"\n## {wl}\n"
    for r in rows:
        have += f"{r['Name'][:110]:110s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e6:9.4f} ms {float(r['TotalDurationNs']) / 1e6:10.3f} ms\n"
open(stats, "w").write(have)
print(stats)
