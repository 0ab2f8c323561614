"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of `bench.py` (C2,
default size) into profiles/pmc_traffic.json, which bench.py reports as
roofline.traffic.  Per MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half the
bytes of 16 B/lane streaming reads on gfx950 (double it), WRITE_SIZE is exact
for 16 B/lane stores; both are in KiB.

usage: python scripts/pmc_traffic.py FETCH_CSV WRITE_CSV NBLOCKS OUT_JSON"""
import csv
import json
import statistics
import sys

KERNEL = "k_dec256v32w"


def per_launch(path, counter):
    def none_mode(name):  # StartMode::None, mangled or demangled
        return KERNEL in name and ("StartModeE0E" in name or "StartMode)0," in name)

    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if none_mode(r["Kernel_Name"]) and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows for {KERNEL}<None> in {path}")
    return statistics.median(vals), len(vals)


def main():
    fetch_csv, write_csv, nblocks, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    f_kib, nf = per_launch(fetch_csv, "FETCH_SIZE")
    w_kib, nw = per_launch(write_csv, "WRITE_SIZE")
    hbm = (2.0 * f_kib + w_kib) * 1024.0
    d = {"workload": "c2", "nblocks": nblocks, "kernel": "tpf::dev::k_dec256v32w<StartMode::None>",
         "FETCH_SIZE_KiB_median": f_kib, "WRITE_SIZE_KiB_median": w_kib, "launches": [nf, nw],
         "hbm_bytes_per_launch": int(hbm),
         "correction": "hbm = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950 FETCH_SIZE halves 16B/lane reads)"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
