"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of `bench.py --workload W`
(default size) into profiles/pmc_traffic.json (one entry per workload), which
bench.py reports as roofline.traffic.  Per MI355X_MICROARCH.md §HBM:
FETCH_SIZE counts half the bytes of 16 B/lane streaming reads on gfx950
(double it), WRITE_SIZE is exact for 16 B/lane stores; both are in KiB.

usage: python scripts/pmc_traffic.py WORKLOAD FETCH_CSV WRITE_CSV NBLOCKS OUT_JSON"""
import csv
import json
import os
import statistics
import sys

# workload -> (kernel name test, description); names appear demangled or mangled
KERNELS = {
    "c2": (lambda n: "k_dec256v32w" in n and ("StartModeE0E" in n or "StartMode)0," in n),
           "tpf::dev::k_dec256v32w<StartMode::None>"),
    "c3": (lambda n: "k_dec256v32w" in n and ("StartModeE1E" in n or "StartMode)1," in n),
           "tpf::dev::k_dec256v32w<StartMode::PerBlock>"),
    "c1": (lambda n: "k_dec_gr" in n and ("FmtE0E" in n or "Fmt)0," in n),
           "tpf::dev::k_dec_gr<Fmt::H32>"),
}


def per_launch(path, counter, test):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if test(r["Kernel_Name"]) and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows for the kernel in {path}")
    return statistics.median(vals), len(vals)


def main():
    wl, fetch_csv, write_csv, nblocks, out = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5]
    test, kname = KERNELS[wl]
    f_kib, nf = per_launch(fetch_csv, "FETCH_SIZE", test)
    w_kib, nw = per_launch(write_csv, "WRITE_SIZE", test)
    hbm = (2.0 * f_kib + w_kib) * 1024.0
    d = {"workload": wl, "nblocks": nblocks, "kernel": kname,
         "FETCH_SIZE_KiB_median": f_kib, "WRITE_SIZE_KiB_median": w_kib, "launches": [nf, nw],
         "hbm_bytes_per_launch": int(hbm),
         "correction": "hbm = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950 FETCH_SIZE halves 16B/lane reads)"}
    allv = {}
    if os.path.exists(out):
        try:
            allv = json.load(open(out))
        except Exception:
            allv = {}
        if "workload" in allv:  # single-entry layout of earlier versions
            allv = {allv["workload"]: allv}
    allv[wl] = d
    json.dump(allv, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
