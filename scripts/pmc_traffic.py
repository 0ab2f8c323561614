"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of `bench.py --workload W`
(default size) into profiles/pmc_traffic.json (one entry per workload), which
bench.py reports as roofline.traffic.  Per MI355X_MICROARCH.md §HBM:
FETCH_SIZE counts half the bytes of 16 B/lane streaming reads on gfx950
(double it), WRITE_SIZE is exact for 16 B/lane stores; both are in KiB.

Each entry records the md5 of the library sources the counters were taken
with (kernel_md5, turbopfor_amd.kernel_md5: the device sources) and a label: bench.py replays the
number only while it runs code built from those same sources, and says so
(roofline.traffic_source).

usage: python scripts/pmc_traffic.py WORKLOAD FETCH_CSV WRITE_CSV NBLOCKS OUT_JSON [LABEL]"""
import csv
import json
import os
import statistics
import sys

def _dec(mode):
    return lambda n: "k_dec256v32w" in n and (f"StartModeE{mode}E" in n or f"StartMode){mode}," in n)


def _dec64(nb, mode):
    """k_dec128v64w<nb, Start64 mode> (mangled or demangled)."""
    return lambda n: "k_dec128v64w" in n and (f"ILj{nb}ELNS0_7Start64E{mode}E" in n or f"<{nb}u, (tpf::dev::Start64){mode}>" in n)


def _enc32(kind, d1):
    return lambda n: f"k_enc256v32_{kind}" in n and (f"ILb{int(d1)}E" in n or f"<{'true' if d1 else 'false'}" in n)


# workload -> (kernel name tests, description): one test per kernel of the
# step; a step's traffic is the sum of each kernel's per-launch median.
# Names appear demangled or mangled.
KERNELS = {
    "c2": ([_dec(0)], "tpf::dev::k_dec256v32w<StartMode::None>"),
    "c5": ([_dec(0)], "tpf::dev::k_dec256v32w<StartMode::None> (C5 shard: bw 8 / bw 16)"),
    "c3": ([_dec(1)], "tpf::dev::k_dec256v32w<StartMode::PerBlock>"),
    "c1": ([lambda n: "k_dec_h32w" in n], "tpf::dev::k_dec_h32w (windowed p4Dec32 batch)"),
    # chained list: phase A (block sums) + phase B (prefix decode); the run
    # scan between them (p4_scan.hip: 156K u32 run sums, ~1 MB) is not counted
    "c3chain": ([lambda n: "k_dsum256v32_lanes" in n, _dec(2)], "k_dsum256v32_lanes (phase A) + k_dec256v32w<Prefix>"),
    # round trip: encoder plan + write passes (non-D1) + decode; the run
    # scan between the passes (625K run totals, ~7.5 MB) is not counted
    "c4": ([_enc32("plan", False), _enc32("write", False), _dec(0)],
           "k_enc256v32_plan<false> + k_enc256v32_write<false> + k_dec256v32w<StartMode::None>"),
    # C4's 64-bit leg (same rocprof runs as c4): 256v64 encode passes + decode
    "c4_64": ([lambda n: "k_enc128v64_plan" in n and ("ILj2ELb0E" in n or "<2u, false" in n),
               lambda n: "k_enc128v64_write" in n and ("ILj2ELb0E" in n or "<2u, false" in n),
               _dec64(2, 0)],
              "k_enc128v64_plan<2,false> + k_enc128v64_write<2,false> + k_dec128v64w<2,None>"),
    # D1 encode of the C3 posting list: plan + write passes (run scan not counted)
    "c3enc": ([_enc32("plan", True), _enc32("write", True)], "k_enc256v32_plan<true> + k_enc256v32_write<true>"),
    # 64-bit chained list: phase A (unit sums) + phase B (prefix decode)
    "c3chain64": ([lambda n: "k_dsum128v64_lanes" in n, _dec64(2, 2)], "k_dsum128v64_lanes (phase A) + k_dec128v64w<2,Prefix>"),
}


def per_launch(path, counter, test):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if test(r["Kernel_Name"]) and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows for the kernel in {path}")
    return statistics.median(vals), len(vals)


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
import turbopfor_amd  # noqa: E402  (kernel_md5 only: no GPU, no torch import)


def main():
    wl, fetch_csv, write_csv, nblocks, out = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5]
    label = sys.argv[6] if len(sys.argv) > 6 else None
    tests, kname = KERNELS[wl]
    f_kib = w_kib = 0.0
    nf, nw = [], []
    for test in tests:
        f, a = per_launch(fetch_csv, "FETCH_SIZE", test)
        w, b = per_launch(write_csv, "WRITE_SIZE", test)
        f_kib, w_kib = f_kib + f, w_kib + w
        nf.append(a)
        nw.append(b)
    hbm = (2.0 * f_kib + w_kib) * 1024.0
    d = {"workload": wl, "nblocks": nblocks, "kernel": kname,
         "FETCH_SIZE_KiB_median": f_kib, "WRITE_SIZE_KiB_median": w_kib, "launches": [nf, nw],
         "hbm_bytes_per_launch": int(hbm), "label": label, "kernel_md5": turbopfor_amd.kernel_md5(), "src_md5": turbopfor_amd.source_md5(),
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
