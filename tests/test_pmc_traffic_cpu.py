"""scripts/pmc_traffic.py (roofline.traffic source): per-launch medians of
FETCH_SIZE / WRITE_SIZE, FETCH doubled per the gfx950 correction, summed over
every kernel of a multi-kernel step (c3chain, c4), merged into one JSON file
per workload.  Synthetic rocprofv3 CSVs; no GPU."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "scripts", "pmc_traffic.py")


def _csv(path, counter, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for name, val in rows:
            w.writerow({"Kernel_Name": name, "Counter_Name": counter, "Counter_Value": val})


def _run(tmp_path, wl, fetch_rows, write_rows, out):
    f, w = tmp_path / f"{wl}_f.csv", tmp_path / f"{wl}_w.csv"
    _csv(f, "FETCH_SIZE", fetch_rows)
    _csv(w, "WRITE_SIZE", write_rows)
    subprocess.run([sys.executable, SCRIPT, wl, str(f), str(w), "1000", str(out)], check=True,
                   capture_output=True)
    return json.load(open(out))[wl]


DEC0 = "void tpf::dev::k_dec256v32w<(tpf::dev::StartMode)0, 16u, 2u, 6u, 7, true>(tpf::dev::DecArgs)"
PLAN = "void tpf::dev::k_enc256v32_plan<false, 0>(unsigned int const*, unsigned long)"
WRITE = "void tpf::dev::k_enc256v32_write<false, 0>(unsigned int const*, unsigned long)"
PLAN_D1 = "void tpf::dev::k_enc256v32_plan<true, 0>(unsigned int const*, unsigned long)"


def test_single_kernel_median_and_correction(tmp_path):
    out = tmp_path / "t.json"
    d = _run(tmp_path, "c2", [(DEC0, 10), (DEC0, 30), (DEC0, 20), ("other_kernel", 999)],
             [(DEC0, 5), (DEC0, 5), (DEC0, 7)], out)
    assert d["FETCH_SIZE_KiB_median"] == 20 and d["WRITE_SIZE_KiB_median"] == 5
    assert d["hbm_bytes_per_launch"] == (2 * 20 + 5) * 1024


def test_step_sums_its_kernels_and_merges(tmp_path):
    out = tmp_path / "t.json"
    _run(tmp_path, "c2", [(DEC0, 1)], [(DEC0, 1)], out)
    d = _run(tmp_path, "c4",
             [(PLAN, 100), (PLAN, 100), (WRITE, 200), (DEC0, 50), (PLAN_D1, 7777)],
             [(PLAN, 1), (WRITE, 60), (DEC0, 100), (PLAN_D1, 7777)], out)
    # the D1 plan kernel is not part of the C4 step
    assert d["FETCH_SIZE_KiB_median"] == 350 and d["WRITE_SIZE_KiB_median"] == 161
    assert d["hbm_bytes_per_launch"] == (2 * 350 + 161) * 1024
    both = json.load(open(out))
    assert set(both) == {"c2", "c4"}


def test_round3_kernels(tmp_path):
    """c3chain = lane-per-block phase A + prefix decode; c1 = the windowed p4Dec32 decoder;
    c4_64 = the 64-bit leg's three kernels (NB = 2, non-D1)."""
    out = tmp_path / "t.json"
    dsum = "void tpf::dev::k_dsum256v32_lanes<16384u>(tpf::dev::DecArgs)"
    dec2 = "void tpf::dev::k_dec256v32w<(tpf::dev::StartMode)2, 16u, 10u, 6u, 7, true>(tpf::dev::DecArgs)"
    d = _run(tmp_path, "c3chain", [(dsum, 10), (dec2, 20)], [(dsum, 0), (dec2, 30)], out)
    assert d["FETCH_SIZE_KiB_median"] == 30 and d["WRITE_SIZE_KiB_median"] == 30
    win = "void tpf::dev::k_dec_h32w<false, 2u>(unsigned char const*, unsigned long)"
    gen = "void tpf::dev::k_dec_gr<(tpf::dev::Fmt)0, false>(unsigned char const*, unsigned long)"
    d = _run(tmp_path, "c1", [(win, 4), (gen, 50)], [(win, 9), (gen, 50)], out)
    assert d["hbm_bytes_per_launch"] == (2 * 4 + 9) * 1024
    p64 = "void tpf::dev::k_enc128v64_plan<2u, false>(unsigned long const*, unsigned long)"
    w64 = "void tpf::dev::k_enc128v64_write<2u, false>(unsigned long const*, unsigned long)"
    d64 = "void tpf::dev::k_dec128v64w<2u, (tpf::dev::Start64)0>(tpf::dev::Dec64Args)"
    d = _run(tmp_path, "c4_64", [(p64, 1), (w64, 2), (d64, 3), (PLAN, 100)], [(p64, 0), (w64, 5), (d64, 6), (PLAN, 100)], out)
    assert d["FETCH_SIZE_KiB_median"] == 6 and d["WRITE_SIZE_KiB_median"] == 11


def test_round4_kernels(tmp_path):
    """c3enc = the D1 encoder's two passes; c3chain64 = the 64-bit chained
    decode's lane-per-unit phase A and its Prefix launch (mangled names, as
    rocprofv3 may print; the decoder's Sum and PerUnit modes are not counted)."""
    out = tmp_path / "t.json"
    pl1 = "_ZN3tpf3dev16k_enc256v32_planILb1ELi0EEEvPKjm"
    wr1 = "_ZN3tpf3dev17k_enc256v32_writeILb1ELi0EEEvPKjm"
    pl0 = "_ZN3tpf3dev16k_enc256v32_planILb0ELi0EEEvPKjm"
    d = _run(tmp_path, "c3enc", [(pl1, 3), (wr1, 4), (pl0, 99)], [(pl1, 0), (wr1, 7), (pl0, 99)], out)
    assert d["FETCH_SIZE_KiB_median"] == 7 and d["WRITE_SIZE_KiB_median"] == 7
    la = "_ZN3tpf3dev18k_dsum128v64_lanesILj2ELj16384EEEvNS0_9Dec64ArgsE"
    s3 = "_ZN3tpf3dev12k_dec128v64wILj2ELNS0_7Start64E3EEEvNS0_9Dec64ArgsE"
    s2 = "_ZN3tpf3dev12k_dec128v64wILj2ELNS0_7Start64E2EEEvNS0_9Dec64ArgsE"
    s1 = "_ZN3tpf3dev12k_dec128v64wILj2ELNS0_7Start64E1EEEvNS0_9Dec64ArgsE"
    d = _run(tmp_path, "c3chain64", [(la, 10), (s2, 20), (s3, 77), (s1, 500)], [(la, 0), (s2, 40), (s3, 77), (s1, 500)], out)
    assert d["FETCH_SIZE_KiB_median"] == 30 and d["WRITE_SIZE_KiB_median"] == 40


def test_committed_traffic_matches_these_kernels():
    """profiles/pmc_traffic.json (the roofline.traffic bench.py replays) holds
    every workload, and each entry names the kernel sources it was measured
    with (turbopfor_amd.kernel_md5: csrc/*.hip, csrc/*.h, the Makefile).  An
    entry of other kernels is STALE: bench.py then reports traffic null, and
    this test says so (skip, not fail: a kernel edit must not break the
    CPU-only suite until the next PMC pass on a GPU box)."""
    import pytest

    sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
    import turbopfor_amd
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    assert {"c1", "c2", "c3", "c3chain", "c4", "c4_64"} <= set(d)
    for wl, v in d.items():
        assert v["hbm_bytes_per_launch"] > 0, wl
    cur = turbopfor_amd.kernel_md5()
    stale = sorted(wl for wl, v in d.items() if v.get("kernel_md5") != cur)
    if stale:
        pytest.skip(f"PMC traffic of {stale} measured with other kernel sources: bench.py reports it as null until re-measured")
