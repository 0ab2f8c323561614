#!/usr/bin/env python3
"""bench.py -- device-resident p4Dec256v32 throughput on MI355X.

Default workload (BASELINE.json configs[1], "C2"): 10M blocks of 256 uint32
per GPU, bit widths 1..32 swept as 32 equal consecutive segments, 10%
exceptions (bw <= 28; benchmarks/ab_test.cpp:1448, :1610-1631), synthetic data
generated on the GPU.  The packed stream is produced by our GPU encoder
(untimed; parity-tested against the reference-pinned oracle) and the timed
decode is verified bit-exact at full size afterwards.  One step = one
tpf_p4dec256v32_batch launch over the whole shard, inputs resident in HBM.

Other workloads (--workload, one JSON line each, for DESIGN.md):
  c1      BASELINE configs[0]: p4Enc32/p4Dec32, n = 127, bw 8, 0% exceptions --
          the reference's own CPU case (ab_test single-block loop, cpu_baseline)
          beside a device batch of 10M such blocks (horizontal format kernels)
  c3      p4D1Dec256v32 on Zipf posting lists (5% big gaps), per-block starts
  c3chain the same list decoded as ONE chained list (only start0 given)
  c4      p4Enc256v32 + p4Dec256v32 round trip (0/5/10/25% exceptions) and
          the 256v64 round trip (bw 1..64 with exceptions above bit 32)
  sweep   SURVEY §8(d): 10M blocks for EACH bit width 1..32, decode vs probe
--e2e adds the host-memory rates (pinned H2D + decode + D2H, tpf_host_dec; and
      the encode trip, tpf_host_enc).

Multi-GPU: `python bench.py --gpus N` (N > 1, WORLD_SIZE unset) starts
`torch.distributed.run` with N ranks as a child process before anything
touches a GPU and exits with its status; under a launcher (WORLD_SIZE set)
every rank owns its own shard (weak scaling); the decode needs no
collective.  RCCL carries the barrier, the max-over-ranks time, the per-rank
kernel times and, for c3chain, the one real exchange step (each shard's delta
total, tpf_shard.chained_base).  --selftest runs the same launcher, process
group and timing plumbing with a CPU stand-in step (gloo; no GPU, no codec)
for the CPU tests.

Rank 0 prints ONE JSON line with `roofline` (decode kernel, HIP events on
the launch stream) and `cpu_baseline` (the reference library compiled from
its own sources, run on this host's cores on a bounded sample).
"""
import argparse
import ctypes
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
import tpf_shard  # noqa: E402
import turbopfor_amd as tpf  # noqa: E402

sys.path.insert(0, ROOT)
import bench_data  # noqa: E402

METRIC = "G int32/s device-resident p4Dec256v32 (+ compressed GB/s vs HBM peak)"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
PROFILE_TRAFFIC = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ------------------------------------------------------------ data (GPU)
# Counter-based generators keyed by the global element index (bench_data.py):
# every rank holds a slice of ONE global stream.  The thin wrappers keep the
# signatures the measurement scripts use.
as_i32 = bench_data.as_i32


def gen_c2(nblocks, exc_pct, seed, dev, pcts=None, first_block=0):
    return bench_data.gen_c2(nblocks, exc_pct, seed, dev, pcts=pcts, first_block=first_block)


def gen_bw(nblocks, bw, exc_pct, seed, dev, first_block=0):
    return bench_data.gen_bw(nblocks, bw, exc_pct, seed, dev, first_block=first_block)


def gen_c3(nblocks, seed, dev, first_block=0, carry_fn=None):
    return bench_data.gen_c3(nblocks, seed, dev, first_block=first_block, carry_fn=carry_fn)


def shard_of(nb, world, rank):
    """Global block range of this rank: one nb-block shard of the world*nb
    global stream (tpf_shard.shard_range, weak scaling)."""
    lo, hi = tpf_shard.shard_range(nb * world, world, rank)
    assert hi - lo == nb
    return lo


_POPCNT = None


def block_mix(packed, offs, chunk=1 << 20):
    """Header-derived block statistics of a 256v32 stream (SURVEY.md §8 d:
    "report the header-derived exception fraction on every run"): fraction
    of vbyte-mode blocks, of bitmap-mode blocks, and exceptions per value
    (vbyte: the xn byte; bitmap: popcount of the 32-byte bitmap)."""
    global _POPCNT
    dev = packed.device
    if _POPCNT is None or _POPCNT.device != dev:
        _POPCNT = torch.tensor([bin(i).count("1") for i in range(256)], dtype=torch.int64, device=dev)
    nb = offs.numel() - 1
    n_vb = n_bm = exc = 0
    ar = torch.arange(32, device=dev)
    for a in range(0, nb, chunk):
        o = offs[a:min(nb, a + chunk)]
        h = packed[o].to(torch.int64)
        x1 = packed[torch.clamp(o + 1, max=packed.numel() - 1)].to(torch.int64)
        vb = (h & 0xC0) == 0x40
        bm = ((h & 0xC0) != 0xC0) & ((h & 0x40) == 0) & ((h & 0x80) != 0)
        n_vb += int(vb.sum().item())
        n_bm += int(bm.sum().item())
        exc += int(torch.where(vb, x1, 0).sum().item())
        ob = o[bm]
        if ob.numel():
            idx = torch.clamp(ob.view(-1, 1) + 2 + ar, max=packed.numel() - 1)
            exc += int(_POPCNT[packed[idx].to(torch.int64)].sum().item())
    return {"vbyte_block_frac": round(n_vb / max(nb, 1), 4), "bitmap_block_frac": round(n_bm / max(nb, 1), 4),
            "exception_frac": round(exc / max(nb * 256, 1), 5)}


def checksum(t, dev, dist_on):
    """Sum of the uint32 values (mod 2^64) over all ranks: the decode's
    checksum of checksums (SURVEY.md §8 e bookkeeping)."""
    c = (t.view(-1).to(torch.int64) & 0xFFFFFFFF).sum().reshape(1)
    if dist_on:
        torch.distributed.all_reduce(c)
    return int(c.item()) & ((1 << 64) - 1)


# --------------------------------------------------------- profile traffic
def src_md5():
    try:
        return tpf.kernel_md5()
    except OSError:
        return None


def pmc_traffic(workload, nblocks):
    """(HBM bytes per step, source) from rocprofv3 PMC counters of exactly this
    workload (profiles/pmc_traffic.json, written by scripts/pmc_traffic.py:
    FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM plus WRITE_SIZE, KiB ->
    bytes).  PMC counters need a rocprofv3 pass of their own, so the number is
    never measured inside this run: it is replayed only when the entry was
    taken with the kernels this process runs (md5 over the device sources,
    turbopfor_amd.kernel_md5), and the source says which measurement it is.  (None, reason) otherwise."""
    src = {"file": os.path.relpath(PROFILE_TRAFFIC, ROOT), "measured_in_this_run": False}
    try:
        d = json.load(open(PROFILE_TRAFFIC)).get(workload, {})
    except Exception:
        d = {}
    if d.get("workload") != workload or int(d.get("nblocks", -1)) != nblocks:
        src["note"] = "no PMC measurement of this workload and size"
        return None, src
    src.update({"label": d.get("label"), "kernel_md5": d.get("kernel_md5")})
    if d.get("kernel_md5") is None or d.get("kernel_md5") != src_md5():
        src["note"] = "PMC measurement taken with other kernel sources: not replayed"
        return None, src
    src["note"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this workload with code built from these kernel sources "
                   "(scripts/gpu.sh pmc:WL)")
    return d.get("hbm_bytes_per_launch"), src


def traffic_fields(workload, nblocks):
    t, src = pmc_traffic(workload, nblocks)
    return {"traffic": t, "traffic_source": src}


def hbm_probes(dev, nbytes=4 << 30):
    """The box's own streaming ceilings, measured in this run with the
    library's probe kernels (tpfm_probe_hbm: 16-B non-temporal read / write /
    copy, grid-stride): bytes moved (read + written) per second."""
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    a.fill_(1)
    res = {}
    for kind, moved in (("read", nbytes), ("write", nbytes), ("copy", nbytes)):
        n = nbytes if kind != "copy" else nbytes // 2
        src, dst = (a, b)
        for _ in range(2):
            tpf.probe_hbm(kind, dst, src, n)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            tpf.probe_hbm(kind, dst, src, n)
        e1.record()
        torch.cuda.synchronize()
        res[kind + "_GBps"] = round(moved * 5 / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
    del a, b
    res["def"] = ("tpfm_probe_hbm over 4 GiB: read-only / write-only / copy (copy counts read + written bytes), "
                  "16-B lanes, non-temporal, 128 WG/CU")
    return res


# ------------------------------------------------------------- cpu baseline
def _cgroup_cpus():
    """CPUs granted by the cgroup (cpu.max quota / period), or None."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                return float(q) / float(per)
        except Exception:
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return q / per
    except Exception:
        pass
    return None


def cpu_host():
    """Threads for the CPU baselines: every CPU this process may run on
    (sched_getaffinity), capped by the cgroup CPU quota when one is set (more
    threads than the quota only queue), and the facts behind the choice."""
    aff = len(os.sched_getaffinity(0))
    quota = _cgroup_cpus()
    threads = aff if quota is None else max(1, min(aff, int(quota)))
    return threads, {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
                     "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"), "model": _cpu_model(),
                     "threads_used": threads}


def cpu_baseline(packed_host, off_host, nblocks, budget_s=12.0, threads=None):
    """Reference library (oracle/_ref: the reference's own sources compiled by
    oracle/Makefile) decoding a bounded sample of the same packed stream with
    `threads` std::threads.  `value` is its bit-exact scalar path
    (turbopfor::scalar::p4Dec256v32, the parity oracle); the AVX2 dispatch
    path (turbopfor::p4Dec256v32) is a labelled side number: it mis-decodes
    bitmap blocks with >= 32 exceptions (src/simd/p4dec256v32.cpp:71-83,
    SURVEY.md 8 a3).  Falls back to the oracle restatement (kind "port")
    if _ref is absent."""
    if threads is None:
        threads, host = cpu_host()
    else:
        host = {"threads_used": threads}
    seg = [(nblocks * s) // 32 for s in range(33)]
    parts, offs = [], [np.zeros(1, dtype=np.uint64)]
    base = 0
    for s in range(32):
        lo = seg[s]
        hi = lo + max(1, (seg[s + 1] - seg[s]) // 16)
        b0, b1 = int(off_host[lo]), int(off_host[hi])
        parts.append(packed_host[b0:b1])
        offs.append(off_host[lo + 1 : hi + 1] - b0 + base)
        base += b1 - b0
    sample = np.concatenate(parts + [np.zeros(64, np.uint8)])
    soff = np.ascontiguousarray(np.concatenate(offs), dtype=np.uint64)
    nb = len(soff) - 1
    out = np.empty((nb, 256), dtype=np.uint32)
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libtpref.so")
    u8p, u32p, u64p = (ctypes.POINTER(t) for t in (ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint64))
    if os.path.exists(ref_so):
        L = ctypes.CDLL(ref_so)
        f = L.tpref_dec256v32_stream_mt
        f.argtypes = [u8p, u64p, ctypes.c_uint64, u32p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        f.restype = ctypes.c_double

        def run():  # scalar: the bit-exact reference path
            return f(sample.ctypes.data_as(u8p), soff.ctypes.data_as(u64p), nb, out.ctypes.data_as(u32p), threads, 0, 0)

        kind, what = "reference", "turbopfor::scalar::p4Dec256v32 (reference scalar, bit-exact, oracle/_ref)"
    else:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib

        L = oracle_lib.lib()

        def run():
            t0 = time.perf_counter()
            L.orc_dec256v32_batch_mt(sample.ctypes.data_as(u8p), soff.ctypes.data_as(u64p), nb,
                                     out.ctypes.data_as(u32p), threads)
            return time.perf_counter() - t0

        kind, what = "port", "oracle restatement"
    run()
    tot, reps = 0.0, 0
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < budget_s:
        tot += run()
        reps += 1
    value = nb * 256 * reps / tot / 1e9
    abt = abtest_single_block(packed_host, off_host, nblocks) if kind == "reference" else None
    avx2 = None
    if kind == "reference":
        # the reference's AVX2 dispatch path over the same sample, shorter budget
        fs = L.tpref_dec256v32_stream_mt
        exp = out.copy()
        fs(sample.ctypes.data_as(u8p), soff.ctypes.data_as(u64p), nb, out.ctypes.data_as(u32p), threads, 1, 0)
        bad = int((out != exp).any(axis=1).sum())
        stot, sreps, s0 = 0.0, 0, time.perf_counter()
        while time.perf_counter() - s0 < budget_s / 3:
            stot += fs(sample.ctypes.data_as(u8p), soff.ctypes.data_as(u64p), nb, out.ctypes.data_as(u32p), threads, 1, 0)
            sreps += 1
        avx2 = {"value": round(nb * 256 * sreps / stot / 1e9, 3), "bit_exact": bad == 0, "blocks_differing_from_scalar": bad,
                "note": "turbopfor::p4Dec256v32 (AVX2 dispatch): mis-decodes bitmap blocks with >= 32 exceptions "
                        "(src/simd/p4dec256v32.cpp:71-83, SURVEY.md 8 a3) -- a speed reference, not a parity one"}
    return {
        "value": round(value, 3),
        "unit": "G int32/s",
        "cores": threads,
        "kind": kind,
        "host": host,
        "avx2_dispatch": avx2,
        "abtest_single_block": abt,
        "sample": f"{nb} blocks (first 1/16 of each bw segment of the same C2 stream) x {reps} passes, "
                  f"{threads} threads, {what} on {host.get('model', _cpu_model())}",
    }


def _cpu_model():
    try:
        return [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        return "unknown"


def _timed_reps(run, budget_s):
    """run() returns its own seconds; one untimed call, then reps until budget_s."""
    if run() < 0:
        raise RuntimeError("cpu baseline run failed")
    tot, reps, t_start = 0.0, 0, time.perf_counter()
    while time.perf_counter() - t_start < budget_s:
        s = run()
        if s < 0:
            raise RuntimeError("cpu baseline run failed")
        tot += s
        reps += 1
    return tot, reps


def cpu_baseline_d1(packed_host, off_host, starts_host, nblocks, chained, budget_s=12.0, threads=None):
    """C3 CPU baseline: the reference library (oracle/_ref) running
    turbopfor::p4D1Dec256v32 over the first 1/8 of the same posting-list
    stream with `threads` std::threads -- per-block starts, or (chained) each
    thread carrying the previous block's last value as its callers do
    (README.md:108-123).  None when oracle/_ref is absent (not built)."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libtpref.so")
    if not os.path.exists(ref_so):
        return None
    threads, host = cpu_host() if threads is None else (threads, {"threads_used": threads})
    nb = max(1, nblocks // 8)
    b1 = int(off_host[nb])
    sample = np.concatenate([packed_host[:b1], np.zeros(64, np.uint8)])
    soff = np.ascontiguousarray(off_host[: nb + 1], dtype=np.uint64)
    st = np.ascontiguousarray(starts_host[:nb], dtype=np.uint32)
    out = np.empty((nb, 256), dtype=np.uint32)
    L = ctypes.CDLL(ref_so)
    f = L.tpref_d1dec256v32_stream_mt
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                  ctypes.c_int, ctypes.c_int]
    f.restype = ctypes.c_double
    run = lambda disp: f(sample.ctypes.data, soff.ctypes.data, st.ctypes.data, nb, out.ctypes.data, threads, disp,
                         int(chained))
    tot, reps = _timed_reps(lambda: run(0), budget_s)
    exp = out.copy()
    dtot, dreps = _timed_reps(lambda: run(1), budget_s / 3)
    bad = int((out != exp).any(axis=1).sum())
    return {"value": round(nb * 256 * reps / tot / 1e9, 3), "unit": "G int32/s", "cores": threads, "kind": "reference",
            "host": host,
            "avx2_dispatch": {"value": round(nb * 256 * dreps / dtot / 1e9, 3), "blocks_differing_from_scalar": bad,
                              "note": "turbopfor::p4D1Dec256v32 AVX2 dispatch (speed reference; its bitmap path is the "
                                      "one of SURVEY.md 8 a3)"},
            "sample": f"first {nb} blocks of the same C3 stream x {reps} passes, {threads} threads, "
                      f"turbopfor::scalar::p4D1Dec256v32 (reference scalar, bit-exact, oracle/_ref; "
                      + ("chained through each block's last value" if chained else "per-block starts")
                      + f") on {_cpu_model()}"}


def cpu_baseline_rt(vals_host, nblocks, budget_s=12.0, threads=None):
    """C4 CPU baseline: the reference library (oracle/_ref) encoding the first
    1/16 of the same C4 values with turbopfor::p4Enc256v32 (chained through
    the returned end pointers) and decoding them back with p4Dec256v32, on
    `threads` std::threads.  None when oracle/_ref is absent."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libtpref.so")
    if not os.path.exists(ref_so):
        return None
    threads, host = cpu_host() if threads is None else (threads, {"threads_used": threads})
    nb = max(1, nblocks // 16)
    # every 16th block: the sample keeps the bw / exception-rate mix of the whole stream
    v = np.ascontiguousarray(vals_host[::16][:nb], dtype=np.uint32)
    slot = 1088
    scratch = np.empty(nb * slot + 64, dtype=np.uint8)
    off = np.empty(nb, dtype=np.uint64)
    out = np.empty((nb, 256), dtype=np.uint32)
    L = ctypes.CDLL(ref_so)
    f = L.tpref_rt256v32_stream_mt
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    f.restype = ctypes.c_double
    run = lambda disp: f(v.ctypes.data, nb, scratch.ctypes.data, slot, off.ctypes.data, out.ctypes.data, threads, disp)
    tot, reps = _timed_reps(lambda: run(0), budget_s)
    bad_scalar = int((out != v).any(axis=1).sum())
    dtot, dreps = _timed_reps(lambda: run(1), budget_s / 3)
    bad_disp = int((out != v).any(axis=1).sum())
    return {"value": round(nb * 256 * reps / tot / 1e9, 3), "unit": "G int32/s", "cores": threads, "kind": "reference",
            "host": host,
            "avx2_dispatch": {"value": round(nb * 256 * dreps / dtot / 1e9, 3), "blocks_not_round_tripped": bad_disp,
                              "note": "turbopfor::p4Enc256v32 + p4Dec256v32 AVX2 dispatch: the decode mis-reads "
                                      "bitmap blocks with >= 32 exceptions (SURVEY.md 8 a3) -- a speed reference"},
            "blocks_not_round_tripped": bad_scalar,
            "sample": f"every 16th block of the same C4 values ({nb} blocks) x {reps} passes, {threads} threads, "
                      f"turbopfor::scalar::p4Enc256v32 then p4Dec256v32 (reference scalar, oracle/_ref) on {_cpu_model()}"}


def abtest_single_block(packed_host, off_host, nblocks):
    """SURVEY §8(d) CPU baseline (i): the ab_test methodology
    (benchmarks/ab_test.cpp:553-701) -- one block L1-hot, 1000 warm-up calls,
    10,000-call chunks, best of 3 -- on one core, for the first block of the
    bw 8, 16 and 24 segments, reference AVX2 dispatch and reference scalar."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libtpref.so")
    L = ctypes.CDLL(ref_so)
    f = L.tpref_abtest_dec256v32
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint, ctypes.c_int]
    f.restype = ctypes.c_double
    res = {}
    for bw in (8, 16, 24):
        i = (nblocks * (bw - 1)) // 32
        b0, b1 = int(off_host[i]), int(off_host[i + 1])
        blk = np.concatenate([packed_host[b0:b1], np.zeros(64, np.uint8)])  # + the reference's read slack
        avx2 = f(blk.ctypes.data, 10000, 3, 1)
        scal = f(blk.ctypes.data, 10000, 3, 0)
        res[f"bw{bw}"] = {"block_bytes": b1 - b0, "avx2_G_int32_per_s": round(256 / avx2 / 1e9, 3),
                          "scalar_G_int32_per_s": round(256 / scal / 1e9, 3)}
    return res


# -------------------------------------------------------------- timing core
class Timer:
    """K launches bracketed by barrier + synchronize; per-launch HIP events
    recorded on the launch stream (torch's current stream, which is the stream
    handed to the C-ABI).  On a CPU device (--selftest) the per-step times are
    host clocks and there is nothing to synchronise."""

    def __init__(self, dist_on, dev):
        self.dist_on, self.dev = dist_on, dev
        self.gpu = torch.device(dev).type == "cuda"

    def _sync(self):
        if self.gpu:
            torch.cuda.synchronize()

    def run(self, fn, steps, warmup):
        for _ in range(warmup):
            fn()
        self._sync()
        if self.dist_on:
            torch.distributed.barrier()
        self._sync()
        if self.gpu:
            stream = torch.cuda.current_stream()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        host = []
        t0 = time.perf_counter()
        for i in range(steps):
            if self.gpu:
                evs[i][0].record(stream)
            h0 = time.perf_counter()
            fn()
            host.append((time.perf_counter() - h0) * 1e3)
            if self.gpu:
                evs[i][1].record(stream)
        self._sync()
        if self.dist_on:
            torch.distributed.barrier()
        self._sync()
        elapsed = time.perf_counter() - t0
        if self.dist_on:
            elapsed = tpf_shard.max_over_ranks(elapsed, self.dev)
        return elapsed, ([a.elapsed_time(b) for a, b in evs] if self.gpu else host)


def per_rank_stats(world, dev, kernel_ms, achieved_GBps):
    """Every rank's average kernel time and HBM fraction (all_gather; rank 0 reports them)."""
    mine = [float(kernel_ms), float(achieved_GBps)]
    rows = tpf_shard.gather_floats(mine, dev) if torch.distributed.is_initialized() else [mine]
    return [{"rank": r, "kernel_ms_avg": round(ms, 4), "achieved_GBps": round(gbs, 1),
             "frac": round(gbs / HBM_PEAK_GBS, 4)} for r, (ms, gbs) in enumerate(rows)]


def line(metric, value, unit, world, steps, warmup, elapsed, dtype, data, config, roofline=None, cpu=None):
    return {
        "metric": metric,
        "value": round(value, 2),
        "unit": unit,
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(elapsed * 1000.0 / steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": data,
        "config": config,
        "roofline": roofline,
        "cpu_baseline": cpu,
    }


# ---------------------------------------------------------------- workloads
def run_c2(args, world, rank, dev, T, c5=False):
    nb = args.nblocks
    t0 = time.time()
    first = shard_of(nb, world, rank)
    if c5:
        vals = bench_data.gen_c5(nb, args.exc, seed=42, dev=dev, first_block=first)
    else:
        vals, seg = gen_c2(nb, args.exc, seed=42, dev=dev, first_block=first)
    packed_full, offs = tpf.enc256v32(vals)
    packed = packed_full.clone()
    del packed_full
    torch.cuda.synchronize()
    pbytes = packed.numel()
    if rank == 0:
        log(f"[bench] {'c5' if c5 else 'c2'}: {nb} blocks generated+encoded in {time.time() - t0:.1f}s, packed {pbytes / 1e9:.3f} GB "
            f"({pbytes / nb:.1f} B/block)")
    out = torch.empty((nb, 256), dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int64, device=dev)
    elapsed, kern_ms = T.run(lambda: tpf.dec256v32(packed, offs, nb, out=out), args.steps, args.warmup)
    tpf.dec256v32(packed, offs, nb, out=out, err=err)
    ok = bool(torch.equal(out, vals)) and int(err.item()) == -1
    sums = {"decoded": checksum(out, dev, T.dist_on), "generated": checksum(vals, dev, T.dist_on)}
    if T.dist_on:
        ok = tpf_shard.all_ok(ok, dev)
    ok = ok and sums["decoded"] == sums["generated"]

    e2e = None
    if args.e2e and rank == 0:
        e2e = measure_e2e(packed, offs, nb, vals)
    # data-movement ceiling of the same access pattern (same kernel, loads
    # and stores only, no decode) -- outside the timed region
    _, probe_ms = T.run(lambda: tpf.probe256v32(packed, offs, nb, out), 10, 2)
    avg_ms = float(np.mean(kern_ms))
    alg = pbytes + nb * (1024 + 8) + 8
    achieved = alg / (avg_ms * 1e-3) / 1e9
    per_rank = per_rank_stats(world, dev, avg_ms, achieved)
    # the box's streaming ceilings (SURVEY §8 d), measured here: rank 0 only,
    # outside the timed region, after the other ranks' work is done
    probes = None
    if rank == 0 and not args.no_probes:
        probes = hbm_probes(dev)
    if rank != 0:
        return None
    probe = alg / (float(np.mean(probe_ms)) * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), **traffic_fields("c5" if c5 else "c2", nb),
            "kernel": "tpf::dev::k_dec256v32w<StartMode::None>", "kernel_ms_avg": round(avg_ms, 4),
            "kernel_ms_median": round(float(np.median(kern_ms)), 4), "kernel_ms_min": round(float(np.min(kern_ms)), 4),
            "alg_bytes_per_launch": int(alg),
            "alg_bytes_def": "packed block bytes + 1024 B decoded + 8 B offset per block",
            "probe_GBps": round(probe, 1), "frac_of_probe": round(achieved / probe, 4),
            "probe_def": "tpfm_probe256v32: the decode kernel's own loads and stores with decoding removed",
            "hbm_probes": probes, "per_rank": per_rank}
    # the CPU baseline is timed at N=1 only (a reported baseline, not a per-rank cost)
    cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline(packed.cpu().numpy(),
                                                                          offs.cpu().numpy().astype(np.uint64), nb)
    value = nb * 256 * world / (elapsed / args.steps) / 1e9
    cfg = {"workload": ("C5: p4Dec256v32 sharded, 10M blocks x 256 u32 per GPU (80M at 8 GPUs), half bw 8 / half "
                        "bw 16, 10% exceptions" if c5 else
                        "C2: p4Dec256v32, 10M blocks x 256 u32 per GPU, bw 1..32 sweep (32 equal segments), "
                        "10% exceptions for bw<=28"),
           "nblocks_per_gpu": nb, "packed_bytes_per_gpu": pbytes, "bytes_per_block": round(pbytes / nb, 1),
           "compressed_GBps": round(pbytes * world / (elapsed / args.steps) / 1e9, 1),
           "parallelism": f"shard{world}", "shard_blocks": [first, first + nb], "verified": ok,
           "checksum_all_ranks": sums}
    if e2e:
        cfg["e2e_host_pinned"] = e2e
    data = (f"synthetic (GPU-generated {'C5' if c5 else 'C2'} values: rank r holds blocks [r*nb, (r+1)*nb) of one "
            "counter-keyed global stream; GPU-encoded; full-size decode verified bit-exact on every rank: "
            + ("ok" if ok else "MISMATCH") + ")")
    return line(METRIC, value, "G int32/s", world, args.steps, args.warmup, elapsed, "u32", data, cfg, roof, cpu), ok


def run_sweep(args, world, rank, dev, T):
    """SURVEY §8(d) per-width sweep at full size: for every bit width 1..32,
    nblocks (default 10M) blocks of that width alone (10 % exceptions for
    bw <= 28), encoded on the GPU, decoded `steps` times (HIP events on the
    launch stream), verified, and timed against the decode kernel's own
    data-movement probe on the same stream.  value = all widths' integers /
    all widths' decode time (each width weighted equally)."""
    nb = args.nblocks
    rows, tot_ms, tot_alg = [], 0.0, 0
    out = torch.empty((nb, 256), dtype=torch.int32, device=dev)
    t_start = time.perf_counter()
    ok = True
    for bw in range(1, 33):
        vals = gen_bw(nb, bw, args.exc, seed=42, dev=dev, first_block=shard_of(nb, world, rank))
        packed_full, offs = tpf.enc256v32(vals)
        packed = packed_full.clone()
        del packed_full
        _, kern_ms = T.run(lambda: tpf.dec256v32(packed, offs, nb, out=out), args.steps, args.warmup)
        good = bool(torch.equal(out, vals))
        _, probe_ms = T.run(lambda: tpf.probe256v32(packed, offs, nb, out), max(3, args.steps // 2), 1)
        ok = ok and good
        ms, pms = float(np.mean(kern_ms)), float(np.mean(probe_ms))
        pbytes = packed.numel()
        alg = pbytes + nb * (1024 + 8) + 8
        row = {"bw": bw, "bytes_per_block": round(pbytes / nb, 1), "ms": round(ms, 4), "G_int32_per_s": round(nb * 256 / ms / 1e6, 1),
               "alg_GBps": round(alg / ms / 1e6, 1), "frac": round(alg / ms / 1e6 / HBM_PEAK_GBS, 4),
               "probe_ms": round(pms, 4), "frac_of_probe": round(pms / ms, 4), "verified": good}
        rows.append(row)
        tot_ms += ms
        tot_alg += alg
        if rank == 0:
            log(f"[sweep] bw={bw:2d} B/blk={row['bytes_per_block']:7.1f} ms={ms:.4f} Gint/s={row['G_int32_per_s']:8.1f} "
                f"alg GB/s={row['alg_GBps']:7.1f} ({row['frac']:.1%} of peak, {row['frac_of_probe']:.1%} of probe)"
                + ("" if good else " MISMATCH"))
        del vals, packed, offs
    elapsed = time.perf_counter() - t_start
    if T.dist_on:
        ok = tpf_shard.all_ok(ok, dev)
    if rank != 0:
        return None
    value = 32 * nb * 256 * world / (tot_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(tot_alg / (tot_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(tot_alg / (tot_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
            "traffic_source": {"note": "no PMC pass for the sweep"}, "kernel": "tpf::dev::k_dec256v32w<StartMode::None>",
            "per_bw": rows}
    cfg = {"workload": f"C2 per-width sweep: {nb} blocks x 256 u32 for EACH bw 1..32, {args.exc:g}% exceptions for bw<=28",
           "nblocks_per_bw": nb, "parallelism": f"shard{world}", "verified": ok}
    res = line("G int32/s device-resident p4Dec256v32, per-width sweep (equal weight)", value, "G int32/s", world,
               32 * args.steps, args.warmup, tot_ms * 1e-3, "u32",
               "synthetic (GPU-generated per-width values, GPU-encoded; every width verified bit-exact)", cfg, roof, None)
    res["wall_s"] = round(elapsed, 1)
    return res, ok


def measure_e2e(packed, offs, nb, vals):
    """Host-memory rates (the north star's end-to-end number): pinned packed
    bytes + offsets in, pinned values out, tpf_host_dec (chunk uploads by
    SDMA overlapped with the decode and the download of the previous chunk);
    and the reverse trip, tpf_host_enc, from pinned values to a pinned
    stream + offsets."""
    L = tpf.lib()
    L.tpf_host_dec.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                               ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
    L.tpf_host_enc.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    h_in = packed.cpu().pin_memory()
    h_off = offs.cpu().pin_memory()
    h_out = torch.empty((nb, 256), dtype=torch.int32).pin_memory()
    reps = 3

    def dec():
        rc = L.tpf_host_dec(2, h_in.data_ptr(), h_in.numel(), h_off.data_ptr(), nb, 256, h_out.data_ptr(), None)
        assert rc == 0, L.tpf_last_error()

    dec()
    t0 = time.perf_counter()
    for _ in range(reps):
        dec()
    dt = (time.perf_counter() - t0) / reps
    ok = bool(torch.equal(h_out, vals.cpu()))
    r = {"G_int32_per_s": round(nb * 256 / dt / 1e9, 2), "s_per_pass": round(dt, 4),
         "pcie_GBps_in_plus_out": round((h_in.numel() + nb * 1032) / dt / 1e9, 2), "verified": ok}
    cap = h_in.numel() + 64
    h_pk = torch.empty(cap, dtype=torch.uint8).pin_memory()
    h_po = torch.empty(nb + 1, dtype=torch.int64).pin_memory()

    def enc():
        rc = L.tpf_host_enc(2, h_out.data_ptr(), nb, 256, 0, None, 0, h_pk.data_ptr(), cap, h_po.data_ptr())
        assert rc == 0, L.tpf_last_error()

    enc()
    t0 = time.perf_counter()
    for _ in range(reps):
        enc()
    dt = (time.perf_counter() - t0) / reps
    ok_e = bool(torch.equal(h_po, h_off.view(torch.int64)) and torch.equal(h_pk[: h_in.numel()], h_in))
    r["enc"] = {"G_int32_per_s": round(nb * 256 / dt / 1e9, 2), "s_per_pass": round(dt, 4),
                "pcie_GBps_in_plus_out": round((h_in.numel() + nb * 1032) / dt / 1e9, 2), "verified": ok_e}
    # the same trips from PAGEABLE host memory (NumPy arrays): the library
    # stages them through its pinned buffers with host copies (it never
    # page-locks caller memory), so this rate is bounded by those copies
    p_in, p_off = h_in.numpy().copy(), h_off.numpy().copy()
    p_out = np.empty((nb, 256), dtype=np.int32)
    L.tpf_host_dec(2, p_in.ctypes.data, p_in.size, p_off.ctypes.data, nb, 256, p_out.ctypes.data, None)
    t0 = time.perf_counter()
    for _ in range(reps):
        assert L.tpf_host_dec(2, p_in.ctypes.data, p_in.size, p_off.ctypes.data, nb, 256, p_out.ctypes.data, None) == 0
    dtp = (time.perf_counter() - t0) / reps
    ok_p = bool(np.array_equal(p_out, h_out.numpy()))
    p_pk = np.empty(cap, dtype=np.uint8)
    p_po = np.empty(nb + 1, dtype=np.uint64)
    L.tpf_host_enc(2, p_out.ctypes.data, nb, 256, 0, None, 0, p_pk.ctypes.data, cap, p_po.ctypes.data)
    t0 = time.perf_counter()
    for _ in range(reps):
        assert L.tpf_host_enc(2, p_out.ctypes.data, nb, 256, 0, None, 0, p_pk.ctypes.data, cap, p_po.ctypes.data) == 0
    dtpe = (time.perf_counter() - t0) / reps
    ok_pe = bool(np.array_equal(p_po.view(np.int64), h_off.numpy())) and bool(np.array_equal(p_pk[: p_in.size], p_in))
    r["pageable"] = {"dec_G_int32_per_s": round(nb * 256 / dtp / 1e9, 2), "enc_G_int32_per_s": round(nb * 256 / dtpe / 1e9, 2),
                     "verified": ok_p and ok_pe,
                     "note": "NumPy (pageable) buffers: staged through the pipeline's pinned buffers by host copies"}
    log(f"[e2e] host-pinned decode/encode: {r}")
    return r


def run_c3(args, world, rank, dev, T, chained):
    nb = args.nblocks
    t0 = time.time()
    # ONE posting list over all ranks: rank r holds its blocks [r*nb, (r+1)*nb);
    # its values continue rank r-1's (the carry is an exclusive prefix of the
    # shards' gap totals, generation only)
    first = shard_of(nb, world, rank)
    carry = (lambda tot: tpf_shard.exclusive_prefix(tot, dev)) if T.dist_on else None
    vals, starts = gen_c3(nb, seed=7, dev=dev, first_block=first, carry_fn=carry)
    packed_full, offs = tpf.enc256v32(vals, d1=True, starts=starts)
    packed = packed_full.clone()
    del packed_full
    torch.cuda.synchronize()
    pbytes = packed.numel()
    mix = block_mix(packed, offs)
    vb_frac = mix["vbyte_block_frac"]
    if rank == 0:
        log(f"[bench] c3: {nb} blocks in {time.time() - t0:.1f}s, {pbytes / nb / 256:.3f} B/int, "
            f"vbyte-mode blocks {vb_frac:.1%}, exception fraction {mix['exception_frac']:.4f}")
    out = torch.empty((nb, 256), dtype=torch.int32, device=dev)
    if chained:
        # phase A (block sums + scan), [all-gather of one u32 per rank], phase B
        # phase A (block sums + scan), [all-gather of one u32 per rank], phase B.
        # start0 = the value before the GLOBAL list's first block (0); every
        # rank's base comes from the exchange, not from its own starts.
        chain = tpf.D1Chain(packed, offs, nb)
        start0 = 0

        def step():
            chain.sums()
            base = tpf_shard.chained_base(chain.total, start0=start0) if T.dist_on else start0
            chain.decode(base, out=out)

        fn = step
    else:
        fn = lambda: tpf.dec256v32(packed, offs, nb, out=out, starts=starts)
    elapsed, kern_ms = T.run(fn, args.steps, args.warmup)
    # every rank checks its slice of the global list (for a chained list this
    # verifies the cross-rank exchange: a wrong base shifts every value)
    ok = bool(torch.equal(out, vals))
    sums = {"decoded": checksum(out, dev, T.dist_on), "generated": checksum(vals, dev, T.dist_on)}
    if T.dist_on:
        ok = tpf_shard.all_ok(ok, dev)
    ok = ok and sums["decoded"] == sums["generated"]
    # data-movement probe of the same stream (decode kernel's loads and stores, no decode)
    _, probe_ms = T.run(lambda: tpf.probe256v32(packed, offs, nb, out), 10, 2)
    avg_ms = float(np.mean(kern_ms))
    alg = pbytes + nb * (1024 + 8 + (0 if chained else 4)) + 8
    per_rank = per_rank_stats(world, dev, avg_ms, alg / (avg_ms * 1e-3) / 1e9)
    if rank != 0:
        return None
    value = nb * 256 * world / (elapsed / args.steps) / 1e9
    probe_alg = pbytes + nb * (1024 + 8) + 8
    roof = {"bound": "hbm", "achieved": round(alg / (avg_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(alg / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            **traffic_fields("c3chain" if chained else "c3", nb),
            "kernel_ms_avg": round(avg_ms, 4),
            "kernel": ("k_dsum256v32_lanes (phase A) + run scan (2 small kernels) + k_dec256v32w<Prefix>" if chained
                       else "tpf::dev::k_dec256v32w<StartMode::PerBlock>"),
            "probe_GBps": round(probe_alg / (float(np.mean(probe_ms)) * 1e-3) / 1e9, 1),
            "ms_vs_probe": round(avg_ms / float(np.mean(probe_ms)), 3),
            "probe_def": "tpfm_probe256v32 on the same stream (loads + stores, no decode; no starts read)",
            "per_rank": per_rank}
    cfg = {"workload": "C3: p4D1Dec256v32 " + ("chained list (start0 only)" if chained else "per-block starts")
                       + ", Zipf(1.1) gaps on [1,64] + 5% 64+U[0,2^16)",
           "nblocks_per_gpu": nb, "bytes_per_int": round(pbytes / nb / 256, 4), **mix,
           "parallelism": f"shard{world}", "shard_blocks": [first, first + nb], "verified": ok,
           "checksum_all_ranks": sums,
           "list": "one posting list over all ranks (rank r: blocks [r*nb, (r+1)*nb), values continue rank r-1's)"}
    metric = "G int32/s device-resident p4D1Dec256v32" + (" (chained list)" if chained else "")
    cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline_d1(
        packed.cpu().numpy(), offs.cpu().numpy().astype(np.uint64), starts.cpu().numpy().view(np.uint32), nb, chained)
    return line(metric, value, "G int32/s", world, args.steps, args.warmup, elapsed, "u32",
                "synthetic (GPU-generated posting list, counter-keyed by global position, GPU-encoded; decode verified "
                "bit-exact on every rank: " + ("ok" if ok else "MISMATCH") + ")", cfg, roof, cpu), ok


def run_c4(args, world, rank, dev, T):
    """BASELINE configs[3]: p4Enc256v32 + p4Dec256v32 round trip (C2 values
    with the exception rate cycling 0/5/10/25% over the bw segments), then
    the same round trip in 64 bits: p4Enc256v64 + p4Dec256v64 over nblocks
    256-value units of bench_data.gen_v64 (bw 1..64, rates 0/5/10/25%,
    exceptions in 32 bits or above bit 32 in alternate segments:
    tests/test_p4_64.cpp:587-611).  value = the 32-bit round trip."""
    nb = args.nblocks
    first = shard_of(nb, world, rank)
    vals, _ = gen_c2(nb, 0, seed=11, dev=dev, pcts=[0, 5, 10, 25], first_block=first)
    cap = int(tpf.lib().tpf_p4enc256v32_bound(nb))
    enc_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    dec_out = torch.empty((nb, 256), dtype=torch.int32, device=dev)
    state = {}

    def rt():
        p, o = tpf.enc256v32(vals, out=enc_out)
        state["p"], state["o"] = p, o
        tpf.dec256v32(p, o, nb, out=dec_out)

    elapsed, rt_ms = T.run(rt, args.steps, args.warmup)
    ok = bool(torch.equal(dec_out, vals))
    # the two halves separately (kernel time, HIP events on the launch stream)
    _, enc_ms = T.run(lambda: tpf.enc256v32(vals, out=enc_out), args.steps, 1)
    _, dec_ms = T.run(lambda: tpf.dec256v32(state["p"], state["o"], nb, out=dec_out), args.steps, 1)
    pbytes = int(state["o"][-1].item())
    cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline_rt(vals.cpu().numpy().view(np.uint32), nb)
    del vals, enc_out, dec_out, state
    torch.cuda.empty_cache()

    # ---- 64-bit leg at the same unit count
    v64 = bench_data.gen_v64(nb, seed=5, dev=dev, first_block=first)
    out64 = torch.empty(nb * 256, dtype=torch.int64, device=dev)
    # encoder output, offsets and workspace allocated once (no allocation in the timed loop)
    bufs64 = {"out": torch.empty(int(tpf.lib().tpf_enc_bound(tpf.FMT["256v64"], nb, 256)), dtype=torch.uint8, device=dev),
              "offs": torch.empty(nb + 1, dtype=torch.int64, device=dev),
              "ws": torch.empty(max(1, int(tpf.lib().tpf_enc_workspace_size(tpf.FMT["256v64"], nb, 256))), dtype=torch.uint8,
                                device=dev)}
    enc64 = {}

    def enc_64():
        enc64["p"], enc64["o"] = tpf.enc_batch("256v64", v64.view(-1), nb, 256, **bufs64)

    def rt64():
        enc_64()
        tpf.dec_batch("256v64", enc64["p"], enc64["o"], nb, 256, out=out64)

    s64 = max(2, args.steps // 2)
    el64, rt64_ms = T.run(rt64, s64, 1)
    ok64 = bool(torch.equal(out64.view(nb, 256), v64))
    _, enc64_ms = T.run(enc_64, s64, 1)
    _, dec64_ms = T.run(lambda: tpf.dec_batch("256v64", enc64["p"], enc64["o"], nb, 256, out=out64), s64, 1)
    p64 = int(enc64["p"].numel())
    # the 256v64 decoder's own data-movement probe on the same stream (its loads and stores, no decode)
    probe64_ms = None
    if os.path.exists(tpf.MEASURE_PATH):
        _, probe64_ms = T.run(lambda: tpf.probe256v64(enc64["p"], enc64["o"], nb, out64), s64, 1)
    del v64, out64, enc64, bufs64
    torch.cuda.empty_cache()

    alg_enc = nb * (1024 + 8) + pbytes + 8
    alg_dec = pbytes + nb * (1024 + 8) + 8
    per_rank = per_rank_stats(world, dev, float(np.mean(rt_ms)), (alg_enc + alg_dec) / (float(np.mean(rt_ms)) * 1e-3) / 1e9)
    ok_all = ok and ok64
    if T.dist_on:
        ok_all = tpf_shard.all_ok(ok_all, dev)
    if rank != 0:
        return None
    value = nb * 256 * world / (elapsed / args.steps) / 1e9
    g = lambda n, ms: round(n * 256 / (float(np.mean(ms)) * 1e-3) / 1e9, 2)
    gbs = lambda b, ms: round(b / (float(np.mean(ms)) * 1e-3) / 1e9, 1)
    a64_enc = nb * (2048 + 8) + p64 + 8
    a64_dec = p64 + nb * (2048 + 8) + 8
    cfg = {"workload": "C4: p4Enc256v32 + p4Dec256v32 round trip, bw 1..32 segments cycling 0/5/10/25% exceptions; "
                       "and p4Enc256v64 + p4Dec256v64 over the same number of 256-value units, bw 1..64 segments "
                       "cycling 0/5/10/25%, exceptions in 32 bits / above bit 32 in alternate segments",
           "nblocks_per_gpu": nb, "parallelism": f"shard{world}", "shard_blocks": [first, first + nb],
           "verified": ok_all, "verified_32": ok, "verified_64": ok64,
           "enc256v32_G_int32_per_s": g(nb, enc_ms), "dec256v32_G_int32_per_s": g(nb, dec_ms),
           "bytes_per_block": round(pbytes / nb, 1),
           "roundtrip_256v64": {"nblocks": nb, "G_int64_per_s": round(nb * 256 / (el64 / s64) / 1e9, 2),
                                "enc_G_int64_per_s": g(nb, enc64_ms), "dec_G_int64_per_s": g(nb, dec64_ms),
                                "packed_bytes_per_unit": round(p64 / nb, 1), "verified": ok64}}
    if probe64_ms is not None:
        cfg["roundtrip_256v64"].update({
            "dec_alg_GBps": gbs(a64_dec, dec64_ms), "probe_GBps": gbs(a64_dec, probe64_ms),
            "dec_ms_vs_probe": round(float(np.mean(dec64_ms)) / float(np.mean(probe64_ms)), 3),
            "probe_def": "tpfm_probe256v64 on the same stream (the decoder's loads + stores, no decode)"})
    # roofline of the step (encode = plan + offset scan + write launches, then
    # the decode launch, all on the launch stream): algorithmic bytes are the
    # encoder's (1024 in + block out + 8 offset) plus the decoder's (block in
    # + 1024 out + 8 offset) per block; the encoder's second read of the
    # values (plan pass, then write pass) is not counted
    rt_gbs = gbs(alg_enc + alg_dec, rt_ms)
    roof = {"bound": "hbm", "achieved": rt_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(rt_gbs / HBM_PEAK_GBS, 4), **traffic_fields("c4", nb),
            "kernel": "round-trip step: k_enc256v32_plan + run scan (2 small kernels) + k_enc256v32_write + k_dec256v32w<None>",
            "kernel_ms_avg": round(float(np.mean(rt_ms)), 4), "alg_bytes_per_launch": int(alg_enc + alg_dec),
            "alg_bytes_def": "encode: 1024 B values + block bytes + 8 B offset; decode: block bytes + 1024 B + 8 B",
            "enc_achieved_GBps": gbs(alg_enc, enc_ms), "enc_frac": round(gbs(alg_enc, enc_ms) / HBM_PEAK_GBS, 4),
            "enc_ms_avg": round(float(np.mean(enc_ms)), 4),
            "dec_achieved_GBps": gbs(alg_dec, dec_ms), "dec_frac": round(gbs(alg_dec, dec_ms) / HBM_PEAK_GBS, 4),
            "dec_ms_avg": round(float(np.mean(dec_ms)), 4),
            "v64": {"kernels": "k_enc128v64_plan + run scan + k_enc128v64_write; k_dec128v64w<2>",
                    "alg_bytes_def": "encode: 2048 B values + unit bytes + 8 B offset; decode: unit bytes + 2048 B + 8 B",
                    "rt_achieved_GBps": gbs(a64_enc + a64_dec, rt64_ms),
                    "rt_frac": round(gbs(a64_enc + a64_dec, rt64_ms) / HBM_PEAK_GBS, 4),
                    "enc_achieved_GBps": gbs(a64_enc, enc64_ms), "enc_frac": round(gbs(a64_enc, enc64_ms) / HBM_PEAK_GBS, 4),
                    "enc_ms_avg": round(float(np.mean(enc64_ms)), 4),
                    "dec_achieved_GBps": gbs(a64_dec, dec64_ms), "dec_frac": round(gbs(a64_dec, dec64_ms) / HBM_PEAK_GBS, 4),
                    "dec_ms_avg": round(float(np.mean(dec64_ms)), 4), **traffic_fields("c4_64", nb)},
            "per_rank": per_rank}
    return line("G int32/s device-resident p4Enc256v32+p4Dec256v32 round trip", value, "G int32/s", world, args.steps,
                args.warmup, elapsed, "u32", "synthetic (GPU-generated, counter-keyed by global position)", cfg, roof,
                cpu), ok_all


def cpu_baseline_d1enc(vals_host, starts_host, nblocks, budget_s=12.0, threads=None):
    """C3 encode CPU baseline: the reference library (oracle/_ref) writing the
    first 1/8 of the same posting list with turbopfor::scalar::p4D1Enc256v32,
    each thread chained through the returned end pointers and the previous
    block's last value (README.md:108-123).  None when oracle/_ref is absent."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libtpref.so")
    if not os.path.exists(ref_so):
        return None
    threads, host = cpu_host() if threads is None else (threads, {"threads_used": threads})
    nb = max(1, nblocks // 8)
    v = np.ascontiguousarray(vals_host[:nb], dtype=np.uint32)
    st = np.ascontiguousarray(starts_host[:nb], dtype=np.uint32)
    slot = 1088
    scratch = np.empty(nb * slot + 64, dtype=np.uint8)
    off = np.empty(nb, dtype=np.uint64)
    L = ctypes.CDLL(ref_so)
    f = L.tpref_d1enc256v32_stream_mt
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                  ctypes.c_int, ctypes.c_int]
    f.restype = ctypes.c_double
    run = lambda disp: f(v.ctypes.data, st.ctypes.data, nb, scratch.ctypes.data, slot, off.ctypes.data, threads, disp)
    tot, reps = _timed_reps(lambda: run(0), budget_s)
    dtot, dreps = _timed_reps(lambda: run(1), budget_s / 3)
    return {"value": round(nb * 256 * reps / tot / 1e9, 3), "unit": "G int32/s", "cores": threads, "kind": "reference",
            "host": host, "avx2_dispatch": {"value": round(nb * 256 * dreps / dtot / 1e9, 3)},
            "sample": f"first {nb} blocks of the same C3 list x {reps} passes, {threads} threads, "
                      f"turbopfor::scalar::p4D1Enc256v32 chained (reference scalar, oracle/_ref) on {_cpu_model()}"}


def run_c3enc(args, world, rank, dev, T):
    """p4D1Enc256v32 on the C3 posting list (the encoder's
    vbyte-heavy case): one chained list per rank-shard, written the way a
    reference caller writes it (block i starts from block i-1's last value:
    start0 + the values themselves, tpf_p4d1enc256v32_batch with no starts).
    Verified: the per-block-start encoding of the same values is identical and
    decode(encode(x)) == x."""
    nb = args.nblocks
    first = shard_of(nb, world, rank)
    carry = (lambda tot: tpf_shard.exclusive_prefix(tot, dev)) if T.dist_on else None
    vals, starts = gen_c3(nb, seed=7, dev=dev, first_block=first, carry_fn=carry)
    start0 = int(starts[0].item()) & 0xFFFFFFFF
    cap = int(tpf.lib().tpf_p4enc256v32_bound(nb))
    enc_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    state = {}

    def enc():
        state["p"], state["o"] = tpf.enc256v32(vals, d1=True, start0=start0, out=enc_out)

    elapsed, kern_ms = T.run(enc, args.steps, args.warmup)
    p1, o1 = state["p"], state["o"]
    pbytes = int(o1[-1].item())
    p2, o2 = tpf.enc256v32(vals, d1=True, starts=starts)
    ok = bool(torch.equal(o1, o2)) and bool(torch.equal(p1[:pbytes], p2[:pbytes]))
    del p2, o2
    out = tpf.dec256v32(p1, o1, nb, starts=starts)
    ok = ok and bool(torch.equal(out, vals))
    del out
    if T.dist_on:
        ok = tpf_shard.all_ok(ok, dev)
    avg_ms = float(np.mean(kern_ms))
    alg = nb * (1024 + 8) + pbytes + 8
    per_rank = per_rank_stats(world, dev, avg_ms, alg / (avg_ms * 1e-3) / 1e9)
    if rank != 0:
        return None
    value = nb * 256 * world / (elapsed / args.steps) / 1e9
    roof = {"bound": "hbm", "achieved": round(alg / (avg_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(alg / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), **traffic_fields("c3enc", nb),
            "kernel": "k_enc256v32_plan<D1> + run scan (2 small kernels) + k_enc256v32_write<D1>",
            "kernel_ms_avg": round(avg_ms, 4), "alg_bytes_per_launch": int(alg),
            "alg_bytes_def": "1024 B values + block bytes + 8 B offset per block (the write pass's second read of the "
                             "values is not counted)",
            "per_rank": per_rank}
    cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline_d1enc(
        vals.cpu().numpy().view(np.uint32), starts.cpu().numpy().view(np.uint32), nb)
    cfg = {"workload": "C3 encode: p4D1Enc256v32 of the C3 Zipf posting list, chained (start0 + the list itself)",
           "nblocks_per_gpu": nb, "bytes_per_int": round(pbytes / nb / 256, 4), **block_mix(p1, o1),
           "parallelism": f"shard{world}", "shard_blocks": [first, first + nb], "verified": ok}
    return line("G int32/s device-resident p4D1Enc256v32 (chained posting list)", value, "G int32/s", world, args.steps,
                args.warmup, elapsed, "u32", "synthetic (GPU-generated C3 posting list; encoding checked against the "
                "per-block-start encoder and decoded back: " + ("ok" if ok else "MISMATCH") + ")", cfg, roof, cpu), ok


def cpu_baseline_d1dec64(packed_host, off_host, starts_host, nunits, budget_s=12.0, threads=None):
    """64-bit chained list CPU baseline: the reference library (oracle/_ref)
    running turbopfor::scalar::p4D1Dec256v64 over the first 1/8 of the same
    stream, each thread chained through the previous unit's last value."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libtpref.so")
    if not os.path.exists(ref_so):
        return None
    threads, host = cpu_host() if threads is None else (threads, {"threads_used": threads})
    nb = max(1, nunits // 8)
    b1 = int(off_host[nb])
    sample = np.concatenate([packed_host[:b1], np.zeros(64, np.uint8)])
    soff = np.ascontiguousarray(off_host[: nb + 1], dtype=np.uint64)
    st = np.ascontiguousarray(starts_host[:nb], dtype=np.uint64)
    out = np.empty((nb, 256), dtype=np.uint64)
    L = ctypes.CDLL(ref_so)
    f = L.tpref_d1dec256v64_stream_mt
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                  ctypes.c_int, ctypes.c_int]
    f.restype = ctypes.c_double
    run = lambda disp: f(sample.ctypes.data, soff.ctypes.data, st.ctypes.data, nb, out.ctypes.data, threads, disp, 1)
    tot, reps = _timed_reps(lambda: run(0), budget_s)
    exp = out.copy()
    dtot, dreps = _timed_reps(lambda: run(1), budget_s / 3)
    return {"value": round(nb * 256 * reps / tot / 1e9, 3), "unit": "G int64/s", "cores": threads, "kind": "reference",
            "host": host, "avx2_dispatch": {"value": round(nb * 256 * dreps / dtot / 1e9, 3),
                                            "units_differing_from_scalar": int((out != exp).any(axis=1).sum())},
            "sample": f"first {nb} units of the same stream x {reps} passes, {threads} threads, "
                      f"turbopfor::scalar::p4D1Dec256v64 chained through each unit's last value (oracle/_ref) on {_cpu_model()}"}


def run_c3chain64(args, world, rank, dev, T):
    """A 64-bit chained posting list (SURVEY §8 f1 widened to
    256v64): the C3 gaps as u64 ids above 2^32, p4D1Enc256v64 units chained the
    way reference callers chain them; decoded from start0 alone by
    tpf_d1dec64_chain_sums (unit totals + u64 run scan) and
    tpf_d1dec64_chain_decode.  Across ranks: one u64 total per rank all-gathered
    (tpf_shard.chained_base64)."""
    nb = args.nblocks
    first = shard_of(nb, world, rank)
    carry = (lambda tot: tpf_shard.exclusive_prefix(tot, dev)) if T.dist_on else None
    vals, starts = bench_data.gen_c3_64(nb, seed=7, dev=dev, first_block=first, carry_fn=carry)
    packed, offs = tpf.enc_batch("256v64", vals.view(-1), nb, 256, d1=True, starts=starts)
    pbytes = int(packed.numel())
    L = tpf.lib()
    fmt = tpf.FMT["256v64"]
    ws = torch.empty(int(L.tpf_d1dec64_chain_workspace_size(nb)), dtype=torch.uint8, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    out = torch.empty((nb, 256), dtype=torch.int64, device=dev)
    start0 = (1 << 40) + 12345  # the value before the GLOBAL list's first unit

    def step():
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        assert L.tpf_d1dec64_chain_sums(fmt, packed.data_ptr(), pbytes, offs.data_ptr(), nb, ws.data_ptr(), ws.numel(),
                                        total.data_ptr(), None, s) == 0
        base = tpf_shard.chained_base64(total, start0=start0) if T.dist_on else start0
        assert L.tpf_d1dec64_chain_decode(fmt, packed.data_ptr(), pbytes, offs.data_ptr(), nb, out.data_ptr(),
                                          ctypes.c_uint64(base), ws.data_ptr(), None, s) == 0

    elapsed, kern_ms = T.run(step, args.steps, args.warmup)
    ok = bool(torch.equal(out, vals))
    if T.dist_on:
        ok = tpf_shard.all_ok(ok, dev)
    _, plain_ms = T.run(lambda: tpf.dec_batch("256v64", packed, offs, nb, 256, starts=starts, out=out.view(-1)), 5, 1)
    ok = ok and bool(torch.equal(out, vals))
    avg_ms = float(np.mean(kern_ms))
    alg = pbytes + nb * (2048 + 8) + 8
    per_rank = per_rank_stats(world, dev, avg_ms, alg / (avg_ms * 1e-3) / 1e9)
    if rank != 0:
        return None
    value = nb * 256 * world / (elapsed / args.steps) / 1e9
    roof = {"bound": "hbm", "achieved": round(alg / (avg_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(alg / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), **traffic_fields("c3chain64", nb),
            "kernel": "k_dsum128v64_lanes (phase A, lane per unit) + run scan (u64) + k_dec128v64w<2, Prefix>", "kernel_ms_avg": round(avg_ms, 4),
            "alg_bytes_per_launch": int(alg),
            "alg_bytes_def": "unit bytes + 2048 B decoded + 8 B offset per unit (phase A's read of the stream not counted)",
            "per_unit_starts_ms_avg": round(float(np.mean(plain_ms)), 4), "per_rank": per_rank}
    cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline_d1dec64(
        packed.cpu().numpy(), offs.cpu().numpy().astype(np.uint64), starts.cpu().numpy().view(np.uint64), nb)
    cfg = {"workload": "C3 as a 64-bit chained list: p4D1Dec256v64 units of the C3 Zipf gaps as u64 ids above 2^32, "
                       "decoded from start0 alone",
           "nunits_per_gpu": nb, "bytes_per_int": round(pbytes / nb / 256, 4), "parallelism": f"shard{world}",
           "shard_units": [first, first + nb], "verified": ok,
           "per_unit_starts_G_int64_per_s": round(nb * 256 / (float(np.mean(plain_ms)) * 1e-3) / 1e9, 2)}
    return line("G int64/s device-resident p4D1Dec256v64 (chained list)", value, "G int64/s", world, args.steps,
                args.warmup, elapsed, "u64", "synthetic (GPU-generated 64-bit posting list, GPU-encoded; chained decode "
                "verified bit-exact on every rank: " + ("ok" if ok else "MISMATCH") + ")", cfg, roof, cpu), ok


def cpu_abtest_c1(vals_host, blk_host, blen, n):
    """ab_test methodology (benchmarks/ab_test.cpp:553-701) on the reference
    library built from its own sources (oracle/_ref): one L1-hot block,
    1000 warm-up calls, 10,000-call chunks, best of 3; turbopfor::p4Dec32 /
    p4Enc32 dispatch path, one core."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libtpref.so")
    if not os.path.exists(ref_so):
        return None
    L = ctypes.CDLL(ref_so)
    f = L.tpref_abtest_p4_32
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_int,
                  ctypes.c_int]
    f.restype = ctypes.c_double
    dec_s = f(vals_host.ctypes.data, blk_host.ctypes.data, n, 10000, 3, 1, 0)
    enc_s = f(vals_host.ctypes.data, blk_host.ctypes.data, n, 10000, 3, 1, 1)
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        model = "unknown"
    return {"value": round(n / dec_s / 1e9, 3), "unit": "G int32/s", "cores": 1, "kind": "reference",
            "sample": f"ab_test loop: one {blen}-B block (n={n}, bw 8, 0% exc), L1-hot, 10,000-call chunks, "
                      f"best of 3, turbopfor::p4Dec32 (oracle/_ref) on {model}",
            "dec_MBps_compressed": round(blen / dec_s / 1e6, 1),
            "enc_G_int32_per_s": round(n / enc_s / 1e9, 3)}


def run_c1(args, world, rank, dev, T):
    """configs[0]: p4Enc32/p4Dec32 with n = 127, bit width 8, no exceptions
    (values uniform in [0, 255] as ab_test.cpp:1610-1631).  Device: a batch of
    nblocks such blocks, encoded and decoded by the horizontal-format kernels
    (tpf_enc_batch / tpf_dec_batch, TPF_FMT_32)."""
    n = 127
    nb = args.nblocks
    vals = bench_data.gen_c1(nb, n, seed=42, dev=dev, first_block=shard_of(nb, world, rank))
    packed, offs = tpf.enc_batch("32", vals, nb, n)
    out = torch.empty_like(vals)
    elapsed, kern_ms = T.run(lambda: tpf.dec_batch("32", packed, offs, nb, n, out=out), args.steps, args.warmup)
    ok = bool(torch.equal(out, vals))
    _, enc_ms = T.run(lambda: tpf.enc_batch("32", vals, nb, n), max(2, args.steps // 4), 1)
    pbytes = int(packed.numel())
    avg_ms = float(np.mean(kern_ms))
    alg = pbytes + nb * (n * 4 + 8) + 8
    per_rank = per_rank_stats(world, dev, avg_ms, alg / (avg_ms * 1e-3) / 1e9)
    if rank != 0:
        return None
    value = nb * n * world / (elapsed / args.steps) / 1e9
    roof = {"bound": "hbm", "achieved": round(alg / (avg_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(alg / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), **traffic_fields("c1", nb),
            "kernel_ms_avg": round(avg_ms, 4),
            "kernel": "tpf::dev::k_dec_h32w (windowed horizontal p4Dec32 batch: 64-block wave runs, windows staged whole, lane-parsed headers)",
            "per_rank": per_rank}
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        blen = int(offs[1].item())
        blk = np.concatenate([packed[:blen].cpu().numpy(), np.zeros(64, np.uint8)])  # + the reference's read slack
        cpu = cpu_abtest_c1(vals[:n].cpu().numpy().view(np.uint32).copy(), blk, blen, n)
    cfg = {"workload": "C1: p4Enc32/p4Dec32, n=127, bw 8, 0% exceptions (configs[0]); device batch of n=127 blocks",
           "nblocks_per_gpu": nb, "bytes_per_block": round(pbytes / nb, 2), "verified": ok,
           "enc32_G_int32_per_s": round(nb * n / (float(np.mean(enc_ms)) * 1e-3) / 1e9, 2), "parallelism": f"shard{world}"}
    return line("G int32/s device-resident p4Dec32 (n=127)", value, "G int32/s", world, args.steps, args.warmup,
                elapsed, "u32", "synthetic (GPU-generated uniform [0,255], GPU-encoded)", cfg, roof, cpu), ok


# ------------------------------------------------------------ launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """--gpus N > 1 without a launcher: run this script under
    torch.distributed.run with N ranks (one per GPU) as a CHILD process --
    nothing here has touched a GPU, and the parent never execs -- and return
    its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] launching {n} ranks: {' '.join(cmd[1:6])} ...")
    return subprocess.call(cmd)


def run_selftest(args, world, rank, dev, T):
    """Launcher / process group / timing plumbing with a CPU stand-in step
    (an integer reduction over a per-rank array; no GPU, no codec): the line
    it prints is marked selftest and carries no throughput claim."""
    x = torch.arange(1 << 20, dtype=torch.int64) + rank
    elapsed, step_ms = T.run(lambda: int(x.sum()), args.steps, args.warmup)
    per_rank = per_rank_stats(world, dev, float(np.mean(step_ms)), 0.0)
    if rank != 0:
        return None
    res = line("selftest (CPU stand-in step, no codec)", 0.0, "none", world, args.steps, args.warmup, elapsed, "int64",
               "synthetic", {"workload": "selftest", "parallelism": f"shard{world}",
                             "world_size": torch.distributed.get_world_size() if T.dist_on else 1,
                             "backend": torch.distributed.get_backend() if T.dist_on else None})
    res["selftest"] = True
    res["per_rank"] = per_rank
    return res, True


# -------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--nblocks", type=int, default=10_000_000, help="blocks per GPU (shard)")
    ap.add_argument("--exc", type=float, default=10.0)
    ap.add_argument("--workload", default="c2", choices=["c1", "c2", "c3", "c3chain", "c3enc", "c3chain64", "c4", "c5", "sweep"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e", action="store_true", help="c2: also measure the pinned host-memory path")
    ap.add_argument("--no-probes", action="store_true", help="c2: skip the in-run HBM read/write/copy probes")
    ap.add_argument("--selftest", action="store_true",
                    help="launcher + process-group plumbing with a CPU stand-in step (gloo, no GPU)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    # under a launcher (WORLD_SIZE set) the process group is used even at
    # world size 1, so `torch.distributed.run --nproc-per-node 1` exercises the
    # RCCL init, barrier, all_gather and all_reduce on a one-GPU box (RCCL
    # refuses two ranks on one device: "Duplicate GPU detected")
    dist_on = world > 1 or "WORLD_SIZE" in os.environ
    # Rehearsal of the multi-rank path on a one-GPU box (never the measured
    # configuration): TPF_BENCH_SAME_GPU=1 puts every rank on cuda:0;
    # TPF_BENCH_BACKEND=gloo carries the collectives over gloo instead of RCCL.
    backend = os.environ.get("TPF_BENCH_BACKEND", "gloo" if args.selftest else "nccl")
    if os.environ.get("TPF_BENCH_SAME_GPU") == "1":
        local = 0
    if args.selftest:
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(local)
        dev = torch.device(f"cuda:{local}")
    if dist_on:
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group(backend)
        assert torch.distributed.get_world_size() == args.gpus == world, "world size != --gpus"
    T = Timer(dist_on, dev)
    if args.selftest:
        res = run_selftest(args, world, rank, dev, T)
    elif args.workload == "c1":
        res = run_c1(args, world, rank, dev, T)
    elif args.workload == "c2":
        res = run_c2(args, world, rank, dev, T)
    elif args.workload == "c5":
        res = run_c2(args, world, rank, dev, T, c5=True)
    elif args.workload == "c3":
        res = run_c3(args, world, rank, dev, T, chained=False)
    elif args.workload == "c3chain":
        res = run_c3(args, world, rank, dev, T, chained=True)
    elif args.workload == "c3enc":
        res = run_c3enc(args, world, rank, dev, T)
    elif args.workload == "c3chain64":
        res = run_c3chain64(args, world, rank, dev, T)
    elif args.workload == "sweep":
        res = run_sweep(args, world, rank, dev, T)
    else:
        res = run_c4(args, world, rank, dev, T)
    ok = True
    if res is not None:
        result, ok = res
        print(json.dumps(result), flush=True)
    if dist_on:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    if rank == 0 and not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
