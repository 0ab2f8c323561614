#!/usr/bin/env python3
"""bench.py -- device-resident p4Dec256v32 throughput on MI355X.

Workload (BASELINE.json configs[1], "C2"): 10M blocks of 256 uint32, bit
widths 1..32 swept as 32 equal consecutive segments, 10% exceptions (bw<=28,
benchmarks/ab_test.cpp:1448/1610-1631), synthetic data generated on the GPU.
The packed stream is produced by our GPU encoder (untimed) and verified by a
full-size round trip after the timed region.  One step = one
tpf_p4dec256v32_batch launch over the whole shard (inputs resident in HBM).

Multi-GPU (torchrun, one process per GPU): every rank decodes its own 10M-block
shard (weak scaling, no collective on the data path); RCCL only carries the
barrier and the max-over-ranks time.

Prints ONE JSON line on rank 0 (see the driver contract in the task prompt),
with a `roofline` object for the decode kernel and a `cpu_baseline` object
(the reference library compiled from /root/reference, run on this host's CPU
on a bounded sample of the same workload).
"""
import argparse
import ctypes
import glob
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
import turbopfor_amd as tpf  # noqa: E402

METRIC = "G int32/s device-resident p4Dec256v32 (+ compressed GB/s vs HBM peak)"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# --------------------------------------------------------------- data (GPU)
def gen_c2(nblocks, exc_pct, seed, dev):
    """uint32 bit patterns (as int32) [nblocks, 256]; 32 equal segments, bw 1..32."""
    vals = torch.empty((nblocks, 256), dtype=torch.int32, device=dev)
    seg = [(nblocks * s) // 32 for s in range(33)]
    g = torch.Generator(device=dev)
    for s in range(32):
        bw = s + 1
        lo, hi = seg[s], seg[s + 1]
        if hi <= lo:
            continue
        g.manual_seed(seed * 1000 + bw)
        n = (hi - lo) * 256
        v = torch.randint(0, 1 << bw, (n,), device=dev, generator=g, dtype=torch.int64)
        if exc_pct > 0 and bw <= 28:
            m = torch.rand(n, device=dev, generator=g) < (exc_pct / 100.0)
            e = torch.randint(1 << bw, 1 << 32, (n,), device=dev, generator=g, dtype=torch.int64)
            v = torch.where(m, e, v)
            del m, e
        vals[lo:hi] = (v - ((v >> 31) << 32)).to(torch.int32).view(hi - lo, 256)
        del v
    return vals, seg


# --------------------------------------------------------- profile traffic
def pmc_traffic(nblocks):
    """HBM bytes per decode launch from the committed rocprofv3 PMC passes
    (profiles/*pmc*.csv), corrected as MI355X_MICROARCH.md §HBM prescribes:
    FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half of a
    wide coalesced stream, so it is doubled.  Returns None when no matching
    profile exists."""
    fetch, write = None, None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*_counter_collection.csv"))):
        try:
            import csv

            with open(path) as f:
                rows = [r for r in csv.DictReader(f) if "k_dec256v32" in r.get("Kernel_Name", "")]
        except Exception:
            continue
        for name in ("FETCH_SIZE", "WRITE_SIZE"):
            vals = [float(r["Counter_Value"]) for r in rows if r.get("Counter_Name") == name]
            if vals:
                med = float(np.median(vals))
                if name == "FETCH_SIZE":
                    fetch = med
                else:
                    write = med
    if fetch is None or write is None:
        return None
    return (2.0 * fetch + write) * 1024.0


# ------------------------------------------------------------- cpu baseline
def cpu_baseline(packed_host, off_host, nblocks, budget_s=12.0, threads=None):
    """Reference library (oracle/_ref, compiled from the reference sources,
    turbopfor::p4Dec256v32 = AVX2 dispatch path) decoding a bounded sample of
    the same packed stream with `threads` std::threads; falls back to the
    oracle restatement (kind "port") when _ref is absent."""
    threads = threads or min(16, os.cpu_count() or 1)
    # sample: the first 1/16 of every bw segment (contiguous bytes per segment)
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
    idx = np.arange(len(soff) - 1)
    nb = len(idx)
    out = np.empty((nb, 256), dtype=np.uint32)
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libtpref.so")
    u8p, u32p, u64p = (ctypes.POINTER(t) for t in (ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint64))
    if os.path.exists(ref_so):
        L = ctypes.CDLL(ref_so)
        f = L.tpref_dec256v32_stream_mt
        f.argtypes = [u8p, u64p, ctypes.c_uint64, u32p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        f.restype = ctypes.c_double
        run = lambda: f(sample.ctypes.data_as(u8p), soff.ctypes.data_as(u64p), nb, out.ctypes.data_as(u32p),
                        threads, 1, 0)
        kind = "reference"
    else:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib

        L = oracle_lib.lib()

        def run():
            t0 = time.perf_counter()
            L.orc_dec256v32_batch_mt(sample.ctypes.data_as(u8p), soff.ctypes.data_as(u64p), nb,
                                     out.ctypes.data_as(u32p), threads)
            return time.perf_counter() - t0

        kind = "port"
    run()  # warm
    tot, reps = 0.0, 0
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < budget_s:
        tot += run()
        reps += 1
    value = nb * 256 * reps / tot / 1e9
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        model = "unknown"
    return {
        "value": round(value, 3),
        "unit": "G int32/s",
        "cores": threads,
        "kind": kind,
        "sample": f"{nb} blocks (first 1/16 of each bw segment of the same C2 stream), {reps} passes, "
                  f"{threads} threads, turbopfor::p4Dec256v32 (AVX2 dispatch) on {model}",
    }


# -------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--nblocks", type=int, default=10_000_000, help="blocks per GPU (shard)")
    ap.add_argument("--exc", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sweep", action="store_true", help="also time each bw segment (stderr table)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        torch.cuda.set_device(local)
        import torch.distributed as td

        td.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    nb = args.nblocks

    t0 = time.time()
    vals, seg = gen_c2(nb, args.exc, seed=42 + rank, dev=dev)
    packed_full, offs = tpf.enc256v32(vals)
    packed = packed_full.clone()
    del packed_full
    torch.cuda.synchronize()
    packed_bytes = packed.numel()
    if rank == 0:
        log(f"[bench] generated+encoded {nb} blocks in {time.time() - t0:.1f}s, packed {packed_bytes / 1e9:.3f} GB "
            f"({packed_bytes / nb:.1f} B/block)")
    out = torch.empty((nb, 256), dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int64, device=dev)

    for _ in range(args.warmup):
        tpf.dec256v32(packed, offs, nb, out=out)
    torch.cuda.synchronize()
    if dist:
        td.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t_start = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        tpf.dec256v32(packed, offs, nb, out=out)
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    if dist:
        td.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    kern_ms = [a.elapsed_time(b) for a, b in evs]
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        td.all_reduce(t, op=td.ReduceOp.MAX)
        elapsed = float(t.item())

    # full-size correctness: decode with the consistency check, compare all values
    tpf.dec256v32(packed, offs, nb, out=out, err=err)
    ok = bool(torch.equal(out, vals)) and int(err.item()) == -1
    if dist:
        okt = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        td.all_reduce(okt, op=td.ReduceOp.MIN)
        ok = bool(okt.item())

    sweep_rows = []
    if args.sweep and rank == 0:
        off_host = offs.cpu().numpy()
        for s in range(32):
            lo, hi = seg[s], seg[s + 1]
            sub_in = packed[int(off_host[lo]) : int(off_host[hi])]
            sub_off = offs[lo : hi + 1] - int(off_host[lo])
            sub_out = out[lo:hi]
            for _ in range(2):
                tpf.dec256v32(sub_in, sub_off, hi - lo, out=sub_out)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                tpf.dec256v32(sub_in, sub_off, hi - lo, out=sub_out)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            nbytes = int(off_host[hi] - off_host[lo])
            gint = (hi - lo) * 256 / ms / 1e6
            gbs = (nbytes + (hi - lo) * 1032) / ms / 1e6
            sweep_rows.append((s + 1, nbytes / (hi - lo), ms, gint, gbs))
            log(f"[sweep] bw={s + 1:2d} B/blk={nbytes / (hi - lo):7.1f} ms={ms:.4f} Gint/s={gint:8.1f} "
                f"alg GB/s={gbs:7.1f} ({gbs / HBM_PEAK_GBS:.1%} of peak)")

    result = None
    if rank == 0:
        steps = args.steps
        ms_per_step = elapsed * 1000.0 / steps
        total_ints = nb * 256 * world
        value = total_ints / elapsed * steps / 1e9  # whole-job G int32/s
        avg_kern_ms = float(np.mean(kern_ms))
        alg_bytes = packed_bytes + nb * (1024 + 8) + 8
        achieved = alg_bytes / (avg_kern_ms * 1e-3) / 1e9
        traffic = pmc_traffic(nb)
        roofline = {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel": "tpf::dev::k_dec256v32<StartMode::None>",
            "kernel_ms_avg": round(avg_kern_ms, 4),
            "alg_bytes_per_launch": int(alg_bytes),
        }
        cpu = None
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(packed.cpu().numpy(), offs.cpu().numpy().astype(np.uint64), nb)
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "G int32/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (GPU-generated C2 values, GPU-encoded; full-size decode verified bit-exact: "
                    + ("ok" if ok else "MISMATCH") + ")",
            "config": {
                "workload": "C2: p4Dec256v32, 10M blocks x 256 u32 per GPU, bw 1..32 sweep (32 equal segments), "
                            "10% exceptions for bw<=28",
                "nblocks_per_gpu": nb,
                "packed_bytes_per_gpu": packed_bytes,
                "bytes_per_block": round(packed_bytes / nb, 1),
                "compressed_GBps": round(packed_bytes * world / (elapsed / steps) / 1e9, 1),
                "parallelism": f"shard{world}",
                "verified": ok,
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    if dist:
        td.barrier()
        td.destroy_process_group()
    if rank == 0 and not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
