"""Synthetic workloads of bench.py (BASELINE.json configs, SURVEY.md §8 d),
generated from a counter-based generator keyed by the GLOBAL element index,
so that every rank of a multi-GPU run holds a slice of ONE global stream and
regenerates it independently (SURVEY.md §8 d: "a counter-based generator ...
so shards regenerate independently").  Torch ops only: the same code runs on
a HIP device (bench) and on the CPU (gloo tests); integer results are
identical on both (tests/test_bench_data_cpu.py, tests/test_gpu_chained.py).

Generator: splitmix64 (Steele, Lea, Flood 2014) of (index * golden + key),
with int64 wrap-around arithmetic and logical shifts written as masks.

Global streams:
  C2 / C5 / sweep  the per-GPU pattern (bw segments) repeats every `period`
                   blocks of the global stream -- weak scaling keeps every
                   rank's shard one period long -- with fresh values in every
                   period (keys: global element index).
  C3 (chained)     ONE sorted posting list over all ranks: gaps are keyed by
                   the global element index, values = start0 + prefix of all
                   gaps, so rank r's first value continues rank r-1's last;
                   the cross-rank carry (sum of every earlier shard's gaps) is
                   an all-gather of one int64 per rank (generation only,
                   outside any timed region).
"""
import torch

GOLDEN = 0x9E3779B97F4A7C15 - (1 << 64)
C1 = 0xBF58476D1CE4E5B9 - (1 << 64)
C2 = 0x94D049BB133111EB - (1 << 64)
KEYMUL = 0xD1B54A32D192ED03 - (1 << 64)
CHUNK = 64 << 20  # elements per generation step


def _srl(x, k):
    """Logical shift right of int64 bit patterns."""
    return (x >> k) & ((1 << (64 - k)) - 1)


def rand64(idx, key):
    """splitmix64 of global indices (int64 tensor) under `key`: int64 bit patterns."""
    z = idx * GOLDEN + (key * KEYMUL & 0x7FFFFFFFFFFFFFFF)
    z = (z ^ _srl(z, 30)) * C1
    z = (z ^ _srl(z, 27)) * C2
    return z ^ _srl(z, 31)


def _u24(r):
    """24-bit uniform integer from the high half."""
    return _srl(r, 40)


def as_i32(v64):
    """uint32 values held in int64 -> int32 bit patterns."""
    return (v64 - ((v64 >> 31) << 32)).to(torch.int32)


def fill_bw(flat, e0, bw, exc_pct, key):
    """flat[k] (int32 view) for global elements e0+k: uniform [0, 2^bw), with
    probability exc_pct % (bw <= 28) an exception uniform in [2^bw, 2^32)
    (benchmarks/ab_test.cpp:1606-1632, :1448)."""
    dev = flat.device
    n = flat.numel()
    for a in range(0, n, CHUNK):
        m = min(CHUNK, n - a)
        idx = torch.arange(e0 + a, e0 + a + m, dtype=torch.int64, device=dev)
        r = rand64(idx, key)
        v = r & ((1 << bw) - 1) if bw < 32 else r & 0xFFFFFFFF
        if exc_pct > 0 and bw <= 28:
            thr = int(exc_pct / 100.0 * (1 << 24))
            r2 = rand64(idx, key + 1)
            e = (1 << bw) + torch.remainder(r2 & 0xFFFFFFFF, (1 << 32) - (1 << bw))
            v = torch.where(_u24(r2) < thr, e, v)
            del r2, e
        flat[a:a + m] = as_i32(v)
        del idx, r, v


def segments(n):
    return [(n * s) // 32 for s in range(33)]


def gen_c2(nblocks, exc_pct, seed, dev, pcts=None, first_block=0):
    """[nblocks, 256] int32 bit patterns: blocks [first_block, first_block +
    nblocks) of the global C2 stream whose period is nblocks: 32 equal
    segments with bw 1..32, exceptions with probability exc_pct (or pcts
    cycling per segment) for bw <= 28.  Returns (values, segment bounds)."""
    vals = torch.empty((nblocks, 256), dtype=torch.int32, device=dev)
    seg = segments(nblocks)
    for s in range(32):
        lo, hi = seg[s], seg[s + 1]
        if hi <= lo:
            continue
        pct = pcts[s % len(pcts)] if pcts else exc_pct
        fill_bw(vals[lo:hi].view(-1), (first_block + lo) * 256, s + 1, pct, seed * 1000 + s + 1)
    return vals, seg


def gen_bw(nblocks, bw, exc_pct, seed, dev, first_block=0):
    """[nblocks, 256] int32 bit patterns of ONE bit width (blocks
    [first_block, first_block + nblocks) of that width's global stream)."""
    vals = torch.empty((nblocks, 256), dtype=torch.int32, device=dev)
    fill_bw(vals.view(-1), first_block * 256, bw, exc_pct, seed * 1000 + bw)
    return vals


def gen_c5(nblocks, exc_pct, seed, dev, first_block=0):
    """C5 shard (SURVEY.md §8 d: 80M blocks as 8 x 10M shards, bw 8 and 16 at
    10% exceptions): in every nblocks-block period the first half bw 8, the
    rest bw 16."""
    h = nblocks // 2
    vals = torch.empty((nblocks, 256), dtype=torch.int32, device=dev)
    fill_bw(vals[:h].view(-1), first_block * 256, 8, exc_pct, seed * 1000 + 8)
    fill_bw(vals[h:].view(-1), (first_block + h) * 256, 16, exc_pct, seed * 1000 + 16)
    return vals


def c3_gaps(e0, m, seed, dev):
    """Gaps of global elements [e0, e0+m) of the C3 posting list (BASELINE.md
    C3): 95% bounded Zipf(s=1.1) on [1, 64] (floored), 5% 64 + U[0, 2^16)."""
    idx = torch.arange(e0, e0 + m, dtype=torch.int64, device=dev)
    r = rand64(idx, seed * 1000 + 901)
    u = _srl(r, 11).to(torch.float64) * (1.0 / (1 << 53))
    s = 1.1
    x = (1.0 + u * (65.0 ** (1 - s) - 1.0)) ** (1.0 / (1 - s))
    gap = torch.clamp(torch.floor(x), 1, 64).to(torch.int64)
    r2 = rand64(idx, seed * 1000 + 902)
    big = _u24(r2) < int(0.05 * (1 << 24))
    return torch.where(big, 64 + (r2 & 0xFFFF), gap)


def gen_c3(nblocks, seed, dev, first_block=0, carry_fn=None, start0=0):
    """Blocks [first_block, first_block + nblocks) of ONE sorted posting list
    (value of global element e = start0 + sum of gaps 0..e, mod 2^32).
    carry_fn(local_gap_total) -> sum of the gaps of every element before
    first_block*256 (a cross-rank all-gather; None: a single-rank list, so
    first_block must be 0).  Returns (values [nblocks,256] int32, per-block
    starts [nblocks] int32: the value preceding each block; the last value of
    the previous shard for block 0)."""
    n = nblocks * 256
    e0 = first_block * 256
    vals = torch.empty(n, dtype=torch.int32, device=dev)
    run = 0  # gaps of this shard so far
    for a in range(0, n, CHUNK):
        m = min(CHUNK, n - a)
        cs = torch.cumsum(c3_gaps(e0 + a, m, seed, dev), 0) + run
        run = int(cs[-1].item())
        vals[a:a + m] = as_i32(cs & 0xFFFFFFFF)
        del cs
    if carry_fn is None:
        assert first_block == 0, "a shard past block 0 needs the carry of the earlier shards"
        before = 0
    else:
        before = int(carry_fn(run))
    base = (start0 + before) & 0xFFFFFFFF
    if base:
        for a in range(0, n, CHUNK):
            m = min(CHUNK, n - a)
            vals[a:a + m] = as_i32((vals[a:a + m].to(torch.int64) + base) & 0xFFFFFFFF)
    vals = vals.view(nblocks, 256)
    starts = torch.empty(nblocks, dtype=torch.int32, device=dev)
    starts[0] = as_i32(torch.tensor([base], dtype=torch.int64))[0]
    starts[1:] = vals[:-1, -1]
    return vals, starts


def gen_c3_64(nunits, seed, dev, first_block=0, carry_fn=None, start0=(1 << 40) + 12345):
    """The C3 posting list as 64-bit ids (p4D1Enc256v64 units of 256): the
    same gaps as gen_c3, values start0 + sum of gaps 0..e (no 2^32 wrap; the
    default start0 puts every id above 2^32).  Returns (values [nunits,256]
    int64, per-unit starts [nunits] int64: the value preceding each unit)."""
    n = nunits * 256
    e0 = first_block * 256
    vals = torch.empty(n, dtype=torch.int64, device=dev)
    run = 0
    for a in range(0, n, CHUNK):
        m = min(CHUNK, n - a)
        vals[a:a + m] = torch.cumsum(c3_gaps(e0 + a, m, seed, dev), 0) + run
        run = int(vals[a + m - 1].item())
    if carry_fn is None:
        assert first_block == 0, "a shard past unit 0 needs the carry of the earlier shards"
        before = 0
    else:
        before = int(carry_fn(run))
    base = start0 + before
    vals += base
    vals = vals.view(nunits, 256)
    starts = torch.empty(nunits, dtype=torch.int64, device=dev)
    starts[0] = base
    starts[1:] = vals[:-1, -1]
    return vals, starts


def gen_c1(nblocks, n, seed, dev, first_block=0):
    """configs[0]: n-value blocks uniform in [0, 255] (ab_test.cpp:1610-1631)."""
    vals = torch.empty(nblocks * n, dtype=torch.int32, device=dev)
    for a in range(0, vals.numel(), CHUNK):
        m = min(CHUNK, vals.numel() - a)
        idx = torch.arange(first_block * n + a, first_block * n + a + m, dtype=torch.int64, device=dev)
        vals[a:a + m] = (rand64(idx, seed * 1000 + 127) & 0xFF).to(torch.int32)
    return vals


def gen_v64(nblocks, seed, dev, first_block=0, pcts=(0, 5, 10, 25)):
    """C4's 64-bit leg ([nblocks, 256] int64 bit patterns of uint64), after
    the reference's 256v64 round-trip patterns (tests/test_p4_64.cpp:587-611,
    fillWithExceptions64 test_helpers.h:142-155: "_32b" exceptions that fit
    in 32 bits and "_64b" exceptions at 2^32 and above): 64 equal segments
    with bw 1..64, exception rates cycling over pcts; an exception's top bit
    is drawn in [bw, 32) in even segments with bw < 32 (32-bit exceptions)
    and in [max(bw, 32), 64) otherwise (exceptions above bit 32), lower bits
    random."""
    vals = torch.empty((nblocks, 256), dtype=torch.int64, device=dev)
    seg = [(nblocks * s) // 64 for s in range(65)]
    for s in range(64):
        lo, hi = seg[s], seg[s + 1]
        if hi <= lo:
            continue
        bw = s + 1
        pct = pcts[s % len(pcts)]
        flat = vals[lo:hi].view(-1)
        e0 = (first_block + lo) * 256
        key = seed * 1000 + 400 + bw
        t_lo, t_hi = (bw, 32) if (s % 2 == 0 and bw < 32) else (max(bw, 32), 64)
        for a in range(0, flat.numel(), CHUNK):
            m = min(CHUNK, flat.numel() - a)
            idx = torch.arange(e0 + a, e0 + a + m, dtype=torch.int64, device=dev)
            r = rand64(idx, key)
            v = r if bw == 64 else r & ((1 << bw) - 1)
            if pct > 0 and bw < 64:
                r2 = rand64(idx, key + 1)
                top = torch.remainder(_srl(r2, 40), t_hi - t_lo) + t_lo
                bit = torch.bitwise_left_shift(torch.ones_like(top), top)
                e = (rand64(idx, key + 2) & (bit - 1)) | bit
                v = torch.where(_u24(r2) < int(pct / 100.0 * (1 << 24)), e, v)
                del r2, top, bit, e
            flat[a:a + m] = v
            del idx, r, v
    return vals
