"""Synthetic inputs shaped like BASELINE.json's configs (numpy, seeded).

C2 / C4: base values U[0, 2^bw), each value an exception with probability
pct, exceptions U[2^bw, 2^32) (benchmarks/ab_test.cpp:1610-1631; exceptions
only for bw <= 28, ab_test.cpp:1448).  C3: sorted posting lists, 95% gaps from a
bounded continuous Zipf(s=1.1) on [1, 64], 5% gaps 64 + U[0, 2^16)."""
import numpy as np


def c2_blocks(nblocks, bw, exc_pct, seed=42):
    rng = np.random.default_rng(seed + bw)
    n = nblocks * 256
    if bw >= 32:
        v = rng.integers(0, 1 << 32, size=n, dtype=np.uint64)
    else:
        v = rng.integers(0, 1 << bw, size=n, dtype=np.uint64)
        if exc_pct > 0 and bw <= 28:
            m = rng.random(n) < exc_pct / 100.0
            v[m] = rng.integers(1 << bw, 1 << 32, size=int(m.sum()), dtype=np.uint64)
    return v.astype(np.uint32).reshape(nblocks, 256)


def zipf_gaps(n, rng):
    s, a, b = 1.1, 1.0, 65.0
    u = rng.random(n)
    x = (a ** (1 - s) + u * (b ** (1 - s) - a ** (1 - s))) ** (1.0 / (1 - s))
    g = np.clip(np.floor(x), 1, 64).astype(np.uint64)
    big = rng.random(n) < 0.05
    g[big] = 64 + rng.integers(0, 1 << 16, size=int(big.sum()), dtype=np.uint64)
    return g


def c3_postings(nblocks, seed=7):
    """Sorted docIDs (mod 2^32) in blocks of 256 + per-block starts (the value
    preceding each block; start of block 0 = 0)."""
    rng = np.random.default_rng(seed)
    g = zipf_gaps(nblocks * 256, rng)
    vals = (np.cumsum(g) & 0xFFFFFFFF).astype(np.uint32).reshape(nblocks, 256)
    starts = np.zeros(nblocks, dtype=np.uint32)
    starts[1:] = vals[:-1, -1]
    return vals, starts


def c4_blocks64(nblocks, bw, exc_pct, seed=11, hi=64):
    rng = np.random.default_rng(seed + bw)
    n = nblocks * 256
    top = (1 << bw) if bw < 64 else None
    if top is None:
        v = rng.integers(0, 1 << 63, size=n, dtype=np.uint64) * 2 + rng.integers(0, 2, size=n, dtype=np.uint64)
    else:
        v = rng.integers(0, top, size=n, dtype=np.uint64)
        if exc_pct > 0 and bw < hi:
            m = rng.random(n) < exc_pct / 100.0
            k = int(m.sum())
            lo = 1 << bw
            span_hi = (1 << hi) if hi < 64 else (1 << 64)
            e = (rng.integers(0, 1 << 62, size=k, dtype=np.uint64).astype(object) * 4 % (span_hi - lo) + lo)
            v[m] = np.array([int(x) for x in e], dtype=np.uint64)
    return v.reshape(nblocks, 256)
