"""Pins the C restatement (oracle/liborc.so) to the REFERENCE's own scalar
codec (oracle/_ref/libtpref.so, compiled from /root/reference/src) on the
distributions the GPU tests and bench.py use, at >= 100k blocks each:

  * C2 / C4-32: datagen.c2_blocks, every bit width 1..32 x 0/5/10/25 %
    exceptions (benchmarks/ab_test.cpp:1610-1631)
  * C3: datagen.c3_postings (Zipf posting lists), delta-1 with per-block
    starts taken from the list (chained) and with independent random starts
  * C4-64: 256v64 blocks, bit widths 1..64, exceptions above bit 32

Encoder bytes must be identical and both decoders must return the input and
end every block exactly at its offset.  The GPU-vs-oracle tests on the same
generators are thereby pinned to the reference transitively (reference:
src/scalar/p4enc256v32_scalar.cpp:216-235, p4dec256v32_scalar.cpp:90-137,
p4d1dec256v32_scalar.cpp:198-268, p4enc256v64_scalar.cpp:15-30).
Skipped where oracle/_ref was not built (no /root/reference)."""
import ctypes

import numpy as np
import pytest

import datagen
import oracle_lib
import ref_lib

pytestmark = pytest.mark.skipif(not ref_lib.available(), reason="oracle/_ref not built")

u8p, u32p, u64p = ref_lib.u8p, ref_lib.u32p, ref_lib.u64p


def _ref():
    L = ref_lib.lib()
    for w, vp in (("32", u32p), ("64", u64p)):
        f = getattr(L, f"tpref_s_enc256v{w}_batch")
        f.argtypes = [vp, ctypes.c_uint64, vp, u8p, u64p]
        f.restype = ctypes.c_uint64
        g = getattr(L, f"tpref_s_dec256v{w}_batch")
        g.argtypes = [u8p, u64p, ctypes.c_uint64, vp, vp]
        g.restype = ctypes.c_int64
    return L


def _p(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def ref_roundtrip(vals, starts=None):
    """Reference scalar: encode (packed, off) and decode back (values, bad block or -1)."""
    L = _ref()
    wide = vals.dtype == np.uint64
    vp = u64p if wide else u32p
    nb = vals.shape[0]
    out = np.zeros(nb * (2400 if wide else 1100) + 4096, np.uint8)
    off = np.zeros(nb + 1, np.uint64)
    st = None if starts is None else np.ascontiguousarray(starts)
    enc = L.tpref_s_enc256v64_batch if wide else L.tpref_s_enc256v32_batch
    dec = L.tpref_s_dec256v64_batch if wide else L.tpref_s_dec256v32_batch
    tot = enc(_p(vals, vp), nb, _p(st, vp), _p(out, u8p), _p(off, u64p))
    packed = out[:tot].copy()
    src = np.concatenate([packed, np.zeros(64, np.uint8)])
    back = np.zeros((nb + 1, 256), vals.dtype)
    bad = dec(_p(src, u8p), _p(off, u64p), nb, _p(st, vp), _p(back, vp))
    return packed, off, back[:nb], bad


def check(vals, starts=None):
    vals = np.ascontiguousarray(vals)
    rp, roff, rback, rbad = ref_roundtrip(vals, starts)
    assert rbad == -1, f"reference decoder end pointer off at block {rbad}"
    np.testing.assert_array_equal(rback, vals)
    if vals.dtype == np.uint64:
        op, ooff = oracle_lib.enc256v64_batch(vals, starts=starts)
        oback = oracle_lib.dec256v64_batch(rp, roff, len(vals), starts=starts)
    else:
        op, ooff = oracle_lib.enc256v32_batch(vals, starts=starts)
        oback = oracle_lib.dec256v32_batch(rp, roff, len(vals), starts=starts)
    np.testing.assert_array_equal(ooff.astype(np.uint64), roff)
    if not np.array_equal(op, rp):
        i = int(np.argmax(op[: len(rp)] != rp[: len(op)]))
        blk = int(np.searchsorted(roff, i, side="right")) - 1
        pytest.fail(f"oracle bytes differ from the reference at byte {i} (block {blk})")
    np.testing.assert_array_equal(oback, vals)
    return len(vals)


def test_c2_every_width_and_rate():
    """C2 and the C4 32-bit mix: 32 widths x 4 exception rates x 800 blocks = 102,400 blocks."""
    total = 0
    for pct in (0, 5, 10, 25):
        blocks = np.concatenate([datagen.c2_blocks(800, bw, pct, seed=42 + pct) for bw in range(1, 33)])
        total += check(blocks)
    assert total >= 100_000


@pytest.mark.parametrize("mode", ["chained", "random_starts"])
def test_c3_postings(mode):
    """C3 Zipf posting lists, 100,000 blocks, p4D1Enc256v32/p4D1Dec256v32."""
    vals, starts = datagen.c3_postings(100_000, seed=7)
    if mode == "random_starts":
        rng = np.random.default_rng(3)
        starts = rng.integers(0, 1 << 32, size=len(vals), dtype=np.uint64).astype(np.uint32)
    assert check(vals, starts) >= 100_000


def _c4_blocks64(nblocks, bw, pct, rng):
    """bw-bit base values; with probability pct an exception whose top bit is in 33..64."""
    n = nblocks * 256
    v = rng.integers(0, 1 << 63, size=n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, size=n, dtype=np.uint64)
    if bw < 64:
        v &= np.uint64((1 << bw) - 1)
        if pct:
            m = rng.random(n) < pct / 100.0
            hi = rng.integers(max(33, bw + 1), 65, size=int(m.sum()))
            e = rng.integers(0, 1 << 63, size=int(m.sum()), dtype=np.uint64) * np.uint64(2) + np.uint64(1)
            e >>= (64 - hi).astype(np.uint64)
            e |= np.uint64(1) << (hi - 1).astype(np.uint64)
            v[m] = e
    return v.reshape(nblocks, 256)


def test_c4_64bit_every_width():
    """C4 64-bit: widths 1..64 x 1,600 blocks (102,400 blocks), 10 % exceptions above bit 32."""
    rng = np.random.default_rng(64)
    blocks = np.concatenate([_c4_blocks64(1600, bw, 10, rng) for bw in range(1, 65)])
    assert check(blocks) >= 100_000
    # delta-1 over sorted 64-bit lists, gaps up to 2^40
    g = rng.integers(1, 1 << 40, size=20_000 * 256, dtype=np.uint64)
    lst = np.cumsum(g).astype(np.uint64).reshape(20_000, 256)
    starts = np.concatenate([[np.uint64(5)], lst[:-1, -1]]).astype(np.uint64)
    check(lst, starts)
