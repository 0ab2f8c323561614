"""GPU parity of the 256v32 batch decoder (p4Dec256v32 / p4D1Dec256v32)
against the golden fixtures (reference src/scalar outputs) and the CPU
restatement in oracle/.  Bit-exact."""
import numpy as np
import pytest

import datagen
import golden_io
import oracle_lib

torch = pytest.importorskip("torch")
tpf = pytest.importorskip("turbopfor_amd")

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
U64MAX = (1 << 64) - 1


def to_dev_stream(blobs, pad_front=0):
    offs = np.zeros(len(blobs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(b) for b in blobs])
    buf = np.frombuffer(b"".join(blobs), dtype=np.uint8)
    full = np.zeros(pad_front + len(buf), dtype=np.uint8)
    full[pad_front:] = buf
    t = torch.from_numpy(full).to(DEV)
    return t[pad_front:], torch.from_numpy(offs).to(DEV)


def as_u32(t):
    return t.cpu().numpy().view(np.uint32)


def assert_blocks_equal(got, exp, what=""):
    got = np.asarray(got).reshape(-1, 256)
    exp = np.asarray(exp).reshape(-1, 256)
    bad = np.nonzero((got != exp).any(axis=1))[0]
    if len(bad):
        i = int(bad[0])
        j = np.nonzero(got[i] != exp[i])[0]
        raise AssertionError(f"{what}: {len(bad)} bad blocks of {len(exp)}, first block {i}, elements {j[:8].tolist()} "
                             f"got {[hex(int(x)) for x in got[i][j[:4]]]} exp {[hex(int(x)) for x in exp[i][j[:4]]]}")


def test_golden_256v32():
    recs = [r for r in golden_io.load("g256v32.bin") if r.n == 256]
    for d1 in (False, True):
        sel = [r for r in recs if r.d1 == d1]
        packed, offs = to_dev_stream([r.enc for r in sel])
        err = torch.zeros(1, dtype=torch.int64, device=DEV)
        starts = None
        if d1:
            starts = torch.tensor(np.array([r.start for r in sel], dtype=np.uint32).view(np.int32), device=DEV)
        out = tpf.dec256v32(packed, offs, len(sel), starts=starts, err=err)
        torch.cuda.synchronize()
        assert int(err.item()) & U64MAX == U64MAX
        got = as_u32(out)
        for i, r in enumerate(sel):
            np.testing.assert_array_equal(got[i], r.values, err_msg=f"golden d1={d1} record {i}")


@pytest.mark.parametrize("pad", [0, 1, 3, 7, 13])
@pytest.mark.parametrize("exc", [0, 5, 10, 25])
def test_c2_sweep_vs_oracle(pad, exc):
    blocks = np.concatenate([datagen.c2_blocks(64, bw, exc, seed=pad * 100 + exc) for bw in range(1, 33)])
    packed_np, off_np = oracle_lib.enc256v32_batch(blocks)
    expect = oracle_lib.dec256v32_batch(packed_np, off_np, len(blocks))
    np.testing.assert_array_equal(expect, blocks)
    packed, offs = to_dev_stream([packed_np.tobytes()], pad_front=pad)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec256v32(packed, torch.from_numpy(off_np.astype(np.int64)).to(DEV), len(blocks), err=err)
    torch.cuda.synchronize()
    assert int(err.item()) & U64MAX == U64MAX
    assert_blocks_equal(as_u32(out), expect, 'decode')


def test_c3_postings_d1_vs_oracle():
    vals, starts = datagen.c3_postings(3000)
    packed_np, off_np = oracle_lib.enc256v32_batch(vals, starts=starts)
    expect = oracle_lib.dec256v32_batch(packed_np, off_np, len(vals), starts=starts)
    np.testing.assert_array_equal(expect, vals)
    packed, _ = to_dev_stream([packed_np.tobytes()])
    out = tpf.dec256v32(packed, torch.from_numpy(off_np.astype(np.int64)).to(DEV), len(vals),
                        starts=torch.from_numpy(starts.view(np.int32)).to(DEV))
    assert_blocks_equal(as_u32(out), vals, 'd1 decode')


def _vbyte_block(rng, b, xn, raw):
    """Hand-built vbyte-mode block (decode-only: valid for the decoder even
    where the reference encoder would pick another mode)."""
    hdr = bytes([0x40 | b, xn])
    payload = rng.integers(0, 256, size=32 * b, dtype=np.uint8).tobytes()
    exc = rng.integers(0, 1 << max(1, 32 - b), size=xn, dtype=np.uint64).astype(np.uint32)
    pos = rng.choice(256, size=xn, replace=False).astype(np.uint8)
    if raw:
        v = b"\xff" + exc.tobytes()
    else:
        v = b""
        for x in exc:
            x = int(x)
            if x < 156:
                v += bytes([x])
            elif x < 16540:
                d = x - 156
                v += bytes([0x9C + (d >> 8), d & 0xFF])
            elif x < 2113692:
                d = x - 16540
                v += bytes([0xDC + (d >> 16), d & 0xFF, (d >> 8) & 0xFF])
            elif x <= 0xFFFFFF:
                v += bytes([0xFC, x & 0xFF, (x >> 8) & 0xFF, (x >> 16) & 0xFF])
            else:
                v += bytes([0xFD]) + int(x).to_bytes(4, "little")
    return hdr + payload + v + pos.tobytes()


@pytest.mark.parametrize("raw", [True, False])
def test_vbyte_heavy_tiles_fallback(raw):
    """Blocks of 1.2-2.3 KB overflow the workgroup staging area and take the
    per-wave staging path; also exercises long compressed vbyte parses."""
    rng = np.random.default_rng(5 if raw else 6)
    blobs = []
    for i in range(200):
        b = int(rng.integers(0, 32))
        xn = int(rng.integers(0, 256))
        blobs.append(_vbyte_block(rng, b, xn, raw))
    expect = np.stack([oracle_lib.decode("256v32", blob, 256)[0] for blob in blobs])
    for blob in blobs:
        assert oracle_lib.decode("256v32", blob, 256)[1] == len(blob)
    packed, offs = to_dev_stream(blobs, pad_front=5)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec256v32(packed, offs, len(blobs), err=err)
    torch.cuda.synchronize()
    assert int(err.item()) & U64MAX == U64MAX
    assert_blocks_equal(as_u32(out), expect, 'decode')


def test_corrupt_offsets_reported():
    blocks = datagen.c2_blocks(500, 9, 10)
    packed_np, off_np = oracle_lib.enc256v32_batch(blocks)
    bad = off_np.astype(np.int64).copy()
    bad[123] += 1  # block 122 now looks one byte longer, block 123 one shorter
    packed, _ = to_dev_stream([packed_np.tobytes()])
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    tpf.dec256v32(packed, torch.from_numpy(bad).to(DEV), len(blocks), err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 122


@pytest.mark.parametrize("pad", [0, 5, 11])
@pytest.mark.parametrize("mix", ["bw1-4", "bw1-4+wide"])
def test_small_block_grouped_path_vs_oracle(pad, mix):
    """Streams averaging under 300 B per block take the grouped-load kernel
    (p4_dec256v32.h dec_grouped, round 5): consecutive blocks that fit one 1
    KB window are staged and decoded together.  Bit-exact vs the oracle at
    odd stream alignments, with blocks larger than a window mixed in (each a
    group of one), and a corrupted offset still reported at its block."""
    rng = np.random.default_rng(pad)
    blocks = np.concatenate([datagen.c2_blocks(400, bw, exc, seed=pad + bw) for bw in (1, 2, 3, 4) for exc in (0, 10)])
    if mix.endswith("wide"):
        # a few bw-32 blocks (1025 B) and vbyte-heavy 24-bit blocks at random places
        wide = np.concatenate([datagen.c2_blocks(6, 32, 0, seed=pad), datagen.c2_blocks(6, 24, 25, seed=pad + 1)])
        at = np.sort(rng.choice(len(blocks), len(wide), replace=False))
        blocks = np.insert(blocks, at, wide, axis=0)
    packed_np, off_np = oracle_lib.enc256v32_batch(blocks)
    assert len(packed_np) < 300 * len(blocks)
    expect = oracle_lib.dec256v32_batch(packed_np, off_np, len(blocks))
    packed, _ = to_dev_stream([packed_np.tobytes()], pad_front=pad)
    offs = torch.from_numpy(off_np.astype(np.int64)).to(DEV)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec256v32(packed, offs, len(blocks), err=err)
    torch.cuda.synchronize()
    assert int(err.item()) & U64MAX == U64MAX
    assert_blocks_equal(as_u32(out), expect, "grouped decode")
    bad = off_np.astype(np.int64).copy()
    bad[777] += 1
    err.zero_()
    out = tpf.dec256v32(packed, torch.from_numpy(bad).to(DEV), len(blocks), err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 776
    assert_blocks_equal(as_u32(out)[:776], expect[:776], "grouped decode before the corruption")


@pytest.mark.parametrize("small", [False, True])
def test_offsets_outside_the_stream_are_reported_not_followed(small):
    """Offsets are input too: a block whose offsets leave the stream (past
    in_bytes, far past it, or ending before they start) loads nothing and is
    reported through d_err; the decoder never bases a load on them (round 5:
    a caller passing too short an offset array made the decoder read garbage
    offsets and fault).  Both pipelines: single-block and grouped (small)."""
    blocks = datagen.c2_blocks(800, 2 if small else 14, 10, seed=3)
    packed_np, off_np = oracle_lib.enc256v32_batch(blocks)
    expect = oracle_lib.dec256v32_batch(packed_np, off_np, len(blocks))
    packed, _ = to_dev_stream([packed_np.tobytes()])
    total = int(off_np[-1])
    for at, bad in ((400, [total + 64, total + 96]), (500, [1 << 40, (1 << 40) + 300]), (600, [2000, 1000]),
                    (700, [(1 << 64) - 256, (1 << 64) - 16])):
        o = off_np.astype(np.uint64).copy()
        o[at], o[at + 1] = bad
        err = torch.zeros(1, dtype=torch.int64, device=DEV)
        out = tpf.dec256v32(packed, torch.from_numpy(o.view(np.int64)).to(DEV), len(blocks), err=err)
        torch.cuda.synchronize()
        # block at-1 ends at the bad offset: it is the first one reported
        assert int(err.item()) == at - 1, (at, int(err.item()))
        assert_blocks_equal(as_u32(out)[:at - 1], expect[:at - 1], f"decode before offsets {at}")
