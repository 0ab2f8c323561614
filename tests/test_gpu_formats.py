"""GPU parity for every format of include/turbopfor.h through the batched
C-ABI (tpf_enc_batch / tpf_dec_batch): byte-exact encoder output and
bit-exact decoding against the golden fixtures generated from the
reference's src/scalar codec, plus oracle cross-checks at larger sizes."""
import collections

import numpy as np
import pytest

import datagen
import golden_io
import oracle_lib

torch = pytest.importorskip("torch")
tpf = pytest.importorskip("turbopfor_amd")

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
U64 = (1 << 64) - 1

FAMILIES = [("g32.bin", "32"), ("g128v32.bin", "128v32"), ("g256v32.bin", "256v32"),
            ("g128v64.bin", "128v64"), ("g256v64.bin", "256v64")]


def to_dev(arr, wide):
    a = np.ascontiguousarray(arr, dtype=np.uint64 if wide else np.uint32)
    return torch.from_numpy(a.view(np.int64 if wide else np.int32)).to(DEV)


def groups(fname, fmt):
    """Golden records by (n, d1).  Batches hold whole 256v64 units; shorter
    256v64 vectors go through the per-block API (test_gpu_dropin.py)."""
    g = collections.defaultdict(list)
    for r in golden_io.load(fname):
        if fmt == "256v64" and r.n != 256:
            continue
        g[(r.n, r.d1)].append(r)
    return g


@pytest.mark.parametrize("fname,fmt", FAMILIES)
def test_golden_encode(fname, fmt):
    wide = fmt in ("64", "128v64", "256v64")
    for (n, d1), recs in groups(fname, fmt).items():
        recs = [r for r in recs if not r.decode_only]
        if not recs:
            continue
        u = tpf.unit_values(fmt, n)
        vals = np.zeros((len(recs), u), dtype=np.uint64 if wide else np.uint32)
        for i, r in enumerate(recs):
            vals[i, :n] = r.values
        starts = to_dev(np.array([r.start for r in recs]), wide) if d1 else None
        packed, offs = tpf.enc_batch(fmt, to_dev(vals.ravel(), wide), len(recs), n, d1=d1, starts=starts)
        pk = packed.cpu().numpy().tobytes()
        of = offs.cpu().numpy()
        for i, r in enumerate(recs):
            mine = pk[of[i]:of[i + 1]]
            if r.padding_unpinned:  # padding bits: the zero convention (oracle), length as the reference
                assert len(mine) == len(r.enc), f"{fmt} n={n} d1={d1} record {i}"
                assert mine == oracle_lib.encode(fmt, r.values, d1=d1, start=r.start), f"{fmt} n={n} record {i}"
            else:
                assert mine == r.enc, f"{fmt} n={n} d1={d1} record {i}"


@pytest.mark.parametrize("fname,fmt", FAMILIES)
def test_golden_decode(fname, fmt):
    wide = fmt in ("64", "128v64", "256v64")
    for (n, d1), recs in groups(fname, fmt).items():
        u = tpf.unit_values(fmt, n)
        offs = np.zeros(len(recs) + 1, dtype=np.int64)
        offs[1:] = np.cumsum([len(r.enc) for r in recs])
        packed = torch.from_numpy(np.frombuffer(b"".join(x.enc for x in recs), dtype=np.uint8).copy()).to(DEV)
        starts = to_dev(np.array([r.start for r in recs]), wide) if d1 else None
        err = torch.zeros(1, dtype=torch.int64, device=DEV)
        out = tpf.dec_batch(fmt, packed, torch.from_numpy(offs).to(DEV), len(recs), n, starts=starts, err=err)
        torch.cuda.synchronize()
        assert int(err.item()) == -1, f"{fmt} n={n}: length check failed at {int(err.item())}"
        got = out.cpu().numpy().view(np.uint64 if wide else np.uint32).reshape(len(recs), u)
        for i, r in enumerate(recs):
            np.testing.assert_array_equal(got[i, :n], r.values, err_msg=f"{fmt} n={n} d1={d1} record {i}")


@pytest.mark.parametrize("bw", [4, 16, 31, 33, 40, 63, 64])
@pytest.mark.parametrize("exc", [0, 5, 25])
def test_256v64_roundtrip_vs_oracle(bw, exc):
    blocks = datagen.c4_blocks64(64, bw, exc, seed=bw * 7 + exc)
    exp_packed, exp_off = oracle_lib.enc256v64_batch(blocks)
    packed, offs = tpf.enc_batch("256v64", to_dev(blocks.ravel(), True), len(blocks), 256)
    np.testing.assert_array_equal(offs.cpu().numpy().astype(np.uint64), exp_off)
    np.testing.assert_array_equal(packed.cpu().numpy(), exp_packed)
    out = tpf.dec_batch("256v64", packed, offs, len(blocks), 256)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64).reshape(-1, 256), blocks)


def test_256v64_d1_chained_vs_oracle():
    rng = np.random.default_rng(3)
    g = rng.integers(1, 1 << 20, size=(300 * 256,), dtype=np.uint64)
    vals = np.cumsum(g).astype(np.uint64).reshape(300, 256)
    starts = np.zeros(300, dtype=np.uint64)
    starts[1:] = vals[:-1, -1]
    exp_packed, exp_off = oracle_lib.enc256v64_batch(vals, starts=starts)
    packed, offs = tpf.enc_batch("256v64", to_dev(vals.ravel(), True), 300, 256, d1=True, start0=0)
    np.testing.assert_array_equal(packed.cpu().numpy(), exp_packed)
    out = tpf.dec_batch("256v64", packed, offs, 300, 256, starts=to_dev(starts, True))
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64).reshape(-1, 256), vals)


@pytest.mark.parametrize("n", [1, 7, 64, 127, 200, 256])
def test_p4enc32_vs_oracle(n):
    """C1-style horizontal blocks (p4Enc32/p4Dec32), incl. n=127 bw=8."""
    rng = np.random.default_rng(n)
    nb = 400
    bw = rng.integers(1, 33, size=(nb, 1))
    vals = (rng.integers(0, 1 << 62, size=(nb, n), dtype=np.uint64) & ((np.uint64(1) << bw.astype(np.uint64)) - np.uint64(1)))
    exc = rng.random((nb, n)) < 0.1
    vals = np.where(exc, rng.integers(0, 1 << 32, size=(nb, n), dtype=np.uint64), vals).astype(np.uint32)
    exp_packed, exp_off = oracle_lib.enc32_batch(vals)
    packed, offs = tpf.enc_batch("32", to_dev(vals.ravel(), False), nb, n)
    np.testing.assert_array_equal(packed.cpu().numpy(), exp_packed)
    out = tpf.dec_batch("32", packed, offs, nb, n)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32).reshape(nb, n), vals)


@pytest.mark.parametrize("n", [127, 256])
def test_p4dec32_corrupt_offsets_reported(n):
    """The run-pipelined generic decoder reports the first block whose parsed
    length disagrees with the offsets (d_err), like the 256v32 kernel."""
    rng = np.random.default_rng(7 + n)
    nb = 300
    vals = rng.integers(0, 1 << 11, size=(nb, n), dtype=np.uint64).astype(np.uint32)
    exp_packed, exp_off = oracle_lib.enc32_batch(vals)
    packed = torch.from_numpy(exp_packed).to(DEV)
    bad = exp_off.astype(np.int64).copy()
    bad[200] += 1  # block 199 looks one byte longer, block 200 one shorter
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    tpf.dec_batch("32", packed, torch.from_numpy(bad).to(DEV), nb, n, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 199
    out = tpf.dec_batch("32", packed, torch.from_numpy(exp_off.astype(np.int64)).to(DEV), nb, n, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == -1  # UINT64_MAX: every block consistent
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32).reshape(nb, n), vals)


def _h32_values(rng, nb, n):
    """Blocks that exercise every p4Dec32 mode the windowed decoder parses:
    constant, plain, bitmap and vbyte exceptions (raw and compressed), at base
    widths 0..32 -- runs of small blocks share one staged window, 1 KB blocks
    split runs into windows of two."""
    bw = rng.integers(0, 33, size=(nb, 1)).astype(np.uint64)
    vals = rng.integers(0, 1 << 62, size=(nb, n), dtype=np.uint64) & ((np.uint64(1) << bw) - np.uint64(1))
    rate = rng.choice([0.0, 0.02, 0.1, 0.3], size=(nb, 1))
    exc = rng.random((nb, n)) < rate
    big = rng.integers(0, 1 << 32, size=(nb, n), dtype=np.uint64) >> rng.integers(0, 24, size=(nb, 1)).astype(np.uint64)
    vals = np.where(exc, big, vals).astype(np.uint32)
    const = rng.random(nb) < 0.1
    vals[const] = vals[const, :1]
    return vals


@pytest.mark.parametrize("n", [1, 33, 64, 65, 127, 128, 129, 255, 256])
@pytest.mark.parametrize("d1", [False, True])
def test_p4dec32_windows_vs_oracle(n, d1):
    """k_dec_h32w (p4Dec32 / p4D1Dec32 batches, n <= 256): mixed modes and
    widths over 64-block wave runs and their staging windows, ragged last run
    (nb % 64 != 0), bit-exact against the oracle's decode of the oracle's
    encoding (reference src/scalar/p4dec32.cpp:70-142, p4d1dec32.cpp)."""
    rng = np.random.default_rng(1000 * n + d1)
    nb = 3001
    vals = _h32_values(rng, nb, n)
    starts = rng.integers(0, 1 << 32, size=nb, dtype=np.uint64).astype(np.uint32) if d1 else None
    if d1:
        # p4D1Enc32 codes vals as strictly increasing deltas from the start
        vals = (np.cumsum(vals.astype(np.uint64) + 1, axis=1) + starts[:, None].astype(np.uint64) - 1).astype(np.uint32)
    packed, off = oracle_lib.enc32_batch(vals, starts=starts)
    exp = oracle_lib.dec32_batch(packed, off, nb, n, starts=starts)
    np.testing.assert_array_equal(exp, vals)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec_batch("32", torch.from_numpy(packed).to(DEV), torch.from_numpy(off.astype(np.int64)).to(DEV), nb, n,
                        starts=to_dev(starts, False) if d1 else None, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == -1
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32).reshape(nb, n), vals)


def test_p4dec32_windows_oversize_block_reported():
    """An offset pair that claims more bytes than a staging window (or runs
    past the stream) is reported through d_err, blocks before it stay exact."""
    rng = np.random.default_rng(5)
    nb, n = 200, 127
    vals = rng.integers(0, 1 << 9, size=(nb, n), dtype=np.uint64).astype(np.uint32)
    packed, off = oracle_lib.enc32_batch(vals)
    pad = np.zeros(len(packed) + 8192, dtype=np.uint8)
    pad[: len(packed)] = packed
    bad = off.astype(np.int64).copy()
    bad[71:] += 4000  # block 70 claims 4000 extra bytes
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec_batch("32", torch.from_numpy(pad).to(DEV), torch.from_numpy(bad).to(DEV), nb, n, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 70
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32).reshape(nb, n)[:70], vals[:70])
    err.zero_()
    short = torch.from_numpy(packed[: int(off[150])].copy()).to(DEV)  # stream ends at block 150
    tpf.dec_batch("32", short, torch.from_numpy(off.astype(np.int64)).to(DEV), nb, n, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 150


def test_256v64_vbyte_every_marker_form():
    """128v64 vbyte exceptions of every vbyte64 length form (1-3 byte markers
    below 0xF8 and the 3..9-byte long forms, p4_scalar_internal.h:638-670):
    few large exceptions over a 3-bit base make the encoder pick vbyte mode;
    bytes against the oracle, values back from the batch decoder (plain and
    D1 per-unit starts)."""
    rng = np.random.default_rng(11)
    nu = 512
    blocks = rng.integers(0, 8, size=(nu, 256), dtype=np.uint64)
    shifts = np.arange(3, 64)
    for i in range(nu):
        pos = rng.choice(256, size=3, replace=False)
        for k, p in enumerate(pos):
            s = int(shifts[(3 * i + k) % len(shifts)])
            blocks[i, p] = np.uint64((1 << s) | int(rng.integers(0, 1 << min(s, 62))))
    exp_packed, exp_off = oracle_lib.enc256v64_batch(blocks)
    packed, offs = tpf.enc_batch("256v64", to_dev(blocks.ravel(), True), nu, 256)
    np.testing.assert_array_equal(offs.cpu().numpy().astype(np.uint64), exp_off)
    np.testing.assert_array_equal(packed.cpu().numpy(), exp_packed)
    heads = exp_packed[exp_off[:-1].astype(np.int64)]
    assert int(((heads & 0xC0) == 0x40).sum()) > nu // 2, "vbyte mode not chosen"
    out = tpf.dec_batch("256v64", packed, offs, nu, 256)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64).reshape(-1, 256), blocks)
    # the same exceptions through D1 (gaps = the blocks' values)
    vals = np.cumsum(blocks.ravel() + np.uint64(1), dtype=np.uint64).reshape(nu, 256) - np.uint64(1)
    starts = np.zeros(nu, dtype=np.uint64)
    starts[1:] = vals[:-1, -1]
    exp_packed, exp_off = oracle_lib.enc256v64_batch(vals, starts=starts)
    packed, offs = tpf.enc_batch("256v64", to_dev(vals.ravel(), True), nu, 256, d1=True, start0=0)
    np.testing.assert_array_equal(packed.cpu().numpy(), exp_packed)
    out = tpf.dec_batch("256v64", packed, offs, nu, 256, starts=to_dev(starts, True))
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64).reshape(-1, 256), vals)
