"""Chained delta-1 decode of 64-bit lists (widening SURVEY.md
§8 f1 to 64-bit): a posting list of u64 ids stored as consecutive
p4D1Enc256v64 (or p4D1Enc128v64) units, each started from the previous
unit's last value the way reference callers chain them (README.md:116-123;
reference decoder p4d1dec256v64_scalar.cpp:15-32).  The device decodes the
whole list from start0 alone (tpf_d1dec64_chained: unit sums + u64 run scan,
then the prefix decode); the expected values come from the oracle decoding
the units one after the other, each from the value the previous call
returned, exactly as a reference caller's loop does."""
import ctypes

import numpy as np
import pytest

import oracle_lib

torch = pytest.importorskip("torch")
tpf = pytest.importorskip("turbopfor_amd")
pytestmark = pytest.mark.gpu
DEV = "cuda:0"
M64 = (1 << 64) - 1


def _list(nu, width, seed, start0):
    """Values of a chained list: per-unit gap widths 0..44 bits, 8% of gaps
    wide (exceptions), some constant-gap units; one unit of huge gaps so the
    list wraps mod 2^64 and the running prefix crosses 2^32 many times."""
    rng = np.random.default_rng(seed)
    bits = rng.integers(0, 45, size=(nu, 1)).astype(np.uint64)
    gaps = rng.integers(0, 1 << 62, size=(nu, width), dtype=np.uint64) & ((np.uint64(1) << bits) - np.uint64(1))
    exc = rng.random((nu, width)) < 0.08
    gaps = np.where(exc, rng.integers(0, 1 << 62, size=(nu, width), dtype=np.uint64) >> np.uint64(20), gaps)
    gaps[::9] = np.uint64(5)  # constant units
    gaps[nu // 3] = np.uint64(1) << np.uint64(61)  # the list wraps mod 2^64 here
    with np.errstate(over="ignore"):
        flat = np.cumsum(gaps.reshape(-1) + np.uint64(1), dtype=np.uint64) + np.uint64(start0)
    return flat.reshape(nu, width)


def _oracle_sequential(fmt, packed, off, nu, width, start0):
    out = np.zeros((nu, width), dtype=np.uint64)
    prev = start0
    for i in range(nu):
        enc = packed[int(off[i]):int(off[i + 1])].tobytes()
        v, used = oracle_lib.decode(fmt, enc, width, d1=True, start=prev)
        assert used == len(enc)
        out[i] = v
        prev = int(v[-1])
    return out


def _dev64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(DEV)


@pytest.mark.parametrize("fmt,nu", [("256v64", 1), ("256v64", 17), ("256v64", 701), ("128v64", 1000)])
def test_chained64_vs_oracle_sequential(fmt, nu):
    width = 256 if fmt == "256v64" else 128
    start0 = (1 << 32) - 1000  # the first unit already crosses 2^32
    vals = _list(nu, width, seed=nu, start0=start0)
    starts = np.concatenate([np.array([start0], dtype=np.uint64), vals[:-1, -1]])  # (a Python int + uint64 would go float64)
    exp_bytes = b"".join(oracle_lib.encode(fmt, vals[i], d1=True, start=int(starts[i])) for i in range(nu))
    packed, offs = tpf.enc_batch(fmt, _dev64(vals.ravel()), nu, width, d1=True, start0=start0)
    pk = packed.cpu().numpy()
    assert np.array_equal(pk, np.frombuffer(exp_bytes, dtype=np.uint8)), "GPU bytes differ from the oracle's"
    exp = _oracle_sequential(fmt, pk, offs.cpu().numpy(), nu, width, start0)
    np.testing.assert_array_equal(exp, vals)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec64_chained(fmt, packed, offs, nu, start0=start0, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == -1
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), exp)


def test_chained64_shards_exchange_totals():
    """A list split over 3 shards (as over 3 GPUs): each shard runs phase A
    (chain_sums -> its u64 total), the totals are exchanged, and each shard
    decodes with base = start0 + the totals of the shards before it."""
    fmt, nu, width, start0 = "256v64", 900, 256, 77
    vals = _list(nu, width, seed=3, start0=start0)
    packed, offs = tpf.enc_batch(fmt, _dev64(vals.ravel()), nu, width, d1=True, start0=start0)
    offs_np = offs.cpu().numpy()
    pk = packed.cpu().numpy()
    L = tpf.lib()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    cuts = [0, 300, 611, nu]
    shards = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        o = offs_np[a:b + 1] - offs_np[a]
        p = torch.from_numpy(pk[offs_np[a]:offs_np[b]].copy()).to(DEV)
        d_off = torch.from_numpy(o.astype(np.int64)).to(DEV)
        ws = torch.empty(int(L.tpf_d1dec64_chain_workspace_size(b - a)), dtype=torch.uint8, device=DEV)
        tot = torch.zeros(1, dtype=torch.int64, device=DEV)
        assert L.tpf_d1dec64_chain_sums(tpf.FMT[fmt], p.data_ptr(), p.numel(), d_off.data_ptr(), b - a, ws.data_ptr(), ws.numel(),
                                        tot.data_ptr(), None, s) == 0
        shards.append((a, b, p, d_off, ws, tot))
    torch.cuda.synchronize()
    base = start0
    for a, b, p, d_off, ws, tot in shards:
        out = torch.empty((b - a, width), dtype=torch.int64, device=DEV)
        assert L.tpf_d1dec64_chain_decode(tpf.FMT[fmt], p.data_ptr(), p.numel(), d_off.data_ptr(), b - a, out.data_ptr(),
                                          ctypes.c_uint64(base), ws.data_ptr(), None, s) == 0
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), vals[a:b])
        base = (base + (int(tot.item()) & M64)) & M64
    assert base == int(vals[-1, -1])


def test_chained64_corrupt_offsets_reported():
    """A unit whose parsed length disagrees with its offsets is reported
    through d_err (first bad unit); the units before it decode exactly."""
    fmt, nu, width = "256v64", 200, 256
    vals = _list(nu, width, seed=11, start0=0)
    packed, offs = tpf.enc_batch(fmt, _dev64(vals.ravel()), nu, width, d1=True, start0=0)
    bad = offs.clone()
    bad[120] += 1
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec64_chained(fmt, packed, bad, nu, start0=0, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 119
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64)[:119], vals[:119])


def test_chained64_large_roundtrip():
    """Size-independent property at 1M units (256M values): encode -> chained
    decode == x, with a start0 above 2^32."""
    nu = 1_000_000
    g = torch.Generator(device=DEV)
    g.manual_seed(17)
    gaps = torch.randint(0, 1 << 20, (nu * 256,), device=DEV, generator=g, dtype=torch.int64)
    gaps[::4099] = 1 << 40
    start0 = (1 << 32) + 5
    vals = (torch.cumsum(gaps + 1, 0) + start0).view(nu, 256)
    del gaps
    packed, offs = tpf.enc_batch("256v64", vals.view(-1), nu, 256, d1=True, start0=start0)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec64_chained("256v64", packed, offs, nu, start0=start0, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == -1
    assert torch.equal(out, vals)


def _vb64_positions(blk):
    """Byte range of the position list of a vbyte-mode 128v64 block (None if
    the block is not in vbyte mode): [0x40|b][xn][16 b base bytes][values][xn
    positions]; values are 0xFF + 8 xn raw words or xn vbyte64 values
    (markers < 0x98: 1 byte, < 0xD8: 2, < 0xF8: 3, else marker - 0xF8 + 4)."""
    h = blk[0]
    if h & 0xC0 != 0x40:
        return None
    b = h & 0x3F
    b = 64 if b == 63 else b
    xn = blk[1]
    c = 2 + 16 * b
    if blk[c] == 0xFF:
        c += 1 + 8 * xn
    else:
        for _ in range(xn):
            m = blk[c]
            c += 1 if m < 0x98 else 2 if m < 0xD8 else 3 if m < 0xF8 else m - 0xF8 + 4
    return c, c + xn


def test_chained64_repeated_positions():
    """Units whose vbyte exception positions repeat (a position byte patched to
    its predecessor's): the reference ORs the two exceptions into one element,
    so the unit's delta total is not base + sum(ex) << b.  Phase A's lane path
    must decline those units (p4_dsum64_lanes.h) and the wave decoder sum them
    exactly; every later unit's start depends on it."""
    fmt, nu, width, start0 = "256v64", 300, 256, 1 << 33
    rng = np.random.default_rng(5)
    gaps = rng.integers(0, 40, size=(nu, width)).astype(np.uint64)
    exc = rng.random((nu, width)) < 0.05
    gaps = np.where(exc, rng.integers(1 << 20, 1 << 30, size=(nu, width), dtype=np.uint64), gaps)
    with np.errstate(over="ignore"):
        vals = (np.cumsum(gaps.reshape(-1) + np.uint64(1), dtype=np.uint64) + np.uint64(start0)).reshape(nu, width)
    starts = np.concatenate([np.array([start0], dtype=np.uint64), vals[:-1, -1]])
    units = [bytearray(oracle_lib.encode(fmt, vals[i], d1=True, start=int(starts[i]))) for i in range(nu)]
    patched = 0
    for i in range(0, nu, 7):
        u = units[i]
        # the unit's first block: its length from a plain oracle decode of 128 values
        _, l0 = oracle_lib.decode("128v64", bytes(u), 128, d1=True, start=0)
        for off0, blk in ((0, u[:l0]), (l0, u[l0:])):
            r = _vb64_positions(bytes(blk))
            if r is not None and r[1] - r[0] >= 2:
                u[off0 + r[0] + 1] = u[off0 + r[0]]
                patched += 1
                break
    assert patched >= 10
    packed_np = np.frombuffer(b"".join(bytes(u) for u in units), dtype=np.uint8)
    offs_np = np.concatenate([[0], np.cumsum([len(u) for u in units])]).astype(np.int64)
    exp = _oracle_sequential(fmt, packed_np, offs_np, nu, width, start0)
    packed = torch.from_numpy(packed_np.copy()).to(DEV)
    offs = torch.from_numpy(offs_np).to(DEV)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec64_chained(fmt, packed, offs, nu, start0=start0, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == -1
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), exp)


def test_dec64_position_past_block_flagged():
    """A 128v64 vbyte block whose position byte points past its 128 values
    (a corrupt stream: an encoder never writes one) is reported through d_err,
    and the exception is dropped instead of being OR-ed into element pos-128
    (ADVICE r4).  Units before it decode exactly, in the plain 256v64 decoder
    and the chained 64-bit decode."""
    fmt, nu, width, start0 = "256v64", 40, 256, 1 << 33
    rng = np.random.default_rng(9)
    gaps = rng.integers(0, 40, size=(nu, width)).astype(np.uint64)
    exc = rng.random((nu, width)) < 0.05
    gaps = np.where(exc, rng.integers(1 << 20, 1 << 30, size=(nu, width), dtype=np.uint64), gaps)
    with np.errstate(over="ignore"):
        vals = (np.cumsum(gaps.reshape(-1) + np.uint64(1), dtype=np.uint64) + np.uint64(start0)).reshape(nu, width)
    starts = np.concatenate([np.array([start0], dtype=np.uint64), vals[:-1, -1]])
    units = [bytearray(oracle_lib.encode(fmt, vals[i], d1=True, start=int(starts[i]))) for i in range(nu)]
    bad_unit = None
    for i in range(5, nu):
        r = _vb64_positions(bytes(units[i]))
        if r is not None and r[1] > r[0]:
            units[i][r[0]] = 200
            bad_unit = i
            break
    assert bad_unit is not None
    packed_np = np.frombuffer(b"".join(bytes(u) for u in units), dtype=np.uint8)
    offs_np = np.concatenate([[0], np.cumsum([len(u) for u in units])]).astype(np.int64)
    packed = torch.from_numpy(packed_np.copy()).to(DEV)
    offs = torch.from_numpy(offs_np).to(DEV)
    st = _dev64(starts)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec_batch(fmt, packed, offs, nu, width, starts=st, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == bad_unit
    got = out.cpu().numpy().view(np.uint64).reshape(nu, width)
    np.testing.assert_array_equal(got[:bad_unit], vals[:bad_unit])
    err.zero_()
    out = tpf.dec64_chained(fmt, packed, offs, nu, start0=start0, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == bad_unit
    got = out.cpu().numpy().view(np.uint64).reshape(nu, width)
    np.testing.assert_array_equal(got[:bad_unit], vals[:bad_unit])
