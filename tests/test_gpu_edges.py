"""Edge cases of the batched device API: empty batches (the reference's n == 0
contract: nothing written, offsets {0}) for every entry point, and a packed
stream larger than 4 GiB (64-bit byte offsets through every kernel of the
256v32 round trip and the chained D1 decode)."""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")
tpf = pytest.importorskip("turbopfor_amd")

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_empty_batches():
    e8 = torch.zeros(64, dtype=torch.uint8, device=DEV)
    off0 = torch.zeros(1, dtype=torch.int64, device=DEV)
    v32 = torch.zeros(0, dtype=torch.int32, device=DEV)
    out = tpf.dec256v32(e8, off0, 0)
    assert out.numel() == 0
    out = tpf.dec256v32(e8, off0, 0, starts=torch.zeros(0, dtype=torch.int32, device=DEV))
    assert out.numel() == 0
    assert tpf.dec256v32_chained(e8, off0, 0, start0=7).numel() == 0
    for d1 in (False, True):
        packed, offs = tpf.enc256v32(v32, d1=d1)
        assert packed.numel() == 0 and offs.cpu().tolist() == [0]
    for fmt, n in (("32", 127), ("128v32", 128), ("256v32", 200), ("64", 64), ("128v64", 128), ("256v64", 256)):
        wide = fmt in ("64", "128v64", "256v64")
        vals = torch.zeros(0, dtype=torch.int64 if wide else torch.int32, device=DEV)
        packed, offs = tpf.enc_batch(fmt, vals, 0, n)
        assert packed.numel() == 0 and offs.cpu().tolist() == [0], fmt
        assert tpf.dec_batch(fmt, e8, off0, 0, n).numel() == 0, fmt
    torch.cuda.synchronize()


def test_stream_over_4gib_roundtrip():
    """4.4M bw-32 blocks (1025 B each, 4.5 GB packed): offsets cross 2^32;
    decode(encode(x)) == x and every block's offset matches its plain-block
    size, for the plain decode and the chained D1 decode."""
    nb = 4_400_000
    g = torch.Generator(device=DEV)
    g.manual_seed(99)
    vals = torch.randint(-(1 << 31), (1 << 31) - 1, (nb, 256), device=DEV, generator=g, dtype=torch.int32)
    vals[:, 0] |= -(1 << 31)  # bit 31 set in every block: b = 32, plain mode, 1025 B
    packed, offs = tpf.enc256v32(vals)
    assert int(offs[-1].item()) == nb * 1025 > (1 << 32)
    step = torch.diff(offs)
    assert bool((step == 1025).all())
    out = tpf.dec256v32(packed, offs, nb)
    assert torch.equal(out, vals)
    del out
    # chained delta-1 list over the same size class (gaps up to 2^31: b = 31)
    gaps = torch.randint(1, 1 << 31, (nb, 256), device=DEV, generator=g, dtype=torch.int64)
    lst = (torch.cumsum(gaps.view(-1), 0) & 0xFFFFFFFF).view(nb, 256)
    lst = (lst - ((lst >> 31) << 32)).to(torch.int32)
    del gaps
    packed, offs = tpf.enc256v32(lst, d1=True, start0=0)
    assert int(offs[-1].item()) > (1 << 32)
    out = tpf.dec256v32_chained(packed, offs, nb, start0=0)
    assert torch.equal(out, lst)


def test_hipgraph_capture_replay():
    """The batched entry points allocate nothing and only launch on the given
    stream, so a decode + chained-D1 decode + encode sequence can be captured
    into one hipGraph (torch.cuda.CUDAGraph on ROCm) and replayed with new
    inputs written into the same buffers."""
    nb = 3000
    g = torch.Generator(device=DEV)
    g.manual_seed(5)

    def fresh():
        bw = torch.randint(1, 33, (nb, 1), device=DEV, generator=g)
        raw = torch.randint(-(1 << 31), (1 << 31) - 1, (nb, 256), device=DEV, generator=g, dtype=torch.int32)
        return torch.where(bw >= 32, raw, raw & ((torch.ones_like(bw) << bw) - 1).to(torch.int32))

    L = tpf.lib()
    vals = fresh()
    cap = int(L.tpf_p4enc256v32_bound(nb))
    packed = torch.zeros(cap, dtype=torch.uint8, device=DEV)
    offs = torch.zeros(nb + 1, dtype=torch.int64, device=DEV)
    wsb = int(L.tpf_p4enc256v32_workspace_size(nb))
    ws = torch.empty(wsb, dtype=torch.uint8, device=DEV)
    out = torch.empty_like(vals)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)

    def seq():
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        assert L.tpf_p4enc256v32_batch(vals.data_ptr(), nb, packed.data_ptr(), cap, offs.data_ptr(), ws.data_ptr(), wsb, s) == 0
        assert L.tpf_p4dec256v32_batch(packed.data_ptr(), cap, offs.data_ptr(), nb, out.data_ptr(), err.data_ptr(), s) == 0

    seq()  # warm-up outside the capture (library load, first-launch setup)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        seq()
    for _ in range(3):
        vals.copy_(fresh())
        out.zero_()
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, vals)
        assert int(err.item()) == -1


def _host_abi():
    L = tpf.lib()
    L.tpf_host_dec.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                               ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
    return L


def test_host_dec_rejects_bad_offsets_and_reports_corrupt_block():
    """tpf_host_dec with caller offsets: decreasing or past in_bytes -> TPF_EINVAL
    before any copy; a block whose parsed length disagrees with its offsets ->
    TPF_ECORRUPT naming the block (offsets were trusted)."""
    import oracle_lib

    rng = np.random.default_rng(5)
    nb = 3000
    vals = rng.integers(0, 1 << 12, size=(nb, 256), dtype=np.uint64).astype(np.uint32)
    packed, off = oracle_lib.enc256v32_batch(vals)
    L = _host_abi()
    out = np.zeros((nb, 256), dtype=np.uint32)

    def run(o, nbytes=len(packed)):
        o = np.ascontiguousarray(o, dtype=np.uint64)
        return L.tpf_host_dec(2, packed.ctypes.data, nbytes, o.ctypes.data, nb, 256, out.ctypes.data, None)

    assert run(off) == 0
    np.testing.assert_array_equal(out, vals)
    bad = off.copy()
    bad[10], bad[11] = bad[11], bad[10]  # a descending pair
    assert run(bad) == -1 and b"decreases" in L.tpf_last_error()
    assert run(off, nbytes=len(packed) - 1) == -1 and b"in_bytes" in L.tpf_last_error()
    bad = off.copy()
    bad[1234] += 1  # block 1233 one byte too long, 1234 one too short
    assert run(bad) == -4
    assert b"block 1233" in L.tpf_last_error()


def test_encoder_rejects_small_out_cap():
    """The encoded sizes are only known on the device: a capacity below the
    bound is rejected up front rather than cutting blocks off silently."""
    L = tpf.lib()
    nb = 64
    vals = torch.zeros((nb, 256), dtype=torch.int32, device=DEV)
    cap = int(L.tpf_p4enc256v32_bound(nb))
    out = torch.empty(cap, dtype=torch.uint8, device=DEV)
    offs = torch.empty(nb + 1, dtype=torch.int64, device=DEV)
    wsb = int(L.tpf_p4enc256v32_workspace_size(nb))
    ws = torch.empty(wsb, dtype=torch.uint8, device=DEV)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert L.tpf_p4enc256v32_batch(vals.data_ptr(), nb, out.data_ptr(), cap - 1, offs.data_ptr(), ws.data_ptr(), wsb, s) == -1
    assert b"out_cap" in L.tpf_last_error()
    assert L.tpf_p4enc256v32_batch(vals.data_ptr(), nb, out.data_ptr(), cap, offs.data_ptr(), ws.data_ptr(), wsb, s) == 0
    torch.cuda.synchronize()


@pytest.mark.parametrize("fmt,n", [("128v32", 100), ("256v32", 200), ("128v64", 100)])
def test_chained_d1_encode_with_short_units(fmt, n):
    """One chained list over units of n < width values: unit i starts from
    unit i-1's value n-1 (the slots after it are padding), as a reference
    caller chaining p4D1Enc<fmt>(in + i*width, n, out, in[i*width + n - 1])."""
    import oracle_lib

    wide = fmt == "128v64"
    dt = np.uint64 if wide else np.uint32
    width = tpf.unit_values(fmt, n)
    nb = 200
    rng = np.random.default_rng(n)
    lst = np.cumsum(rng.integers(1, 300, size=nb * n)).astype(dt).reshape(nb, n)
    vals = np.zeros((nb, width), dtype=dt)
    vals[:, :n] = lst
    vals[:, n:] = 0xDEAD  # padding must not feed the next unit's start
    start0 = 17
    exp = b"".join(oracle_lib.encode(fmt, lst[i], d1=True, start=int(lst[i - 1, -1]) if i else start0) for i in range(nb))
    t = torch.from_numpy(vals.view(np.int64 if wide else np.int32).ravel()).to(DEV)
    packed, offs = tpf.enc_batch(fmt, t, nb, n, d1=True, start0=start0)
    assert packed.cpu().numpy().tobytes() == exp


@pytest.mark.parametrize("nruns", [0, 1, 15, 4095, 4096, 4097, 1024 * 4096 + 3, 9_000_000])
def test_run_scan_matches_cumsum(nruns):
    """The run scan between every two-pass kernel pair (p4_scan.h): exclusive
    u64 prefix of u32 run totals near 2^32 (carries), across tile borders
    and across the single-workgroup top scan's 1024-tile steps (> 4M runs:
    sizes the encoders only reach at > 67M blocks)."""
    M = tpf.measure()  # the test hook lives in the measurement library
    rng = np.random.default_rng(nruns)
    tot = rng.integers(0xF0000000, 1 << 32, nruns, dtype=np.uint64).astype(np.uint32)
    d_tot = torch.from_numpy(tot.view(np.int32)).to(DEV)
    d_base = torch.zeros(max(nruns, 1), dtype=torch.int64, device=DEV)
    d_total = torch.full((1,), -1, dtype=torch.int64, device=DEV)
    wsb = int(M.tpfm_run_scan_workspace_size(nruns))
    ws = torch.empty(wsb, dtype=torch.uint8, device=DEV)
    rc = M.tpfm_run_scan(d_tot.data_ptr(), nruns, d_base.data_ptr(), d_total.data_ptr(), ws.data_ptr(), wsb,
                         torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    incl = np.cumsum(tot.astype(np.uint64), dtype=np.uint64)
    excl = np.concatenate([np.zeros(1, np.uint64), incl[:-1]]) if nruns else np.zeros(0, np.uint64)
    got = d_base.cpu().numpy().view(np.uint64)[:nruns]
    assert np.array_equal(got, excl)
    assert int(d_total.cpu().numpy().view(np.uint64)[0]) == (int(incl[-1]) if nruns else 0)


def test_out_of_format_widths_reported():
    """a block whose width field is outside its format (32-bit: b or
    bx > 32; p4Dec32 constant: b > 32) is rejected by the host framing
    (tpf_scan_offsets) AND reported by every device decoder through d_err,
    even when the caller's offsets match the clamped parse; the blocks before
    it decode exactly."""
    import oracle_lib

    L = tpf.lib()
    rng = np.random.default_rng(8)
    good = rng.integers(0, 1 << 9, size=(5, 256), dtype=np.uint64).astype(np.uint32)
    gp, go = oracle_lib.enc256v32_batch(good)
    bad_blocks = [bytes([0x21]) + bytes(32 * 32),              # plain, b = 33 (clamped parse: 1025 B)
                  bytes([0x85, 40]) + bytes(32) + bytes(32 * 5),  # bitmap, bx = 40, no exceptions
                  bytes([0x40 | 33, 1]) + bytes(32 * 32) + bytes([7, 3])]  # vbyte, b = 33
    for k, blk in enumerate(bad_blocks):
        stream = np.concatenate([gp, np.frombuffer(blk, np.uint8), gp[: go[1]]])
        offs = np.concatenate([go, [go[-1] + len(blk), go[-1] + len(blk) + go[1]]]).astype(np.int64)
        nb = len(offs) - 1
        L.tpf_scan_offsets.restype = ctypes.c_int64
        scanned = np.zeros(nb + 1, dtype=np.uint64)
        assert L.tpf_scan_offsets(2, ctypes.c_void_p(stream.ctypes.data), ctypes.c_uint64(len(stream)), 256, ctypes.c_uint64(nb),
                                  ctypes.c_void_p(scanned.ctypes.data)) < 0, k
        err = torch.zeros(1, dtype=torch.int64, device=DEV)
        out = tpf.dec256v32(torch.from_numpy(stream).to(DEV), torch.from_numpy(offs).to(DEV), nb, err=err)
        torch.cuda.synchronize()
        assert int(err.item()) == 5, k
        np.testing.assert_array_equal(out[:5].cpu().numpy().view(np.uint32), good)
        err.zero_()
        out = tpf.dec_batch("256v32", torch.from_numpy(stream).to(DEV), torch.from_numpy(offs).to(DEV), nb, 200, err=err)
        torch.cuda.synchronize()
        assert int(err.item()) == 5, ("generic", k)
    # p4Dec32 constant block wider than 32 bits: 1 + 5 bytes by the clamped parse
    g32 = rng.integers(0, 200, size=(3, 127), dtype=np.uint64).astype(np.uint32)
    p32, o32 = oracle_lib.enc32_batch(g32)
    blk = bytes([0xC0 | 40]) + bytes(5)
    stream = np.concatenate([p32, np.frombuffer(blk, np.uint8)])
    offs = np.concatenate([o32, [o32[-1] + len(blk)]]).astype(np.int64)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec_batch("32", torch.from_numpy(stream).to(DEV), torch.from_numpy(offs).to(DEV), 4, 127, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 3
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32).reshape(4, 127)[:3], g32)
