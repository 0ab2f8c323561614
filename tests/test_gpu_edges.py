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
