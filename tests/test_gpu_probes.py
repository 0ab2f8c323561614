"""The measurement-only probes bench.py divides the decoders by
(tpfm_probe256v32, tpfm_probe256v64 of the measurement library: the decode
kernels' loads and stores with the decoding removed).  No reference counterpart; these check that they run
through the C-ABI on real streams and move the bytes they claim to: each
unit's output starts with the first 16 bytes of its 16-aligned staged image."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
tpf = pytest.importorskip("turbopfor_amd")

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _expected_first16(packed, offs, nunits):
    """Lane 0's word of each unit's staged image (p4_dec_run.h RunPlaneT):
    bytes [cb, cb+16) with cb = the unit's start rounded down to 16, OR-ed
    with the words at cb + 1024k the probe also loads for a unit over 1 KB;
    zeros for a unit the plane stages by guarded loads (span + 16 past the
    stream end)."""
    p = packed.cpu().numpy()
    o = offs.cpu().numpy().astype(np.int64)
    out = np.zeros((nunits, 16), dtype=np.uint8)
    for i in range(nunits):
        cb = o[i] & ~15
        span = o[i + 1] - cb
        if span + 16 > len(p) - cb:
            continue
        for k in range(0, span, 1024):
            out[i] |= p[cb + k:cb + k + 16]
    return out


def _check(out, packed, offs, nunits, unit_bytes):
    got = out.view(torch.uint8).view(nunits, unit_bytes)[:, :16].cpu().numpy()
    exp = _expected_first16(packed, offs, nunits)
    bad = np.nonzero((got != exp).any(axis=1))[0]
    assert bad.size == 0, bad[:10]


def test_probe256v32_moves_the_staged_bytes():
    g = torch.Generator(device="cpu").manual_seed(3)
    nb = 3000
    # widths 8..20: blocks average well over 300 B, so the probe (like the
    # decoder) takes the single-block pipeline, not the grouped one
    vals = (torch.randint(0, 1 << 20, (nb, 256), generator=g, dtype=torch.int64) >> torch.randint(0, 12, (nb, 1), generator=g)).to(torch.int32).to(DEV)
    packed, offs = tpf.enc256v32(vals)
    assert packed.numel() >= 300 * nb
    out = torch.empty((nb, 256), dtype=torch.int32, device=DEV)
    tpf.probe256v32(packed, offs, nb, out)
    torch.cuda.synchronize()
    _check(out, packed, offs, nb, 1024)


def test_probe256v64_moves_the_staged_bytes():
    g = torch.Generator(device="cpu").manual_seed(4)
    nb = 3000
    vals = (torch.randint(0, 1 << 62, (nb, 256), generator=g, dtype=torch.int64) >> torch.randint(0, 62, (nb, 1), generator=g)).to(DEV)
    packed, offs = tpf.enc_batch("256v64", vals.view(-1), nb, 256)
    out = torch.empty(nb * 256, dtype=torch.int64, device=DEV)
    tpf.probe256v64(packed, offs, nb, out)
    torch.cuda.synchronize()
    _check(out, packed, offs, nb, 2048)
    # both 1 KB halves of a unit carry the same image
    ob = out.view(torch.uint8).view(nb, 2, 1024)
    assert torch.equal(ob[:, 0], ob[:, 1])
