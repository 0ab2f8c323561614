"""GPU parity of the n-variant stream API (SURVEY.md §8 f2,
include/turbopfor_gpu.h tpf_p4nenc256v32 / tpf_p4ndec256v32): n values of
any count as 256v32 blocks plus one p4Enc32 tail, byte-exact against the
oracle composition (pinned to the reference chained call by call in
tests/test_nstream_cpu.py) and bit-exact on decode, plain and delta-1."""
import ctypes

import numpy as np
import pytest

import oracle_lib as orc

torch = pytest.importorskip("torch")
tpf = pytest.importorskip("turbopfor_amd")

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

SIZES = [0, 1, 5, 127, 255, 256, 257, 511, 512, 1000, 4097, 256 * 3000 + 77]


def _values(n, seed):
    r = np.random.default_rng(seed)
    bw = r.integers(0, 33, size=n // 64 + 1)
    raw = r.integers(0, 1 << 32, size=n, dtype=np.uint64)
    mask = np.array([(1 << int(b)) - 1 for b in bw], dtype=np.uint64).repeat(64)[:n]
    v = (raw & mask).astype(np.uint32)
    hit = r.random(n) < 0.05
    v[hit] = r.integers(0, 1 << 32, size=int(hit.sum()), dtype=np.uint64).astype(np.uint32)
    return v


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(DEV)


def _host(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("n", SIZES)
def test_plain_stream(n):
    v = _values(n, n)
    packed, offs = tpf.encn256v32(_dev(v))
    want, woff = orc.encn256v32(v)
    assert offs.numel() == tpf.n_units(n) + 1
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), woff)
    assert bytes(packed.cpu().numpy()) == bytes(want)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.decn256v32(packed, offs, n, err=err)
    assert np.array_equal(_host(out), v)
    assert int(err.item()) == -1


@pytest.mark.parametrize("n", SIZES)
def test_d1_stream(n):
    r = np.random.default_rng(11 + n)
    v = (np.cumsum(r.integers(1, 1 << 14, size=n, dtype=np.uint64)) + 50).astype(np.uint32)
    packed, offs = tpf.encn256v32(_dev(v), d1=True, start0=49)
    want, woff = orc.encn256v32(v, d1=True, start0=49)
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), woff)
    assert bytes(packed.cpu().numpy()) == bytes(want)
    out = tpf.decn256v32(packed, offs, n, d1=True, start0=49)
    assert np.array_equal(_host(out), v)


@pytest.mark.parametrize("n", [200, 256 * 5 + 100])
def test_tail_error_index(n):
    """A tail whose offsets disagree with its bytes is reported as block
    n // 256 (the full blocks' errors, if any, come first)."""
    v = _values(n, 3)
    packed, offs = tpf.encn256v32(_dev(v))
    bad = offs.clone()
    bad[-1] += 1
    pad = torch.zeros(packed.numel() + 64, dtype=torch.uint8, device=DEV)
    pad[: packed.numel()] = packed
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    tpf.decn256v32(pad, bad, n, err=err)
    assert int(err.item()) == n // 256


def test_small_capacity_refused():
    L = tpf.lib()
    n = 300
    v = _dev(_values(n, 1))
    ws_bytes = int(L.tpf_p4nenc256v32_workspace_size(n))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=DEV)
    out = torch.empty(16, dtype=torch.uint8, device=DEV)
    offs = torch.empty(3, dtype=torch.int64, device=DEV)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = L.tpf_p4nenc256v32(v.data_ptr(), n, 0, 0, out.data_ptr(), 16, offs.data_ptr(), ws.data_ptr(), ws_bytes, s)
    assert rc != 0 and b"out_cap" in L.tpf_last_error()
