"""GPU parity of the 256v32 batch encoder (p4Enc256v32 / p4D1Enc256v32):
byte-exact against the golden fixtures (reference src/scalar outputs) and the
CPU restatement, plus encode->decode round trips at larger sizes."""
import numpy as np
import pytest

import datagen
import golden_io
import oracle_lib

torch = pytest.importorskip("torch")
tpf = pytest.importorskip("turbopfor_amd")

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dev_u32(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(DEV)


def test_golden_256v32_encode():
    recs = [r for r in golden_io.load("g256v32.bin") if r.n == 256 and not r.decode_only]
    for d1 in (False, True):
        sel = [r for r in recs if r.d1 == d1]
        vals = np.stack([r.values for r in sel])
        starts = dev_u32(np.array([r.start for r in sel], dtype=np.uint32)) if d1 else None
        packed, offs = tpf.enc256v32(dev_u32(vals), d1=d1, starts=starts)
        packed = packed.cpu().numpy().tobytes()
        offs = offs.cpu().numpy()
        assert offs[-1] == sum(len(r.enc) for r in sel)
        for i, r in enumerate(sel):
            assert packed[offs[i]:offs[i + 1]] == r.enc, f"golden d1={d1} record {i}"


@pytest.mark.parametrize("exc", [0, 5, 10, 25])
def test_c2_encode_vs_oracle(exc):
    blocks = np.concatenate([datagen.c2_blocks(48, bw, exc, seed=exc + 3) for bw in range(1, 33)])
    exp_packed, exp_off = oracle_lib.enc256v32_batch(blocks)
    packed, offs = tpf.enc256v32(dev_u32(blocks))
    np.testing.assert_array_equal(offs.cpu().numpy().astype(np.uint64), exp_off)
    np.testing.assert_array_equal(packed.cpu().numpy(), exp_packed)


def test_c3_d1_encode_chained_and_starts():
    vals, starts = datagen.c3_postings(2000)
    exp_packed, exp_off = oracle_lib.enc256v32_batch(vals, starts=starts)
    p1, o1 = tpf.enc256v32(dev_u32(vals), d1=True, starts=dev_u32(starts))
    np.testing.assert_array_equal(p1.cpu().numpy(), exp_packed)
    p2, o2 = tpf.enc256v32(dev_u32(vals), d1=True, start0=0)  # chained: same starts
    np.testing.assert_array_equal(p2.cpu().numpy(), exp_packed)
    np.testing.assert_array_equal(o2.cpu().numpy().astype(np.uint64), exp_off)


def test_roundtrip_large_mixed():
    """Size-independent property at scale: decode(encode(x)) == x."""
    g = torch.Generator(device=DEV)
    g.manual_seed(1234)
    nb = 200_000
    bw = torch.randint(1, 33, (nb, 1), device=DEV, generator=g)
    raw = torch.randint(0, 1 << 62, (nb, 256), device=DEV, generator=g, dtype=torch.int64)
    base = raw & ((1 << bw) - 1)
    exc = (torch.rand((nb, 256), device=DEV, generator=g) < 0.1) & (bw <= 28)
    vals = torch.where(exc, raw >> 30, base).to(torch.int64) & 0xFFFFFFFF
    vals = (vals - ((vals >> 31) << 32)).to(torch.int32)  # uint32 bit pattern as int32
    packed, offs = tpf.enc256v32(vals)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec256v32(packed, offs, nb, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == -1
    assert torch.equal(out, vals.view(nb, 256))


def test_full_size_c2_sample_vs_oracle():
    """At the bench's full size (10M blocks, C2 generator: bw 1..32 segments,
    10% exceptions) the GPU encoder's bytes for 4,000 sampled blocks equal the
    oracle's encoding of those blocks, their offsets step by exactly that
    size, and the GPU decoder returns the sampled blocks' values."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    nb = 10_000_000
    vals, _ = bench.gen_c2(nb, 10.0, seed=1, dev=torch.device(DEV))
    packed, offs = tpf.enc256v32(vals)
    rng = np.random.default_rng(0)
    idx = np.sort(rng.choice(nb, 4000, replace=False))
    idx_t = torch.from_numpy(idx).to(DEV)
    sample = vals[idx_t].cpu().numpy().view(np.uint32)
    exp_packed, exp_off = oracle_lib.enc256v32_batch(sample)
    o = offs.cpu().numpy()
    pk = packed.cpu().numpy()
    for i, b in enumerate(idx):
        got = pk[o[b]:o[b + 1]]
        want = exp_packed[exp_off[i]:exp_off[i + 1]]
        assert np.array_equal(got, want), f"block {b}"
    out = tpf.dec256v32(packed, offs, nb)
    assert torch.equal(out[idx_t], vals[idx_t])


def test_full_size_c5_shard_sample_vs_oracle():
    """C5's single-GPU shard at full size (bench.py --workload c5: 10M blocks,
    the first half bw 8, the rest bw 16, 10% exceptions; BASELINE configs[4]
    is 8 such shards): the GPU encoder's bytes for 4,000 sampled blocks equal
    the oracle's, offsets step by exactly those sizes, the decoder returns the
    sampled blocks, and the whole shard's decode equals its values."""
    import bench_data

    nb = 10_000_000
    vals = bench_data.gen_c5(nb, 10.0, 1, torch.device(DEV))
    packed, offs = tpf.enc256v32(vals)
    rng = np.random.default_rng(5)
    idx = np.sort(np.concatenate([rng.choice(nb, 3998, replace=False), [nb // 2 - 1, nb // 2]]))
    idx = np.unique(idx)
    idx_t = torch.from_numpy(idx).to(DEV)
    sample = vals[idx_t].cpu().numpy().view(np.uint32)
    exp_packed, exp_off = oracle_lib.enc256v32_batch(sample)
    o = offs.cpu().numpy()
    pk = packed.cpu().numpy()
    for i, b in enumerate(idx):
        assert np.array_equal(pk[o[b]:o[b + 1]], exp_packed[exp_off[i]:exp_off[i + 1]]), f"block {b}"
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec256v32(packed, offs, nb, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == -1
    assert torch.equal(out, vals)


def test_full_size_c3_sample_vs_oracle():
    """Full-size C3 (10M blocks of Zipf posting lists, per-block starts):
    p4D1Enc256v32 bytes of 4,000 sampled blocks equal the oracle's, and the
    D1 decode (per-block starts) and the chained decode return them."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    nb = 10_000_000
    vals, starts = bench.gen_c3(nb, seed=7, dev=torch.device(DEV))
    packed, offs = tpf.enc256v32(vals, d1=True, starts=starts)
    rng = np.random.default_rng(1)
    idx = np.sort(rng.choice(nb, 4000, replace=False))
    idx_t = torch.from_numpy(idx).to(DEV)
    sample = vals[idx_t].cpu().numpy().view(np.uint32)
    sst = starts[idx_t].cpu().numpy().view(np.uint32)
    exp_packed, exp_off = oracle_lib.enc256v32_batch(sample, starts=sst)
    o = offs.cpu().numpy()
    pk = packed.cpu().numpy()
    for i, b in enumerate(idx):
        assert np.array_equal(pk[o[b]:o[b + 1]], exp_packed[exp_off[i]:exp_off[i + 1]]), f"block {b}"
    out = tpf.dec256v32(packed, offs, nb, starts=starts)
    assert torch.equal(out[idx_t], vals[idx_t])
    out2 = tpf.dec256v32_chained(packed, offs, nb, start0=int(starts[0].item()) & 0xFFFFFFFF)
    assert torch.equal(out2, vals)


@pytest.mark.parametrize("mode", [0, 3, 4, 5])
@pytest.mark.parametrize("nb", [1, 15, 16, 17, 31, 33, 1000, 20_000])
def test_encoder_entries_vs_oracle(mode, nb):
    """The 256v32 encoder through the batch entry (mode 0: the library's
    two-pass encoder) and through the measurement library (tpfm_enc256v32):
    3 = two-pass (plan, run scan, write), 4 / 5 = the slot encoder (plan +
    build into per-run slots, run scan, compaction; with / without the fused
    scans), measured and not adopted but kept byte-exact for A/B runs.  Byte-exact vs the
    oracle, mixed widths and exception rates, ragged last runs (a run is 16
    blocks)."""
    blocks = mixed_blocks(nb, nb + mode)
    exp_packed, exp_off = oracle_lib.enc256v32_batch(blocks)
    vals = dev_u32(blocks)
    if mode == 0:
        packed, offs = tpf.enc256v32(vals)
        packed = packed.cpu().numpy()
    else:
        cap = int(tpf.lib().tpf_p4enc256v32_bound(nb))
        out = torch.zeros(cap, dtype=torch.uint8, device=DEV)
        offs = tpf.enc256v32_path(mode, vals, out)
        packed = out.cpu().numpy()[:int(offs[-1].item())]
    np.testing.assert_array_equal(offs.cpu().numpy().astype(np.uint64), exp_off)
    np.testing.assert_array_equal(packed, exp_packed)


@pytest.mark.parametrize("mode", [3, 4, 5])
@pytest.mark.parametrize("chained", [True, False])
def test_encoder_paths_d1_vs_oracle(mode, chained):
    """p4D1Enc256v32 through both forced paths, one chained C3 list (start0 +
    the list itself) and per-block starts: byte-exact vs the oracle, and the
    compaction's writes leave the bytes past the stream untouched."""
    pv, st = datagen.c3_postings(3001)
    exp_packed, exp_off = oracle_lib.enc256v32_batch(pv, starts=st)
    vals = dev_u32(pv)
    cap = int(tpf.lib().tpf_p4enc256v32_bound(len(pv)))
    out = torch.full((cap,), 0xA5, dtype=torch.uint8, device=DEV)
    starts = None if chained else dev_u32(st)
    offs = tpf.enc256v32_path(mode, vals, out, d1=True, starts=starts, start0=int(st[0]))
    got = out.cpu().numpy()
    total = int(offs[-1].item())
    np.testing.assert_array_equal(offs.cpu().numpy().astype(np.uint64), exp_off)
    np.testing.assert_array_equal(got[:total], exp_packed)
    assert (got[total:total + 4096] == 0xA5).all()


def mixed_blocks(nb, seed):
    rng = np.random.default_rng(seed)
    bws = rng.integers(1, 33, nb)
    if nb <= 1000:
        return np.concatenate([datagen.c2_blocks(1, int(bw), int(rng.choice([0, 5, 10, 25])), seed=int(i))
                               for i, bw in enumerate(bws)])
    return np.concatenate([datagen.c2_blocks(nb // 32 + 1, bw, 10, seed=bw) for bw in range(1, 33)])[:nb]


@pytest.mark.parametrize("d1", [False, True])
@pytest.mark.parametrize("nb", [1, 7, 16, 31, 32, 33, 65, 257])
def test_tiny_blocks_run_copy(d1, nb):
    """Round 5's run copy-out (RunCopy: whole 16-byte chunks, the chunk a
    block ends in carried into the next block of the wave's run) on runs of
    1-5 byte blocks -- all-zero blocks (1 byte), constant blocks (2-5 bytes),
    D1 lists with a constant step (constant deltas) -- mixed with ordinary
    blocks, ragged run ends (runs are 16 blocks, 32 for D1): byte-exact vs
    the oracle, and no byte past the stream is written."""
    rng = np.random.default_rng(nb * 7 + d1)
    kinds = rng.integers(0, 4, nb)
    blocks = np.zeros((nb, 256), dtype=np.uint32)
    for i, k in enumerate(kinds):
        if k == 1:
            blocks[i] = np.uint32(rng.integers(1, 1 << 31))  # constant block
        elif k == 2:
            blocks[i] = datagen.c2_blocks(1, int(rng.integers(1, 33)), 10, seed=i)[0]
        elif k == 3:
            blocks[i] = np.uint32(rng.integers(0, 256))
    starts = None
    if d1:
        # D1 input: running sums of (delta + 1) so that each block's deltas are `blocks`
        flat = np.cumsum(blocks.astype(np.uint64).reshape(-1) + 1) + np.uint64(12345)
        vals = (flat & 0xFFFFFFFF).astype(np.uint32).reshape(nb, 256)
        st = np.empty(nb, dtype=np.uint32)
        st[0] = 12345
        st[1:] = vals[:-1, -1]
        starts = st
    else:
        vals = blocks
    exp_packed, exp_off = oracle_lib.enc256v32_batch(vals, starts=starts)
    cap = int(tpf.lib().tpf_p4enc256v32_bound(nb))
    out = torch.full((cap,), 0xA5, dtype=torch.uint8, device=DEV)
    if d1:
        packed, offs = tpf.enc256v32(dev_u32(vals), d1=True, start0=12345, out=out)
    else:
        packed, offs = tpf.enc256v32(dev_u32(vals), out=out)
    total = int(offs[-1].item())
    got = out.cpu().numpy()
    np.testing.assert_array_equal(offs.cpu().numpy().astype(np.uint64), exp_off)
    np.testing.assert_array_equal(got[:total], exp_packed)
    assert (got[total:] == 0xA5).all()
