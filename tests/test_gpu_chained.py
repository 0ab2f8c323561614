"""Chained delta-1 decode (one posting list over many 256v32 blocks, only the
list's start given) on the GPU, single shard and simulated multi-shard
exchange, against the original values (bit-exact)."""
import numpy as np
import pytest

import datagen
import oracle_lib

torch = pytest.importorskip("torch")
tpf = pytest.importorskip("turbopfor_amd")
pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _list(nb, start0, seed):
    vals, _ = datagen.c3_postings(nb, seed=seed)
    vals = (vals.astype(np.uint64) + start0 + 1).astype(np.uint32)
    starts = np.concatenate([[start0], vals[:-1, -1]]).astype(np.uint32)
    return vals, starts


@pytest.mark.parametrize("start0,nb", [(0, 5000), (7, 5000), (0xFFFFFF00, 5000), (5, 1), (5, 3), (5, 4), (5, 5), (9, 16), (9, 17), (9, 31),
                                      (9, 32), (9, 33), (9, 48), (9, 65), (9, 130), (9, 4111),
                                       (5, 257), (11, 200003)])
def test_chained_single(start0, nb):
    vals, starts = _list(nb, start0, seed=3)
    packed_np, off_np = oracle_lib.enc256v32_batch(vals, starts=starts)
    packed = torch.from_numpy(packed_np).to(DEV)
    offs = torch.from_numpy(off_np.astype(np.int64)).to(DEV)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec256v32_chained(packed, offs, len(vals), start0=start0, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == -1
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), vals)


def test_chained_corrupt_offsets():
    vals, starts = _list(3000, 1, seed=5)
    packed_np, off_np = oracle_lib.enc256v32_batch(vals, starts=starts)
    off_bad = off_np.astype(np.int64).copy()
    off_bad[1234] += 1  # blocks 1233 and 1234 disagree with their headers
    packed = torch.from_numpy(packed_np).to(DEV)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    tpf.dec256v32_chained(packed, torch.from_numpy(off_bad).to(DEV), len(vals), start0=1, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 1233


def test_chained_sharded_exchange():
    import tpf_shard

    start0 = 99
    vals, starts = _list(7001, start0, seed=4)
    packed_np, off_np = oracle_lib.enc256v32_batch(vals, starts=starts)
    world = 3
    chains, totals = [], []
    for r in range(world):
        lo, hi = tpf_shard.shard_range(len(vals), world, r)
        loff, (b0, b1) = tpf_shard.rebase(off_np.astype(np.int64), lo, hi)
        c = tpf.D1Chain(torch.from_numpy(packed_np[b0:b1].copy()).to(DEV), torch.from_numpy(loff).to(DEV), hi - lo)
        totals.append(int(c.sums().item()) & 0xFFFFFFFF)
        chains.append((c, lo, hi))
    for r, (c, lo, hi) in enumerate(chains):
        base = (start0 + sum(totals[:r])) & 0xFFFFFFFF
        out = c.decode(base)
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), vals[lo:hi], err_msg=f"shard {r}")


def test_chained_ws_reuse_and_modes():
    """Same workspace across calls (status words re-zeroed per launch) and a
    list mixing bitmap-, vbyte- and constant-mode blocks."""
    rng = np.random.default_rng(12)
    nb = 40000
    gaps = rng.integers(0, 1 << rng.integers(0, 20, size=(nb, 1)), size=(nb, 256), dtype=np.uint64)
    exc = rng.random((nb, 256)) < 0.1
    gaps = np.where(exc, rng.integers(0, 1 << 31, size=(nb, 256), dtype=np.uint64), gaps)
    gaps[::7] = 0  # constant blocks
    flat = (np.cumsum(gaps.reshape(-1) + 1) + 3) & 0xFFFFFFFF
    vals = flat.astype(np.uint32).reshape(nb, 256)
    start0 = 3
    starts = np.concatenate([[start0], vals[:-1, -1]]).astype(np.uint32)
    packed_np, off_np = oracle_lib.enc256v32_batch(vals, starts=starts)
    packed = torch.from_numpy(packed_np).to(DEV)
    offs = torch.from_numpy(off_np.astype(np.int64)).to(DEV)
    ws = torch.empty(int(tpf.lib().tpf_p4d1dec256v32_chain_workspace_size(nb)), dtype=torch.uint8, device=DEV)
    for _ in range(3):
        out = tpf.dec256v32_chained(packed, offs, nb, start0=start0, ws=ws)
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), vals)
