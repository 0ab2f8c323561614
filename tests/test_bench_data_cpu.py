"""bench_data.py, the counter-keyed synthetic workloads of bench.py: a shard
generated on its own equals the same slice of the whole stream (so ranks hold
slices of ONE stream), and the distributions are the configured ones."""
import numpy as np
import torch

import bench_data as B


def test_c2_slices_are_one_stream():
    whole, _ = B.gen_c2(64, 10, 42, "cpu", first_block=0)
    for w in range(1, 4):
        # period = shard size: a shard of the global stream is one period
        sh, _ = B.gen_c2(64, 10, 42, "cpu", first_block=64 * w)
        assert not torch.equal(sh, whole)  # fresh values in every period
    a = B.gen_bw(100, 9, 10, 42, "cpu")
    b = B.gen_bw(40, 9, 10, 42, "cpu", first_block=60)
    assert torch.equal(a[60:], b)


def test_c2_distribution():
    v, seg = B.gen_c2(3200, 10, 42, "cpu")
    u = v.numpy().view(np.uint32)
    for s in range(32):
        blk = u[seg[s]:seg[s + 1]]
        bw = s + 1
        exc = (blk >= (1 << bw)).mean() if bw < 32 else 0.0
        if bw <= 28:
            assert 0.08 < exc < 0.12, (bw, exc)
        else:
            assert exc == 0.0


def test_c3_one_list_across_shards():
    nb, world = 30, 3
    whole, wst = B.gen_c3(nb * world, 7, "cpu")
    w = whole.numpy().view(np.uint32).ravel().astype(np.int64)
    assert (np.diff(w) >= 1).all()  # strictly increasing (no wrap at this size)
    gaps = []
    for r in range(world):
        n = nb * 256
        gaps.append(int(B.c3_gaps(r * n, n, 7, "cpu").sum()))
    for r in range(world):
        before = sum(gaps[:r])
        v, st = B.gen_c3(nb, 7, "cpu", first_block=r * nb, carry_fn=lambda tot, b=before: b)
        assert torch.equal(v, whole[r * nb:(r + 1) * nb])
        assert torch.equal(st, wst[r * nb:(r + 1) * nb])
    d = np.diff(np.concatenate([[0], w]))
    assert 0.04 < (d > 64).mean() < 0.06


def test_v64_segments():
    v = B.gen_v64(640, 5, "cpu").numpy().view(np.uint64)
    for s in range(64):
        blk = v[s * 10:(s + 1) * 10]
        bw = s + 1
        if bw == 64:
            continue
        big = blk >= np.uint64(1 << bw)
        rate = [0, 5, 10, 25][s % 4] / 100
        assert abs(big.mean() - rate) < 0.03, (bw, big.mean())
        if big.any():
            top = np.array([int(x).bit_length() for x in blk[big]])
            if s % 2 == 0 and bw < 32:
                assert top.max() <= 32
            else:
                assert top.min() > 32
