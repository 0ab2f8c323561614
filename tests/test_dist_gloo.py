"""world_size-2 gloo tests of the multi-GPU path (tpf_shard), run on CPU:
sharding + offset rebasing, and the one real exchange step (delta-1 list
chained across shards), with the oracle standing in for the per-shard GPU
decode."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import datagen
import oracle_lib
import tpf_shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        vals, starts = datagen.c3_postings(600, seed=11)
        start0 = 12345
        vals = (vals.astype(np.uint64) + start0).astype(np.uint32)  # list continues after start0
        starts = np.concatenate([[start0], vals[:-1, -1]]).astype(np.uint32)
        packed, off = oracle_lib.enc256v32_batch(vals, starts=starts)  # chained D1 encoding
        lo, hi = tpf_shard.shard_range(len(vals), world, rank)
        loff, (b0, b1) = tpf_shard.rebase(off, lo, hi)
        shard = packed[b0:b1]
        # phase A on this shard: delta sums per block (decode with start 0, last value = total)
        raw = oracle_lib.dec256v32_batch(shard, loff, hi - lo, starts=np.zeros(hi - lo, np.uint32))
        sums = ((raw[:, -1].astype(np.uint64)) & 0xFFFFFFFF).astype(np.uint64)
        local_total = int(sums.sum() & 0xFFFFFFFF)
        base = tpf_shard.chained_base(torch.tensor([local_total]), start0=start0)
        # phase B: per-block starts from base + local prefix
        pref = np.concatenate([[0], np.cumsum(sums)[:-1]]).astype(np.uint64)
        bst = ((pref + base) & 0xFFFFFFFF).astype(np.uint32)
        got = oracle_lib.dec256v32_batch(shard, loff, hi - lo, starts=bst)
        ok = np.array_equal(got, vals[lo:hi])
        ok_all = tpf_shard.all_ok(ok, "cpu")
        tmax = tpf_shard.max_over_ranks(float(rank + 1), "cpu")
        q.put((rank, ok, ok_all, tmax, (lo, hi)))
    finally:
        dist.destroy_process_group()


def test_chained_d1_across_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert [r[1] for r in res] == [True, True]
    assert all(r[2] for r in res)
    assert all(r[3] == 2.0 for r in res)
    assert res[0][4] == (0, 300) and res[1][4] == (300, 600)


def _global_list_worker(rank, world, port, nb, q):
    """Rank `rank` of bench.py's multi-GPU C3 path on the CPU: its slice of
    ONE global posting list (bench_data.gen_c3, carry over earlier ranks by
    all-gather), chained-D1 encoded (the oracle standing in for the GPU
    encoder), phase A (block sums), the exchange (tpf_shard.chained_base),
    phase B -- checked against the generated slice, and the shard's bytes
    against the global list's encoding cut by shard_range / rebase."""
    import bench_data

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = tpf_shard.shard_range(world * nb, world, rank)
        vals, starts = bench_data.gen_c3(hi - lo, 7, "cpu", first_block=lo,
                                         carry_fn=lambda tot: tpf_shard.exclusive_prefix(tot, "cpu"))
        v = vals.numpy().view(np.uint32)
        st = starts.numpy().view(np.uint32)
        packed, off = oracle_lib.enc256v32_batch(v, starts=st)
        # phase A: each block's delta total (decode from start 0: last value)
        raw = oracle_lib.dec256v32_batch(packed, off, hi - lo, starts=np.zeros(hi - lo, np.uint32))
        sums = raw[:, -1].astype(np.uint64)
        total = int(sums.sum() & 0xFFFFFFFF)
        base = tpf_shard.chained_base(torch.tensor([total]), start0=0)
        pref = np.concatenate([[0], np.cumsum(sums)[:-1]]).astype(np.uint64)
        got = oracle_lib.dec256v32_batch(packed, off, hi - lo, starts=((pref + base) & 0xFFFFFFFF).astype(np.uint32))
        ok = bool(np.array_equal(got, v)) and base == int(st[0])
        # the same slice cut out of the whole list's encoding (one process)
        gv, gst = bench_data.gen_c3(world * nb, 7, "cpu")
        gp, goff = oracle_lib.enc256v32_batch(gv.numpy().view(np.uint32), starts=gst.numpy().view(np.uint32))
        loff, (b0, b1) = tpf_shard.rebase(goff, lo, hi)
        cut_ok = bool(np.array_equal(gp[b0:b1], packed)) and bool(np.array_equal(loff, off))
        q.put((rank, ok, cut_ok, tpf_shard.all_ok(ok and cut_ok, "cpu"), base))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_global_posting_list_across_ranks(world):
    """bench.py's C3 at world > 1 is ONE list: rank r's first value continues
    rank r-1's last, and the chained decode's cross-rank exchange must rebuild
    it exactly (the bench used to stitch unrelated lists and skip
    the check)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_global_list_worker, args=(r, world, port, 40, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] for r in res), res
    assert all(r[2] for r in res), res
    assert all(r[3] for r in res)
    assert res[0][4] == 0 and all(r[4] != 0 for r in res[1:])


def test_shard_range_covers():
    for n in (1, 7, 100, 80_000_000):
        for w in (1, 2, 3, 8):
            rs = [tpf_shard.shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))


def _global_list64_worker(rank, world, port, nb, q):
    """bench.py's c3chain64 path on the CPU: rank r's slice of ONE 64-bit
    posting list (bench_data.gen_c3_64, carry by all-gather), p4D1Enc256v64
    units (the oracle standing in for the GPU), phase A (unit delta totals
    mod 2^64), the exchange (tpf_shard.chained_base64), phase B."""
    import bench_data

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = tpf_shard.shard_range(world * nb, world, rank)
        start0 = (1 << 40) + 12345
        vals, starts = bench_data.gen_c3_64(hi - lo, 7, "cpu", first_block=lo,
                                            carry_fn=lambda tot: tpf_shard.exclusive_prefix(tot, "cpu"), start0=start0)
        v = vals.numpy().view(np.uint64)
        st = starts.numpy().view(np.uint64)
        packed, off = oracle_lib.enc256v64_batch(v, starts=st)
        raw = oracle_lib.dec256v64_batch(packed, off, hi - lo, starts=np.zeros(hi - lo, np.uint64))
        sums = raw[:, -1].astype(np.uint64)  # each unit's total from start 0
        with np.errstate(over="ignore"):
            total = int(sums.sum(dtype=np.uint64))
        base = tpf_shard.chained_base64(torch.tensor([total - (1 << 64) if total >= 1 << 63 else total]), start0=start0)
        with np.errstate(over="ignore"):
            pref = np.concatenate([np.zeros(1, np.uint64), np.cumsum(sums, dtype=np.uint64)[:-1]]) + np.uint64(base)
        got = oracle_lib.dec256v64_batch(packed, off, hi - lo, starts=pref)
        ok = bool(np.array_equal(got, v)) and base == int(st[0])
        q.put((rank, ok, tpf_shard.all_ok(ok, "cpu"), base))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_global_posting_list64_across_ranks(world):
    """The 64-bit chained list across ranks: one u64 total per rank
    all-gathered (mod 2^64), every rank's slice rebuilt exactly."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_global_list64_worker, args=(r, world, port, 24, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] for r in res), res
    assert all(r[2] for r in res)
    assert res[0][3] == (1 << 40) + 12345 and all(r[3] > res[0][3] for r in res[1:])
