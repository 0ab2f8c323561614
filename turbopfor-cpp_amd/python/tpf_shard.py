"""Multi-GPU sharding of P4 block streams (SURVEY.md §8 e).

Blocks are independent given their offsets (and their delta-1 start), so a
stream is split into contiguous block ranges, one per rank, each rebased to
its own byte range and placed in that rank's HBM: the decode itself needs no
collective.  The only exchange step is for ONE delta-1 list chained across
shards: every rank contributes its shard total (one uint32) and starts from
start0 + the totals of all earlier ranks (mod 2^32).  Bookkeeping collectives
(max of per-rank time, min of per-rank verification) ride on the same
process group.  Backend-agnostic: RCCL ("nccl") on MI355X, gloo for the CPU
tests.
"""
import torch
import torch.distributed as dist


def shard_range(nblocks, world, rank):
    """Contiguous block range [lo, hi) of `rank` (sizes differ by at most 1)."""
    lo = nblocks * rank // world
    hi = nblocks * (rank + 1) // world
    return lo, hi


def rebase(offsets, lo, hi):
    """Offsets of blocks [lo, hi) rebased to the shard's first byte, and the
    shard's byte range in the full stream."""
    b0, b1 = int(offsets[lo]), int(offsets[hi])
    return offsets[lo : hi + 1] - b0, (b0, b1)


def chained_base(local_total, start0=0, group=None):
    """Exchange step for a delta-1 list sharded over ranks: all-gather every
    rank's shard total (uint32 carried in an int64 tensor on the group's
    device) and return this rank's base = start0 + sum of earlier totals mod 2^32."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    t = local_total.to(torch.int64).reshape(1) & 0xFFFFFFFF
    gathered = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(gathered, t, group=group)
    earlier = sum(int(g.item()) for g in gathered[:rank])
    return (start0 + earlier) & 0xFFFFFFFF


def chained_base64(local_total, start0=0, group=None):
    """chained_base for a 64-bit list (tpf_d1dec64_chain_sums totals): this
    rank's base = start0 + the earlier ranks' totals, mod 2^64."""
    rank = dist.get_rank(group)
    t = local_total.to(torch.int64).reshape(1)
    gathered = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(gathered, t, group=group)
    return (start0 + sum(int(g.item()) & 0xFFFFFFFFFFFFFFFF for g in gathered[:rank])) & 0xFFFFFFFFFFFFFFFF


def exclusive_prefix(value, device, group=None):
    """Sum of `value` (a Python int, e.g. a shard's gap total) over the ranks
    before this one: all-gather of one int64 per rank."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    gathered = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(gathered, t, group=group)
    return sum(int(g.item()) for g in gathered[:rank])


def max_over_ranks(x, device, group=None):
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def gather_floats(values, device, group=None):
    """Every rank's list of floats (same length on every rank), rank order."""
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    return [[float(v) for v in o.cpu().tolist()] for o in out]


def all_ok(ok, device, group=None):
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())
