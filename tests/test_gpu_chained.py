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


def test_bench_data_same_on_gpu_and_cpu():
    """bench.py generates on the GPU, the gloo tests on the CPU: the
    counter-keyed generators give the same integers on both."""
    import bench_data as B

    for f in (lambda d: B.gen_c2(640, 10, 42, d, first_block=6400)[0],
              lambda d: B.gen_c5(200, 10, 42, d, first_block=400),
              lambda d: B.gen_c3(300, 7, d, first_block=300, carry_fn=lambda tot: 123456789)[0],
              lambda d: B.gen_v64(640, 5, d, first_block=64),
              lambda d: B.gen_c1(100, 127, 42, d, first_block=7)):
        assert torch.equal(f("cpu"), f(DEV).cpu())


@pytest.mark.timeout(400)
@pytest.mark.parametrize("workload", ["c3chain", "c3", "c2", "c5", "c3chain64", "c3enc", "c4"])
def test_bench_two_ranks_one_gpu(workload, tmp_path):
    """bench.py --gpus 2 (launcher, two ranks sharing cuda:0 over gloo: RCCL
    refuses two ranks on one device) on a small shard: rank 1's slice
    continues rank 0's list, the chained decode's exchange rebuilds it, and
    the printed `verified` is computed on every rank."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, TPF_BENCH_SAME_GPU="1", TPF_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--workload", workload,
                        "--nblocks", "20000", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-probes"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["verified"] is True
    if "checksum_all_ranks" in res["config"]:
        assert res["config"]["checksum_all_ranks"]["decoded"] == res["config"]["checksum_all_ranks"]["generated"]
    assert res["config"].get("shard_blocks", res["config"].get("shard_units")) == [0, 20000]


@pytest.mark.parametrize("misalign", [0, 1, 3])
def test_chained_duplicate_positions(misalign):
    """A chained list with length-consistent vbyte blocks whose exceptions
    repeat a position (raw-escape and compressed): the reference ORs them
    (p4d1dec256v32_scalar.cpp:260; tests/test_oracle_dup_positions.py pins
    the oracle to it), so every later block's start depends on the OR.
    Phase A declines such blocks to the wave decoder (p4_dsum_lanes.h)."""
    import dup_positions

    packed_np, off_np, start0, mod, kinds = dup_positions.dup_list()
    nb = len(off_np) - 1
    exp = dup_positions.chained_decode_oracle(packed_np, off_np, nb, start0)
    buf = torch.zeros(len(packed_np) + 16, dtype=torch.uint8, device=DEV)
    buf[misalign:misalign + len(packed_np)] = torch.from_numpy(packed_np).to(DEV)
    packed = buf[misalign:misalign + len(packed_np)]
    offs = torch.from_numpy(off_np.astype(np.int64)).to(DEV)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec256v32_chained(packed, offs, nb, start0=start0, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == -1
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), exp)
    # per-block starts through the plain D1 decode agree too
    st = np.concatenate([[start0], exp[:-1, -1]]).astype(np.uint32)
    o2 = tpf.dec256v32(packed, offs, nb, starts=torch.from_numpy(st.view(np.int32)).to(DEV))
    np.testing.assert_array_equal(o2.cpu().numpy().view(np.uint32), exp)


@pytest.mark.parametrize("maxgap_bits,exc", [(4, 0.0), (9, 0.05), (17, 0.1), (24, 0.3), (31, 0.0)])
def test_chained_widths_and_big_runs(maxgap_bits, exc):
    """Phase A across base widths and block sizes: small blocks (many per
    staging window), runs of ~1 KB blocks (several window passes per run),
    bitmap and vbyte exceptions, constant blocks; bit-exact vs the oracle's
    sequential chained decode."""
    rng = np.random.default_rng(maxgap_bits)
    nb = 6000
    bits = rng.integers(0, maxgap_bits + 1, size=(nb, 1))
    gaps = rng.integers(0, 1 << 62, size=(nb, 256), dtype=np.uint64) & ((np.uint64(1) << bits.astype(np.uint64)) - np.uint64(1))
    ex = rng.random((nb, 256)) < exc
    gaps = np.where(ex, rng.integers(0, 1 << 32, size=(nb, 256), dtype=np.uint64) >> np.uint64(1), gaps)
    gaps[::11] = 0
    flat = (np.cumsum(gaps.reshape(-1) + np.uint64(1)) + np.uint64(7)) & np.uint64(0xFFFFFFFF)
    vals = flat.astype(np.uint32).reshape(nb, 256)
    starts = np.concatenate([[7], vals[:-1, -1]]).astype(np.uint32)
    packed_np, off_np = oracle_lib.enc256v32_batch(vals, starts=starts)
    out = tpf.dec256v32_chained(torch.from_numpy(packed_np).to(DEV), torch.from_numpy(off_np.astype(np.int64)).to(DEV), nb,
                                start0=7)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), vals)


def test_chained_random_bytes_with_huge_blocks():
    """Random bytes cut into blocks of 1 B .. 40 KB (larger than phase A's
    staging window): no fault, an error is reported, and a clean prefix
    still decodes exactly."""
    rng = np.random.default_rng(5)
    vals, starts = _list(3000, 1, seed=8)
    packed_np, off_np = oracle_lib.enc256v32_batch(vals, starts=starts)
    nbad = 2000
    lens = rng.integers(1, 2400, size=nbad)
    lens[::50] = rng.integers(16000, 40000, size=len(lens[::50]))
    garbage = rng.integers(0, 256, size=int(lens.sum()), dtype=np.uint8)
    allp = np.concatenate([packed_np, garbage])
    offs = np.concatenate([off_np.astype(np.int64), off_np[-1].astype(np.int64) + np.cumsum(lens)])
    nb = len(offs) - 1
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec256v32_chained(torch.from_numpy(allp).to(DEV), torch.from_numpy(offs).to(DEV), nb, start0=1, err=err)
    torch.cuda.synchronize()
    assert 3000 <= int(err.item()) < nb
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32)[:3000], vals)


@pytest.mark.parametrize("narrow,wide", [(1, 6), (2, 6), (3, 6), (1, 2), (2, 3), (1, 17), (2, 17), (3, 9), (1, 32), (2, 32), (3, 31)])
def test_chained_mixed_width_runs(narrow, wide):
    """Phase A sums a wave's lanes with the fold depth of the wave's
    narrowest block: every run here mixes one or a few narrow blocks (more
    pre-fold levels) into wide ones, at every lane position."""
    rng = np.random.default_rng(narrow * 100 + wide)
    nb = 64 * 6 + 13
    bits = np.full((nb, 1), wide, dtype=np.uint64)
    for r in range(nb // 64 + 1):
        lanes = rng.choice(64, size=1 + r % 3, replace=False)
        for j in lanes:
            if r * 64 + j < nb:
                bits[r * 64 + j, 0] = narrow
    gaps = rng.integers(0, 1 << 62, size=(nb, 256), dtype=np.uint64) & ((np.uint64(1) << bits) - np.uint64(1))
    gaps[:, 5] = (np.uint64(1) << bits[:, 0]) - np.uint64(1)  # every block needs exactly its width
    flat = (np.cumsum(gaps.reshape(-1) + np.uint64(1)) + np.uint64(3)) & np.uint64(0xFFFFFFFF)
    vals = flat.astype(np.uint32).reshape(nb, 256)
    starts = np.concatenate([[3], vals[:-1, -1]]).astype(np.uint32)
    packed_np, off_np = oracle_lib.enc256v32_batch(vals, starts=starts)
    out = tpf.dec256v32_chained(torch.from_numpy(packed_np).to(DEV), torch.from_numpy(off_np.astype(np.int64)).to(DEV), nb,
                                start0=3)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), vals)
