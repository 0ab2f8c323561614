"""Robustness of the device decoders on corrupted and random streams (the
reference's decoders have undefined behaviour there; ours are memory-safe by
construction: range-checked buffer loads, clamped widths, LDS-bounded reads).

Valid streams (from the GPU encoder, checked against the oracle elsewhere)
get random bytes flipped inside randomly chosen blocks, headers included;
offsets stay as encoded.  Every decoder must finish, report through d_err
either nothing (-1: the flips left every parse length unchanged) or a block
at or after the first corrupted one, and decode every block before the first
corrupted one bit-exactly.  Pure random bytes with random block lengths must
decode without a fault and report a block in range."""
import numpy as np
import pytest

import datagen

torch = pytest.importorskip("torch")
tpf = pytest.importorskip("turbopfor_amd")

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dev_u32(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(DEV)


def corrupt(packed, offs, nb, rng, nbad):
    """Flip 1-3 random bytes (the header byte in a third of the cases) in
    nbad random blocks; returns the corrupted copy and the first block hit."""
    p = packed.copy()
    hit = np.sort(rng.choice(nb, size=nbad, replace=False))
    for b in hit:
        lo, hi = int(offs[b]), int(offs[b + 1])
        k = int(rng.integers(1, 4))
        pos = rng.integers(lo, hi, size=k)
        if rng.random() < 0.34:
            pos[0] = lo
        p[pos] ^= rng.integers(1, 256, size=k, dtype=np.uint8)
    return p, int(hit[0])


def check_err(err, first_bad, nb):
    e = int(err.item())
    assert e == -1 or first_bad <= e < nb, (e, first_bad, nb)
    return e


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_256v32_plain_d1_chained(seed):
    rng = np.random.default_rng(100 + seed)
    nb = 3000
    bws = rng.integers(1, 33, nb // 100)
    vals = np.concatenate([datagen.c2_blocks(100, int(bw), int(rng.choice([0, 5, 10, 25])), seed=seed) for bw in bws])
    packed, offs = tpf.enc256v32(dev_u32(vals))
    pk, oh = packed.cpu().numpy(), offs.cpu().numpy()
    bad, first = corrupt(pk, oh, nb, rng, nbad=int(rng.integers(1, 40)))
    dbad = torch.from_numpy(bad).to(DEV)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec256v32(dbad, offs, nb, err=err)
    torch.cuda.synchronize()
    check_err(err, first, nb)
    assert np.array_equal(out.cpu().numpy().view(np.uint32)[:first], vals[:first])

    # delta-1 lists: per-block starts and one chained list
    pv, st = datagen.c3_postings(nb, seed=seed)
    p1, o1 = tpf.enc256v32(dev_u32(pv), d1=True, starts=dev_u32(st))
    bad1, first1 = corrupt(p1.cpu().numpy(), o1.cpu().numpy(), nb, rng, nbad=int(rng.integers(1, 40)))
    d1 = torch.from_numpy(bad1).to(DEV)
    err.zero_()
    o = tpf.dec256v32(d1, o1, nb, starts=dev_u32(st), err=err)
    torch.cuda.synchronize()
    check_err(err, first1, nb)
    assert np.array_equal(o.cpu().numpy().view(np.uint32)[:first1], pv[:first1])
    err.zero_()
    oc = tpf.dec256v32_chained(d1, o1, nb, start0=int(st[0]), err=err)
    torch.cuda.synchronize()
    check_err(err, first1, nb)
    assert np.array_equal(oc.cpu().numpy().view(np.uint32)[:first1], pv[:first1])


@pytest.mark.parametrize("fmt,n", [("32", 127), ("128v32", 128), ("256v64", 256), ("128v64", 100)])
def test_fuzz_generic_formats(fmt, n):
    rng = np.random.default_rng(7 + n)
    nb = 2000
    uv = tpf.unit_values(fmt, n)
    wide = fmt in ("256v64", "128v64", "64")
    if wide:
        raw = rng.integers(0, 1 << 63, size=(nb, uv), dtype=np.uint64) >> rng.integers(0, 63, size=(nb, 1)).astype(np.uint64)
        vals = torch.from_numpy(raw.view(np.int64)).to(DEV)
    else:
        raw = rng.integers(0, 1 << 32, size=(nb, uv), dtype=np.uint64) >> rng.integers(0, 32, size=(nb, 1)).astype(np.uint64)
        raw = raw.astype(np.uint32)
        vals = dev_u32(raw)
    packed, offs = tpf.enc_batch(fmt, vals.view(-1), nb, n)
    bad, first = corrupt(packed.cpu().numpy(), offs.cpu().numpy(), nb, rng, nbad=25)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = tpf.dec_batch(fmt, torch.from_numpy(bad).to(DEV), offs, nb, n, err=err)
    torch.cuda.synchronize()
    check_err(err, first, nb)
    got = out.cpu().numpy().reshape(nb, uv)[:first]
    want = raw.reshape(nb, uv)[:first].view(np.int64 if wide else np.int32)
    # values past n in a unit are layout padding: compare the n real ones
    assert np.array_equal(got[:, :n], want[:, :n])


@pytest.mark.parametrize("fmt,n", [("256v32", 256), ("32", 127), ("256v64", 256)])
def test_random_bytes_do_not_fault(fmt, n):
    rng = np.random.default_rng(99)
    nb = 4000
    lens = rng.integers(1, 2400, size=nb)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    garbage = rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    dg, do = torch.from_numpy(garbage).to(DEV), torch.from_numpy(offs).to(DEV)
    if fmt == "256v32":
        tpf.dec256v32(dg, do, nb, err=err)
        torch.cuda.synchronize()
        check_err(err, 0, nb)
        err.zero_()
        tpf.dec256v32_chained(dg, do, nb, err=err)
    else:
        tpf.dec_batch(fmt, dg, do, nb, n, err=err)
    torch.cuda.synchronize()
    assert check_err(err, 0, nb) >= 0  # 4000 random headers: some parse length disagrees
