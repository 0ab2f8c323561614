"""n-variant streams (include/turbopfor_gpu.h
tpf_p4nenc256v32): the oracle composition -- 256v32 blocks then one p4Enc32
tail -- against the reference library chained call by call, the way a
reference caller writes a list of any length (reference include/turbopfor.h:9,
:33).  Skipped where oracle/_ref was not built (no /root/reference)."""
import numpy as np
import pytest

import oracle_lib as orc
import ref_lib

pytestmark = pytest.mark.skipif(not ref_lib.available(), reason="oracle/_ref not built")

SIZES = [1, 5, 127, 255, 256, 257, 511, 512, 1000, 4097]


def _values(n, seed):
    r = np.random.default_rng(seed)
    bw = r.integers(0, 33, size=n // 64 + 1)
    raw = r.integers(0, 1 << 32, size=n, dtype=np.uint64)
    mask = np.array([(1 << int(b)) - 1 for b in bw], dtype=np.uint64).repeat(64)[:n]
    v = (raw & mask).astype(np.uint32)
    v[r.random(n) < 0.05] = r.integers(0, 1 << 32, dtype=np.uint64)  # exceptions
    return v


@pytest.mark.parametrize("n", SIZES)
def test_plain_composition_matches_reference(n):
    v = _values(n, n)
    packed, off = orc.encn256v32(v)
    assert bytes(packed) == ref_lib.encn256v32_stream(v)
    assert len(off) == n // 256 + (n % 256 != 0) + 1 and int(off[-1]) == len(packed)


@pytest.mark.parametrize("n", SIZES)
def test_d1_composition_matches_reference(n):
    r = np.random.default_rng(7 + n)
    v = (np.cumsum(r.integers(1, 1 << 12, size=n, dtype=np.uint64)) + 1000).astype(np.uint32)
    packed, off = orc.encn256v32(v, d1=True, start0=999)
    assert bytes(packed) == ref_lib.encn256v32_stream(v, d1=True, start0=999)
