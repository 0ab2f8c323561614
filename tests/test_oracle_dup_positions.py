"""Pins the oracle's handling of repeated vbyte positions (OR) to the
reference's own decoder (oracle/_ref, compiled from /root/reference/src):
raw-escape and compressed vbyte blocks, plain and delta-1, block by block
through a chained list.  Skipped where oracle/_ref was not built."""
import ctypes

import numpy as np
import pytest

import dup_positions
import oracle_lib
import ref_lib

pytestmark = pytest.mark.skipif(not ref_lib.available(), reason="oracle/_ref not built")


def test_dup_positions_oracle_matches_reference():
    packed, off, start0, mod, kinds = dup_positions.dup_list()
    assert len(mod) >= 20 and "raw" in kinds and "vbyte" in kinds
    L = ref_lib.lib()
    nb = len(off) - 1
    src = np.zeros(len(packed) + 64, dtype=np.uint8)
    src[: len(packed)] = packed
    prev = start0
    exp = dup_positions.chained_decode_oracle(packed, off, nb, start0)
    base = src.ctypes.data
    for i in range(nb):
        out = np.zeros(256 + 64, dtype=np.uint32)
        end = L.tpref_s_p4d1dec256v32(ctypes.cast(base + int(off[i]), ref_lib.u8p), 256, out.ctypes.data_as(ref_lib.u32p),
                                      prev)
        assert end - base == int(off[i + 1]), i
        np.testing.assert_array_equal(out[:256], exp[i], err_msg=f"block {i}")
        prev = int(out[255])
        # plain (non-D1) decode of the same bytes too
        o2 = np.zeros(256 + 64, dtype=np.uint32)
        L.tpref_s_p4dec256v32(ctypes.cast(base + int(off[i]), ref_lib.u8p), 256, o2.ctypes.data_as(ref_lib.u32p))
        v, _ = oracle_lib.decode("256v32", bytes(packed[int(off[i]):int(off[i + 1])]), 256)
        np.testing.assert_array_equal(o2[:256], v, err_msg=f"block {i} (plain)")
