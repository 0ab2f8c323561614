"""Chained delta-1 lists whose vbyte-exception blocks carry REPEATED
positions.  The reference encoder never writes such a block, but its decoder
accepts it and ORs the exceptions that share a position
(src/scalar/p4d1dec256v32_scalar.cpp:260: out[ip[i]] |= exceptions[i] << b),
and the block length does not change -- so a chained decode must carry the OR
into every later block's start."""
import numpy as np

import datagen
import oracle_lib


def dup_list(nb=3000, seed=21, every=37, start0=5):
    """(packed, offsets, start0, modified block indices, per-block raw/compressed
    kind): a C3 posting list, D1-encoded as one chained list, with positions
    [1] (and [2] every other time) of every `every`-th vbyte block with >= 3
    exceptions overwritten by position [0]."""
    vals, _ = datagen.c3_postings(nb, seed=seed)
    vals = (vals.astype(np.uint64) + start0 + 1).astype(np.uint32)
    starts = np.concatenate([[start0], vals[:-1, -1]]).astype(np.uint32)
    packed, off = oracle_lib.enc256v32_batch(vals, starts=starts)
    packed = packed.copy()
    mod, kinds, seen = [], [], 0
    for i in range(nb):
        o, e = int(off[i]), int(off[i + 1])
        h = int(packed[o])
        if (h & 0xC0) != 0x40:
            continue
        xn = int(packed[o + 1])
        if xn < 3:
            continue
        seen += 1
        if seen % every:
            continue
        b = h & 0x3F
        raw = packed[o + 2 + 32 * b] == 0xFF
        pos = e - xn  # the position bytes end the block
        packed[pos + 1] = packed[pos]
        if len(mod) % 2:
            packed[pos + 2] = packed[pos]
        mod.append(i)
        kinds.append("raw" if raw else "vbyte")
    return packed, off, start0, mod, kinds


def chained_decode_oracle(packed, off, nb, start0):
    """Sequential chained decode, block by block (each block starts from the
    previous block's last decoded value), with the oracle."""
    out = np.zeros((nb, 256), dtype=np.uint32)
    prev = start0
    for i in range(nb):
        blk = bytes(packed[int(off[i]):int(off[i + 1])])
        v, used = oracle_lib.decode("256v32", blk, 256, d1=True, start=prev)
        assert used == len(blk)
        out[i] = v
        prev = int(v[-1])
    return out
