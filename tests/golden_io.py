"""Reader for tests/golden/*.bin (written by oracle/gen_golden.cpp from the
reference's own src/scalar codec).  Test infrastructure only."""
import os
import struct

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class Record:
    __slots__ = ("d1", "decode_only", "padding_unpinned", "n", "start", "esize", "values", "enc")

    def __init__(self, flags, n, start, esize, values, enc):
        self.d1 = bool(flags & 1)
        self.decode_only = bool(flags & 2)
        # flag 4: n below the layout width and the reference's bytes for the
        # padding slots depend on its uninitialised stack (oracle/gen_golden.cpp
        # gen64_short): compare the length and the decoded values, not the bytes
        self.padding_unpinned = bool(flags & 4)
        self.n = n
        self.start = start
        self.esize = esize
        self.values = values
        self.enc = enc


def load(name):
    path = os.path.join(GOLDEN_DIR, name)
    with open(path, "rb") as f:
        data = f.read()
    assert data[:4] == b"TPFG", path
    ver, count = struct.unpack_from("<II", data, 4)
    assert ver == 1
    pos = 12
    recs = []
    for _ in range(count):
        flags, n, start, esize, enc_len = struct.unpack_from("<IIQII", data, pos)
        pos += 24
        dt = np.uint32 if esize == 4 else np.uint64
        vals = np.frombuffer(data, dtype=dt, count=n, offset=pos).copy()
        pos += n * esize
        enc = data[pos : pos + enc_len]
        pos += enc_len
        recs.append(Record(flags, n, start, esize, vals, enc))
    assert pos == len(data)
    return recs
