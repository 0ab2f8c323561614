"""Debug: phase A block sums (D1Chain.sums workspace) vs the oracle's, for a
datagen posting list; prints the first mismatching blocks and their headers."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import turbopfor_amd as tpf  # noqa: E402
import datagen  # noqa: E402
import oracle_lib  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 200003
start0 = 11
vals, _ = datagen.c3_postings(nb, seed=3)
vals = (vals.astype(np.uint64) + start0 + 1).astype(np.uint32)
starts = np.concatenate([[start0], vals[:-1, -1]]).astype(np.uint32)
pk, off = oracle_lib.enc256v32_batch(vals, starts=starts)
exp = ((vals[:, -1].astype(np.int64) - starts.astype(np.int64)) & 0xFFFFFFFF).astype(np.uint32)
dev = "cuda:0"
packed = torch.from_numpy(pk).to(dev)
offs = torch.from_numpy(off.astype(np.int64)).to(dev)
ch = tpf.D1Chain(packed, offs, nb)
err = torch.zeros(1, dtype=torch.int64, device=dev)
ch.sums(err=err)
torch.cuda.synchronize()
got = ch.ws[: 4 * nb].view(torch.int32).cpu().numpy().view(np.uint32)
bad = np.nonzero(got != exp)[0]
print("err", int(err.item()), "bad blocks", len(bad), "first", bad[:20].tolist())
for i in bad[:8]:
    o = int(off[i])
    print(i, "run", i // 64, "lane", i % 64, "h", hex(pk[o]), "x1", pk[o + 1], "len", int(off[i + 1] - off[i]),
          "got", got[i], "exp", exp[i], "diff", (int(got[i]) - int(exp[i])) & 0xFFFFFFFF)
