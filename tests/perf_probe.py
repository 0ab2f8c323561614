"""Quick decode-throughput probe (development aid, not the bench): reference-
encodes C2-style blocks per bit width on the CPU, then times the GPU decoder."""
import sys
import time

import numpy as np
import torch

_T = __file__.rsplit("/", 1)[0]
sys.path.insert(0, _T)
sys.path.insert(0, _T + "/../turbopfor-cpp_amd/python")
import datagen  # noqa: E402
import ref_lib  # noqa: E402
import turbopfor_amd as tpf  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 400000
    rows = []
    for bw in [1, 4, 8, 12, 16, 20, 24, 28, 32]:
        t0 = time.time()
        blocks = datagen.c2_blocks(nb, bw, 10)
        packed, off = ref_lib.enc256v32_stream(blocks)
        tenc = time.time() - t0
        d_in = torch.from_numpy(packed).cuda()
        d_off = torch.from_numpy(off.astype(np.int64)).cuda()
        out = torch.empty((nb, 256), dtype=torch.int32, device="cuda")
        err = torch.zeros(1, dtype=torch.int64, device="cuda")
        tpf.dec256v32(d_in, d_off, nb, out=out, err=err)
        torch.cuda.synchronize()
        ok = np.array_equal(out.cpu().numpy().view(np.uint32), blocks)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            tpf.dec256v32(d_in, d_off, nb, out=out)
        reps = 20
        e0.record()
        for _ in range(reps):
            tpf.dec256v32(d_in, d_off, nb, out=out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        gint = nb * 256 / ms / 1e6
        bpb = len(packed) / nb
        gbs = (len(packed) + nb * (1024 + 8)) / ms / 1e6
        rows.append((bw, bpb, ms, gint, gbs, ok, int(err.item())))
        print(f"bw={bw:2d} B/blk={bpb:7.1f} ms={ms:7.3f} Gint/s={gint:8.1f} GB/s={gbs:7.1f} ok={ok} err={int(err.item())} enc_s={tenc:.1f}",
              flush=True)


if __name__ == "__main__":
    main()
