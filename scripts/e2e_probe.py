"""Host-path probe (measurement tool): how fast can values reach pinned host
memory?  (a) tpf_host_dec (H2D / decode / D2H chunks on 3 streams), (b) plain
pinned copies, (c) the decode kernel storing straight into pinned host memory
(input in HBM), (d) the kernel reading its input from pinned host memory too.
usage: python scripts/e2e_probe.py [nblocks]"""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, ROOT)
import turbopfor_amd as tpf  # noqa: E402
import bench  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    dev = torch.device("cuda:0")
    vals, _ = bench.gen_c2(nb, 10.0, seed=1, dev=dev)
    packed, offs = tpf.enc256v32(vals)
    packed = packed.clone()
    torch.cuda.synchronize()
    L = tpf.lib()
    h_in = packed.cpu().pin_memory()
    h_off = offs.cpu().pin_memory()
    h_out = torch.empty((nb, 256), dtype=torch.int32).pin_memory()
    ints = nb * 256
    L.tpf_host_dec.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                               ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]

    def host_dec():
        assert L.tpf_host_dec(2, h_in.data_ptr(), h_in.numel(), h_off.data_ptr(), nb, 256, h_out.data_ptr(), None) == 0

    t = timed(host_dec)
    ok = torch.equal(h_out, vals.cpu())
    print(f"(a) tpf_host_dec          {ints / t / 1e9:7.2f} G int32/s  ok={ok}")
    d_out = torch.empty((nb, 256), dtype=torch.int32, device=dev)
    t = timed(lambda: h_out.copy_(d_out, non_blocking=True))
    print(f"(b) D2H copy              {h_out.numel() * 4 / t / 1e9:7.2f} GB/s")
    t = timed(lambda: packed.copy_(h_in, non_blocking=True))
    print(f"(b) H2D copy              {h_in.numel() / t / 1e9:7.2f} GB/s")
    h_out.zero_()
    t = timed(lambda: tpf.dec256v32(packed, offs, nb, out=h_out))
    ok = torch.equal(h_out, vals.cpu())
    print(f"(c) kernel -> host        {ints / t / 1e9:7.2f} G int32/s  ({ints * 4 / t / 1e9:.1f} GB/s written)  ok={ok}")
    h_out.zero_()
    t = timed(lambda: tpf.dec256v32(h_in, offs, nb, out=h_out))
    ok = torch.equal(h_out, vals.cpu())
    print(f"(d) host -> kernel -> host {ints / t / 1e9:7.2f} G int32/s  ok={ok}")


if __name__ == "__main__":
    main()
