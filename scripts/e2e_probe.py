"""Host-path probe (measurement tool): how fast can values reach pinned host
memory?  (a) tpf_host_dec (H2D / decode / D2H chunks on 3 streams), (b) plain
pinned copies, (c) the decode kernel storing straight into pinned host memory
(input in HBM), (d) the kernel reading its input from pinned host memory too, (e) SDMA upload
and SDMA download at once on two streams, (f) SDMA upload and the copy kernel
writing host memory at once, (g) the copy kernel alone, (h) tpf_host_enc.
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

    for mode in ("sdma", "kernel"):
        os.environ["TPF_HOST_DOWN"] = mode
        h_out.zero_()
        t = timed(host_dec)
        ok = torch.equal(h_out, vals.cpu())
        print(f"(a) tpf_host_dec [{mode:6s}] {ints / t / 1e9:7.2f} G int32/s  ok={ok}")
    os.environ.pop("TPF_HOST_DOWN")
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

    # (e)/(f)/(g): do the two directions overlap?
    n_up = h_in.numel()
    d_in2 = torch.empty_like(packed)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    L.tpf_copy_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]

    def both_sdma():
        with torch.cuda.stream(s1):
            d_in2.copy_(h_in, non_blocking=True)
        with torch.cuda.stream(s2):
            h_out.copy_(d_out, non_blocking=True)

    t = timed(both_sdma)
    print(f"(e) SDMA up + SDMA down    {(n_up + ints * 4) / t / 1e9:7.2f} GB/s combined ({t * 1e3:.1f} ms)")

    def kdown():
        assert L.tpf_copy_async(h_out.data_ptr(), d_out.data_ptr(), ints * 4, ctypes.c_void_p(s2.cuda_stream)) == 0

    def sdma_up_kdown():
        with torch.cuda.stream(s1):
            d_in2.copy_(h_in, non_blocking=True)
        kdown()

    t = timed(sdma_up_kdown)
    print(f"(f) SDMA up + kernel down  {(n_up + ints * 4) / t / 1e9:7.2f} GB/s combined ({t * 1e3:.1f} ms)")
    t = timed(kdown)
    print(f"(g) kernel down            {ints * 4 / t / 1e9:7.2f} GB/s")
    d_out.copy_(vals)
    h_out.zero_()
    kdown()
    torch.cuda.synchronize()
    print(f"(g) kernel down verified   {torch.equal(h_out, d_out.cpu())}")
    # (h) host encode
    L.tpf_host_enc.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    h_vals = vals.cpu().pin_memory()
    cap = nb * 1040 + 64
    h_pk = torch.empty(cap, dtype=torch.uint8).pin_memory()
    h_po = torch.empty(nb + 1, dtype=torch.int64).pin_memory()

    def host_enc():
        assert L.tpf_host_enc(2, h_vals.data_ptr(), nb, 256, 0, None, 0, h_pk.data_ptr(), cap, h_po.data_ptr()) == 0

    for mode in ("sdma", "kernel"):
        os.environ["TPF_HOST_DOWN"] = mode
        h_pk.zero_()
        t = timed(host_enc)
        ok = torch.equal(h_po, h_off.view(torch.int64)) and torch.equal(h_pk[: h_in.numel()], h_in)
        print(f"(h) tpf_host_enc [{mode:6s}] {ints / t / 1e9:7.2f} G int32/s  ok={ok}")
    os.environ.pop("TPF_HOST_DOWN")


if __name__ == "__main__":
    main()
