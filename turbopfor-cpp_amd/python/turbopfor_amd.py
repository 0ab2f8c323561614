"""Python host binding of libturbopfor_amd.so (ctypes over the C-ABI in
include/turbopfor_gpu.h).  Device buffers are torch tensors on a HIP device;
kernels run on torch's current stream.  There is no CPU fallback: every
entry point raises if the HIP library or device is missing.

Reference interface mirrored: include/turbopfor.h of amosbird/TurboPFor-CPP
(per-block p4Enc*/p4Dec*), lifted to batches of blocks with explicit byte
offsets (the reference's callers chain blocks through the returned pointer).
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(_HERE)
# TPF_LIB: load another build of the library (A/B measurements only)
LIB_PATH = os.environ.get("TPF_LIB") or os.path.join(PKG_DIR, "lib", "libturbopfor_amd.so")

_lib = None

c_u64 = ctypes.c_uint64
c_vp = ctypes.c_void_p


class TpfError(RuntimeError):
    pass


def build():
    subprocess.check_call(["make", "-s", "-C", PKG_DIR, f"-j{min(os.cpu_count() or 4, 16)}"])


def _md5(files, root):
    import hashlib

    h = hashlib.md5()
    for f in sorted(files):
        h.update(os.path.relpath(f, root).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def source_md5():
    """md5 over the library's sources (turbopfor-cpp_amd/csrc/*, its Makefile
    and include/*.h, sorted by path; path and contents): the identity of the
    build (build_stamp.json).  (The built .so's own bytes differ when the same
    sources are rebuilt elsewhere -- e.g. a build on the GPU box embeds that
    box's paths -- so they do not identify the code.)"""
    root = os.path.dirname(PKG_DIR)
    files = [os.path.join(PKG_DIR, "Makefile")]
    for d in (os.path.join(PKG_DIR, "csrc"), os.path.join(root, "include")):
        files += [os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".hip", ".cpp"))]
    return _md5(files, root)


def kernel_md5():
    """md5 over the DEVICE code only (csrc/*.hip, csrc/*.h, the Makefile's
    flags): the identity of the kernels a PMC traffic measurement was taken
    with.  Host-side edits (host_api.cpp, host_stream.cpp, include/) do not
    change what a kernel moves, so they do not invalidate the measurement."""
    root = os.path.dirname(PKG_DIR)
    d = os.path.join(PKG_DIR, "csrc")
    files = [os.path.join(PKG_DIR, "Makefile")] + [os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".hip"))]
    return _md5(files, root)


def lib():
    """Load (building if needed) the in-tree HIP library."""
    global _lib
    if _lib is None:
        # torch bundles its own libamdhip64 (soname libamdhip64.so.7, file
        # name libamdhip64.so).  Load it first so our library binds to that
        # same HIP runtime instead of a second copy from /opt/rocm.
        import torch  # noqa: F401

        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.tpf_last_error.restype = ctypes.c_char_p
        L.tpf_device_count.restype = ctypes.c_int
        L.tpf_p4dec256v32_batch.argtypes = [c_vp, c_u64, c_vp, c_u64, c_vp, c_vp, c_vp]
        L.tpf_p4d1dec256v32_batch.argtypes = [c_vp, c_u64, c_vp, c_u64, c_vp, c_vp, c_vp, c_vp]
        L.tpf_p4enc256v32_bound.argtypes = [c_u64]
        L.tpf_p4enc256v32_bound.restype = c_u64
        L.tpf_p4enc256v32_workspace_size.argtypes = [c_u64]
        L.tpf_p4enc256v32_workspace_size.restype = ctypes.c_size_t
        L.tpf_p4enc256v32_batch.argtypes = [c_vp, c_u64, c_vp, c_u64, c_vp, c_vp, ctypes.c_size_t, c_vp]
        L.tpf_p4d1enc256v32_batch.argtypes = [c_vp, c_u64, c_vp, ctypes.c_uint32, c_vp, c_u64, c_vp, c_vp,
                                              ctypes.c_size_t, c_vp]
        L.tpf_enc_bound.argtypes = [ctypes.c_int, c_u64, ctypes.c_uint]
        L.tpf_enc_bound.restype = c_u64
        L.tpf_enc_workspace_size.argtypes = [ctypes.c_int, c_u64, ctypes.c_uint]
        L.tpf_enc_workspace_size.restype = ctypes.c_size_t
        L.tpf_dec_batch.argtypes = [ctypes.c_int, c_vp, c_u64, c_vp, c_u64, ctypes.c_uint, c_vp, c_vp, c_vp, c_vp]
        L.tpf_enc_batch.argtypes = [ctypes.c_int, c_vp, c_u64, ctypes.c_uint, ctypes.c_int, c_vp, c_u64, c_vp, c_u64,
                                    c_vp, c_vp, ctypes.c_size_t, c_vp]
        L.tpf_p4d1dec256v32_chain_workspace_size.argtypes = [c_u64]
        L.tpf_p4d1dec256v32_chain_workspace_size.restype = ctypes.c_size_t
        L.tpf_p4d1dec256v32_chained.argtypes = [c_vp, c_u64, c_vp, c_u64, c_vp, ctypes.c_uint32, c_vp, ctypes.c_size_t,
                                                c_vp, c_vp]
        L.tpf_p4d1dec256v32_chain_sums.argtypes = [c_vp, c_u64, c_vp, c_u64, c_vp, ctypes.c_size_t, c_vp, c_vp, c_vp]
        L.tpf_p4d1dec256v32_chain_decode.argtypes = [c_vp, c_u64, c_vp, c_u64, c_vp, ctypes.c_uint32, c_vp, c_vp, c_vp]
        L.tpf_p4nenc256v32_bound.argtypes = [c_u64]
        L.tpf_p4nenc256v32_bound.restype = c_u64
        L.tpf_p4nenc256v32_workspace_size.argtypes = [c_u64]
        L.tpf_p4nenc256v32_workspace_size.restype = ctypes.c_size_t
        L.tpf_p4nenc256v32.argtypes = [c_vp, c_u64, ctypes.c_int, ctypes.c_uint32, c_vp, c_u64, c_vp, c_vp,
                                       ctypes.c_size_t, c_vp]
        L.tpf_p4ndec256v32_workspace_size.argtypes = [c_u64]
        L.tpf_p4ndec256v32_workspace_size.restype = ctypes.c_size_t
        L.tpf_p4ndec256v32.argtypes = [c_vp, c_u64, c_vp, c_u64, ctypes.c_int, ctypes.c_uint32, c_vp, c_vp,
                                       ctypes.c_size_t, c_vp, c_vp]
        # round-4 entry points: absent from older builds loaded through TPF_LIB for A/B runs
        if hasattr(L, "tpf_d1dec64_chained"):
            L.tpf_d1dec64_chain_workspace_size.argtypes = [c_u64]
            L.tpf_d1dec64_chain_workspace_size.restype = ctypes.c_size_t
            L.tpf_d1dec64_chained.argtypes = [ctypes.c_int, c_vp, c_u64, c_vp, c_u64, c_vp, c_u64, c_vp, ctypes.c_size_t, c_vp, c_vp]
            L.tpf_d1dec64_chain_sums.argtypes = [ctypes.c_int, c_vp, c_u64, c_vp, c_u64, c_vp, ctypes.c_size_t, c_vp, c_vp, c_vp]
            L.tpf_d1dec64_chain_decode.argtypes = [ctypes.c_int, c_vp, c_u64, c_vp, c_u64, c_vp, c_u64, c_vp, c_vp, c_vp]
            for name in ("tpf_d1dec64_chained", "tpf_d1dec64_chain_sums", "tpf_d1dec64_chain_decode"):
                getattr(L, name).restype = ctypes.c_int
        for name in ("tpf_p4nenc256v32", "tpf_p4ndec256v32", "tpf_p4dec256v32_batch", "tpf_p4d1dec256v32_batch", "tpf_p4enc256v32_batch",
                     "tpf_p4d1enc256v32_batch", "tpf_dec_batch", "tpf_enc_batch", "tpf_p4d1dec256v32_chained",
                     "tpf_p4d1dec256v32_chain_sums", "tpf_p4d1dec256v32_chain_decode"):
            getattr(L, name).restype = ctypes.c_int
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise TpfError(f"turbopfor_amd error {rc}: {lib().tpf_last_error().decode()}")


def _stream(torch):
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def dec256v32(packed, offsets, nblocks, out=None, starts=None, err=None):
    """Decode nblocks 256v32 blocks.  packed: uint8 CUDA tensor; offsets:
    int64 CUDA tensor [nblocks+1]; starts: optional int32 [nblocks] for the
    delta-1 variant (p4D1Dec256v32).  Returns int32 tensor [nblocks, 256]
    (bit pattern = uint32)."""
    import torch

    if out is None:
        out = torch.empty((nblocks, 256), dtype=torch.int32, device=packed.device)
    L = lib()
    if starts is None:
        rc = L.tpf_p4dec256v32_batch(_ptr(packed), packed.numel(), _ptr(offsets), nblocks, _ptr(out), _ptr(err),
                                     _stream(torch))
    else:
        rc = L.tpf_p4d1dec256v32_batch(_ptr(packed), packed.numel(), _ptr(offsets), nblocks, _ptr(out),
                                       _ptr(starts), _ptr(err), _stream(torch))
    _check(rc)
    return out


# ---- the measurement / test library (measure/tpf_measure.h) --------------
# Not the codec: kernel probes, device ceilings, forced encoder paths and the
# run-scan test hook, loaded only by bench.py, the GPU tests and scripts/.
MEASURE_PATH = os.path.join(PKG_DIR, "lib", "libtpf_measure.so")
_mlib = None


def measure():
    """Load lib/libtpf_measure.so (after the codec library it links)."""
    global _mlib
    if _mlib is None:
        lib()
        if not os.path.exists(MEASURE_PATH):
            build()
        M = ctypes.CDLL(MEASURE_PATH)
        M.tpfm_probe256v32.argtypes = [c_vp, c_u64, c_vp, c_u64, c_vp, c_vp]
        M.tpfm_dec256v32_path.argtypes = [ctypes.c_int, c_vp, c_u64, c_vp, c_u64, c_vp, c_vp]
        M.tpfm_probe256v64.argtypes = [c_vp, c_u64, c_vp, c_u64, c_vp, c_vp]
        M.tpfm_probe_hbm.argtypes = [ctypes.c_int, c_vp, c_vp, c_u64, c_vp]
        M.tpfm_enc256v32.argtypes = [ctypes.c_int, c_vp, c_u64, ctypes.c_int, c_vp, ctypes.c_uint32, c_vp, c_u64, c_vp, c_vp,
                                     ctypes.c_size_t, c_vp]
        M.tpfm_enc256v32_workspace_size.argtypes = [ctypes.c_int, c_u64]
        M.tpfm_enc256v32_workspace_size.restype = ctypes.c_size_t
        M.tpfm_run_scan_workspace_size.argtypes = [c_u64]
        M.tpfm_run_scan_workspace_size.restype = ctypes.c_size_t
        M.tpfm_run_scan.argtypes = [c_vp, c_u64, c_vp, c_vp, c_vp, ctypes.c_size_t, c_vp]
        for name in ("tpfm_probe256v32", "tpfm_probe256v64", "tpfm_probe_hbm", "tpfm_enc256v32", "tpfm_run_scan"):
            getattr(M, name).restype = ctypes.c_int
        _mlib = M
    return _mlib


def _mcheck(rc, what):
    if rc != 0:
        raise TpfError(f"{what}: measurement library error {rc}")


def probe256v64(packed, offsets, nunits, out):
    """Measurement only: the 256v64 decode kernel's loads and stores without
    the decoding (tpfm_probe256v64)."""
    import torch

    _mcheck(measure().tpfm_probe256v64(_ptr(packed), packed.numel(), _ptr(offsets), nunits, _ptr(out), _stream(torch)),
            "tpfm_probe256v64")
    return out


def probe256v32(packed, offsets, nblocks, out):
    """Measurement only: the decode kernel's loads and stores without the
    decoding (data-movement ceiling of the hot path's access pattern)."""
    import torch

    _mcheck(measure().tpfm_probe256v32(_ptr(packed), packed.numel(), _ptr(offsets), nblocks, _ptr(out), _stream(torch)),
            "tpfm_probe256v32")
    return out


def dec256v32_path(grouped, packed, offsets, nblocks, out):
    """Measurement only: the plain 256v32 decode through a forced load path
    (tpfm_dec256v32_path: grouped 0 = single-block pipeline, 1 = grouped 1 KB
    loads; the library chooses per launch)."""
    import torch

    _mcheck(measure().tpfm_dec256v32_path(1 if grouped else 0, _ptr(packed), packed.numel(), _ptr(offsets), nblocks, _ptr(out),
                                          _stream(torch)), "tpfm_dec256v32_path")
    return out


def probe_hbm(kind, dst, src, nbytes):
    """Measurement only: streaming ceiling kernels (tpfm_probe_hbm): kind
    "read" (src), "write" (dst) or "copy" (src -> dst) of nbytes bytes."""
    import torch

    k = {"read": 0, "write": 1, "copy": 2}[kind]
    _mcheck(measure().tpfm_probe_hbm(k, _ptr(dst), _ptr(src), nbytes, _stream(torch)), "tpfm_probe_hbm")


def enc256v32_path(mode, values, out, d1=False, starts=None, start0=0):
    """The 256v32 encoder through a forced path (tpfm_enc256v32): mode 1 =
    plan pass as a wave OR, 2 = write pass copying values (plain only, not a
    valid stream), 3 = the two-pass encoder (the library's), 4 / 5 = the slot
    encoder with / without the fused scans (measured, not adopted).  Returns
    the offsets tensor [nblocks+1]."""
    import torch

    nb = values.numel() // 256
    offs = torch.empty(nb + 1, dtype=torch.int64, device=values.device)
    ws_bytes = int(measure().tpfm_enc256v32_workspace_size(mode, nb))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=values.device)
    _mcheck(measure().tpfm_enc256v32(mode, _ptr(values), nb, 1 if d1 else 0, _ptr(starts), ctypes.c_uint32(start0 & 0xFFFFFFFF),
                                     _ptr(out), out.numel(), _ptr(offs), _ptr(ws), ws_bytes, _stream(torch)), "tpfm_enc256v32")
    return offs


def enc256v32(values, d1=False, starts=None, start0=0, out=None):
    """Encode values (int32/uint32-bit CUDA tensor, nblocks*256 elements) as
    256v32 P4 blocks.  Returns (packed uint8 tensor sized to the encoded
    total, offsets int64 tensor [nblocks+1]).  d1 selects p4D1Enc256v32:
    starts (int32 [nblocks]) gives each block's preceding value, or with
    starts=None the blocks form one chained list starting after start0."""
    import torch

    assert values.is_cuda and values.dtype in (torch.int32,) and values.numel() % 256 == 0
    values = values.contiguous()
    nb = values.numel() // 256
    L = lib()
    cap = int(L.tpf_p4enc256v32_bound(nb))
    if out is None:
        out = torch.empty(cap, dtype=torch.uint8, device=values.device)
    offs = torch.empty(nb + 1, dtype=torch.int64, device=values.device)
    ws_bytes = int(L.tpf_p4enc256v32_workspace_size(nb))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=values.device)
    if d1:
        rc = L.tpf_p4d1enc256v32_batch(_ptr(values), nb, _ptr(starts), ctypes.c_uint32(start0 & 0xFFFFFFFF),
                                       _ptr(out), out.numel(), _ptr(offs), _ptr(ws), ws_bytes, _stream(torch))
    else:
        rc = L.tpf_p4enc256v32_batch(_ptr(values), nb, _ptr(out), out.numel(), _ptr(offs), _ptr(ws), ws_bytes,
                                     _stream(torch))
    _check(rc)
    total = int(offs[-1].item())
    return out[:total], offs


# ---- every turbopfor.h family (include/turbopfor_gpu.h tpf_{enc,dec}_batch) ----
FMT = {"32": 0, "128v32": 1, "256v32": 2, "64": 3, "128v64": 4, "256v64": 5}
_WIDE = {"64", "128v64", "256v64"}
_UNIT = {"128v32": 128, "256v32": 256, "128v64": 128, "256v64": 256}


def unit_values(fmt, n):
    return _UNIT.get(fmt, n)


def enc_batch(fmt, values, nblocks, n, d1=False, starts=None, start0=0, out=None, offs=None, ws=None):
    """values: int32/int64 CUDA tensor with nblocks*unit_values(fmt, n)
    elements (bit patterns of uint32/uint64).  Returns (packed, offsets).
    out / offs / ws: optional preallocated buffers (reused across calls)."""
    import torch

    values = values.contiguous()
    assert values.numel() == nblocks * unit_values(fmt, n)
    L = lib()
    f = FMT[fmt]
    cap = int(L.tpf_enc_bound(f, nblocks, n))
    if out is None:
        out = torch.empty(cap, dtype=torch.uint8, device=values.device)
    assert out.numel() >= cap
    cap = out.numel()
    if offs is None:
        offs = torch.empty(nblocks + 1, dtype=torch.int64, device=values.device)
    wsb = int(L.tpf_enc_workspace_size(f, nblocks, n))
    if ws is None or ws.numel() < wsb:
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=values.device)
    wsb = ws.numel()
    rc = L.tpf_enc_batch(f, _ptr(values), nblocks, n, 1 if d1 else 0, _ptr(starts),
                         ctypes.c_uint64(start0 & ((1 << 64) - 1)), _ptr(out), cap, _ptr(offs), _ptr(ws), wsb,
                         _stream(torch))
    _check(rc)
    return out[: int(offs[-1].item())], offs


def dec_batch(fmt, packed, offsets, nblocks, n, starts=None, err=None, out=None):
    import torch

    dt = torch.int64 if fmt in _WIDE else torch.int32
    if out is None:
        out = torch.zeros(nblocks * unit_values(fmt, n), dtype=dt, device=packed.device)
    L = lib()
    rc = L.tpf_dec_batch(FMT[fmt], _ptr(packed), packed.numel(), _ptr(offsets), nblocks, n, _ptr(out), _ptr(starts),
                         _ptr(err), _stream(torch))
    _check(rc)
    return out


# ---- chained delta-1 decode of one posting list (f1) ----------------------
class D1Chain:
    """Two-phase chained p4D1Dec256v32 over one list: sums() decodes every
    block's delta sum and its prefix (returns the shard total as a 1-element
    int32 CUDA tensor), decode(base) writes the values.  A multi-GPU list
    runs sums() on every shard, exchanges the totals, then decode() with
    base = start0 + sum of earlier shards' totals (mod 2^32)."""

    def __init__(self, packed, offsets, nblocks):
        import torch

        self.packed, self.offsets, self.nblocks = packed, offsets, nblocks
        L = lib()
        self.ws_bytes = int(L.tpf_p4d1dec256v32_chain_workspace_size(nblocks))
        self.ws = torch.empty(max(self.ws_bytes, 1), dtype=torch.uint8, device=packed.device)
        self.total = torch.zeros(1, dtype=torch.int32, device=packed.device)

    def sums(self, err=None):
        import torch

        rc = lib().tpf_p4d1dec256v32_chain_sums(_ptr(self.packed), self.packed.numel(), _ptr(self.offsets), self.nblocks,
                                                _ptr(self.ws), self.ws_bytes, _ptr(self.total), _ptr(err),
                                                _stream(torch))
        _check(rc)
        return self.total

    def decode(self, base, out=None, err=None):
        import torch

        if out is None:
            out = torch.empty((self.nblocks, 256), dtype=torch.int32, device=self.packed.device)
        rc = lib().tpf_p4d1dec256v32_chain_decode(_ptr(self.packed), self.packed.numel(), _ptr(self.offsets),
                                                  self.nblocks, _ptr(out), ctypes.c_uint32(base & 0xFFFFFFFF),
                                                  _ptr(self.ws), _ptr(err), _stream(torch))
        _check(rc)
        return out


def dec256v32_chained(packed, offsets, nblocks, start0=0, out=None, err=None, ws=None):
    """One chained list (block i starts from block i-1's last value, block 0
    from start0): tpf_p4d1dec256v32_chained (block sums + scan, then decode).
    ws: optional reusable uint8 workspace tensor."""
    import torch

    if out is None:
        out = torch.empty((nblocks, 256), dtype=torch.int32, device=packed.device)
    L = lib()
    ws_bytes = int(L.tpf_p4d1dec256v32_chain_workspace_size(nblocks))
    if ws is None or ws.numel() < ws_bytes:
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=packed.device)
    rc = L.tpf_p4d1dec256v32_chained(_ptr(packed), packed.numel(), _ptr(offsets), nblocks, _ptr(out),
                                     ctypes.c_uint32(start0 & 0xFFFFFFFF), _ptr(ws), ws.numel(), _ptr(err),
                                     _stream(torch))
    _check(rc)
    return out


def dec64_chained(fmt, packed, offsets, nunits, start0=0, out=None, err=None, ws=None):
    """One chained 64-bit list of fmt "256v64" or "128v64" units (unit i
    starts from unit i-1's last value, unit 0 from start0): tpf_d1dec64_chained
    (unit sums + scan, then decode).  Returns int64 [nunits, 256 or 128]."""
    import torch

    width = _UNIT[fmt]
    if out is None:
        out = torch.empty((nunits, width), dtype=torch.int64, device=packed.device)
    L = lib()
    ws_bytes = int(L.tpf_d1dec64_chain_workspace_size(nunits))
    if ws is None or ws.numel() < ws_bytes:
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=packed.device)
    rc = L.tpf_d1dec64_chained(FMT[fmt], _ptr(packed), packed.numel(), _ptr(offsets), nunits, _ptr(out),
                               ctypes.c_uint64(start0 & 0xFFFFFFFFFFFFFFFF), _ptr(ws), ws.numel(), _ptr(err), _stream(torch))
    _check(rc)
    return out


# ---- n-variant streams (include/turbopfor_gpu.h tpf_p4nenc256v32) ----------
def n_units(n):
    """Blocks in an n-value stream: n // 256 256v32 blocks + one p4Enc32 tail."""
    return n // 256 + (1 if n % 256 else 0)


def encn256v32(values, d1=False, start0=0):
    """Encode any number of int32 values as the stream the reference produces
    by chaining p4Enc256v32 over the full 256-blocks and p4Enc32 over the
    remainder (p4D1* with d1, one list starting after start0).  Returns
    (packed uint8 tensor, offsets int64 [n_units(n) + 1])."""
    import torch

    assert values.is_cuda and values.dtype == torch.int32
    values = values.contiguous().view(-1)
    n = values.numel()
    L = lib()
    cap = int(L.tpf_p4nenc256v32_bound(n))
    out = torch.empty(cap, dtype=torch.uint8, device=values.device)
    offs = torch.empty(n_units(n) + 1, dtype=torch.int64, device=values.device)
    ws_bytes = int(L.tpf_p4nenc256v32_workspace_size(n))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=values.device)
    _check(L.tpf_p4nenc256v32(_ptr(values), n, int(bool(d1)), ctypes.c_uint32(start0 & 0xFFFFFFFF), _ptr(out), cap,
                              _ptr(offs), _ptr(ws), ws_bytes, _stream(torch)))
    return out[:int(offs[-1].item())], offs


def decn256v32(packed, offsets, n, d1=False, start0=0, out=None, err=None):
    """Decode an n-value stream of encn256v32's layout (offsets: n_units(n)+1)."""
    import torch

    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=packed.device)
    L = lib()
    ws_bytes = int(L.tpf_p4ndec256v32_workspace_size(n))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=packed.device)
    _check(L.tpf_p4ndec256v32(_ptr(packed), packed.numel(), _ptr(offsets), n, int(bool(d1)),
                              ctypes.c_uint32(start0 & 0xFFFFFFFF), _ptr(out), _ptr(ws), ws_bytes, _ptr(err),
                              _stream(torch)))
    return out
