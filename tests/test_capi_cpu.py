"""CPU-only checks of the drop-in boundary: the HIP library loads without a
GPU, exports every symbol include/*.h declares (C-ABI names and the C++
turbopfor:: mangled names), reports TPF_ENODEV instead of falling back to a
CPU codec, and its host-side framing (block lengths / stream offsets) agrees
with the golden fixtures from the reference."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import golden_io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "turbopfor-cpp_amd", "lib", "libturbopfor_amd.so")
FMT = {"32": 0, "128v32": 1, "256v32": 2, "64": 3, "128v64": 4, "256v64": 5}


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "turbopfor-cpp_amd"), "-j8"])
    return ctypes.CDLL(LIB)


def declared_c_symbols():
    names = set()
    for h in ("turbopfor_gpu.h", "turbopfor_capi.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names |= set(re.findall(r"\b(tpf_\w+)\s*\(", txt))
    return names


def test_exports_every_declared_symbol(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = sorted(s for s in declared_c_symbols() if s not in exported)
    assert not missing, missing
    # the C++ turbopfor:: surface of include/turbopfor.h (24 functions)
    cpp = [s for s in exported if s.startswith("_ZN9turbopfor")]
    assert len(cpp) == 24, sorted(cpp)
    assert "_ZN9turbopfor11p4Dec256v32EPKhjPj" in exported  # mangled name of the reference's p4Dec256v32


def test_no_cpu_fallback_without_device(lib):
    if subprocess.run(["python", "-c", "import torch,sys;sys.exit(0 if torch.cuda.is_available() else 1)"]).returncode == 0:
        pytest.skip("a HIP device is visible")
    lib.tpf_p4dec256v32_batch.restype = ctypes.c_int
    rc = lib.tpf_p4dec256v32_batch(None, 0, None, ctypes.c_uint64(1), None, None, None)
    assert rc == -3  # TPF_ENODEV
    lib.tpf_last_error.restype = ctypes.c_char_p
    assert b"no CPU fallback" in lib.tpf_last_error()
    # the host-stream entry points (one and several GPUs) fail the same way
    devs = (ctypes.c_int * 2)(0, 1)
    data = (ctypes.c_uint8 * 64)()
    vals = (ctypes.c_uint32 * 256)()
    lib.tpf_host_dec_multi.restype = ctypes.c_int
    assert lib.tpf_host_dec_multi(devs, 2, 2, data, ctypes.c_uint64(64), None, ctypes.c_uint64(1), 256, vals, None) == -3
    assert b"no CPU fallback" in lib.tpf_last_error()
    lib.tpf_p4Dec256v32.restype = ctypes.c_void_p
    buf = (ctypes.c_uint8 * 64)()
    out = (ctypes.c_uint32 * 256)()
    assert lib.tpf_p4Dec256v32(buf, 256, out) is None


def test_perblock_mode_query_and_set(lib):
    """tpf_perblock_mode: < 0 queries, 0/1/2 select a design, anything else
    means the default (0); each call returns the previous mode.  No server
    exists on a machine without a device, so the switch touches no GPU."""
    lib.tpf_perblock_mode.restype = ctypes.c_int
    lib.tpf_perblock_mode.argtypes = [ctypes.c_int]
    prev = lib.tpf_perblock_mode(-1)
    try:
        assert lib.tpf_perblock_mode(2) == prev
        assert lib.tpf_perblock_mode(-1) == 2
        assert lib.tpf_perblock_mode(1) == 2
        assert lib.tpf_perblock_mode(7) == 1
        assert lib.tpf_perblock_mode(-5) == 0
    finally:
        lib.tpf_perblock_mode(prev)


@pytest.mark.parametrize("fname,fmt", [("g32.bin", "32"), ("g128v32.bin", "128v32"), ("g256v32.bin", "256v32"),
                                       ("g128v64.bin", "128v64"), ("g256v64.bin", "256v64")])
def test_framing_matches_golden(lib, fname, fmt):
    lib.tpf_block_size.restype = ctypes.c_uint64
    lib.tpf_block_size.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint,
                                   ctypes.POINTER(ctypes.c_int)]
    lib.tpf_scan_offsets.restype = ctypes.c_int64
    lib.tpf_scan_offsets.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_uint64,
                                     ctypes.POINTER(ctypes.c_uint64)]
    recs = golden_io.load(fname)
    w = ctypes.c_int()
    for i, r in enumerate(recs):
        assert lib.tpf_block_size(FMT[fmt], r.enc, len(r.enc), r.n, ctypes.byref(w)) == len(r.enc), (fmt, i)
        assert lib.tpf_block_size(FMT[fmt], r.enc, len(r.enc) - 1, r.n, None) == 0, (fmt, i)  # truncated
    by_n = {}
    for r in recs:
        by_n.setdefault(r.n, []).append(r.enc)
    for n, encs in by_n.items():
        stream = b"".join(encs)
        off = (ctypes.c_uint64 * (len(encs) + 1))()
        assert lib.tpf_scan_offsets(FMT[fmt], stream, len(stream), n, len(encs), off) == len(stream)
        exp = np.concatenate([[0], np.cumsum([len(e) for e in encs])])
        assert list(off) == exp.tolist()


@pytest.mark.skipif(not os.path.exists("/opt/rocm/include/hip/hip_runtime.h"), reason="no HIP headers")
def test_nested_perblock_pauses(lib, tmp_path):
    """round 4's hs_pause A/B variant aborted with EDEADLK --
    one thread locked the per-block pause (a std::shared_mutex) while holding
    it.  tpf::PerblockPause now counts its own per-thread depth, so nested
    pauses, tpf_perblock_quiesce and tpf_host_release inside a pause, on four
    threads at once, neither throw nor hang (host only: no server runs)."""
    exe = tmp_path / "pause_nesting"
    subprocess.check_call(["g++", "-std=c++20", "-O1", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                           os.path.join(ROOT, "tests", "cpp", "pause_nesting.cpp"), "-L", os.path.dirname(LIB),
                           "-lturbopfor_amd", "-Wl,-rpath," + os.path.dirname(LIB), "-lpthread", "-o", str(exe)])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "pause nesting ok" in r.stdout


def test_host_entries_check_offsets_before_the_device(lib):
    """h_off has nblocks + 1 entries (turbopfor_capi.h).  The
    host entries cannot see the array's length, but they reject what a short
    or foreign array yields -- offsets that decrease or run past in_bytes --
    and a bad (fmt, n) with TPF_EINVAL, on the host, before any device is
    touched: the same answer with or without a GPU."""
    lib.tpf_last_error.restype = ctypes.c_char_p
    lib.tpf_host_dec.restype = ctypes.c_int
    lib.tpf_host_dec_multi.restype = ctypes.c_int
    data = (ctypes.c_uint8 * 4096)()
    vals = (ctypes.c_uint32 * (256 * 4))()
    devs = (ctypes.c_int * 2)(0, 0)
    u64 = ctypes.c_uint64
    cases = [
        ((ctypes.c_uint64 * 5)(0, 10, 20, 30, 5000), b"past in_bytes"),   # ends past the 4096-byte stream
        ((ctypes.c_uint64 * 5)(0, 10, 5, 30, 40), b"decreases at block 1"),
        ((ctypes.c_uint64 * 5)(0, 10, 20, 30, 2 ** 63), b"past in_bytes"),  # garbage read past a short array
    ]
    for off, msg in cases:
        assert lib.tpf_host_dec(2, data, u64(4096), off, u64(4), 256, vals, None) == -1
        assert msg in lib.tpf_last_error(), lib.tpf_last_error()
        assert lib.tpf_host_dec_multi(devs, 2, 2, data, u64(4096), off, u64(4), 256, vals, None) == -1
        assert msg in lib.tpf_last_error(), lib.tpf_last_error()
    good = (ctypes.c_uint64 * 5)(0, 10, 20, 30, 40)
    assert lib.tpf_host_dec(2, data, u64(4096), good, u64(4), 300, vals, None) == -1  # n past the 256v32 unit
    assert b"unsupported" in lib.tpf_last_error()
    assert lib.tpf_host_dec(2, None, u64(4096), good, u64(4), 256, vals, None) == -1
    assert lib.tpf_host_dec_multi(None, 0, 2, data, u64(4096), good, u64(4), 256, vals, None) == -1
