"""The drop-in boundary on the GPU: the extern "C" per-block mirrors
(include/turbopfor_capi.h, one symbol per reference function) reproduce the
golden fixtures byte- and bit-exact; a reference-style C++ caller linked
against include/turbopfor.h round-trips; the host-memory streams
(tpf_host_dec / tpf_host_enc) match the oracle."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import datagen
import golden_io
import oracle_lib

torch = pytest.importorskip("torch")
tpf = pytest.importorskip("turbopfor_amd")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = {"32": "32", "128v32": "128v32", "256v32": "256v32", "128v64": "128v64", "256v64": "256v64"}


def capi():
    L = tpf.lib()
    return L


@pytest.mark.parametrize("fname,fmt", [("g32.bin", "32"), ("g128v32.bin", "128v32"), ("g256v32.bin", "256v32"),
                                       ("g128v64.bin", "128v64"), ("g256v64.bin", "256v64")])
def test_per_block_mirrors_match_golden(fname, fmt):
    L = capi()
    wide = fmt in ("128v64", "256v64")
    dt = np.uint64 if wide else np.uint32
    vt = ctypes.c_uint64 if wide else ctypes.c_uint32
    recs = golden_io.load(fname)
    step = max(1, len(recs) // 120)  # per-block calls are latency-bound: sample
    for i, r in enumerate(recs[::step]):
        full = tpf.unit_values(fmt, r.n)
        src = np.zeros(full + 64, dtype=dt)
        src[: r.n] = r.values
        out = np.zeros(len(r.enc) + 4096, dtype=np.uint8)
        if not r.decode_only:
            if r.d1:
                f = getattr(L, f"tpf_p4D1Enc{fmt}")
                f.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p, vt]
            else:
                f = getattr(L, f"tpf_p4Enc{fmt}")
                f.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
            f.restype = ctypes.c_void_p
            args = [src.ctypes.data, r.n, out.ctypes.data] + ([r.start] if r.d1 else [])
            end = f(*args)
            assert end is not None, L.tpf_last_error()
            assert bytes(out[: end - out.ctypes.data]) == r.enc, (fmt, i)
        enc = np.frombuffer(r.enc + bytes(64), dtype=np.uint8).copy()
        dec = np.zeros(full + 64, dtype=dt)
        if r.d1:
            g = getattr(L, f"tpf_p4D1Dec{fmt}")
            g.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p, vt]
        else:
            g = getattr(L, f"tpf_p4Dec{fmt}")
            g.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
        g.restype = ctypes.c_void_p
        end = g(*([enc.ctypes.data, r.n, dec.ctypes.data] + ([r.start] if r.d1 else [])))
        assert end - enc.ctypes.data == len(r.enc), (fmt, i)
        np.testing.assert_array_equal(dec[: r.n], r.values, err_msg=f"{fmt} record {i}")


def test_reference_style_cpp_caller(tmp_path):
    exe = tmp_path / "dropin_example"
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "dropin_example.cpp"), "-o", str(exe),
                           "-L", os.path.join(ROOT, "turbopfor-cpp_amd", "lib"), "-lturbopfor_amd",
                           "-Wl,-rpath," + os.path.join(ROOT, "turbopfor-cpp_amd", "lib")])
    res = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.startswith("ok:"), res.stdout


def test_host_streams_vs_oracle():
    L = capi()
    L.tpf_host_dec.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                               ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
    L.tpf_host_enc.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    blocks = np.concatenate([datagen.c2_blocks(3000, bw, 10, seed=5) for bw in (3, 9, 17, 26, 32)])
    exp_packed, exp_off = oracle_lib.enc256v32_batch(blocks)
    nb = len(blocks)
    cap = nb * 1800 + 64
    out = np.zeros(cap, dtype=np.uint8)
    off = np.zeros(nb + 1, dtype=np.uint64)
    rc = L.tpf_host_enc(2, blocks.ctypes.data, nb, 256, 0, None, 0, out.ctypes.data, cap, off.ctypes.data)
    assert rc == 0, L.tpf_last_error()
    np.testing.assert_array_equal(off, exp_off)
    np.testing.assert_array_equal(out[: off[-1]], exp_packed)
    back = np.zeros_like(blocks)
    rc = L.tpf_host_dec(2, exp_packed.ctypes.data, len(exp_packed), None, nb, 256, back.ctypes.data, None)
    assert rc == 0, L.tpf_last_error()
    np.testing.assert_array_equal(back, blocks)
    # delta-1 chained posting list through the host stream
    vals, starts = datagen.c3_postings(5000)
    exp_p, exp_o = oracle_lib.enc256v32_batch(vals, starts=starts)
    out2 = np.zeros(5000 * 1800, dtype=np.uint8)
    off2 = np.zeros(5001, dtype=np.uint64)
    rc = L.tpf_host_enc(2, vals.ctypes.data, 5000, 256, 1, None, 0, out2.ctypes.data, len(out2), off2.ctypes.data)
    assert rc == 0, L.tpf_last_error()
    np.testing.assert_array_equal(out2[: off2[-1]], exp_p)
    back2 = np.zeros_like(vals)
    rc = L.tpf_host_dec(2, exp_p.ctypes.data, len(exp_p), exp_o.ctypes.data, 5000, 256, back2.ctypes.data,
                        starts.ctypes.data)
    assert rc == 0, L.tpf_last_error()
    np.testing.assert_array_equal(back2, vals)
