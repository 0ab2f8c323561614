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


@pytest.fixture(params=[0, 1, 2], ids=["server", "launch", "server-hostmail"])
def perblock_mode(request):
    """Every per-block design (tpf_perblock_mode): the resident block server
    with request mailboxes in device memory (default), one launch +
    synchronise per call, and the server with request mailboxes in host
    memory."""
    L = capi()
    L.tpf_perblock_mode.restype = ctypes.c_int
    L.tpf_perblock_mode.argtypes = [ctypes.c_int]
    prev = L.tpf_perblock_mode(request.param)
    yield request.param
    L.tpf_perblock_mode(prev)


@pytest.mark.parametrize("fname,fmt", [("g32.bin", "32"), ("g128v32.bin", "128v32"), ("g256v32.bin", "256v32"),
                                       ("g128v64.bin", "128v64"), ("g256v64.bin", "256v64")])
def test_per_block_mirrors_match_golden(fname, fmt, perblock_mode):
    L = capi()
    wide = fmt in ("128v64", "256v64")
    dt = np.uint64 if wide else np.uint32
    vt = ctypes.c_uint64 if wide else ctypes.c_uint32
    recs = golden_io.load(fname)
    step = max(1, len(recs) // 120)  # per-block calls are latency-bound: sample
    # ... but keep every unit shorter than the layout width (128v64 n < 128,
    # 256v64 n < 256: split into 128v64 blocks like the reference)
    short = [r for r in recs if wide and r.n < tpf.unit_values(fmt, r.n)]
    for i, r in enumerate(recs[::step] + short):
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
            mine = bytes(out[: end - out.ctypes.data])
            if r.padding_unpinned:  # reference padding bits came from its stack: length + values
                assert len(mine) == len(r.enc), (fmt, i)
                assert mine == oracle_lib.encode(fmt, r.values, d1=r.d1, start=r.start), (fmt, i)
            else:
                assert mine == r.enc, (fmt, i)
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


@pytest.mark.parametrize("chunk_bytes", [None, 1000 * 1024, 777 * 1024])
def test_host_streams_vs_oracle(chunk_bytes, monkeypatch):
    """Pageable numpy buffers (staged through the pipeline's pinned buffers by
    host copies); with small chunks the pipeline runs many chunks through its
    3 slots."""
    if chunk_bytes:
        monkeypatch.setenv("TPF_HOST_CHUNK_BYTES", str(chunk_bytes))
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


@pytest.mark.parametrize("down", ["sdma", "kernel"])
def test_host_streams_pinned_torch(down, monkeypatch):
    """Pinned (hipHostMalloc) torch buffers, odd destination phase.  down=sdma
    (default): results come back by hipMemcpyAsync; down=kernel: decode
    stores straight into host memory and encode copies its bytes out with the
    copy kernel at whatever byte phase each chunk lands on."""
    monkeypatch.setenv("TPF_HOST_CHUNK_BYTES", str(513 * 1024))
    monkeypatch.setenv("TPF_HOST_DOWN", down)
    L = capi()
    L.tpf_host_dec.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                               ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
    L.tpf_host_enc.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    blocks = np.concatenate([datagen.c2_blocks(1500, bw, 10, seed=9) for bw in (1, 5, 12, 20, 28, 32)])
    exp_packed, exp_off = oracle_lib.enc256v32_batch(blocks)
    nb = len(blocks)
    h_vals = torch.from_numpy(blocks.view(np.int32)).pin_memory()
    cap = nb * 1100 + 64
    h_pk = torch.zeros(cap + 3, dtype=torch.uint8).pin_memory()
    h_po = torch.zeros(nb + 1, dtype=torch.int64).pin_memory()
    base = h_pk.data_ptr() + 3  # odd destination phase
    assert L.tpf_host_enc(2, h_vals.data_ptr(), nb, 256, 0, None, 0, base, cap, h_po.data_ptr()) == 0, L.tpf_last_error()
    np.testing.assert_array_equal(h_po.numpy().view(np.uint64), exp_off)
    np.testing.assert_array_equal(h_pk.numpy()[3:3 + len(exp_packed)], exp_packed)
    assert not h_pk.numpy()[:3].any() and not h_pk.numpy()[3 + len(exp_packed):].any()
    h_back = torch.zeros_like(h_vals).pin_memory()
    assert L.tpf_host_dec(2, base, len(exp_packed), h_po.data_ptr(), nb, 256, h_back.data_ptr(), None) == 0, \
        L.tpf_last_error()
    np.testing.assert_array_equal(h_back.numpy().view(np.uint32), blocks)


def test_copy_async_phases():
    """tpf_copy_async (the pipelines' download path): every source/destination
    phase mod 16 class, lengths around the 16-byte vector edges, device ->
    pinned host, pinned host -> device and device -> device."""
    L = capi()
    L.tpf_copy_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    rng = np.random.default_rng(3)
    n = (1 << 20) + 64
    src_h = torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8))
    src_d = src_h.cuda()
    src_p = src_h.pin_memory()
    dst_d = torch.empty(n, dtype=torch.uint8, device="cuda")
    dst_p = torch.empty(n, dtype=torch.uint8).pin_memory()
    cases = [(sp, dp, ln) for sp in (0, 1, 3, 4, 8, 13) for dp in (0, 2, 5, 15)
             for ln in (0, 1, 15, 16, 17, 31, 100, 4099)]
    cases += [(7, 0, n - 64), (0, 0, n - 64), (4, 12, 65536 + 3)]
    stream = torch.cuda.current_stream().cuda_stream
    for sp, dp, ln in cases:
        for src, dst in ((src_d, dst_p), (src_p, dst_d), (src_d, dst_d)):
            dst.fill_(0xAB)
            assert L.tpf_copy_async(dst.data_ptr() + dp, src.data_ptr() + sp, ln, stream) == 0, L.tpf_last_error()
            torch.cuda.synchronize()
            got = dst.cpu().numpy()
            want = src_h.numpy()
            np.testing.assert_array_equal(got[dp:dp + ln], want[sp:sp + ln], err_msg=f"{sp} {dp} {ln}")
            assert (got[:dp] == 0xAB).all() and (got[dp + ln:dp + ln + 64] == 0xAB).all(), (sp, dp, ln)


def test_host_streams_concurrent_threads(monkeypatch):
    """Two host threads decoding and encoding through the pooled pipelines at
    once (each call leases its own pipeline; ctypes releases the GIL)."""
    import threading

    monkeypatch.setenv("TPF_HOST_CHUNK_BYTES", str(300 * 1024))
    L = capi()
    L.tpf_host_dec.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                               ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
    L.tpf_host_enc.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    jobs = []
    for seed in (11, 12, 13, 14):
        blocks = np.concatenate([datagen.c2_blocks(800, bw, 10, seed=seed) for bw in (4, 13, 22, 31)])
        exp_packed, exp_off = oracle_lib.enc256v32_batch(blocks)
        jobs.append((blocks, exp_packed, exp_off))
    errors = []

    def work(blocks, exp_packed, exp_off):
        try:
            for _ in range(3):
                nb = len(blocks)
                back = np.zeros_like(blocks)
                assert L.tpf_host_dec(2, exp_packed.ctypes.data, len(exp_packed), exp_off.ctypes.data, nb, 256,
                                      back.ctypes.data, None) == 0
                np.testing.assert_array_equal(back, blocks)
                out = np.zeros(nb * 1100 + 64, dtype=np.uint8)
                off = np.zeros(nb + 1, dtype=np.uint64)
                assert L.tpf_host_enc(2, blocks.ctypes.data, nb, 256, 0, None, 0, out.ctypes.data, len(out),
                                      off.ctypes.data) == 0
                np.testing.assert_array_equal(off, exp_off)
                np.testing.assert_array_equal(out[: off[-1]], exp_packed)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    threads = [threading.Thread(target=work, args=j) for j in jobs]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert not errors, errors


def test_host_streams_of_two_threads_overlap():
    """host-stream calls of different threads run AT THE SAME TIME
    (each on its own pooled pipeline); only the library's buffer frees and
    allocations pause the per-block server.  Two threads start a decode of the
    same pageable stream together; their call intervals must intersect, and
    both results are exact."""
    import threading
    import time

    L = capi()
    L.tpf_host_dec.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                               ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
    unit = np.concatenate([datagen.c2_blocks(100, bw, 10, seed=21) for bw in (6, 15, 27)])
    up, uo = oracle_lib.enc256v32_batch(unit)
    reps = 200  # 60,000 blocks, 61 MB of values per call
    packed = np.tile(up, reps)
    off = np.concatenate([np.zeros(1, np.uint64)] + [uo[1:] + np.uint64(i * len(up)) for i in range(reps)])
    nb = len(unit) * reps
    bar = threading.Barrier(2)
    spans, errors = [None, None], []

    def work(i):
        try:
            back = np.empty((nb, 256), dtype=np.uint32)
            # warm (pipeline leased and staging grown), then the timed call
            assert L.tpf_host_dec(2, packed.ctypes.data, len(packed), off.ctypes.data, nb, 256, back.ctypes.data, None) == 0
            bar.wait()
            t0 = time.perf_counter()
            assert L.tpf_host_dec(2, packed.ctypes.data, len(packed), off.ctypes.data, nb, 256, back.ctypes.data, None) == 0
            spans[i] = (t0, time.perf_counter())
            np.testing.assert_array_equal(back[: len(unit)], unit)
            np.testing.assert_array_equal(back[-len(unit):], unit)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ts = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors
    (a0, a1), (b0, b1) = spans
    assert max(a0, b0) < min(a1, b1), f"calls ran one after the other: {spans}"


@pytest.mark.parametrize("nthreads", [16, 80, 128])
def test_per_block_server_concurrent_threads(nthreads):
    """16 threads (each its own mailbox), 80 and 128 (more than the server's
    64 mailboxes: callers wait for a free one and, with more threads than
    CPUs, sleep while they wait) call at once: every thread's
    encode -> decode round trip of its own blocks is byte-exact (oracle),
    bit-exact, and every returned end pointer is right."""
    import threading

    L = capi()
    L.tpf_p4Enc256v32.restype = ctypes.c_void_p
    L.tpf_p4Enc256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
    L.tpf_p4D1Dec256v32.restype = ctypes.c_void_p
    L.tpf_p4D1Dec256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p, ctypes.c_uint32]
    L.tpf_p4Dec256v32.restype = ctypes.c_void_p
    L.tpf_p4Dec256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
    errors = []

    def worker(k):
        try:
            blocks = datagen.c2_blocks(40 if nthreads <= 16 else 12, 1 + (3 * k) % 32, 10, seed=k)
            for v in blocks:
                v = np.ascontiguousarray(v)
                buf = np.zeros(4096, np.uint8)
                end = L.tpf_p4Enc256v32(v.ctypes.data, 256, buf.ctypes.data)
                assert end is not None
                enc = bytes(buf[: end - buf.ctypes.data])
                assert enc == oracle_lib.encode("256v32", v)
                out = np.zeros(256, np.uint32)
                assert L.tpf_p4Dec256v32(buf.ctypes.data, 256, out.ctypes.data) == end
                assert np.array_equal(out, v)
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors


def test_per_block_pause_and_mode_switch_during_calls():
    """Round 5: a pause takes every mailbox, so tpf_perblock_quiesce and
    tpf_perblock_mode may run while other threads are inside per-block calls
    (each waits for the calls in flight; new calls wait for it).  8 caller
    threads round-trip their blocks while a 9th switches the mailbox half
    (mode 0 <-> 2) and quiesces the server over and over: every result stays
    byte-exact and no call hangs."""
    import threading

    L = capi()
    L.tpf_p4Enc256v32.restype = ctypes.c_void_p
    L.tpf_p4Enc256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
    L.tpf_p4Dec256v32.restype = ctypes.c_void_p
    L.tpf_p4Dec256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
    L.tpf_perblock_mode.restype = ctypes.c_int
    L.tpf_perblock_mode.argtypes = [ctypes.c_int]
    old = L.tpf_perblock_mode(-1)
    errors = []
    done = threading.Event()

    def worker(k):
        try:
            for v in datagen.c2_blocks(60, 1 + (5 * k) % 32, 10, seed=100 + k):
                v = np.ascontiguousarray(v)
                buf = np.zeros(4096, np.uint8)
                end = L.tpf_p4Enc256v32(v.ctypes.data, 256, buf.ctypes.data)
                assert end is not None
                assert bytes(buf[: end - buf.ctypes.data]) == oracle_lib.encode("256v32", v)
                out = np.zeros(256, np.uint32)
                assert L.tpf_p4Dec256v32(buf.ctypes.data, 256, out.ctypes.data) == end
                assert np.array_equal(out, v)
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))

    def switcher():
        try:
            i = 0
            while not done.is_set():
                L.tpf_perblock_mode(2 if i % 2 == 0 else 0)
                L.tpf_perblock_quiesce()
                i += 1
        except Exception as e:  # noqa: BLE001
            errors.append(("switcher", repr(e)))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    sw = threading.Thread(target=switcher)
    sw.start()
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    done.set()
    sw.join(timeout=60)
    L.tpf_perblock_mode(old)
    assert not any(t.is_alive() for t in ts + [sw]), "a per-block call or the switcher hung"
    assert not errors, errors


def test_per_block_server_idle_exit_and_mode_switch():
    """The block server leaves after 10 ms without a request and the next call
    relaunches it; switching between the server layouts (device / host
    request mailboxes) and launch + synchronise between calls keeps every
    answer exact (stale request words of the unused layout must not be taken
    for new requests)."""
    import time

    L = capi()
    L.tpf_perblock_mode.restype = ctypes.c_int
    L.tpf_perblock_mode.argtypes = [ctypes.c_int]
    L.tpf_p4Enc256v32.restype = ctypes.c_void_p
    L.tpf_p4Enc256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
    L.tpf_p4Dec256v32.restype = ctypes.c_void_p
    L.tpf_p4Dec256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
    prev = L.tpf_perblock_mode(-1)
    blocks = datagen.c2_blocks(12, 9, 10, seed=5)
    try:
        for step, mode in enumerate([0, 0, 2, 2, 1, 0, 2, 0]):
            L.tpf_perblock_mode(mode)
            for v in blocks[step % 3::3]:
                v = np.ascontiguousarray(v)
                buf = np.zeros(4096, np.uint8)
                end = L.tpf_p4Enc256v32(v.ctypes.data, 256, buf.ctypes.data)
                assert end is not None
                assert bytes(buf[: end - buf.ctypes.data]) == oracle_lib.encode("256v32", v)
                out = np.zeros(256, np.uint32)
                assert L.tpf_p4Dec256v32(buf.ctypes.data, 256, out.ctypes.data) == end
                assert np.array_equal(out, v), (step, mode)
            if step in (1, 3, 6):
                time.sleep(0.05)  # past the server's 10 ms idle exit
    finally:
        L.tpf_perblock_mode(prev)


def test_per_block_calls_beside_host_stream_frees(monkeypatch):
    """a thread making per-block calls (resident server running)
    while another thread's host-stream calls grow -- i.e. free and reallocate --
    their staging buffers.  HIP's frees wait for every stream of the device,
    the server's included; the library stops the server around its own frees
    and holds back per-block calls meanwhile (tpf::PerblockPause).  Both sides
    must finish promptly and exactly; tpf_perblock_quiesce() is callable."""
    import threading
    import time

    L = capi()
    L.tpf_p4Enc256v32.restype = ctypes.c_void_p
    L.tpf_p4Enc256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
    L.tpf_p4Dec256v32.restype = ctypes.c_void_p
    L.tpf_p4Dec256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
    L.tpf_host_dec.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                               ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
    L.tpf_host_release.restype = None
    L.tpf_perblock_quiesce.restype = None
    stop = threading.Event()
    errors, calls = [], [0]
    pb = datagen.c2_blocks(16, 11, 10, seed=3)

    def per_block():
        try:
            while not stop.is_set():
                for v in pb:
                    v = np.ascontiguousarray(v)
                    buf = np.zeros(4096, np.uint8)
                    end = L.tpf_p4Enc256v32(v.ctypes.data, 256, buf.ctypes.data)
                    out = np.zeros(256, np.uint32)
                    assert L.tpf_p4Dec256v32(buf.ctypes.data, 256, out.ctypes.data) == end
                    assert np.array_equal(out, v)
                    calls[0] += 1
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = threading.Thread(target=per_block)
    th.start()
    try:
        t0 = time.time()
        for k, nb in enumerate((500, 2000, 8000, 500, 16000)):
            # a growing chunk size makes the pooled pipeline free and reallocate its staging
            monkeypatch.setenv("TPF_HOST_CHUNK_BYTES", str((64 << 10) * (k + 1)))
            blocks = np.concatenate([datagen.c2_blocks(nb // 4, bw, 10, seed=k) for bw in (5, 12, 20, 29)])
            exp_packed, exp_off = oracle_lib.enc256v32_batch(blocks)
            back = np.zeros_like(blocks)
            assert L.tpf_host_dec(2, exp_packed.ctypes.data, len(exp_packed), exp_off.ctypes.data, len(blocks), 256,
                                  back.ctypes.data, None) == 0
            np.testing.assert_array_equal(back, blocks)
            if k == 2:
                L.tpf_host_release()  # frees every pooled pipeline while per-block calls run
            L.tpf_perblock_quiesce()
        assert time.time() - t0 < 60
    finally:
        stop.set()
        th.join(timeout=60)
    assert not th.is_alive()
    assert not errors, errors
    assert calls[0] > 0


def test_host_dec_multi_vs_single():
    """tpf_host_dec_multi (SURVEY.md 8 f3 across GPUs): the stream cut into
    shards, one pipeline thread per listed device -- on a one-GPU box the same
    device listed 1, 2 and 3 times -- matches tpf_host_dec and the oracle for
    plain and delta-1 decodes (pageable numpy buffers, registered once for
    all shards), and a corrupt block fails the call naming its shard."""
    L = capi()
    L.tpf_host_dec_multi.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
    ndev = torch.cuda.device_count()
    blocks = np.concatenate([datagen.c2_blocks(2000, bw, 10, seed=9) for bw in (2, 11, 23, 32)])
    packed, off = oracle_lib.enc256v32_batch(blocks)
    nb = len(blocks)
    vals, starts = datagen.c3_postings(4001)
    p1, o1 = oracle_lib.enc256v32_batch(vals, starts=starts)
    for k in (1, 2, 3):
        devs = np.array([i % ndev for i in range(k)], dtype=np.int32)
        back = np.zeros_like(blocks)
        rc = L.tpf_host_dec_multi(devs.ctypes.data, k, 2, packed.ctypes.data, len(packed), off.ctypes.data, nb, 256,
                                  back.ctypes.data, None)
        assert rc == 0, L.tpf_last_error()
        np.testing.assert_array_equal(back, blocks)
        back = np.zeros_like(blocks)  # offsets scanned from the headers
        assert L.tpf_host_dec_multi(devs.ctypes.data, k, 2, packed.ctypes.data, len(packed), None, nb, 256,
                                    back.ctypes.data, None) == 0, L.tpf_last_error()
        np.testing.assert_array_equal(back, blocks)
        back1 = np.zeros_like(vals)
        assert L.tpf_host_dec_multi(devs.ctypes.data, k, 2, p1.ctypes.data, len(p1), o1.ctypes.data, 4001, 256,
                                    back1.ctypes.data, starts.ctypes.data) == 0, L.tpf_last_error()
        np.testing.assert_array_equal(back1, vals)
    bad = off.astype(np.uint64).copy()
    bad[7000] += 1  # block 6999 one byte too long: shard 1 of 2 (blocks 4000.. hold the wider widths' bytes)
    devs = np.zeros(2, dtype=np.int32)
    back = np.zeros_like(blocks)
    rc = L.tpf_host_dec_multi(devs.ctypes.data, 2, 2, packed.ctypes.data, len(packed), bad.ctypes.data, nb, 256,
                              back.ctypes.data, None)
    assert rc == -4
    assert b"shard" in L.tpf_last_error()
    assert L.tpf_host_dec_multi(devs.ctypes.data, 0, 2, packed.ctypes.data, len(packed), off.ctypes.data, nb, 256,
                                back.ctypes.data, None) == -1


def test_host_dec_multi_p4dec32():
    """tpf_host_dec_multi on a p4Dec32 (n=127) stream: shards cut at block
    granularity of 128-byte blocks decode through the windowed kernel, two
    pipelines on the same device."""
    L = capi()
    L.tpf_host_dec_multi.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
    rng = np.random.default_rng(127)
    nb, n = 50001, 127
    vals = rng.integers(0, 256, size=(nb, n), dtype=np.uint64).astype(np.uint32)
    packed, off = oracle_lib.enc32_batch(vals)
    devs = np.zeros(2, dtype=np.int32)
    back = np.zeros_like(vals)
    rc = L.tpf_host_dec_multi(devs.ctypes.data, 2, 0, packed.ctypes.data, len(packed), off.ctypes.data, nb, n,
                              back.ctypes.data, None)
    assert rc == 0, L.tpf_last_error()
    np.testing.assert_array_equal(back, vals)


def test_host_enc_multi_vs_single():
    """tpf_host_enc_multi (SURVEY.md 8 f3 across GPUs, encode side): shards of
    equal block counts encoded by one pipeline thread per listed device (on a
    one-GPU box the same device listed 2 and 3 times), the later shards moved
    behind the earlier ones: bytes and offsets identical to the oracle's for
    plain 256v32, a chained D1 list (each shard continues from the value
    before its first block), per-unit starts, 256v64, and fewer blocks than
    devices."""
    L = capi()
    L.tpf_host_enc_multi.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_uint, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_void_p]
    ndev = torch.cuda.device_count()
    blocks = np.concatenate([datagen.c2_blocks(333, bw, 10, seed=4) for bw in (3, 14, 25)])
    vals, starts = datagen.c3_postings(1001)
    v64 = datagen.c4_blocks64(301, 37, 5, seed=2)
    cases = [("256v32 plain", 2, blocks, 0, None, 0, oracle_lib.enc256v32_batch(blocks)),
             ("256v32 D1 chained", 2, vals, 1, None, int(starts[0]), oracle_lib.enc256v32_batch(vals, starts=starts)),
             ("256v32 D1 starts", 2, vals, 1, starts, 0, oracle_lib.enc256v32_batch(vals, starts=starts)),
             ("256v64 plain", 5, v64, 0, None, 0, oracle_lib.enc256v64_batch(v64)),
             ("2 blocks", 2, blocks[:2], 0, None, 0, oracle_lib.enc256v32_batch(blocks[:2]))]
    L.tpf_enc_bound.restype = ctypes.c_uint64
    L.tpf_enc_bound.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint]
    for k in (2, 3):
        devs = np.array([i % ndev for i in range(k)], dtype=np.int32)
        for name, fmt, v, d1, st, s0, (exp_p, exp_o) in cases:
            nb = len(v)
            # roomy output: shards written in place at provisional offsets and
            # moved down; exactly the bound: shards through scratch buffers
            for cap in (nb * 2200 + 64 * k + 64, int(L.tpf_enc_bound(fmt, nb, 256))):
                out = np.zeros(cap, dtype=np.uint8)
                off = np.zeros(nb + 1, dtype=np.uint64)
                rc = L.tpf_host_enc_multi(devs.ctypes.data, k, fmt, v.ctypes.data, nb, 256, d1,
                                          None if st is None else st.ctypes.data, s0, out.ctypes.data, len(out), off.ctypes.data)
                assert rc == 0, (name, k, cap, L.tpf_last_error())
                np.testing.assert_array_equal(off, exp_o, err_msg=f"{name} k={k} cap={cap}")
                assert np.array_equal(out[: int(off[-1])], exp_p), (name, k, cap)
    # bad (fmt, n) is rejected before any shard reads the caller's array
    # (a chained shard read value n-1 of the unit before it first)
    devs = np.zeros(2, dtype=np.int32)
    out = np.zeros(len(vals) * 2200, dtype=np.uint8)
    off = np.zeros(len(vals) + 1, dtype=np.uint64)
    for fmt, n in ((2, 0), (2, 300), (2, 257), (5, 100), (99, 256)):
        assert L.tpf_host_enc_multi(devs.ctypes.data, 2, fmt, vals.ctypes.data, len(vals), n, 1, None, 0,
                                    out.ctypes.data, len(out), off.ctypes.data) == -1, (fmt, n)
    small = np.zeros(16, dtype=np.uint8)
    off = np.zeros(len(blocks) + 1, dtype=np.uint64)
    devs = np.zeros(2, dtype=np.int32)
    assert L.tpf_host_enc_multi(devs.ctypes.data, 2, 2, blocks.ctypes.data, len(blocks), 256, 0, None, 0, small.ctypes.data,
                                len(small), off.ctypes.data) == -1


def test_device_synchronize_beside_busy_per_block_caller():
    """A thread issuing per-block calls back to back keeps the resident block
    server busy; hipDeviceSynchronize (torch.cuda.synchronize) in another
    thread waits for every stream of the device, the server's included.  The
    server leaves after 5 ms of service even when busy (the next call
    relaunches it), so such waits return promptly instead of never (round 4:
    found with scripts/graph_canary.py)."""
    import threading
    import time

    L = capi()
    L.tpf_p4Enc256v32.restype = ctypes.c_void_p
    L.tpf_p4Enc256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
    L.tpf_p4Dec256v32.restype = ctypes.c_void_p
    L.tpf_p4Dec256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
    stop = threading.Event()
    errors, calls = [], [0]
    v = np.ascontiguousarray(datagen.c2_blocks(1, 12, 10, seed=6)[0])

    def busy():
        try:
            buf = np.zeros(4096, np.uint8)
            out = np.zeros(256, np.uint32)
            while not stop.is_set():
                end = L.tpf_p4Enc256v32(v.ctypes.data, 256, buf.ctypes.data)
                assert L.tpf_p4Dec256v32(buf.ctypes.data, 256, out.ctypes.data) == end
                calls[0] += 1
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = threading.Thread(target=busy)
    th.start()
    try:
        time.sleep(0.05)
        x = torch.arange(1 << 20, device="cuda", dtype=torch.int64)
        t0 = time.time()
        for _ in range(20):
            x.add_(1)
            torch.cuda.synchronize()
        dt = time.time() - t0
    finally:
        stop.set()
        th.join(timeout=60)
    assert not errors, errors
    assert calls[0] > 0
    assert dt < 10.0, f"20 device-wide synchronizes took {dt:.1f} s beside a busy per-block caller"
    assert int(x[0].item()) == 20


def test_block_server_launches_track_its_lifetime():
    """the idle-exit test could wrap (the clock read before another
    workgroup published a later activity time) and end the whole server early.
    A launch now leaves only after 10 ms idle, after its 5 ms lifetime, or
    when stopped: under continuous calls from 8 threads for ~0.3 s the
    launches stay within the lifetime's count (plus slack for the first
    launch and the relaunch gaps)."""
    import threading
    import time

    L = capi()
    L.tpf_p4Enc256v32.restype = ctypes.c_void_p
    L.tpf_p4Enc256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
    L.tpf_perblock_launches.restype = ctypes.c_uint64
    v = np.ascontiguousarray(datagen.c2_blocks(1, 9, 10, seed=3)[0])
    buf0 = np.zeros(4096, np.uint8)
    assert L.tpf_p4Enc256v32(v.ctypes.data, 256, buf0.ctypes.data) is not None  # server up
    stop = time.monotonic() + 0.3
    calls = [0] * 8
    errors = []

    def worker(k):
        buf = np.zeros(4096, np.uint8)
        try:
            while time.monotonic() < stop:
                assert L.tpf_p4Enc256v32(v.ctypes.data, 256, buf.ctypes.data) is not None
                calls[k] += 1
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    l0 = L.tpf_perblock_launches()
    t0 = time.monotonic()
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    dt = time.monotonic() - t0
    launches = L.tpf_perblock_launches() - l0
    assert not errors, errors
    assert sum(calls) > 100
    assert launches <= dt / 0.005 * 1.25 + 4, (launches, dt, sum(calls))
