// host_stream.cpp -- end-to-end host-memory streams: blocks
// and values live in host memory; chunks are uploaded to HBM, decoded/encoded
// by the batched kernels and the results brought back, with the upload of
// chunk k+1 (copy stream, SDMA) overlapping the kernel and the download of
// chunk k (kernel stream).  PCIe is full duplex and the kernels run at HBM
// speed, so the PCIe link bounds this path.
//
// Downloads go by SDMA (hipMemcpyAsync on the kernel stream): an SDMA upload
// and an SDMA download on two streams overlap on MI355X (82 GB/s combined vs
// 57 GB/s one way, scripts/e2e_probe.py).  TPF_HOST_DOWN=kernel instead has
// the decode kernel store straight into the mapped host array and encode
// move its bytes with the copy kernel (host_copy.hip); measured 4-8% slower
// (profiles/r1_v4_e2e_probe.txt), kept for A/B.
//
// The staging buffers, streams and events of a pipeline are pooled across
// calls (per device): allocating ~200 MB of HBM and pinned offset staging per
// call cost more than the transfers (8.4 -> 12.5 G int32/s end to end).
// tpf_host_release() frees the pool.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <optional>
#include <thread>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/turbopfor_capi.h"
#include "../../include/turbopfor_gpu.h"
#include "shard_exec.h"
#include "tpf_kernels.h"

namespace tpf
{
void set_last_error(const std::string & msg);
}

namespace
{

constexpr int kSlots = 3;

// chunk = this many bytes of values: small enough that the first upload (not
// overlapped) is short, large enough to fill the GPU per launch.
// TPF_HOST_CHUNK_BYTES overrides it (tests drive many chunks through small inputs).
uint64_t chunk_value_bytes()
{
    if (const char * e = std::getenv("TPF_HOST_CHUNK_BYTES"))
        if (const uint64_t v = std::strtoull(e, nullptr, 10))
            return v;
    return 64ull << 20;
}

bool sdma_down()
{
    const char * e = std::getenv("TPF_HOST_DOWN");
    return !(e && std::strcmp(e, "kernel") == 0);
}

bool wide_fmt(int fmt) { return fmt == TPF_FMT_64 || fmt == TPF_FMT_128V64 || fmt == TPF_FMT_256V64; }

unsigned unit_values(int fmt, unsigned n)
{
    switch (fmt)
    {
        case TPF_FMT_128V32:
        case TPF_FMT_128V64:
            return 128;
        case TPF_FMT_256V32:
        case TPF_FMT_256V64:
            return 256;
        default:
            return n;
    }
}

struct Err : std::runtime_error
{
    int code;
    Err(int c, const std::string & m) : std::runtime_error(m), code(c) { }
};

void hc(hipError_t e, const char * what)
{
    if (e != hipSuccess)
        throw Err(TPF_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

void tc(int rc)
{
    if (rc != TPF_OK)
        throw Err(rc, tpf_last_error());
}

// Can the copy engines (and, mapped, the kernels) use the host range
// [p, p + bytes) as it is?  Yes when HIP knows both its ends as page-locked
// host memory (hipHostMalloc'd or caller-registered; `d` = its device
// address) or as device memory.  A pageable range -- or one whose far end
// lies outside any registration -- is STAGED: host threads
// copy it into / out of the pipeline's pinned buffers.  The library never
// page-locks caller memory.  (Until round 3 it did, hipHostRegister for the
// length of a call: a call's registration and release of pageable pages that
// the interpreter's heap hands to the next arrays was the one library action
// that changed the GPU's view of caller memory, and the suspect of the r3r
// hipErrorIllegalAddress on a later pageable torch copy)
struct Reach
{
    bool direct = true;
    bool dev = false; // device (or managed) memory handed over as a host pointer
    void * d = nullptr;
    // copy kinds for a direct range (explicit rather than hipMemcpyDefault)
    hipMemcpyKind up() const { return dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice; }
    hipMemcpyKind down() const { return dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost; }
};

bool lookup(const void * q, hipPointerAttribute_t & a)
{
    a = hipPointerAttribute_t{};
    const bool ok = hipPointerGetAttributes(&a, q) == hipSuccess && a.type != hipMemoryTypeUnregistered;
    if (!ok)
        (void)hipGetLastError();
    return ok;
}

Reach reach(const void * ptr, size_t bytes)
{
    Reach r;
    if (!ptr || !bytes)
        return r;
    const uint8_t * lo = static_cast<const uint8_t *>(ptr);
    const uint8_t * hi = lo + bytes - 1;
    hipPointerAttribute_t a{}, b{};
    if (!lookup(lo, a) || !lookup(hi, b))
    {
        r.direct = false;
        return r;
    }
    if (a.type == hipMemoryTypeHost && b.type == hipMemoryTypeHost)
    {
        // both ends page-locked.  (Not "one hostPointer": for an interior
        // pointer -- torch's pinned caching allocator hands those out -- HIP
        // reports the queried address, so that test sent every pinned torch
        // buffer through the pageable staging: host encode 12.9 -> 9.8 G
        // int32/s, decode 12.3 -> 10.9, round 4.)
        // Both ends must lie in ONE allocation: the mapped device address r.d
        // is derived from lo's, and the kernels' direct paths address the whole
        // range through it.  A range across two registrations,
        // or one HIP cannot size, is staged.
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        if (hipMemGetAddressRange(&base, &size, const_cast<uint8_t *>(lo)) != hipSuccess || !base ||
            hi >= static_cast<const uint8_t *>(base) + size || lo < static_cast<const uint8_t *>(base))
        {
            (void)hipGetLastError();
            r.direct = false;
            return r;
        }
        if (a.devicePointer && a.hostPointer)
            r.d = static_cast<uint8_t *>(a.devicePointer) + (lo - static_cast<const uint8_t *>(a.hostPointer));
        return r;
    }
    // device (or managed) memory handed over as a host pointer: the copy engines take it as it is
    r.direct = (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) && a.type == b.type;
    r.dev = r.direct;
    return r;
}

// Host copies between pageable caller memory and pinned staging, split over
// up to TPF_HOST_COPY_THREADS (default 8) threads: one core copies ~10 GB/s,
// the link moves ~57 GB/s one way.
void par_copy(void * dst, const void * src, size_t n)
{
    static const size_t nthr = [] {
        const char * e = std::getenv("TPF_HOST_COPY_THREADS");
        const long v = e ? std::strtol(e, nullptr, 10) : 8;
        return static_cast<size_t>(std::clamp<long>(v, 1, 64));
    }();
    constexpr size_t kPiece = 4u << 20;
    const size_t nt = std::min(nthr, std::max<size_t>(1, n / kPiece));
    if (nt <= 1)
    {
        std::memcpy(dst, src, n);
        return;
    }
    const size_t per = ((n + nt - 1) / nt + 4095) & ~size_t(4095);
    std::vector<std::thread> th;
    th.reserve(nt);
    for (size_t o = per; o < n; o += per)
        th.emplace_back([=] { std::memcpy(static_cast<uint8_t *>(dst) + o, static_cast<const uint8_t *>(src) + o, std::min(per, n - o)); });
    std::memcpy(dst, src, std::min(per, n));
    for (std::thread & t : th)
        t.join();
}

// The per-block server must not run while HIP frees, allocates or tears down
// the library's own buffers and streams (HIP waits for every stream of the
// device there, the server's included), so those -- and only those -- hold
// tpf::PerblockPause.  Host-stream calls of different threads otherwise run
// concurrently (the whole call used to hold it).  Reentrant per
// thread (tpf::PerblockPause counts its own depth).
using FreePause = tpf::PerblockPause;

// A grow-only device (or pinned host) buffer.
struct Buf
{
    void * p = nullptr;
    size_t cap = 0;
    bool host = false;
    explicit Buf(bool h = false) : host(h) { }
    void * get(size_t n)
    {
        if (n <= cap && p)
            return p;
        const FreePause fp;
        release();
        n = std::max<size_t>(n, 256);
        if (host)
            hc(hipHostMalloc(&p, n, hipHostMallocDefault), "hipHostMalloc staging");
        else
            hc(hipMalloc(&p, n), "hipMalloc staging");
        cap = n;
        return p;
    }
    void release()
    {
        if (p)
        {
            const FreePause fp;
            (void)(host ? hipHostFree(p) : hipFree(p));
        }
        p = nullptr;
        cap = 0;
    }
    ~Buf() { release(); }
};

// One pipeline slot: per-chunk buffers; events: `up` = the chunk's uploads
// landed (copy stream), `mid` = encode offsets reached the host, `done` = the
// kernel stream finished with the slot.  hin / hout / hst: pinned staging of
// pageable caller ranges; `pend` = the host copy-out of a staged result,
// done once `done` has completed.
struct Slot
{
    hipEvent_t up = nullptr, mid = nullptr, done = nullptr;
    Buf in, vals, ws, start, off, hoff{true}, hin{true}, hout{true}, hst{true};
    struct Pending
    {
        void * dst = nullptr;
        const void * src = nullptr;
        size_t n = 0;
    } pend;
    Slot()
    {
        for (hipEvent_t * e : {&up, &mid, &done})
            hc(hipEventCreateWithFlags(e, hipEventDisableTiming), "event");
    }
    ~Slot()
    {
        for (hipEvent_t e : {up, mid, done})
            if (e)
                (void)hipEventDestroy(e);
    }
    // wait until the kernel stream is done with the slot, then finish its staged copy-out
    void drain()
    {
        hc(hipEventSynchronize(done), "wait slot");
        if (pend.n)
            par_copy(pend.dst, pend.src, pend.n);
        pend = Pending{};
    }
};

struct Pipeline
{
    int dev = -1;
    hipStream_t cs = nullptr, ks = nullptr; // copy stream, kernel stream
    Slot slots[kSlots];
    Buf errs;          // decode: one first-inconsistent-block word per chunk, read back once at the end
    Buf herrs{true};   // their pinned host copy
    explicit Pipeline(int d) : dev(d)
    {
        hc(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking), "stream");
        hc(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking), "stream");
    }
    ~Pipeline()
    {
        for (hipStream_t s : {cs, ks})
            if (s)
            {
                (void)hipStreamSynchronize(s);
                (void)hipStreamDestroy(s);
            }
    }
};

// The device discipline of the pool and of the shard threads lives in
// shard_exec.h (HIP-free, driven by a mock device map in
// tests/cpp/shard_exec_mock.cpp); these are its HIP operations.
struct HipOps
{
    int get_dev()
    {
        int d = 0;
        hc(hipGetDevice(&d), "hipGetDevice");
        return d;
    }
    bool set_dev(int d) { return hipSetDevice(d) == hipSuccess; }
    Pipeline * make(int d) { return new Pipeline(d); } // streams, events and buffers of the current device d
};

tpf::DevicePool<Pipeline> g_pool; // idle pipelines, keyed by device

// Exclusive use of a pooled pipeline of the calling thread's device for one
// call; on return the streams are drained and the pipeline goes back to the
// pool (or is destroyed -- with its own device selected -- after an error,
// when its state is unknown).
struct Lease
{
    Pipeline * p = nullptr;
    bool ok = false;
    Lease()
    {
        HipOps ops;
        p = g_pool.acquire(ops);
        for (Slot & s : p->slots)
            s.pend = Slot::Pending{};
    }
    ~Lease()
    {
        const bool drained = hipStreamSynchronize(p->ks) == hipSuccess && hipStreamSynchronize(p->cs) == hipSuccess;
        if (ok && drained)
            g_pool.give_back(p);
        else
        {
            const FreePause fp;
            HipOps ops;
            try
            {
                tpf::DevicePool<Pipeline>::destroy(ops, p);
            }
            catch (...)
            {
            }
        }
    }
};

int report(const std::exception & e, int code)
{
    tpf::set_last_error(e.what());
    return code;
}

void need_device()
{
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= 0)
        throw Err(TPF_ENODEV, "no HIP device visible (turbopfor_amd has no CPU fallback)");
}

int host_dec_impl(int fmt, const uint8_t * h_in, uint64_t in_bytes, const uint64_t * h_off, uint64_t nblocks, unsigned n,
                  void * h_vals, const void * h_starts);

} // namespace

extern "C" {

// Decode: chunk k's bytes (+ offsets, starts) go up by SDMA on the copy
// stream while the kernel stream decodes chunk k-1 into HBM and downloads it
// (or, TPF_HOST_DOWN=kernel with a mappable host array, decodes straight
// into host memory).
int tpf_host_dec(int fmt, const uint8_t * h_in, uint64_t in_bytes, const uint64_t * h_off, uint64_t nblocks, unsigned n,
                 void * h_vals, const void * h_starts)
{
    return host_dec_impl(fmt, h_in, in_bytes, h_off, nblocks, n, h_vals, h_starts);
}

} // extern "C"

namespace
{
int host_dec_impl(int fmt, const uint8_t * h_in, uint64_t in_bytes, const uint64_t * h_off, uint64_t nblocks, unsigned n,
                  void * h_vals, const void * h_starts)
{
    try
    {
        if (nblocks == 0)
            return TPF_OK;
        // The arguments are checked on the host before anything touches a
        // device (round 6: the same answer with or without a GPU).
        // h_off has nblocks + 1 entries (turbopfor_capi.h): a shorter array
        // cannot be detected, but what it usually yields -- offsets that
        // decrease or run past in_bytes -- is rejected here, before any copy.
        if (!h_in || !h_vals)
            throw Err(TPF_EINVAL, "tpf_host_dec: null pointer");
        if (!tpf::fmt_ok(fmt, n))
            throw Err(TPF_EINVAL, "tpf_host_dec: unsupported (fmt, n)");
        std::vector<uint64_t> scanned;
        if (!h_off)
        {
            scanned.resize(nblocks + 1);
            if (tpf_scan_offsets(fmt, h_in, in_bytes, n, nblocks, scanned.data()) < 0)
                throw Err(TPF_ECORRUPT, "tpf_host_dec: malformed block while scanning offsets");
            h_off = scanned.data();
        }
        else
        {
            // caller-supplied offsets bound every upload: they must rise and stay inside h_in
            const int64_t bad = tpf_check_offsets(h_off, nblocks, in_bytes);
            if (bad == -static_cast<int64_t>(nblocks) - 1)
                throw Err(TPF_EINVAL, "tpf_host_dec: h_off[nblocks] is past in_bytes");
            if (bad < 0)
                throw Err(TPF_EINVAL, "tpf_host_dec: h_off decreases at block " + std::to_string(-bad - 1));
        }
        need_device();
        const size_t es = wide_fmt(fmt) ? 8 : 4;
        const size_t uv = unit_values(fmt, n);
        const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(nblocks, chunk_value_bytes() / (es * uv)));
        // only this call's byte range of h_in (a shard of tpf_host_dec_multi reads no more)
        const Reach r_in = reach(h_in + h_off[0], h_off[nblocks] - h_off[0]);
        const Reach r_vals = reach(h_vals, nblocks * uv * es);
        const Reach r_st = h_starts ? reach(h_starts, nblocks * es) : Reach{};
        uint8_t * dv = (sdma_down() || !r_vals.direct) ? nullptr : static_cast<uint8_t *>(r_vals.d);
        size_t max_in = 0;
        for (uint64_t c0 = 0; c0 < nblocks; c0 += chunk)
        {
            const uint64_t c1 = std::min(nblocks, c0 + chunk);
            max_in = std::max<size_t>(max_in, h_off[c1] - h_off[c0]);
        }
        Lease lease;
        Pipeline & P = *lease.p;
        // per chunk, the first block whose parsed length disagrees with its
        // offsets: a device word each, brought back with ONE copy at the end
        // (a small device-to-host copy per chunk can stall the host loop)
        const uint64_t nchunks = (nblocks + chunk - 1) / chunk;
        auto * d_errs = static_cast<uint64_t *>(P.errs.get(nchunks * 8));
        auto * h_errs = static_cast<uint64_t *>(P.herrs.get(nchunks * 8));
        uint64_t k = 0;
        for (uint64_t c0 = 0; c0 < nblocks; c0 += chunk, ++k)
        {
            Slot & sl = P.slots[k % kSlots];
            sl.drain(); // chunk k-kSlots is done with the slot (and its staged values are out)
            const uint64_t c1 = std::min(nblocks, c0 + chunk);
            const uint64_t nb = c1 - c0;
            const uint64_t b0 = h_off[c0], bytes = h_off[c1] - b0;
            auto * d_in = static_cast<uint8_t *>(sl.in.get(max_in + 64));
            auto * d_off = static_cast<uint64_t *>(sl.off.get((chunk + 1) * 8));
            auto * st_off = static_cast<uint64_t *>(sl.hoff.get((chunk + 1) * 8));
            void * d_start = h_starts ? sl.start.get(chunk * es) : nullptr;
            void * out = dv ? static_cast<void *>(dv + c0 * uv * es) : sl.vals.get(chunk * uv * es);
            for (uint64_t i = 0; i <= nb; ++i)
                st_off[i] = h_off[c0 + i] - b0;
            const void * src_in = h_in + b0;
            if (!r_in.direct)
            {
                void * s = sl.hin.get(max_in + 64);
                par_copy(s, src_in, bytes);
                src_in = s;
            }
            hc(hipMemcpyAsync(d_off, st_off, (nb + 1) * 8, hipMemcpyHostToDevice, P.cs), "H2D off");
            hc(hipMemcpyAsync(d_in, src_in, bytes, r_in.direct ? r_in.up() : hipMemcpyHostToDevice, P.cs), "H2D bytes");
            if (h_starts)
            {
                const void * src_st = static_cast<const uint8_t *>(h_starts) + c0 * es;
                if (!r_st.direct)
                {
                    void * s = sl.hst.get(chunk * es);
                    std::memcpy(s, src_st, nb * es);
                    src_st = s;
                }
                hc(hipMemcpyAsync(d_start, src_st, nb * es, r_st.direct ? r_st.up() : hipMemcpyHostToDevice, P.cs), "H2D starts");
            }
            hc(hipEventRecord(sl.up, P.cs), "record up");
            hc(hipStreamWaitEvent(P.ks, sl.up, 0), "wait up");
            tc(tpf_dec_batch(fmt, d_in, bytes, d_off, nb, n, out, d_start, d_errs + k, P.ks));
            if (!dv)
            {
                uint8_t * dst = static_cast<uint8_t *>(h_vals) + c0 * uv * es;
                if (r_vals.direct)
                    hc(hipMemcpyAsync(dst, out, nb * uv * es, r_vals.down(), P.ks), "D2H vals");
                else
                {
                    void * s = sl.hout.get(chunk * uv * es);
                    hc(hipMemcpyAsync(s, out, nb * uv * es, hipMemcpyDeviceToHost, P.ks), "D2H vals");
                    sl.pend = {dst, s, nb * uv * es};
                }
            }
            hc(hipEventRecord(sl.done, P.ks), "record done");
        }
        hc(hipMemcpyAsync(h_errs, d_errs, nchunks * 8, hipMemcpyDeviceToHost, P.ks), "D2H errs");
        hc(hipStreamSynchronize(P.ks), "sync");
        for (Slot & sl : P.slots)
            sl.drain();
        lease.ok = true;
        uint64_t bad = ~0ull; // first block whose parsed length disagrees with its offsets
        for (uint64_t i = 0; i < nchunks; ++i)
            if (h_errs[i] != ~0ull)
            {
                bad = i * chunk + h_errs[i];
                break;
            }
        if (bad != ~0ull)
            throw Err(TPF_ECORRUPT, "tpf_host_dec: block " + std::to_string(bad) + " parses to a length other than its offsets");
        return TPF_OK;
    }
    catch (const Err & e)
    {
        return report(e, e.code);
    }
    catch (const std::exception & e)
    {
        return report(e, TPF_EHIP);
    }
}

} // namespace

extern "C" {

// Multi-GPU decode of one host stream ("across streams and
// GPUs"): the blocks are cut into ndev contiguous shards of about equal
// bytes, and shard d runs tpf_host_dec's pipeline on device devs[d] from a
// thread of its own (each device has its own PCIe link and copy engines).
// Each shard reaches (or stages) only its own byte range of the input and its
// own values.
int tpf_host_dec_multi(const int * devs, int ndev, int fmt, const uint8_t * h_in, uint64_t in_bytes, const uint64_t * h_off,
                       uint64_t nblocks, unsigned n, void * h_vals, const void * h_starts)
{
    try
    {
        if (nblocks == 0)
            return TPF_OK;
        if (!devs || ndev < 1 || ndev > 64)
            throw Err(TPF_EINVAL, "tpf_host_dec_multi: need 1..64 devices");
        if (!h_in || !h_vals)
            throw Err(TPF_EINVAL, "tpf_host_dec_multi: null pointer");
        if (!tpf::fmt_ok(fmt, n))
            throw Err(TPF_EINVAL, "tpf_host_dec_multi: unsupported (fmt, n)");
        std::vector<uint64_t> scanned;
        if (!h_off)
        {
            scanned.resize(nblocks + 1);
            if (tpf_scan_offsets(fmt, h_in, in_bytes, n, nblocks, scanned.data()) < 0)
                throw Err(TPF_ECORRUPT, "tpf_host_dec_multi: malformed block while scanning offsets");
            h_off = scanned.data();
        }
        else
        {
            const int64_t bad = tpf_check_offsets(h_off, nblocks, in_bytes);
            if (bad == -static_cast<int64_t>(nblocks) - 1)
                throw Err(TPF_EINVAL, "tpf_host_dec_multi: h_off[nblocks] is past in_bytes");
            if (bad < 0)
                throw Err(TPF_EINVAL, "tpf_host_dec_multi: h_off decreases at block " + std::to_string(-bad - 1));
        }
        need_device();
        int cnt = 0;
        hc(hipGetDeviceCount(&cnt), "hipGetDeviceCount");
        for (int d = 0; d < ndev; ++d)
            if (devs[d] < 0 || devs[d] >= cnt)
                throw Err(TPF_EINVAL, "tpf_host_dec_multi: device " + std::to_string(devs[d]) + " is not visible");
        const size_t es = wide_fmt(fmt) ? 8 : 4;
        const size_t uv = unit_values(fmt, n);
        // shard cuts: equal shares of the stream's bytes (block granularity)
        std::vector<uint64_t> cut(static_cast<size_t>(ndev) + 1, nblocks);
        cut[0] = 0;
        const uint64_t total = h_off[nblocks] - h_off[0];
        for (int d = 1; d < ndev; ++d)
        {
            const uint64_t target = h_off[0] + total / static_cast<uint64_t>(ndev) * static_cast<uint64_t>(d);
            cut[d] = std::max<uint64_t>(cut[d - 1], static_cast<uint64_t>(std::lower_bound(h_off, h_off + nblocks, target) - h_off));
        }
        // one thread per shard, bound to its device first (shard_exec.h)
        const std::vector<tpf::ShardResult> res = tpf::run_shards(
            devs, ndev, [](int dev) { return hipSetDevice(dev) == hipSuccess; },
            [&](int d, std::string & msg) {
                const uint64_t b0 = cut[d], nb = cut[d + 1] - cut[d];
                if (nb == 0)
                    return TPF_OK;
                const int rc = host_dec_impl(fmt, h_in, in_bytes, h_off + b0, nb, n, static_cast<uint8_t *>(h_vals) + b0 * uv * es,
                                             h_starts ? static_cast<const uint8_t *>(h_starts) + b0 * es : nullptr);
                if (rc != TPF_OK)
                    msg = tpf_last_error(); // thread-local: carried to the caller's thread below
                return rc;
            },
            TPF_EHIP, TPF_EHIP);
        for (int d = 0; d < ndev; ++d)
            if (res[d].rc != TPF_OK)
                throw Err(res[d].rc, "tpf_host_dec_multi: shard " + std::to_string(d) + " (device " + std::to_string(devs[d]) + ", blocks " +
                                         std::to_string(cut[d]) + ".." + std::to_string(cut[d + 1]) +
                                         ", block numbers below are shard-relative): " + res[d].msg);
        return TPF_OK;
    }
    catch (const Err & e)
    {
        return report(e, e.code);
    }
    catch (const std::exception & e)
    {
        return report(e, TPF_EHIP);
    }
}

// Encode: chunk k's values go up by SDMA on the copy stream; the kernel
// stream encodes it and brings its offsets to the host; once the host knows
// where chunk k-1 lands (one-chunk lag), the kernel stream downloads chunk
// k-1's bytes into the host stream, concurrently with the next upload.
int tpf_host_enc(int fmt, const void * h_vals, uint64_t nblocks, unsigned n, int d1, const void * h_starts, uint64_t start0,
                 uint8_t * h_out, uint64_t out_cap, uint64_t * h_off)
{
    try
    {
        if (!h_off)
            throw Err(TPF_EINVAL, "tpf_host_enc: h_off is required");
        h_off[0] = 0;
        if (nblocks == 0)
            return TPF_OK;
        need_device();
        const size_t es = wide_fmt(fmt) ? 8 : 4;
        const size_t uv = unit_values(fmt, n);
        const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(nblocks, chunk_value_bytes() / (es * uv)));
        const Reach r_vals = reach(h_vals, nblocks * uv * es), r_out = reach(h_out, out_cap);
        const Reach r_st = (d1 && h_starts) ? reach(h_starts, nblocks * es) : Reach{};
        uint8_t * dout = (sdma_down() || !r_out.direct) ? nullptr : static_cast<uint8_t *>(r_out.d);
        const size_t cap = tpf_enc_bound(fmt, chunk, n);
        const size_t wsb = std::max<size_t>(tpf_enc_workspace_size(fmt, chunk, n), 256);
        Lease lease;
        Pipeline & P = *lease.p;
        uint64_t pos = 0;
        std::vector<uint64_t> c0s;
        auto finish = [&](uint64_t kk) {
            Slot & sl = P.slots[kk % kSlots];
            hc(hipEventSynchronize(sl.mid), "wait offsets");
            const uint64_t c0 = c0s[kk];
            const uint64_t nb = std::min(nblocks, c0 + chunk) - c0;
            const auto * st_off = static_cast<const uint64_t *>(sl.hoff.p);
            const uint64_t total = st_off[nb];
            if (pos + total > out_cap)
                throw Err(TPF_EINVAL, "tpf_host_enc: out_cap too small");
            for (uint64_t i = 1; i <= nb; ++i)
                h_off[c0 + i] = pos + st_off[i];
            if (dout)
                tc(tpf_copy_async(dout + pos, sl.in.p, total, P.ks));
            else if (r_out.direct)
                hc(hipMemcpyAsync(h_out + pos, sl.in.p, total, r_out.down(), P.ks), "D2H bytes");
            else
            {
                void * st = sl.hout.get(cap);
                hc(hipMemcpyAsync(st, sl.in.p, total, hipMemcpyDeviceToHost, P.ks), "D2H bytes");
                sl.pend = {h_out + pos, st, total};
            }
            hc(hipEventRecord(sl.done, P.ks), "record done");
            pos += total;
        };
        uint64_t k = 0;
        for (uint64_t c0 = 0; c0 < nblocks; c0 += chunk, ++k)
        {
            Slot & sl = P.slots[k % kSlots];
            sl.drain(); // chunk k-kSlots is done with the slot (and its staged bytes are out)
            c0s.push_back(c0);
            const uint64_t nb = std::min(nblocks, c0 + chunk) - c0;
            auto * d_pk = static_cast<uint8_t *>(sl.in.get(cap));
            void * d_vals = sl.vals.get(chunk * uv * es);
            void * d_ws = sl.ws.get(wsb);
            auto * d_off = static_cast<uint64_t *>(sl.off.get((chunk + 1) * 8));
            void * st_off = sl.hoff.get((chunk + 1) * 8);
            const void * src_vals = static_cast<const uint8_t *>(h_vals) + c0 * uv * es;
            if (!r_vals.direct)
            {
                void * st = sl.hin.get(chunk * uv * es);
                par_copy(st, src_vals, nb * uv * es);
                src_vals = st;
            }
            hc(hipMemcpyAsync(d_vals, src_vals, nb * uv * es, r_vals.direct ? r_vals.up() : hipMemcpyHostToDevice, P.cs), "H2D vals");
            const void * dstart = nullptr;
            uint64_t s0 = start0;
            if (d1 && h_starts)
            {
                void * d_start = sl.start.get(chunk * es);
                const void * src_st = static_cast<const uint8_t *>(h_starts) + c0 * es;
                if (!r_st.direct)
                {
                    void * st = sl.hst.get(chunk * es);
                    std::memcpy(st, src_st, nb * es);
                    src_st = st;
                }
                hc(hipMemcpyAsync(d_start, src_st, nb * es, r_st.direct ? r_st.up() : hipMemcpyHostToDevice, P.cs), "H2D starts");
                dstart = d_start;
            }
            else if (d1 && c0 > 0)
            {
                // chained list: this chunk starts after the previous chunk's last
                // input value (the previous unit's value n-1: slots past n are padding)
                const uint8_t * last = static_cast<const uint8_t *>(h_vals) + ((c0 - 1) * uv + n - 1) * es;
                s0 = 0;
                std::memcpy(&s0, last, es);
            }
            hc(hipEventRecord(sl.up, P.cs), "record up");
            hc(hipStreamWaitEvent(P.ks, sl.up, 0), "wait up");
            tc(tpf_enc_batch(fmt, d_vals, nb, n, d1, dstart, s0, d_pk, cap, d_off, d_ws, wsb, P.ks));
            hc(hipMemcpyAsync(st_off, d_off, (nb + 1) * 8, hipMemcpyDeviceToHost, P.ks), "D2H offsets");
            hc(hipEventRecord(sl.mid, P.ks), "record offsets");
            if (k >= 1)
                finish(k - 1);
        }
        finish(k - 1);
        hc(hipStreamSynchronize(P.ks), "sync");
        for (Slot & sl : P.slots)
            sl.drain();
        lease.ok = true;
        return TPF_OK;
    }
    catch (const Err & e)
    {
        return report(e, e.code);
    }
    catch (const std::exception & e)
    {
        return report(e, TPF_EHIP);
    }
}

int tpf_host_enc_multi(const int * devs, int ndev, int fmt, const void * h_vals, uint64_t nblocks, unsigned n, int d1,
                       const void * h_starts, uint64_t start0, uint8_t * h_out, uint64_t out_cap, uint64_t * h_off)
{
    try
    {
        if (!h_off)
            throw Err(TPF_EINVAL, "tpf_host_enc_multi: h_off is required");
        h_off[0] = 0;
        if (nblocks == 0)
            return TPF_OK;
        // validate before any shard reads the caller's array (a chained D1
        // shard reads the value before its first block: with n == 0 or n past
        // the unit that read would leave the array)
        if (!tpf::fmt_ok(fmt, n))
            throw Err(TPF_EINVAL, "tpf_host_enc_multi: unsupported (fmt, n)");
        if (!h_vals || !h_out)
            throw Err(TPF_EINVAL, "tpf_host_enc_multi: null pointer");
        need_device();
        int cnt = 0;
        hc(hipGetDeviceCount(&cnt), "hipGetDeviceCount");
        if (!devs || ndev < 1 || ndev > 64)
            throw Err(TPF_EINVAL, "tpf_host_enc_multi: need 1..64 devices");
        for (int d = 0; d < ndev; ++d)
            if (devs[d] < 0 || devs[d] >= cnt)
                throw Err(TPF_EINVAL, "tpf_host_enc_multi: device " + std::to_string(devs[d]) + " is not visible");
        const size_t es = wide_fmt(fmt) ? 8 : 4;
        const size_t uv = unit_values(fmt, n);
        const auto * vals = static_cast<const uint8_t *>(h_vals);
        std::vector<uint64_t> cut(static_cast<size_t>(ndev) + 1);
        for (int d = 0; d <= ndev; ++d)
            cut[d] = nblocks * static_cast<uint64_t>(d) / static_cast<uint64_t>(ndev);
        // Shard d > 0 writes at a provisional offset: the worst case of the
        // shards before it, inside the caller's own output when out_cap holds
        // every shard's bound (then each shard is moved down into place once
        // the earlier sizes are known: final <= provisional), else into a
        // scratch buffer of its bound (no zero-fill).  ADVICE r4: the first
        // version always used zero-filled pageable vectors, copied twice.
        std::vector<uint64_t> prov(static_cast<size_t>(ndev) + 1, 0);
        for (int d = 0; d < ndev; ++d)
            prov[d + 1] = prov[d] + tpf_enc_bound(fmt, cut[d + 1] - cut[d], n);
        const bool in_place = prov[ndev] <= out_cap;
        std::vector<std::unique_ptr<uint8_t[]>> tmp(static_cast<size_t>(ndev));
        std::vector<std::vector<uint64_t>> toff(static_cast<size_t>(ndev));
        const std::vector<tpf::ShardResult> res = tpf::run_shards(
            devs, ndev, [](int dev) { return hipSetDevice(dev) == hipSuccess; },
            [&](int d, std::string & msg) {
                const uint64_t b0 = cut[d], nb = cut[d + 1] - cut[d];
                if (nb == 0)
                    return TPF_OK;
                // a chained D1 list (no per-unit starts): shard d starts after the
                // previous unit's value n-1 (slots past n are padding)
                uint64_t s0 = start0;
                if (d1 && !h_starts && b0 > 0)
                {
                    s0 = 0;
                    std::memcpy(&s0, vals + ((b0 - 1) * uv + n - 1) * es, es);
                }
                const void * st = (d1 && h_starts) ? static_cast<const uint8_t *>(h_starts) + b0 * es : nullptr;
                int rc;
                if (d == 0)
                    rc = tpf_host_enc(fmt, vals, nb, n, d1, st, s0, h_out, out_cap, h_off);
                else
                {
                    const uint64_t cap = prov[d + 1] - prov[d];
                    uint8_t * dst = h_out + prov[d];
                    if (!in_place)
                    {
                        tmp[d].reset(new uint8_t[cap]); // (a bad_alloc is recorded for this shard by run_shards)
                        dst = tmp[d].get();
                    }
                    toff[d].resize(nb + 1);
                    rc = tpf_host_enc(fmt, vals + b0 * uv * es, nb, n, d1, st, s0, dst, cap, toff[d].data());
                }
                if (rc != TPF_OK)
                    msg = tpf_last_error(); // thread-local: carried to the caller's thread below
                return rc;
            },
            TPF_EHIP, TPF_EHIP);
        for (int d = 0; d < ndev; ++d)
            if (res[d].rc != TPF_OK)
                throw Err(res[d].rc, "tpf_host_enc_multi: shard " + std::to_string(d) + " (device " + std::to_string(devs[d]) + ", blocks " +
                                         std::to_string(cut[d]) + ".." + std::to_string(cut[d + 1]) + "): " + res[d].msg);
        // move the later shards into place behind the earlier ones, in order
        // (each destination ends at or before its provisional source)
        for (int d = 1; d < ndev; ++d)
        {
            const uint64_t b0 = cut[d], nb = cut[d + 1] - cut[d];
            if (nb == 0)
                continue;
            const uint64_t pos = h_off[b0], total = toff[d][nb];
            if (pos + total > out_cap)
                throw Err(TPF_EINVAL, "tpf_host_enc_multi: out_cap too small");
            const uint8_t * src = in_place ? h_out + prov[d] : tmp[d].get();
            if (!in_place || pos + total <= prov[d])
                par_copy(h_out + pos, src, total); // disjoint ranges
            else if (pos != prov[d])
                std::memmove(h_out + pos, src, total);
            tmp[d].reset();
            for (uint64_t i = 1; i <= nb; ++i)
                h_off[b0 + i] = pos + toff[d][i];
        }
        return TPF_OK;
    }
    catch (const Err & e)
    {
        return report(e, e.code);
    }
    catch (const std::exception & e)
    {
        return report(e, TPF_EHIP);
    }
}

void tpf_host_release(void)
{
    const FreePause fp; // the frees below wait on every stream of the device
    HipOps ops;
    try
    {
        g_pool.drain(ops); // each pipeline destroyed with its own device selected
    }
    catch (const std::exception & e)
    {
        tpf::set_last_error(e.what());
    }
}

} // extern "C"
