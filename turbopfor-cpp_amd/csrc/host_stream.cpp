// host_stream.cpp -- end-to-end host-memory streams: blocks
// and values live in host memory; chunks are copied to HBM, decoded/encoded
// by the batched kernels and copied back, with H2D, kernels and D2H of
// different chunks overlapped on kSets HIP streams (PCIe is full duplex, the
// kernels run at HBM speed, so the PCIe links bound this path).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/turbopfor_capi.h"
#include "../../include/turbopfor_gpu.h"

namespace tpf
{
void set_last_error(const std::string & msg);
}

namespace
{

constexpr int kSets = 3;

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

// Page-lock a host range for the duration of a call unless it already is.
struct Pin
{
    void * p = nullptr;
    Pin(const void * ptr, size_t bytes)
    {
        if (!ptr || !bytes)
            return;
        hipPointerAttribute_t a{};
        if (hipPointerGetAttributes(&a, ptr) == hipSuccess && a.type != hipMemoryTypeUnregistered)
            return;
        (void)hipGetLastError();
        if (hipHostRegister(const_cast<void *>(ptr), bytes, hipHostRegisterDefault) == hipSuccess)
            p = const_cast<void *>(ptr);
        else
            (void)hipGetLastError();
    }
    ~Pin()
    {
        if (p)
            (void)hipHostUnregister(p);
    }
};

struct Set
{
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr;
    void *d_in = nullptr, *d_vals = nullptr, *d_ws = nullptr, *d_start = nullptr;
    uint64_t * d_off = nullptr;
    uint64_t * h_off = nullptr; // pinned, chunk-local offsets
    size_t in_cap = 0, ws_cap = 0;
    ~Set()
    {
        if (s)
            (void)hipStreamSynchronize(s);
        for (void * p : {d_in, d_vals, d_ws, d_start, static_cast<void *>(d_off)})
            if (p)
                (void)hipFree(p);
        if (h_off)
            (void)hipHostFree(h_off);
        if (done)
            (void)hipEventDestroy(done);
        if (s)
            (void)hipStreamDestroy(s);
    }
};

} // namespace

extern "C" {

int tpf_host_dec(int fmt, const uint8_t * h_in, uint64_t in_bytes, const uint64_t * h_off, uint64_t nblocks, unsigned n,
                 void * h_vals, const void * h_starts)
{
    try
    {
        if (nblocks == 0)
            return TPF_OK;
        int cnt = 0;
        if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= 0)
            throw Err(TPF_ENODEV, "no HIP device visible (turbopfor_amd has no CPU fallback)");
        std::vector<uint64_t> scanned;
        if (!h_off)
        {
            scanned.resize(nblocks + 1);
            if (tpf_scan_offsets(fmt, h_in, in_bytes, n, nblocks, scanned.data()) < 0)
                throw Err(TPF_ECORRUPT, "tpf_host_dec: malformed block while scanning offsets");
            h_off = scanned.data();
        }
        const size_t es = wide_fmt(fmt) ? 8 : 4;
        const size_t uv = unit_values(fmt, n);
        const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(nblocks, (256ull << 20) / (es * uv)));
        Pin pin_in(h_in, in_bytes), pin_vals(h_vals, nblocks * uv * es);
        Set sets[kSets];
        size_t max_in = 0;
        for (uint64_t c0 = 0; c0 < nblocks; c0 += chunk)
        {
            const uint64_t c1 = std::min(nblocks, c0 + chunk);
            max_in = std::max<size_t>(max_in, h_off[c1] - h_off[c0]);
        }
        for (Set & st : sets)
        {
            hc(hipStreamCreateWithFlags(&st.s, hipStreamNonBlocking), "stream");
            hc(hipEventCreateWithFlags(&st.done, hipEventDisableTiming), "event");
            hc(hipMalloc(&st.d_in, max_in + 64), "hipMalloc in");
            hc(hipMalloc(&st.d_vals, chunk * uv * es), "hipMalloc vals");
            hc(hipMalloc(reinterpret_cast<void **>(&st.d_off), (chunk + 1) * 8), "hipMalloc off");
            hc(hipHostMalloc(reinterpret_cast<void **>(&st.h_off), (chunk + 1) * 8, hipHostMallocDefault), "hipHostMalloc off");
            if (h_starts)
                hc(hipMalloc(&st.d_start, chunk * es), "hipMalloc starts");
        }
        uint64_t k = 0;
        for (uint64_t c0 = 0; c0 < nblocks; c0 += chunk, ++k)
        {
            Set & st = sets[k % kSets];
            hc(hipEventSynchronize(st.done), "wait set"); // h_off staging and buffers free again
            const uint64_t c1 = std::min(nblocks, c0 + chunk);
            const uint64_t nb = c1 - c0;
            const uint64_t b0 = h_off[c0], bytes = h_off[c1] - b0;
            for (uint64_t i = 0; i <= nb; ++i)
                st.h_off[i] = h_off[c0 + i] - b0;
            hc(hipMemcpyAsync(st.d_off, st.h_off, (nb + 1) * 8, hipMemcpyHostToDevice, st.s), "H2D off");
            hc(hipMemcpyAsync(st.d_in, h_in + b0, bytes, hipMemcpyHostToDevice, st.s), "H2D bytes");
            if (h_starts)
                hc(hipMemcpyAsync(st.d_start, static_cast<const uint8_t *>(h_starts) + c0 * es, nb * es, hipMemcpyHostToDevice, st.s),
                   "H2D starts");
            const int rc = tpf_dec_batch(fmt, static_cast<const uint8_t *>(st.d_in), bytes, st.d_off, nb, n, st.d_vals,
                                         h_starts ? st.d_start : nullptr, nullptr, st.s);
            if (rc != TPF_OK)
                throw Err(rc, tpf_last_error());
            hc(hipMemcpyAsync(static_cast<uint8_t *>(h_vals) + c0 * uv * es, st.d_vals, nb * uv * es, hipMemcpyDeviceToHost, st.s),
               "D2H vals");
            hc(hipEventRecord(st.done, st.s), "record");
        }
        for (Set & st : sets)
            hc(hipStreamSynchronize(st.s), "sync");
        return TPF_OK;
    }
    catch (const Err & e)
    {
        tpf::set_last_error(e.what());
        return e.code;
    }
    catch (const std::exception & e)
    {
        tpf::set_last_error(e.what());
        return TPF_EHIP;
    }
}

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
        int cnt = 0;
        if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= 0)
            throw Err(TPF_ENODEV, "no HIP device visible (turbopfor_amd has no CPU fallback)");
        const size_t es = wide_fmt(fmt) ? 8 : 4;
        const size_t uv = unit_values(fmt, n);
        const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(nblocks, (256ull << 20) / (es * uv)));
        Pin pin_vals(h_vals, nblocks * uv * es), pin_out(h_out, out_cap);
        Set sets[kSets];
        const size_t cap = tpf_enc_bound(fmt, chunk, n);
        const size_t wsb = std::max<size_t>(tpf_enc_workspace_size(fmt, chunk, n), 256);
        for (Set & st : sets)
        {
            hc(hipStreamCreateWithFlags(&st.s, hipStreamNonBlocking), "stream");
            hc(hipEventCreateWithFlags(&st.done, hipEventDisableTiming), "event");
            hc(hipMalloc(&st.d_in, cap), "hipMalloc out");
            hc(hipMalloc(&st.d_vals, chunk * uv * es), "hipMalloc vals");
            hc(hipMalloc(&st.d_ws, wsb), "hipMalloc ws");
            hc(hipMalloc(reinterpret_cast<void **>(&st.d_off), (chunk + 1) * 8), "hipMalloc off");
            hc(hipHostMalloc(reinterpret_cast<void **>(&st.h_off), (chunk + 1) * 8, hipHostMallocDefault), "hipHostMalloc off");
            if (d1 && h_starts)
                hc(hipMalloc(&st.d_start, chunk * es), "hipMalloc starts");
        }
        // chunk k is encoded on set k%kSets; its bytes are copied out once the
        // previous chunk's total (its host position) is known: one-chunk lag.
        uint64_t pos = 0;
        std::vector<uint64_t> c0s;
        auto finish = [&](uint64_t kk) {
            Set & st = sets[kk % kSets];
            hc(hipEventSynchronize(st.done), "wait offsets");
            const uint64_t c0 = c0s[kk];
            const uint64_t nb = std::min(nblocks, c0 + chunk) - c0;
            const uint64_t total = st.h_off[nb];
            if (pos + total > out_cap)
                throw Err(TPF_EINVAL, "tpf_host_enc: out_cap too small");
            for (uint64_t i = 1; i <= nb; ++i)
                h_off[c0 + i] = pos + st.h_off[i];
            hc(hipMemcpyAsync(h_out + pos, st.d_in, total, hipMemcpyDeviceToHost, st.s), "D2H bytes");
            hc(hipEventRecord(st.done, st.s), "record");
            pos += total;
        };
        uint64_t k = 0;
        for (uint64_t c0 = 0; c0 < nblocks; c0 += chunk, ++k)
        {
            if (k >= 1)
                finish(k - 1);
            Set & st = sets[k % kSets];
            hc(hipEventSynchronize(st.done), "wait set");
            c0s.push_back(c0);
            const uint64_t nb = std::min(nblocks, c0 + chunk) - c0;
            hc(hipMemcpyAsync(st.d_vals, static_cast<const uint8_t *>(h_vals) + c0 * uv * es, nb * uv * es, hipMemcpyHostToDevice, st.s),
               "H2D vals");
            const void * dstart = nullptr;
            uint64_t s0 = start0;
            if (d1 && h_starts)
            {
                hc(hipMemcpyAsync(st.d_start, static_cast<const uint8_t *>(h_starts) + c0 * es, nb * es, hipMemcpyHostToDevice, st.s),
                   "H2D starts");
                dstart = st.d_start;
            }
            else if (d1 && c0 > 0)
            {
                // chained list: this chunk starts after the previous chunk's last input value
                const uint8_t * last = static_cast<const uint8_t *>(h_vals) + (c0 * uv - 1) * es;
                s0 = 0;
                std::memcpy(&s0, last, es);
            }
            const int rc = tpf_enc_batch(fmt, st.d_vals, nb, n, d1, dstart, s0, static_cast<uint8_t *>(st.d_in), cap, st.d_off,
                                         st.d_ws, wsb, st.s);
            if (rc != TPF_OK)
                throw Err(rc, tpf_last_error());
            hc(hipMemcpyAsync(st.h_off, st.d_off, (nb + 1) * 8, hipMemcpyDeviceToHost, st.s), "D2H off");
            hc(hipEventRecord(st.done, st.s), "record");
        }
        finish(k - 1);
        for (Set & st : sets)
            hc(hipStreamSynchronize(st.s), "sync");
        return TPF_OK;
    }
    catch (const Err & e)
    {
        tpf::set_last_error(e.what());
        return e.code;
    }
    catch (const std::exception & e)
    {
        tpf::set_last_error(e.what());
        return TPF_EHIP;
    }
}

} // extern "C"
