// capi.cpp -- extern "C" entry points of include/turbopfor_gpu.h.
// Argument checking, error reporting and launch sizing; the kernels live in
// the *.hip files.  There is deliberately no CPU fallback: without a HIP
// device every entry point fails with TPF_ENODEV.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/turbopfor_gpu.h"
#include "tpf_kernels.h"

#include <algorithm>

namespace
{
thread_local std::string g_err;

int fail(int code, const std::string & msg)
{
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char * where)
{
    return fail(TPF_EHIP, std::string(where) + ": " + hipGetErrorString(e));
}

int check_device()
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(TPF_ENODEV, "no HIP device visible (turbopfor_amd has no CPU fallback)");
    return TPF_OK;
}

// d_err handling: init to UINT64_MAX before the kernel.
int prep_err(uint64_t * d_err, hipStream_t s)
{
    if (!d_err)
        return TPF_OK;
    hipError_t e = tpf::fill_u32(d_err, 0xFFFFFFFFu, 2, s);
    return e == hipSuccess ? TPF_OK : hip_fail(e, "init d_err");
}
} // namespace

namespace tpf
{
void set_last_error(const std::string & msg) { g_err = msg; }

uint64_t grid_cap(hipStream_t, uint32_t per_cu)
{
    static int cus[64] = {0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64)
        dev = 0;
    if (cus[dev] == 0)
    {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        cus[dev] = n;
    }
    return static_cast<uint64_t>(cus[dev]) * per_cu;
}
} // namespace tpf

extern "C" {

const char * tpf_last_error(void) { return g_err.c_str(); }

int tpf_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    return n;
}

int tpf_p4dec256v32_batch(const uint8_t * d_in, uint64_t in_bytes, const uint64_t * d_off, uint64_t nblocks, uint32_t * d_out,
                          uint64_t * d_err, void * stream)
{
    if (int rc = check_device())
        return rc;
    if (nblocks && (!d_in || !d_off || !d_out))
        return fail(TPF_EINVAL, "tpf_p4dec256v32_batch: null pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (int rc = prep_err(d_err, s))
        return rc;
    hipError_t e = tpf::launch_dec256v32(d_in, in_bytes, d_off, nblocks, d_out, nullptr,
                                         reinterpret_cast<unsigned long long *>(d_err), s);
    return e == hipSuccess ? TPF_OK : hip_fail(e, "tpf_p4dec256v32_batch");
}


int tpf_p4d1dec256v32_batch(const uint8_t * d_in, uint64_t in_bytes, const uint64_t * d_off, uint64_t nblocks, uint32_t * d_out,
                            const uint32_t * d_starts, uint64_t * d_err, void * stream)
{
    if (int rc = check_device())
        return rc;
    if (nblocks && (!d_in || !d_off || !d_out || !d_starts))
        return fail(TPF_EINVAL, "tpf_p4d1dec256v32_batch: null pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (int rc = prep_err(d_err, s))
        return rc;
    hipError_t e = tpf::launch_dec256v32(d_in, in_bytes, d_off, nblocks, d_out, d_starts,
                                         reinterpret_cast<unsigned long long *>(d_err), s);
    return e == hipSuccess ? TPF_OK : hip_fail(e, "tpf_p4d1dec256v32_batch");
}

size_t tpf_p4d1dec256v32_chain_workspace_size(uint64_t nblocks) { return tpf::d1chain_workspace(nblocks); }

int tpf_p4d1dec256v32_chain_sums(const uint8_t * d_in, uint64_t in_bytes, const uint64_t * d_off, uint64_t nblocks, void * d_ws,
                                 size_t ws_bytes, uint32_t * d_total, uint64_t * d_err, void * stream)
{
    if (int rc = check_device())
        return rc;
    if (nblocks && (!d_in || !d_off || !d_ws))
        return fail(TPF_EINVAL, "tpf_p4d1dec256v32_chain_sums: null pointer");
    if (ws_bytes < tpf_p4d1dec256v32_chain_workspace_size(nblocks))
        return fail(TPF_EINVAL, "tpf_p4d1dec256v32_chain_sums: workspace too small");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (int rc = prep_err(d_err, s))
        return rc;
    hipError_t e = tpf::launch_d1chain_sums(d_in, in_bytes, d_off, nblocks, d_ws, ws_bytes, d_total,
                                            reinterpret_cast<unsigned long long *>(d_err), s);
    return e == hipSuccess ? TPF_OK : hip_fail(e, "tpf_p4d1dec256v32_chain_sums");
}

int tpf_p4d1dec256v32_chain_decode(const uint8_t * d_in, uint64_t in_bytes, const uint64_t * d_off, uint64_t nblocks, uint32_t * d_out,
                                   uint32_t base, const void * d_ws, uint64_t * d_err, void * stream)
{
    if (int rc = check_device())
        return rc;
    if (nblocks && (!d_in || !d_off || !d_out || !d_ws))
        return fail(TPF_EINVAL, "tpf_p4d1dec256v32_chain_decode: null pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (int rc = prep_err(d_err, s))
        return rc;
    hipError_t e = tpf::launch_d1chain_decode(d_in, in_bytes, d_off, nblocks, d_out, d_ws, base,
                                              reinterpret_cast<unsigned long long *>(d_err), s);
    return e == hipSuccess ? TPF_OK : hip_fail(e, "tpf_p4d1dec256v32_chain_decode");
}

int tpf_p4d1dec256v32_chained(const uint8_t * d_in, uint64_t in_bytes, const uint64_t * d_off, uint64_t nblocks, uint32_t * d_out,
                              uint32_t start0, void * d_ws, size_t ws_bytes, uint64_t * d_err, void * stream)
{
    // Two phases (block sums + scan, then decode).  A one-launch variant
    // (per-run sum pass, decoupled look-back, decode pass) measured 335 vs
    // 580 G int32/s on C3 and was dropped.
    if (int rc = tpf_p4d1dec256v32_chain_sums(d_in, in_bytes, d_off, nblocks, d_ws, ws_bytes, nullptr, d_err, stream))
        return rc;
    // phase B re-checks lengths; keep the first error index from phase A
    return tpf_p4d1dec256v32_chain_decode(d_in, in_bytes, d_off, nblocks, d_out, start0, d_ws, nullptr, stream);
}

// ---- 64-bit chained delta-1 decode (128v64 / 256v64 units) ----------------
static int chain64_nb(int fmt) { return fmt == TPF_FMT_256V64 ? 2 : fmt == TPF_FMT_128V64 ? 1 : 0; }

size_t tpf_d1dec64_chain_workspace_size(uint64_t nunits) { return tpf::d1chain64_workspace(nunits); }

int tpf_d1dec64_chain_sums(int fmt, const uint8_t * d_in, uint64_t in_bytes, const uint64_t * d_off, uint64_t nunits, void * d_ws,
                           size_t ws_bytes, uint64_t * d_total, uint64_t * d_err, void * stream)
{
    if (int rc = check_device())
        return rc;
    const int nb = chain64_nb(fmt);
    if (!nb)
        return fail(TPF_EINVAL, "tpf_d1dec64_chain_sums: fmt must be TPF_FMT_128V64 or TPF_FMT_256V64");
    if (nunits && (!d_in || !d_off || !d_ws))
        return fail(TPF_EINVAL, "tpf_d1dec64_chain_sums: null pointer");
    if (ws_bytes < tpf_d1dec64_chain_workspace_size(nunits))
        return fail(TPF_EINVAL, "tpf_d1dec64_chain_sums: workspace too small");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (int rc = prep_err(d_err, s))
        return rc;
    hipError_t e = tpf::launch_d1chain64_sums(static_cast<uint32_t>(nb), d_in, in_bytes, d_off, nunits, d_ws, ws_bytes, d_total,
                                              reinterpret_cast<unsigned long long *>(d_err), s);
    return e == hipSuccess ? TPF_OK : hip_fail(e, "tpf_d1dec64_chain_sums");
}

int tpf_d1dec64_chain_decode(int fmt, const uint8_t * d_in, uint64_t in_bytes, const uint64_t * d_off, uint64_t nunits, uint64_t * d_out,
                             uint64_t base, const void * d_ws, uint64_t * d_err, void * stream)
{
    if (int rc = check_device())
        return rc;
    const int nb = chain64_nb(fmt);
    if (!nb)
        return fail(TPF_EINVAL, "tpf_d1dec64_chain_decode: fmt must be TPF_FMT_128V64 or TPF_FMT_256V64");
    if (nunits && (!d_in || !d_off || !d_out || !d_ws))
        return fail(TPF_EINVAL, "tpf_d1dec64_chain_decode: null pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (int rc = prep_err(d_err, s))
        return rc;
    hipError_t e = tpf::launch_d1chain64_decode(static_cast<uint32_t>(nb), d_in, in_bytes, d_off, nunits, d_out, d_ws, base,
                                                reinterpret_cast<unsigned long long *>(d_err), s);
    return e == hipSuccess ? TPF_OK : hip_fail(e, "tpf_d1dec64_chain_decode");
}

int tpf_d1dec64_chained(int fmt, const uint8_t * d_in, uint64_t in_bytes, const uint64_t * d_off, uint64_t nunits, uint64_t * d_out,
                        uint64_t start0, void * d_ws, size_t ws_bytes, uint64_t * d_err, void * stream)
{
    if (int rc = tpf_d1dec64_chain_sums(fmt, d_in, in_bytes, d_off, nunits, d_ws, ws_bytes, nullptr, d_err, stream))
        return rc;
    // phase B re-checks lengths; keep the first error index from phase A
    return tpf_d1dec64_chain_decode(fmt, d_in, in_bytes, d_off, nunits, d_out, start0, d_ws, nullptr, stream);
}

int tpf_p4d1dec256v64_chained(const uint8_t * d_in, uint64_t in_bytes, const uint64_t * d_off, uint64_t nunits, uint64_t * d_out,
                              uint64_t start0, void * d_ws, size_t ws_bytes, uint64_t * d_err, void * stream)
{
    return tpf_d1dec64_chained(TPF_FMT_256V64, d_in, in_bytes, d_off, nunits, d_out, start0, d_ws, ws_bytes, d_err, stream);
}

int tpf_p4d1dec128v64_chained(const uint8_t * d_in, uint64_t in_bytes, const uint64_t * d_off, uint64_t nunits, uint64_t * d_out,
                              uint64_t start0, void * d_ws, size_t ws_bytes, uint64_t * d_err, void * stream)
{
    return tpf_d1dec64_chained(TPF_FMT_128V64, d_in, in_bytes, d_off, nunits, d_out, start0, d_ws, ws_bytes, d_err, stream);
}

uint64_t tpf_p4enc256v32_bound(uint64_t nblocks) { return nblocks * 1800u + 64u; }

size_t tpf_p4enc256v32_workspace_size(uint64_t nblocks) { return tpf::enc256v32_workspace(nblocks); }

static int enc256v32_common(const uint32_t * d_in, uint64_t nblocks, const uint32_t * d_starts, uint32_t start0, bool d1,
                            uint8_t * d_out, uint64_t out_cap, uint64_t * d_off, void * d_ws, size_t ws_bytes, void * stream,
                            const char * name)
{
    if (int rc = check_device())
        return rc;
    if (!d_off || (nblocks && (!d_in || !d_out || !d_ws)))
        return fail(TPF_EINVAL, std::string(name) + ": null pointer");
    if (ws_bytes < tpf::enc256v32_workspace(nblocks))
        return fail(TPF_EINVAL, std::string(name) + ": workspace too small");
    // the encoded sizes are known only on the device: the caller's capacity
    // must cover the worst case, or a block could be cut off unreported
    if (nblocks && out_cap < tpf_p4enc256v32_bound(nblocks))
        return fail(TPF_EINVAL, std::string(name) + ": out_cap below tpf_p4enc256v32_bound(nblocks)");
    hipError_t e = tpf::launch_enc256v32(d_in, nblocks, d_starts, start0, d1, d_out, out_cap, d_off, d_ws, ws_bytes,
                                         static_cast<hipStream_t>(stream));
    return e == hipSuccess ? TPF_OK : hip_fail(e, name);
}

int tpf_p4enc256v32_batch(const uint32_t * d_in, uint64_t nblocks, uint8_t * d_out, uint64_t out_cap, uint64_t * d_off, void * d_ws,
                          size_t ws_bytes, void * stream)
{
    return enc256v32_common(d_in, nblocks, nullptr, 0, false, d_out, out_cap, d_off, d_ws, ws_bytes, stream, "tpf_p4enc256v32_batch");
}


int tpf_p4d1enc256v32_batch(const uint32_t * d_in, uint64_t nblocks, const uint32_t * d_starts, uint32_t start0, uint8_t * d_out,
                            uint64_t out_cap, uint64_t * d_off, void * d_ws, size_t ws_bytes, void * stream)
{
    return enc256v32_common(d_in, nblocks, d_starts, start0, true, d_out, out_cap, d_off, d_ws, ws_bytes, stream,
                            "tpf_p4d1enc256v32_batch");
}

extern "C++" {
namespace tpf
{
// (fmt, n) pairs the batch entry points accept (also checked by the host
// streams before they cut a batch into shards)
bool fmt_ok(int fmt, unsigned n)
{
    switch (fmt)
    {
        case TPF_FMT_32:
        case TPF_FMT_64:
            return n >= 1 && n <= 256;
        case TPF_FMT_128V32:
            return n >= 1 && n <= 128;
        case TPF_FMT_256V32:
            return n >= 1 && n <= 256;
        case TPF_FMT_128V64: // n < 128: bitmap of pad8(n), exceptions over n values, full-width base
            return n >= 1 && n <= 128;
        case TPF_FMT_256V64: // batches of 256v64 units hold full units (the per-block API splits n < 256)
            return n == 256;
        default:
            return false;
    }
}
} // namespace tpf
}
using tpf::fmt_ok;

static unsigned unit_values(int fmt, unsigned n)
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

uint64_t tpf_enc_bound(int fmt, uint64_t nblocks, unsigned n)
{
    const bool wide = fmt == TPF_FMT_64 || fmt == TPF_FMT_128V64 || fmt == TPF_FMT_256V64;
    return nblocks * (64u + (wide ? 18u : 8u) * unit_values(fmt, n)) + 64u;
}

size_t tpf_enc_workspace_size(int fmt, uint64_t nblocks, unsigned n)
{
    if (fmt == TPF_FMT_256V32 && n == 256)
        return tpf::enc256v32_workspace(nblocks);
    if ((fmt == TPF_FMT_128V64 && n == 128) || fmt == TPF_FMT_256V64)
        return tpf::enc128v64_workspace(nblocks);
    return tpf::generic_workspace(nblocks);
}

int tpf_dec_batch(int fmt, const uint8_t * d_in, uint64_t in_bytes, const uint64_t * d_off, uint64_t nblocks, unsigned n, void * d_vals,
                  const void * d_starts, uint64_t * d_err, void * stream)
{
    if (int rc = check_device())
        return rc;
    if (!fmt_ok(fmt, n))
        return fail(TPF_EINVAL, "tpf_dec_batch: unsupported (fmt, n)");
    if (nblocks && (!d_in || !d_off || !d_vals))
        return fail(TPF_EINVAL, "tpf_dec_batch: null pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (int rc = prep_err(d_err, s))
        return rc;
    hipError_t e;
    if (fmt == TPF_FMT_256V32 && n == 256)
        e = tpf::launch_dec256v32(d_in, in_bytes, d_off, nblocks, static_cast<uint32_t *>(d_vals),
                                  static_cast<const uint32_t *>(d_starts), reinterpret_cast<unsigned long long *>(d_err), s);
    else
        e = tpf::launch_dec_generic(fmt, d_in, in_bytes, d_off, nblocks, n, d_vals, d_starts,
                                    reinterpret_cast<unsigned long long *>(d_err), s);
    return e == hipSuccess ? TPF_OK : hip_fail(e, "tpf_dec_batch");
}

int tpf_enc_batch(int fmt, const void * d_vals, uint64_t nblocks, unsigned n, int d1, const void * d_starts, uint64_t start0,
                  uint8_t * d_out, uint64_t out_cap, uint64_t * d_off, void * d_ws, size_t ws_bytes, void * stream)
{
    if (int rc = check_device())
        return rc;
    if (!fmt_ok(fmt, n))
        return fail(TPF_EINVAL, "tpf_enc_batch: unsupported (fmt, n)");
    if (!d_off || (nblocks && (!d_vals || !d_out || !d_ws)))
        return fail(TPF_EINVAL, "tpf_enc_batch: null pointer");
    if (ws_bytes < tpf_enc_workspace_size(fmt, nblocks, n))
        return fail(TPF_EINVAL, "tpf_enc_batch: workspace too small");
    if (nblocks && out_cap < tpf_enc_bound(fmt, nblocks, n))
        return fail(TPF_EINVAL, "tpf_enc_batch: out_cap below tpf_enc_bound(fmt, nblocks, n)");
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e;
    if (fmt == TPF_FMT_256V32 && n == 256)
        e = tpf::launch_enc256v32(static_cast<const uint32_t *>(d_vals), nblocks, static_cast<const uint32_t *>(d_starts),
                                  static_cast<uint32_t>(start0), d1 != 0, d_out, out_cap, d_off, d_ws, ws_bytes, s);
    else if ((fmt == TPF_FMT_128V64 && n == 128) || fmt == TPF_FMT_256V64)
        e = tpf::launch_enc128v64(fmt == TPF_FMT_256V64 ? 2u : 1u, static_cast<const uint64_t *>(d_vals), nblocks, d1 != 0,
                                  static_cast<const uint64_t *>(d_starts), start0, d_out, out_cap, d_off, d_ws, ws_bytes, s);
    else
        e = tpf::launch_enc_generic(fmt, d_vals, nblocks, n, d1 != 0, d_starts, start0, d_out, out_cap, d_off, d_ws, ws_bytes, s);
    return e == hipSuccess ? TPF_OK : hip_fail(e, "tpf_enc_batch");
}

// ---- n-variant streams: floor(n/256) 256v32 blocks + one
// p4Enc32 tail block.  Workspace: [0,256) scalars (tail start, tail error,
// tail offsets), then the tail's scratch image (encode), then the
// sub-call's own workspace.
static constexpr size_t kNHead = 256;

static size_t ntail_image(uint64_t) { return (tpf_enc_bound(TPF_FMT_32, 1, 256) + 255) & ~size_t(255); }

uint64_t tpf_p4nenc256v32_bound(uint64_t n) { return tpf_p4enc256v32_bound(n / 256) + tpf_enc_bound(TPF_FMT_32, 1, 256); }

size_t tpf_p4nenc256v32_workspace_size(uint64_t n)
{
    const size_t full = tpf::enc256v32_workspace(n / 256), tail = tpf_enc_workspace_size(TPF_FMT_32, 1, 256);
    return kNHead + ntail_image(n) + (full > tail ? full : tail);
}

int tpf_p4nenc256v32(const uint32_t * d_in, uint64_t n, int d1, uint32_t start0, uint8_t * d_out, uint64_t out_cap, uint64_t * d_off,
                     void * d_ws, size_t ws_bytes, void * stream)
{
    if (int rc = check_device())
        return rc;
    if (!d_off || (n && (!d_in || !d_out || !d_ws)))
        return fail(TPF_EINVAL, "tpf_p4nenc256v32: null pointer");
    if (ws_bytes < tpf_p4nenc256v32_workspace_size(n))
        return fail(TPF_EINVAL, "tpf_p4nenc256v32: workspace too small");
    if (n && out_cap < tpf_p4nenc256v32_bound(n)) // the tail lands at an offset only the device knows
        return fail(TPF_EINVAL, "tpf_p4nenc256v32: out_cap below tpf_p4nenc256v32_bound(n)");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t nfull = n / 256;
    const unsigned tail = static_cast<unsigned>(n % 256);
    uint8_t * ws = static_cast<uint8_t *>(d_ws);
    uint8_t * sub_ws = ws + kNHead + ntail_image(n);
    const size_t sub_bytes = ws_bytes - kNHead - ntail_image(n);
    if (nfull || !tail)
        if (int rc = enc256v32_common(d_in, nfull, nullptr, start0, d1 != 0, d_out, out_cap, d_off, sub_ws, sub_bytes, stream,
                                      "tpf_p4nenc256v32"))
            return rc;
    if (!tail)
        return TPF_OK;
    // D1 tail: its start is the last value of the full blocks (device) or start0
    const uint32_t * starts = (d1 && nfull) ? d_in + nfull * 256 - 1 : nullptr;
    if (!nfull) // the whole stream is the tail block
        return tpf_enc_batch(TPF_FMT_32, d_in, 1, tail, d1, nullptr, start0, d_out, out_cap, d_off, sub_ws, sub_bytes, stream);
    uint64_t * tail_off = reinterpret_cast<uint64_t *>(ws + 16);
    uint8_t * img = ws + kNHead;
    if (int rc = tpf_enc_batch(TPF_FMT_32, d_in + nfull * 256, 1, tail, d1, starts, start0, img, ntail_image(n), tail_off, sub_ws,
                               sub_bytes, stream))
        return rc;
    hipError_t e = tpf::launch_append(d_out, img, d_off + nfull, tail_off + 1, d_off + nfull + 1, s);
    return e == hipSuccess ? TPF_OK : hip_fail(e, "tpf_p4nenc256v32");
}

size_t tpf_p4ndec256v32_workspace_size(uint64_t n) { return kNHead + tpf_p4d1dec256v32_chain_workspace_size(n / 256); }

int tpf_p4ndec256v32(const uint8_t * d_in, uint64_t in_bytes, const uint64_t * d_off, uint64_t n, int d1, uint32_t start0,
                     uint32_t * d_out, void * d_ws, size_t ws_bytes, uint64_t * d_err, void * stream)
{
    if (int rc = check_device())
        return rc;
    if (n && (!d_in || !d_off || !d_out || !d_ws))
        return fail(TPF_EINVAL, "tpf_p4ndec256v32: null pointer");
    if (ws_bytes < tpf_p4ndec256v32_workspace_size(n))
        return fail(TPF_EINVAL, "tpf_p4ndec256v32: workspace too small");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t nfull = n / 256;
    const unsigned tail = static_cast<unsigned>(n % 256);
    uint8_t * ws = static_cast<uint8_t *>(d_ws);
    if (nfull)
    {
        int rc = d1 ? tpf_p4d1dec256v32_chained(d_in, in_bytes, d_off, nfull, d_out, start0, ws + kNHead, ws_bytes - kNHead, d_err, stream)
                    : tpf_p4dec256v32_batch(d_in, in_bytes, d_off, nfull, d_out, d_err, stream);
        if (rc)
            return rc;
    }
    else if (int rc = prep_err(d_err, s))
        return rc;
    if (!tail)
        return TPF_OK;
    uint32_t * start = reinterpret_cast<uint32_t *>(ws);
    const uint32_t * starts = nullptr;
    if (d1)
    {
        if (nfull)
            starts = d_out + nfull * 256 - 1;
        else
        {
            hipError_t e = tpf::fill_u32(start, start0, 1, s);
            if (e != hipSuccess)
                return hip_fail(e, "tpf_p4ndec256v32");
            starts = start;
        }
    }
    uint64_t * tail_err = d_err ? reinterpret_cast<uint64_t *>(ws + 8) : nullptr;
    if (int rc = tpf_dec_batch(TPF_FMT_32, d_in, in_bytes, d_off + nfull, 1, tail, d_out + nfull * 256, starts, tail_err, stream))
        return rc;
    if (!d_err)
        return TPF_OK;
    hipError_t e = tpf::launch_err_merge(reinterpret_cast<unsigned long long *>(d_err), reinterpret_cast<unsigned long long *>(tail_err),
                                         nfull, s);
    return e == hipSuccess ? TPF_OK : hip_fail(e, "tpf_p4ndec256v32");
}

int tpf_copy_async(void * dst, const void * src, uint64_t bytes, void * stream)
{
    if (int rc = check_device())
        return rc;
    if (bytes && (!dst || !src))
        return fail(TPF_EINVAL, "tpf_copy_async: null pointer");
    hipError_t e = tpf::launch_copy(dst, src, bytes, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? TPF_OK : hip_fail(e, "tpf_copy_async");
}

} // extern "C"
