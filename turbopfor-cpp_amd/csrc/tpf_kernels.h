// tpf_kernels.h -- host-side launch functions of the HIP kernels (internal).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

namespace tpf
{

// Stops the resident per-block servers (host_api.cpp) and keeps them
// stopped -- no per-block call starts -- while alive: wrap every hipFree /
// hipHostFree / hipHostUnregister of the library's own buffers in one, since
// HIP waits for all of the device's streams there, the server's included.
// Reentrant per thread (a thread-local depth: only the outermost pause takes
// the lock), and a per-block call made by a thread that holds a pause does not
// take the shared side (a std::shared_mutex locked again by its holder throws
// EDEADLK; round 4's hs_pause variant hit exactly that).
struct PerblockPause
{
    PerblockPause();
    ~PerblockPause();
    PerblockPause(const PerblockPause &) = delete;
    PerblockPause & operator=(const PerblockPause &) = delete;
};

// Workgroups to launch for a grid-stride kernel: per_cu workgroups on every
// CU of the current device (cached per device).
uint64_t grid_cap(hipStream_t stream, uint32_t per_cu);

// format ids (== TPF_FMT_* of include/turbopfor_gpu.h)
enum : int
{
    FMT_32 = 0,
    FMT_128V32 = 1,
    FMT_256V32 = 2,
    FMT_64 = 3,
    FMT_128V64 = 4,
    FMT_256V64 = 5,
};

// Kernel copy (16-B non-temporal stores) for moving data to/from pinned host
// memory concurrently with an SDMA copy in the other direction (host_copy.hip).
hipError_t launch_copy(void * dst, const void * src, uint64_t bytes, hipStream_t s);
// n-variant streams: device-positioned append of a scratch-encoded block, and
// merging a sub-batch's error index into the caller's.
hipError_t launch_append(uint8_t * dst, const uint8_t * src, const uint64_t * pos, const uint64_t * len, uint64_t * pos_out,
                         hipStream_t s);
hipError_t launch_err_merge(unsigned long long * err, const unsigned long long * sub_err, uint64_t base, hipStream_t s);
// p[0 .. n) = v, n <= 64 dwords, as a kernel (not a memset: see host_copy.hip)
hipError_t fill_u32(void * p, uint32_t v, uint32_t n, hipStream_t s);
// Per-block block server (p4_server.hip, tpf_server.h).
struct ServerReq;
struct ServerAns;
struct ServerCtl;
hipError_t launch_block_server(ServerReq * d_req, ServerAns * d_ans, ServerCtl * d_ctl, hipStream_t s);

// (fmt, n) accepted by the batch entry points (capi.cpp)
bool fmt_ok(int fmt, unsigned n);

size_t generic_workspace(uint64_t nblocks);
hipError_t launch_dec_generic(int fmt, const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t n,
                              void * out, const void * starts, unsigned long long * err, hipStream_t s);
hipError_t launch_enc_generic(int fmt, const void * in, uint64_t nblocks, uint32_t n, bool d1, const void * starts, uint64_t start0,
                              uint8_t * out, uint64_t out_cap, uint64_t * off, void * ws, size_t ws_bytes, hipStream_t s);

hipError_t launch_dec256v32(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t * out,
                            const uint32_t * starts, unsigned long long * err, hipStream_t stream);


// run scan test hook (p4_scan.hip)
size_t d1chain_workspace(uint64_t nblocks);
hipError_t launch_d1chain_sums(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, void * ws, size_t ws_bytes,
                               uint32_t * total, unsigned long long * err, hipStream_t stream);
hipError_t launch_d1chain_decode(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t * out,
                                 const void * ws, uint32_t base, unsigned long long * err, hipStream_t stream);

hipError_t launch_dec128v64(uint32_t nb, const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nunits,
                            uint64_t * out, const uint64_t * starts, unsigned long long * err, hipStream_t s);

size_t d1chain64_workspace(uint64_t nunits);
hipError_t launch_d1chain64_sums(uint32_t nb, const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nunits, void * ws,
                                 size_t ws_bytes, uint64_t * total, unsigned long long * err, hipStream_t s);
hipError_t launch_d1chain64_decode(uint32_t nb, const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nunits,
                                   uint64_t * out, const void * ws, uint64_t base, unsigned long long * err, hipStream_t s);

size_t enc128v64_workspace(uint64_t nunits);
hipError_t launch_enc128v64(uint32_t nb, const uint64_t * in, uint64_t nunits, bool d1, const uint64_t * starts, uint64_t start0,
                            uint8_t * out, uint64_t out_cap, uint64_t * off, void * ws, size_t ws_bytes, hipStream_t s);

size_t enc256v32_workspace(uint64_t nblocks);
hipError_t launch_enc256v32(const uint32_t * in, uint64_t nblocks, const uint32_t * starts, uint32_t start0, bool d1,
                            uint8_t * out, uint64_t out_cap, uint64_t * off, void * ws, size_t ws_bytes, hipStream_t stream);

} // namespace tpf
