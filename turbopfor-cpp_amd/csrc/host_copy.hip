// host_copy.hip -- copy kernel for the host pipelines.
//
// Moving decoded values (or encoded bytes) between HBM and pinned host memory
// with a kernel instead of an SDMA engine (the host pipelines' A/B
// alternative, TPF_HOST_DOWN=kernel: measured 54 GB/s to the host vs 57 GB/s
// for SDMA, so SDMA stays the default).  Each lane moves 16-byte vectors with
// non-temporal stores; the head/tail bytes that are not 16-byte aligned at
// the destination go byte by byte.
#include <hip/hip_runtime.h>

#include "tpf_device.h"
#include "tpf_kernels.h"

namespace tpf::dev
{

// Destination-aligned copy: vector i covers dst[head + 16i, +16).  When the
// source shares the destination's phase mod 16 it is read with 16-byte loads;
// otherwise with five aligned dword loads and v_alignbyte (every dword read
// holds at least one byte of the source range, so nothing outside the
// source's pages is touched).  Edge bytes (head, tail) go one by one.
template <bool kAligned>
__global__ __launch_bounds__(256) void k_copy16(uint8_t * __restrict__ dst, const uint8_t * __restrict__ src, uint64_t head,
                                                uint64_t nvec, uint64_t bytes)
{
    const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    u32x4 * d = reinterpret_cast<u32x4 *>(dst + head);
    if constexpr (kAligned)
    {
        const u32x4 * s = reinterpret_cast<const u32x4 *>(src + head);
        for (uint64_t i = gid; i < nvec; i += stride)
            __builtin_nontemporal_store(s[i], d + i);
    }
    else
    {
        const uintptr_t s0 = reinterpret_cast<uintptr_t>(src + head);
        const uint32_t sh = static_cast<uint32_t>(s0 & 3u);
        const uint32_t * w = reinterpret_cast<const uint32_t *>(s0 & ~uintptr_t(3));
        for (uint64_t i = gid; i < nvec; i += stride)
        {
            const uint32_t * q = w + 4u * i;
            const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
            u32x4 v{__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                    __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
            __builtin_nontemporal_store(v, d + i);
        }
    }
    // unaligned head [0, head) and tail [head + 16 nvec, bytes)
    const uint64_t tail0 = head + nvec * 16u;
    const uint64_t nedge = head + (bytes - tail0);
    for (uint64_t i = gid; i < nedge; i += stride)
    {
        const uint64_t p = i < head ? i : tail0 + (i - head);
        dst[p] = src[p];
    }
}

// n-variant streams: append a block that was encoded into scratch at a
// position known only on the device (the total of the blocks before it):
// dst[*pos .. *pos + *len) = src[0 .. *len), then *pos_out = *pos + *len.
__global__ __launch_bounds__(256) void k_append(uint8_t * __restrict__ dst, const uint8_t * __restrict__ src, const uint64_t * pos,
                                                const uint64_t * len, uint64_t * pos_out)
{
    const uint64_t p = *pos, n = *len;
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x)
        dst[p + i] = src[i];
    if (threadIdx.x == 0)
        *pos_out = p + n;
}

// p[0 .. n) = v (n <= 64 dwords): the device-side initialisations of the
// batch entry points (d_err = ~0, empty totals and offsets) as a kernel
// rather than hipMemsetAsync.  Captured into a hipGraph a memset becomes a
// memset node, and replays of those nodes wrote a foreign byte pattern
// (0x11.., 0xd3..) while another thread of the process launched kernels
// (the block server): scripts/graph_canary.py, DESIGN.md 7.  A kernel node
// carries its value in its own arguments.
__global__ void k_fill_u32(uint32_t * p, uint32_t v, uint32_t n)
{
    if (threadIdx.x < n)
        p[threadIdx.x] = v;
}

// *err = min(*err, base + *sub_err) when the sub-batch reported a block.
__global__ void k_err_merge(unsigned long long * err, const unsigned long long * sub_err, uint64_t base)
{
    const unsigned long long e = *sub_err;
    if (threadIdx.x == 0 && e != ~0ull && base + e < *err)
        *err = base + e;
}

} // namespace tpf::dev

namespace tpf
{

hipError_t launch_append(uint8_t * dst, const uint8_t * src, const uint64_t * pos, const uint64_t * len, uint64_t * pos_out,
                         hipStream_t s)
{
    hipLaunchKernelGGL(dev::k_append, dim3(1), dim3(256), 0, s, dst, src, pos, len, pos_out);
    return hipGetLastError();
}

hipError_t fill_u32(void * p, uint32_t v, uint32_t n, hipStream_t s)
{
    if (n == 0)
        return hipSuccess;
    if (n > 64u)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(dev::k_fill_u32, dim3(1), dim3(64), 0, s, static_cast<uint32_t *>(p), v, n);
    return hipGetLastError();
}

hipError_t launch_err_merge(unsigned long long * err, const unsigned long long * sub_err, uint64_t base, hipStream_t s)
{
    hipLaunchKernelGGL(dev::k_err_merge, dim3(1), dim3(64), 0, s, err, sub_err, base);
    return hipGetLastError();
}

hipError_t launch_copy(void * dst, const void * src, uint64_t bytes, hipStream_t s)
{
    if (bytes == 0)
        return hipSuccess;
    const uintptr_t d = reinterpret_cast<uintptr_t>(dst), sp = reinterpret_cast<uintptr_t>(src);
    uint64_t head = (16u - (d & 15u)) & 15u;
    if (head > bytes)
        head = bytes;
    uint64_t nvec = (bytes - head) / 16u;
    const bool aligned = ((d ^ sp) & 15u) == 0;
    // the shifted reader loads one dword past each vector: keep the last
    // vector only if that dword still holds source bytes
    if (!aligned && nvec && (((sp + head + 16u * nvec) & 3u) == 0) && head + 16u * nvec == bytes)
        --nvec;
    const uint64_t want = (nvec + 32u + 255u) / 256u;
    const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>(want, grid_cap(s, 4)));
    if (aligned)
        hipLaunchKernelGGL(dev::k_copy16<true>, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, static_cast<uint8_t *>(dst),
                           static_cast<const uint8_t *>(src), head, nvec, bytes);
    else
        hipLaunchKernelGGL(dev::k_copy16<false>, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, static_cast<uint8_t *>(dst),
                           static_cast<const uint8_t *>(src), head, nvec, bytes);
    return hipGetLastError();
}

} // namespace tpf
