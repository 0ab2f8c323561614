// p4_enc256v32.hip -- batch encode of 256v32 P4 blocks (p4Enc256v32 /
// p4D1Enc256v32, reference src/scalar/p4enc256v32_scalar.cpp:216-235 and
// p4d1enc256v32_scalar.cpp:7-15) on gfx950.
//
// Three launches:
//   1. plan  : one wave per block evaluates p4Bits32 (parallel cost model,
//              p4_enc32.h) and the exact encoded size -> d_off[i], plan word.
//   2. scan  : exclusive sum of sizes in place (hipcub/rocPRIM) -> byte offsets.
//   3. write : one wave per block scatters header, bitmap / exceptions / base
//              payload / vbytes into a zeroed LDS image whose dword phase
//              matches the destination, then streams it out with dword stores
//              (byte stores only on the two edge dwords shared with the
//              neighbouring blocks).
#include <hipcub/hipcub.hpp>

#include "p4_enc32.h"
#include "tpf_kernels.h"

namespace tpf::dev
{

constexpr uint32_t kImgU32 = 576; // 2304 bytes per wave image (max block 1792 B + phase)

__device__ __forceinline__ u32x4 load_block_values(const uint32_t * __restrict in, uint64_t blk, uint32_t t)
{
    return reinterpret_cast<const u32x4 *>(in + blk * 256u)[t];
}

// deltaEnc1 (p4_scalar_internal.h:711-719): d[i] = in[i] - in[i-1] - 1, in[-1] = start.
__device__ __forceinline__ u32x4 delta_encode(const u32x4 & v, uint32_t start, uint32_t t)
{
    uint32_t prev = static_cast<uint32_t>(__shfl_up(static_cast<int>(v.w), 1, 64));
    if (t == 0)
        prev = start;
    return u32x4{v.x - prev - 1u, v.y - v.x - 1u, v.z - v.y - 1u, v.w - v.z - 1u};
}

template <bool D1>
__device__ __forceinline__ uint32_t block_start(const uint32_t * in, const uint32_t * starts, uint32_t start0, uint64_t blk)
{
    if constexpr (!D1)
        return 0u;
    if (starts)
        return starts[blk];
    return blk == 0 ? start0 : in[blk * 256u - 1u]; // chained posting list
}

__device__ __forceinline__ uint32_t plan_word(const Plan32 & P)
{
    return P.b | (P.bx << 8) | (P.xn << 16) | (P.raw << 25);
}

__device__ __forceinline__ Plan32 unplan(uint32_t w, uint32_t size)
{
    Plan32 P;
    P.b = w & 0xFFu;
    P.bx = (w >> 8) & 0xFFu;
    P.xn = (w >> 16) & 0x1FFu;
    P.raw = (w >> 25) & 1u;
    P.size = size;
    return P;
}

template <bool D1>
__global__ __launch_bounds__(256) void k_enc256v32_plan(const uint32_t * __restrict in, uint64_t nblocks,
                                                         const uint32_t * __restrict starts, uint32_t start0,
                                                         uint64_t * __restrict sizes, uint32_t * __restrict plan)
{
    __shared__ uint32_t hist[4][64];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint64_t nw = static_cast<uint64_t>(gridDim.x) * 4u;
    for (uint64_t blk = static_cast<uint64_t>(blockIdx.x) * 4u + wv; blk < nblocks; blk += nw)
    {
        u32x4 v = load_block_values(in, blk, t);
        if constexpr (D1)
            v = delta_encode(v, block_start<D1>(in, starts, start0, blk), t);
        const Plan32 P = plan_block256(v, hist[wv], t);
        if (t == 0)
        {
            sizes[blk] = P.size;
            plan[blk] = plan_word(P);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        sizes[nblocks] = 0; // exclusive scan over nblocks+1 entries yields the total
}

template <bool D1>
__global__ __launch_bounds__(256) void k_enc256v32_write(const uint32_t * __restrict in, uint64_t nblocks,
                                                          const uint32_t * __restrict starts, uint32_t start0,
                                                          const uint64_t * __restrict off, const uint32_t * __restrict plan,
                                                          uint8_t * __restrict out, uint64_t out_cap)
{
    __shared__ uint32_t img_all[4][kImgU32 + 8];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t * img = img_all[wv];
    const uint64_t nw = static_cast<uint64_t>(gridDim.x) * 4u;
    const uint64_t out_base = reinterpret_cast<uint64_t>(out);
    for (uint64_t blk = static_cast<uint64_t>(blockIdx.x) * 4u + wv; blk < nblocks; blk += nw)
    {
        u32x4 v = load_block_values(in, blk, t);
        if constexpr (D1)
            v = delta_encode(v, block_start<D1>(in, starts, start0, blk), t);
        const uint64_t o = off[blk];
        const uint32_t size = static_cast<uint32_t>(off[blk + 1] - o);
        const Plan32 P = unplan(plan[blk], size);
        for (uint32_t i = t; i < kImgU32 + 8; i += 64)
            img[i] = 0u;
        wave_lds_sync();
        const uint64_t dst = out_base + o;
        const uint32_t phase = static_cast<uint32_t>(dst & 3u);
        emit_block256(img, phase, P, v, t);
        wave_lds_sync();
        const uint64_t a0 = dst & ~3ull;
        const uint32_t end = phase + size; // image bytes [phase, end) are the block
        const uint32_t nd = (end + 3u) >> 2;
        const uint64_t cap_end = out_base + out_cap;
        for (uint32_t d = t; d < nd; d += 64)
        {
            const uint64_t ga = a0 + 4u * d;
            const uint32_t w = img[d];
            const uint32_t lo = 4u * d, hi = lo + 4u;
            if (lo >= phase && hi <= end && ga + 4u <= cap_end)
            {
                *reinterpret_cast<uint32_t *>(ga) = w;
            }
            else
            {
                for (uint32_t x = 0; x < 4; ++x)
                {
                    const uint32_t bi = lo + x;
                    if (bi >= phase && bi < end && ga + x < cap_end)
                        *reinterpret_cast<uint8_t *>(ga + x) = static_cast<uint8_t>(w >> (8u * x));
                }
            }
        }
        wave_lds_sync();
    }
}

} // namespace tpf::dev

namespace tpf
{

size_t enc256v32_workspace(uint64_t nblocks)
{
    size_t scan_bytes = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, static_cast<uint64_t *>(nullptr),
                                     static_cast<int>(std::min<uint64_t>(nblocks + 1, 0x7FFFFFFF)));
    return ((nblocks * 4u + 255u) & ~size_t(255)) + scan_bytes + 256;
}

hipError_t launch_enc256v32(const uint32_t * in, uint64_t nblocks, const uint32_t * starts, uint32_t start0, bool d1,
                            uint8_t * out, uint64_t out_cap, uint64_t * off, void * ws, size_t ws_bytes, hipStream_t stream)
{
    if (nblocks == 0)
        return hipMemsetAsync(off, 0, sizeof(uint64_t), stream);
    if (nblocks + 1 > 0x7FFFFFFFull)
        return hipErrorInvalidValue;
    uint32_t * plan = static_cast<uint32_t *>(ws);
    const size_t plan_bytes = (nblocks * 4u + 255u) & ~size_t(255);
    void * scan_tmp = static_cast<uint8_t *>(ws) + plan_bytes;
    size_t scan_bytes = ws_bytes > plan_bytes ? ws_bytes - plan_bytes : 0;
    const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>((nblocks + 3) / 4, grid_cap(stream, 8)));
    if (d1)
        hipLaunchKernelGGL(dev::k_enc256v32_plan<true>, dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan);
    else
        hipLaunchKernelGGL(dev::k_enc256v32_plan<false>, dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return e;
    e = hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, off, static_cast<int>(nblocks + 1), stream);
    if (e != hipSuccess)
        return e;
    if (d1)
        hipLaunchKernelGGL(dev::k_enc256v32_write<true>, dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan,
                           out, out_cap);
    else
        hipLaunchKernelGGL(dev::k_enc256v32_write<false>, dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan,
                           out, out_cap);
    return hipGetLastError();
}

} // namespace tpf
