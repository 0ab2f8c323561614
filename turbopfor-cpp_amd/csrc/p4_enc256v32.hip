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
// Both kernels walk runs of 16 consecutive blocks per wave with the values of
// the next two blocks in flight (the first version loaded one block per loop
// iteration and waited for it: 5.0 and 5.4 ms per 10M blocks, latency-bound).
//
// probe != 0 (measurement only, reachable only through the separate
// tpf_probe_enc256v32 entry point -- the output is NOT a valid stream): 1 =
// plan kernel with the cost model replaced by a wave OR, 2 = write kernel
// copying the staged values instead of building blocks; same loads and
// stores, so they time each pass's data-movement ceiling
// (scripts/gpu_enc_probe.sh, profiles/r1_v4_enc_probe.txt).
#include <hipcub/hipcub.hpp>

#include "p4_enc32.h"
#include "tpf_kernels.h"

namespace tpf::dev
{

constexpr uint32_t kImgU32 = 592; // bytes per wave image: 4..7 lead + block (<= 2276 B) + slack, 16-B multiple
constexpr uint32_t kEncRun = 16;  // blocks per wave run
constexpr uint32_t kEncNC = 3;    // value chunks in flight per wave (block j+1, j+2 while j is encoded)

// deltaEnc1 (p4_scalar_internal.h:711-719): d[i] = in[i] - in[i-1] - 1, in[-1] = start.
__device__ __forceinline__ u32x4 delta_encode(const u32x4 & v, uint32_t start, uint32_t t)
{
    uint32_t prev = static_cast<uint32_t>(__shfl_up(static_cast<int>(v.w), 1, 64));
    if (t == 0)
        prev = start;
    return u32x4{v.x - prev - 1u, v.y - v.x - 1u, v.z - v.y - 1u, v.w - v.z - 1u};
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

// A wave's run of up to kEncRun consecutive blocks of 256 values.  Values
// arrive through a buffer descriptor over exactly the run's n KB, so the
// pipelined loads of blocks >= n return zeros without memory traffic and
// every path has the same vmcnt pattern (see RunPlane, p4_dec_run.h).
struct EncRun
{
    uint64_t first;
    uint32_t n;
    __amdgpu_buffer_rsrc_t rs;

    __device__ __forceinline__ bool init(const uint32_t * in, uint64_t nblocks, uint32_t wv)
    {
        first = (static_cast<uint64_t>(blockIdx.x) * 4u + wv) * kEncRun;
        if (first >= nblocks)
            return false;
        n = static_cast<uint32_t>(min_u64(kEncRun, nblocks - first));
        rs = make_rsrc(in + first * 256u, n * 1024u);
        return true;
    }

    __device__ __forceinline__ u32x4 load(uint32_t jj, uint32_t t) const
    {
        return __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(jj * 1024u + 16u * t), 0, 0);
    }

    // Start value of block first+t for delta-1 (lanes t < n): the given
    // starts, or for one chained list the last value of the previous block.
    __device__ __forceinline__ uint32_t start_lane(const uint32_t * in, const uint32_t * starts, uint32_t start0,
                                                    uint32_t t) const
    {
        if (t >= n)
            return 0u;
        const uint64_t blk = first + t;
        if (starts)
            return starts[blk];
        return blk == 0 ? start0 : in[blk * 256u - 1u];
    }

    // Pipelined walk: body(v, jj) for jj = 0..n-1 with NC blocks in flight.
    template <class Body>
    __device__ __forceinline__ void walk(uint32_t t, Body && body) const
    {
        u32x4 C[kEncNC];
#pragma unroll
        for (uint32_t u = 0; u + 1 < kEncNC; ++u)
            C[u] = load(u, t);
        bool more = true;
        for (uint32_t j = 0; more; j += kEncNC)
        {
#pragma unroll
            for (uint32_t u = 0; u < kEncNC; ++u)
            {
                if (more)
                {
                    C[(u + kEncNC - 1) % kEncNC] = load(j + u + kEncNC - 1, t);
                    body(C[u], j + u);
                    more = j + u + 1 < n;
                }
            }
        }
    }
};

__device__ __forceinline__ uint32_t rl32(uint32_t v, uint32_t lane)
{
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(lane)));
}

template <bool D1, int PROBE = 0>
__global__ __launch_bounds__(256) void k_enc256v32_plan(const uint32_t * __restrict in, uint64_t nblocks,
                                                         const uint32_t * __restrict starts, uint32_t start0,
                                                         uint64_t * __restrict sizes, uint32_t * __restrict plan)
{
    __shared__ __attribute__((aligned(16))) uint32_t hist[4][kPlanHistU32];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    if (blockIdx.x == 0 && threadIdx.x == 0)
        sizes[nblocks] = 0; // exclusive scan over nblocks+1 entries yields the total
    EncRun R;
    if (!R.init(in, nblocks, wv))
        return;
    const uint32_t stv = D1 ? R.start_lane(in, starts, start0, t) : 0u;
    uint32_t szv = 0u, pwv = 0u; // lane j: block first+j
    R.walk(t, [&](u32x4 v, uint32_t jj) {
        if constexpr (D1)
            v = delta_encode(v, rl32(stv, jj), t);
        Plan32 P;
        if constexpr (PROBE == 1)
        {
            P.b = bw32(uni(wave_or(v.x | v.y | v.z | v.w)));
            P.bx = 0;
            P.size = 1 + 32 * P.b;
            P.xn = 0;
            P.raw = 0;
        }
        else
            P = plan_block256(v, hist[wv], t);
        szv = t == jj ? P.size : szv;
        pwv = t == jj ? plan_word(P) : pwv;
    });
    if (t < R.n)
    {
        sizes[R.first + t] = szv;
        plan[R.first + t] = pwv;
    }
}

template <bool D1, int PROBE = 0>
__global__ __launch_bounds__(256) void k_enc256v32_write(const uint32_t * __restrict in, uint64_t nblocks,
                                                          const uint32_t * __restrict starts, uint32_t start0,
                                                          const uint64_t * __restrict off, const uint32_t * __restrict plan,
                                                          uint8_t * __restrict out, uint64_t out_cap)
{
    __shared__ __attribute__((aligned(16))) uint32_t img_all[4][kImgU32];
    __shared__ __attribute__((aligned(16))) uint32_t val_all[4][kEncValU32];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t * img = img_all[wv];
    EncRun R;
    if (!R.init(in, nblocks, wv))
        return;
    const uint32_t stv = D1 ? R.start_lane(in, starts, start0, t) : 0u;
    // lane j: destination offset (64-bit), size and plan of block first+j
    const uint64_t ov = t < R.n ? off[R.first + t] : 0ull;
    const uint64_t ev = t < R.n ? off[R.first + t + 1u] : 0ull;
    const uint32_t szv = static_cast<uint32_t>(ev - ov);
    const uint32_t pwv = t < R.n ? plan[R.first + t] : 0u;
    const uint32_t olo = static_cast<uint32_t>(ov), ohi = static_cast<uint32_t>(ov >> 32);
    const uint64_t out_base = reinterpret_cast<uint64_t>(out);
    const uint64_t cap_end = out_base + out_cap;
    zero_image(img, kImgU32 / 4u, t);
    wave_lds_sync();
    R.walk(t, [&](u32x4 v, uint32_t jj) {
        if constexpr (D1)
            v = delta_encode(v, rl32(stv, jj), t);
        const uint32_t size = rl32(szv, jj);
        const Plan32 P = unplan(rl32(pwv, jj), size);
        const uint64_t dst = out_base + ((static_cast<uint64_t>(rl32(ohi, jj)) << 32) | rl32(olo, jj));
        if constexpr (PROBE == 2)
        {
            reinterpret_cast<u32x4 *>(img)[4 + t] = v;
            wave_lds_sync();
            copy_out_image16(img, kImgLead, dst, size, cap_end, t);
            wave_lds_sync();
            return;
        }
        const uint32_t sb = emit_block256<true>(img, val_all[wv], P, v, t);
        wave_lds_sync();
        copy_out_image16(img, sb, dst, size, cap_end, t);
        wave_lds_sync();
        // only [0, sb + size) can be non-zero: clear it for the next block
        zero_image(img, min((sb + size + 15u) >> 4, kImgU32 / 4u), t);
        wave_lds_sync();
    });
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
                            uint8_t * out, uint64_t out_cap, uint64_t * off, void * ws, size_t ws_bytes, hipStream_t stream,
                            int probe)
{
    if (nblocks == 0)
        return hipMemsetAsync(off, 0, sizeof(uint64_t), stream);
    if (nblocks + 1 > 0x7FFFFFFFull)
        return hipErrorInvalidValue;
    uint32_t * plan = static_cast<uint32_t *>(ws);
    const size_t plan_bytes = (nblocks * 4u + 255u) & ~size_t(255);
    void * scan_tmp = static_cast<uint8_t *>(ws) + plan_bytes;
    size_t scan_bytes = ws_bytes > plan_bytes ? ws_bytes - plan_bytes : 0;
    const uint64_t per_wg = 4ull * dev::kEncRun;
    const uint32_t grid = static_cast<uint32_t>((nblocks + per_wg - 1) / per_wg);
    if (d1)
        hipLaunchKernelGGL(dev::k_enc256v32_plan<true>, dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan);
    else if (probe == 1)
        hipLaunchKernelGGL((dev::k_enc256v32_plan<false, 1>), dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan);
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
    else if (probe == 2)
        hipLaunchKernelGGL((dev::k_enc256v32_write<false, 2>), dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan,
                           out, out_cap);
    else
        hipLaunchKernelGGL(dev::k_enc256v32_write<false>, dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan,
                           out, out_cap);
    return hipGetLastError();
}

} // namespace tpf
