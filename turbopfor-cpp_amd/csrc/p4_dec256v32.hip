// p4_dec256v32.hip -- batch decode of 256v32 P4 blocks (p4Dec256v32 /
// p4D1Dec256v32, reference src/scalar/p4dec256v32_scalar.cpp:90-137 and
// p4d1dec256v32_scalar.cpp:198-268) on gfx950: the hot path.
//
// Design notes (measured on MI355X): a first version staged
// tiles of 8 consecutive blocks per workgroup with one coalesced sweep and
// __syncthreads; it was latency-bound (one tile in flight per workgroup,
// 39% of HBM peak).  The kernel below runs every wave independently with a
// software pipeline and no workgroup barrier.
#include "p4_block32.h"
#include "tpf_kernels.h"

#include <hipcub/hipcub.hpp>

#include <cstdlib>

namespace tpf::dev
{

enum class StartMode : int
{
    None = 0,     // p4Dec256v32
    PerBlock = 1, // p4D1Dec256v32, start of block i = starts[i]
    Prefix = 2,   // chained list: start of block i = base + incl[i-1] (incl = prefix of block sums)
    SumOnly = 3,  // no output: sums[i] = sum over the block of (v + 1) mod 2^32
};

struct DecArgs
{
    const uint8_t * in;
    uint64_t in_bytes;
    const uint64_t * off;
    uint64_t nblocks;
    uint32_t * out;
    const uint32_t * starts; // PerBlock: starts; Prefix: inclusive block-sum prefix
    uint32_t base;           // Prefix: value preceding block 0
    uint32_t * sums;         // SumOnly
    unsigned long long * err;
};

// ---------------------------------------------------------------------------
// Wave-independent variant: every wave owns a private LDS slot and walks
// blocks wg, wg+W, wg+2W (W = all waves of the grid) with a software
// pipeline: while block k is decoded, the bytes of block k+1 are already in
// flight (two unconditional 16-byte buffer loads per lane = 2 KB per wave) and
// the offsets of block k+2 are prefetched through the scalar cache.  The loop
// is unrolled by two with separate register sets (A/B) so no in-flight load
// result is ever copied (a copy would force s_waitcnt vmcnt(0) at the loop
// head).  No workgroup barriers at all.
constexpr uint32_t kSlotBytes = 2304 + 64;

struct Chunk
{
    u32x4 a, b;    // bytes [0,1024) and [1024,2048) of the 16-aligned block image
    uint64_t base; // 16-aligned absolute start
    uint32_t span; // bytes to stage from base
    uint32_t avail;
};

// Always issues exactly two loads (a block that does not exist gets an empty
// descriptor: the loads return zeros without touching memory) so every path
// through the pipelined loop has the same vmcnt pattern and the compiler can
// wait with vmcnt(N > 0) instead of draining.
__device__ __forceinline__ void issue_chunk(Chunk & c, uint64_t in_base, uint64_t in_end, uint64_t o, uint64_t e, bool valid,
                                            uint32_t t)
{
    c.base = (in_base + o) & ~15ull;
    c.span = static_cast<uint32_t>(min_u64(sub_sat(in_base + e, c.base), kSlotBytes - 64));
    c.avail = valid ? static_cast<uint32_t>(min_u64(sub_sat(in_end, c.base), kSlotBytes)) : 0u;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const void *>(c.base), c.avail);
    // lanes past the block get an out-of-range offset: no memory traffic, zeros
    const uint32_t oa = 16u * t < c.span ? 16u * t : 0x80000000u;
    const uint32_t ob = 1024u + 16u * t < c.span ? 1024u + 16u * t : 0x80000000u;
    c.a = buf_load16(rs, oa);
    c.b = buf_load16(rs, ob);
}

template <StartMode SM>
__device__ __forceinline__ bool consume_chunk(const Chunk & c, uint64_t in_base, uint64_t o, uint64_t e, uint64_t blk,
                                              uint32_t * slot, uint32_t * scr, const DecArgs & A, uint32_t t)
{
    reinterpret_cast<u32x4 *>(slot)[t] = c.a;
    if (c.span > 1024u)
        reinterpret_cast<u32x4 *>(slot)[64 + t] = c.b;
    if (c.span > 2048u || c.span + 16u > c.avail)
    {
        // rare: > 2 KB blocks (third chunk) or the chunk straddling the end of
        // the stream (a raw buffer load that crosses num_records returns 0)
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const void *>(c.base), c.avail);
        const uint8_t * bp = reinterpret_cast<const uint8_t *>(c.base);
        for (uint32_t x = 16u * t; x < c.span; x += 1024u)
            reinterpret_cast<u32x4 *>(slot)[x >> 4] = load16_guarded(bp, rs, x, c.avail);
    }
    wave_lds_sync();
    u32x4 v;
    const uint32_t used = decode_block256v32(slot, static_cast<uint32_t>(in_base + o - c.base), scr, t, v);
    if constexpr (SM == StartMode::SumOnly)
    {
        const uint32_t s = wave_sum(v.x + v.y + v.z + v.w + 4u);
        if (t == 0)
            A.sums[blk] = s;
    }
    else
    {
        if constexpr (SM == StartMode::PerBlock)
            apply_delta1_256(v, A.starts[blk]);
        if constexpr (SM == StartMode::Prefix)
            apply_delta1_256(v, A.base + (blk ? A.starts[blk - 1] : 0u));
        reinterpret_cast<u32x4 *>(A.out + blk * 256u)[t] = v;
    }
    wave_lds_sync();
    return static_cast<uint64_t>(used) == e - o;
}

// Each wave decodes a contiguous run of kRun blocks [first, first+kRun): the
// run's kRun+1 offsets arrive with one vector load (lane i holds off[first+i])
// and are broadcast with v_readlane, so the per-block control path issues no
// memory instruction besides the pipelined data loads.  The grid is NOT
// persistent: ~nblocks/(4*kRun) workgroups let the dispatcher balance the CUs
// (a persistent grid larger than the resident set leaves a tail wave).
constexpr uint32_t kRun = 16;

__device__ __forceinline__ uint64_t lane_u64(uint64_t v, uint32_t lane)
{
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), lane);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), lane);
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

template <StartMode SM, int MINW>
__global__ __launch_bounds__(256, MINW) void k_dec256v32w(const DecArgs A)
{
    const uint8_t * in = A.in;
    const uint64_t in_bytes = A.in_bytes;
    const uint64_t * off = A.off;
    const uint64_t nblocks = A.nblocks;
    __shared__ uint32_t slots[4][kSlotBytes / 4];
    __shared__ uint32_t scratch[4][kWaveScratchU32];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t * slot = slots[wv];
    uint32_t * scr = scratch[wv];
    const uint64_t in_base = reinterpret_cast<uint64_t>(in);
    const uint64_t in_end = in_base + in_bytes;

    const uint64_t first = (static_cast<uint64_t>(blockIdx.x) * 4u + wv) * kRun;
    if (first >= nblocks)
        return;
    const uint32_t n = static_cast<uint32_t>(min_u64(kRun, nblocks - first));
    const uint64_t offv = t <= n ? off[first + t] : 0ull;
    uint64_t bad = ~0ull;

    // Three register chunks rotate (unrolled by three, no copies): while block
    // j is decoded, blocks j+1 and j+2 are in flight.
    Chunk C0, C1, C2;
    auto issue = [&](Chunk & c, uint32_t jj) {
        const uint32_t q = min(jj, n - 1);
        issue_chunk(c, in_base, in_end, lane_u64(offv, q), lane_u64(offv, q + 1), jj < n, t);
    };
    auto consume = [&](const Chunk & c, uint32_t jj) {
        const uint64_t o = lane_u64(offv, jj), e = lane_u64(offv, jj + 1);
        if (!consume_chunk<SM>(c, in_base, o, e, first + jj, slot, scr, A, t))
            bad = min_u64(bad, first + jj);
    };
    issue(C0, 0);
    issue(C1, 1);
    for (uint32_t j = 0;; j += 3)
    {
        issue(C2, j + 2);
        consume(C0, j);
        if (j + 1 >= n)
            break;
        issue(C0, j + 3);
        consume(C1, j + 1);
        if (j + 2 >= n)
            break;
        issue(C1, j + 4);
        consume(C2, j + 2);
        if (j + 3 >= n)
            break;
    }
    if (A.err != nullptr && t == 0 && bad != ~0ull)
        atomicMin(A.err, static_cast<unsigned long long>(bad));
}

} // namespace tpf::dev

namespace tpf
{

namespace
{
// TPF_DEC_MINW selects the occupancy the register allocator targets
// (launch-bounds minimum waves per SIMD; A/B knob, default measured best).
int dec_minw()
{
    static const int v = [] {
        const char * e = std::getenv("TPF_DEC_MINW");
        return e ? std::atoi(e) : 7;
    }();
    return v;
}

template <dev::StartMode SM>
hipError_t launch_mode(const dev::DecArgs & A, hipStream_t stream)
{
    const uint64_t per_wg = 4ull * dev::kRun;
    const uint32_t grid = static_cast<uint32_t>((A.nblocks + per_wg - 1) / per_wg);
    switch (dec_minw())
    {
        case 8:
            hipLaunchKernelGGL((dev::k_dec256v32w<SM, 8>), dim3(grid), dim3(256), 0, stream, A);
            break;
        case 6:
            hipLaunchKernelGGL((dev::k_dec256v32w<SM, 1>), dim3(grid), dim3(256), 0, stream, A);
            break;
        default:
            hipLaunchKernelGGL((dev::k_dec256v32w<SM, 7>), dim3(grid), dim3(256), 0, stream, A);
            break;
    }
    return hipGetLastError();
}
} // namespace

hipError_t launch_dec256v32(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t * out,
                            const uint32_t * starts, unsigned long long * err, hipStream_t stream)
{
    if (nblocks == 0)
        return hipSuccess;
    const dev::DecArgs A{in, in_bytes, off, nblocks, out, starts, 0u, nullptr, err};
    return starts ? launch_mode<dev::StartMode::PerBlock>(A, stream) : launch_mode<dev::StartMode::None>(A, stream);
}

// Chained delta-1: phase A computes every block's sum of
// (v+1) and their inclusive prefix in `incl` (device, nblocks u32); phase B
// decodes with start(i) = base + incl[i-1].  A shard of a multi-GPU list runs
// A, exchanges its total incl[n-1] with the other ranks, then B with its base.
size_t d1chain_workspace(uint64_t nblocks)
{
    size_t scan_bytes = 0;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, static_cast<uint32_t *>(nullptr), static_cast<uint32_t *>(nullptr),
                                           static_cast<int>(std::min<uint64_t>(nblocks, 0x7FFFFFFF)));
    return scan_bytes + 256;
}

hipError_t launch_d1chain_sums(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t * incl,
                               void * ws, size_t ws_bytes, unsigned long long * err, hipStream_t stream)
{
    if (nblocks == 0)
        return hipSuccess;
    if (nblocks > 0x7FFFFFFFull)
        return hipErrorInvalidValue;
    const dev::DecArgs A{in, in_bytes, off, nblocks, nullptr, nullptr, 0u, incl, err};
    hipError_t e = launch_mode<dev::StartMode::SumOnly>(A, stream);
    if (e != hipSuccess)
        return e;
    size_t sb = ws_bytes;
    return hipcub::DeviceScan::InclusiveSum(ws, sb, incl, incl, static_cast<int>(nblocks), stream);
}

hipError_t launch_d1chain_decode(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t * out,
                                 const uint32_t * incl, uint32_t base, unsigned long long * err, hipStream_t stream)
{
    if (nblocks == 0)
        return hipSuccess;
    const dev::DecArgs A{in, in_bytes, off, nblocks, out, incl, base, nullptr, err};
    return launch_mode<dev::StartMode::Prefix>(A, stream);
}

} // namespace tpf
