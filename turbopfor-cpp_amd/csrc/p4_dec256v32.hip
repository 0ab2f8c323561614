// p4_dec256v32.hip -- batch decode of 256v32 P4 blocks (p4Dec256v32 /
// p4D1Dec256v32, reference src/scalar/p4dec256v32_scalar.cpp:90-137 and
// p4d1dec256v32_scalar.cpp:198-268) on gfx950.
//
// Geometry: a 256-thread workgroup walks tiles of kTile consecutive blocks
// (grid-stride).  Because the blocks of a tile are contiguous in the packed
// stream, the whole tile [off[i0], off[i0+kTile]) is staged into LDS with one
// coalesced sweep of 16-byte buffer loads (the bytes of ~8 blocks in flight
// per workgroup), then each wave decodes blocks w, w+4 of the tile from LDS
// and writes 1 KB per block with one global_store_dwordx4 per lane.  Tiles
// larger than the staging area (only possible with vbyte-heavy blocks) fall
// back to per-wave staging of single blocks.
#include "p4_block32.h"
#include "tpf_kernels.h"

#include <cstdlib>

namespace tpf::dev
{

constexpr uint32_t kTile = 8;             // blocks per workgroup tile
constexpr uint32_t kStage = 10240;        // staging bytes per workgroup
constexpr uint32_t kWaveSlot = kStage / 4; // per-wave staging in the fallback
constexpr uint32_t kWG = 256;

enum class StartMode : int
{
    None = 0,     // p4Dec256v32
    PerBlock = 1, // p4D1Dec256v32 with starts[i]
};

template <StartMode SM>
__global__ __launch_bounds__(256) void k_dec256v32(const uint8_t * __restrict in, uint64_t in_bytes,
                                                    const uint64_t * __restrict off, uint64_t nblocks,
                                                    uint32_t * __restrict out, const uint32_t * __restrict starts,
                                                    unsigned long long * __restrict err)
{
    __shared__ uint32_t stage[(kStage + 64) / 4];
    __shared__ uint32_t scratch[4 * kWaveScratchU32];
    __shared__ uint64_t toff[kTile + 1];

    const uint32_t tid = threadIdx.x;
    const uint32_t t = tid & 63u;
    const uint32_t wv = uni(tid >> 6);
    uint32_t * scr = scratch + wv * kWaveScratchU32;
    const uint64_t ntiles = (nblocks + kTile - 1) / kTile;
    const uint64_t in_base = reinterpret_cast<uint64_t>(in);
    const uint64_t in_end = in_base + in_bytes;

    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x)
    {
        const uint64_t i0 = tile * kTile;
        const uint32_t nb = static_cast<uint32_t>(min_u64(kTile, nblocks - i0));
        if (tid <= nb)
            toff[tid] = off[i0 + tid];
        __syncthreads();
        const uint64_t a0 = (in_base + toff[0]) & ~15ull;
        const uint64_t aend = in_base + toff[nb];
        const uint64_t span = aend > a0 ? aend - a0 : 0;

        if (span <= kStage)
        {
            const uint32_t avail = static_cast<uint32_t>(min_u64(in_end > a0 ? in_end - a0 : 0, kStage));
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const void *>(a0), avail);
            for (uint32_t x = tid * 16u; x < span; x += kWG * 16u)
                *reinterpret_cast<u32x4 *>(reinterpret_cast<uint8_t *>(stage) + x) =
                    load16_guarded(reinterpret_cast<const uint8_t *>(a0), rs, x, avail);
            __syncthreads();
            for (uint32_t j = wv; j < nb; j += 4)
            {
                const uint64_t bo = toff[j];
                const uint32_t s = static_cast<uint32_t>(in_base + bo - a0);
                u32x4 v;
                const uint32_t used = decode_block256v32(stage, s, scr, t, v);
                const uint64_t blk = i0 + j;
                if constexpr (SM == StartMode::PerBlock)
                    apply_delta1_256(v, starts[blk]);
                reinterpret_cast<u32x4 *>(out + blk * 256u)[t] = v;
                if (err != nullptr && t == 0 && static_cast<uint64_t>(used) != toff[j + 1] - bo)
                    atomicMin(err, static_cast<unsigned long long>(blk));
            }
        }
        else
        {
            // Fallback: each wave stages one block at a time into its quarter.
            uint32_t * slot = stage + wv * (kWaveSlot / 4);
            for (uint32_t j = wv; j < nb; j += 4)
            {
                const uint64_t babs = in_base + toff[j];
                const uint64_t ba = babs & ~15ull;
                const uint64_t bend = in_base + toff[j + 1];
                const uint32_t bspan = static_cast<uint32_t>(min_u64(bend > ba ? bend - ba : 0, kWaveSlot - 64));
                const uint32_t avail = static_cast<uint32_t>(min_u64(in_end > ba ? in_end - ba : 0, kWaveSlot - 64));
                const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const void *>(ba), avail);
                for (uint32_t x = t * 16u; x < bspan; x += kWave * 16u)
                    *reinterpret_cast<u32x4 *>(reinterpret_cast<uint8_t *>(slot) + x) =
                        load16_guarded(reinterpret_cast<const uint8_t *>(ba), rs, x, avail);
                wave_lds_sync();
                u32x4 v;
                const uint32_t used = decode_block256v32(slot, static_cast<uint32_t>(babs - ba), scr, t, v);
                const uint64_t blk = i0 + j;
                if constexpr (SM == StartMode::PerBlock)
                    apply_delta1_256(v, starts[blk]);
                reinterpret_cast<u32x4 *>(out + blk * 256u)[t] = v;
                if (err != nullptr && t == 0 && static_cast<uint64_t>(used) != toff[j + 1] - toff[j])
                    atomicMin(err, static_cast<unsigned long long>(blk));
                wave_lds_sync();
            }
        }
        __syncthreads();
    }
}


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
                                              uint32_t * slot, uint32_t * scr, uint32_t * __restrict out,
                                              const uint32_t * __restrict starts, uint32_t t)
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
    if constexpr (SM == StartMode::PerBlock)
        apply_delta1_256(v, starts[blk]);
    reinterpret_cast<u32x4 *>(out + blk * 256u)[t] = v;
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

template <StartMode SM>
__global__ __launch_bounds__(256) void k_dec256v32w(const uint8_t * __restrict in, uint64_t in_bytes,
                                                     const uint64_t * __restrict off, uint64_t nblocks,
                                                     uint32_t * __restrict out, const uint32_t * __restrict starts,
                                                     unsigned long long * __restrict err)
{
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
        if (!consume_chunk<SM>(c, in_base, o, e, first + jj, slot, scr, out, starts, t))
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
    if (err != nullptr && t == 0 && bad != ~0ull)
        atomicMin(err, static_cast<unsigned long long>(bad));
}

} // namespace tpf::dev

namespace tpf
{

hipError_t launch_dec256v32(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t * out,
                            const uint32_t * starts, unsigned long long * err, hipStream_t stream)
{
    if (nblocks == 0)
        return hipSuccess;
    static const int variant = [] {
        const char * e = std::getenv("TPF_DEC_VARIANT");
        return e ? std::atoi(e) : 1;
    }();
    if (variant == 1)
    {
        const uint64_t per_wg = 4ull * dev::kRun;
        const uint32_t grid = static_cast<uint32_t>((nblocks + per_wg - 1) / per_wg);
        if (starts)
            hipLaunchKernelGGL(dev::k_dec256v32w<dev::StartMode::PerBlock>, dim3(grid), dim3(256), 0, stream, in, in_bytes,
                               off, nblocks, out, starts, err);
        else
            hipLaunchKernelGGL(dev::k_dec256v32w<dev::StartMode::None>, dim3(grid), dim3(256), 0, stream, in, in_bytes, off,
                               nblocks, out, starts, err);
        return hipGetLastError();
    }
    const uint64_t ntiles = (nblocks + dev::kTile - 1) / dev::kTile;
    const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(ntiles, grid_cap(stream, 8)));
    if (starts)
        hipLaunchKernelGGL(dev::k_dec256v32<dev::StartMode::PerBlock>, dim3(grid), dim3(dev::kWG), 0, stream, in, in_bytes,
                           off, nblocks, out, starts, err);
    else
        hipLaunchKernelGGL(dev::k_dec256v32<dev::StartMode::None>, dim3(grid), dim3(dev::kWG), 0, stream, in, in_bytes, off,
                           nblocks, out, starts, err);
    return hipGetLastError();
}

} // namespace tpf
