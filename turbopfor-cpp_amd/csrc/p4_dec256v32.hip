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
        const uint32_t nb = static_cast<uint32_t>(min<uint64_t>(kTile, nblocks - i0));
        if (tid <= nb)
            toff[tid] = off[i0 + tid];
        __syncthreads();
        const uint64_t a0 = (in_base + toff[0]) & ~15ull;
        const uint64_t aend = in_base + toff[nb];
        const uint64_t span = aend > a0 ? aend - a0 : 0;

        if (span <= kStage)
        {
            const uint32_t avail = static_cast<uint32_t>(min<uint64_t>(in_end > a0 ? in_end - a0 : 0, kStage));
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
                const uint32_t bspan = static_cast<uint32_t>(min<uint64_t>(bend > ba ? bend - ba : 0, kWaveSlot - 64));
                const uint32_t avail = static_cast<uint32_t>(min<uint64_t>(in_end > ba ? in_end - ba : 0, kWaveSlot - 64));
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

} // namespace tpf::dev

namespace tpf
{

hipError_t launch_dec256v32(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t * out,
                            const uint32_t * starts, unsigned long long * err, hipStream_t stream)
{
    if (nblocks == 0)
        return hipSuccess;
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
