// tpf_device.h -- CDNA4 (gfx950) device helpers shared by the P4 kernels.
//
// All kernels decode/encode ONE P4 block per wave64.  Packed bytes are staged
// into LDS with coalesced 16-byte buffer loads and read back with aligned
// ds_read_b32 + v_alignbyte/v_alignbit funnel shifts, so no kernel ever issues
// an unaligned memory access although P4 blocks start at arbitrary bytes.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tpf::dev
{

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kWave = 64;

__device__ __forceinline__ uint32_t lane_id()
{
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// Broadcast lane 0's value: tells the compiler the value is wave-uniform so
// the mode dispatch becomes scalar branches.
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint64_t uni64(uint64_t x)
{
    uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x));
    uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x >> 32));
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

// SGPR budget of the generic encoder passes (k_enc_gr; 0 = the compiler's
// choice).  MI355X_MICROARCH.md: a .sgpr_count of 82-96 allows 7 waves per
// SIMD and 98+ 6, although the occupancy report says 8 / 7; k_enc_gr sat at
// 83-106.  A cap of 80 (a few SGPRs spill to VGPR lanes): C1 encode 344-346
// -> 356-358 G int32/s; on the 256v32 writer (86) it was neutral
// (profiles/r3_enc_sgpr_cap_ab.txt).
#define TPF_SGPR_ATTR __attribute__((amdgpu_num_sgpr(80)))

// Integer min (HIP's min<uint64_t> can resolve to a double overload).
__device__ __forceinline__ uint64_t min_u64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t sub_sat(uint64_t a, uint64_t b) { return a > b ? a - b : 0u; }

// v_readlane of a 64-bit value.  (__builtin_amdgcn_readlane returns int: OR-ing
// it into a uint64_t directly would sign-extend the low word.)
__device__ __forceinline__ uint64_t readlane_u64(uint64_t x, uint32_t l)
{
    const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(x)), l));
    const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(x >> 32)), l));
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

// OR-ed into a block decoder's consumed-byte count when a width field is
// outside its format (a 32-bit block with b or bx > 32, a 64-bit one with
// > 64): the count then disagrees with any offsets, so the batch decoders
// report the block through d_err exactly as the host framing rejects it
// (framing.cpp one_block).  Decoders clamp the widths to stay in
// bounds; the flag keeps the clamped parse from passing for a valid one.
constexpr uint32_t kWidthBad = 0x80000000u;

__device__ __forceinline__ uint32_t mask32(uint32_t b) { return b >= 32u ? 0xFFFFFFFFu : ((1u << b) - 1u); }

__device__ __forceinline__ uint32_t shl32(uint32_t v, uint32_t b) { return b >= 32u ? 0u : (v << b); }

// Order LDS traffic between lanes of ONE wave (a wave's DS ops execute in
// order; this only stops the compiler from moving them across the point).
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- LDS byte-stream readers (pos = byte offset into the dword array) -----
__device__ __forceinline__ uint32_t lds_byte(const uint32_t * w, uint32_t pos)
{
    return reinterpret_cast<const uint8_t *>(w)[pos];
}

// 32 bits starting at byte pos (any alignment).
__device__ __forceinline__ uint32_t lds_u32(const uint32_t * w, uint32_t pos)
{
    uint32_t q = pos >> 2;
    return __builtin_amdgcn_alignbyte(w[q + 1], w[q], pos & 3u);
}

// nb (<= 32) bits starting at absolute bit position bp.
__device__ __forceinline__ uint32_t lds_bits(const uint32_t * w, uint32_t bp, uint32_t nb)
{
    uint32_t q = bp >> 5;
    return __builtin_amdgcn_alignbit(w[q + 1], w[q], bp & 31u) & mask32(nb);
}

// Lane t gets x of lane t-1, lane 0 gets `first` (DPP wave_shr:1, one VALU
// op; __shfl_up is a ds_bpermute through the LDS pipe).  Round 4.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x, uint32_t first)
{
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(first), static_cast<int>(x), 0x138, 0xf, 0xf, false));
}
// Lane t gets x of lane t+1, lane 63 gets `last` (DPP wave_shl:1).
__device__ __forceinline__ uint32_t wave_shl1(uint32_t x, uint32_t last)
{
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(last), static_cast<int>(x), 0x130, 0xf, 0xf, false));
}

// ---- wave64 inclusive scan (DPP row_shr + row_bcast, gfx9 idiom) ----------
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x)
{
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false); // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false); // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false); // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false); // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false); // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false); // row_bcast:31
    return x;
}

// 64-bit inclusive scan (mod 2^64) from three 32-bit DPP scans: x = H 2^32 +
// M 2^16 + L with 16-bit M and L, whose scans over 64 lanes stay below 2^22
// (exact), and H scanned mod 2^32; then (SH << 32) + (SM << 16) + SL mod 2^64
// is the exact scan.  (Round 4: it replaced six 64-bit __shfl_up steps, i.e.
// twelve ds_bpermute through the LDS pipe, per scan: every 64-bit delta-1
// block and the 64-bit chained decode's unit sums pay one.)
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t x)
{
    const uint32_t sh = wave_incl_scan(static_cast<uint32_t>(x >> 32));
    const uint32_t sm = wave_incl_scan(static_cast<uint32_t>(x >> 16) & 0xFFFFu);
    const uint32_t sl = wave_incl_scan(static_cast<uint32_t>(x) & 0xFFFFu);
    return (static_cast<uint64_t>(sh) << 32) + (static_cast<uint64_t>(sm) << 16) + sl;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x)
{
    uint32_t s = wave_incl_scan(x);
    return __builtin_amdgcn_readlane(s, 63);
}

// Wave-wide OR / unsigned min, result in every lane: DPP inclusive scan
// (VALU, a few cycles per step) then a broadcast of lane 63 -- the
// __shfl_xor butterfly would be six ds_bpermute round trips through LDS.
__device__ __forceinline__ uint32_t wave_or(uint32_t x)
{
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false); // row_shr:1
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false); // row_shr:2
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false); // row_shr:4
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false); // row_shr:8
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false); // row_bcast:15
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false); // row_bcast:31
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(x), 63));
}

__device__ __forceinline__ uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }

__device__ __forceinline__ uint32_t wave_min(uint32_t x)
{
    constexpr uint32_t I = 0xFFFFFFFFu; // identity for lanes without a source
    x = umin32(x, __builtin_amdgcn_update_dpp(I, x, 0x111, 0xf, 0xf, false));
    x = umin32(x, __builtin_amdgcn_update_dpp(I, x, 0x112, 0xf, 0xf, false));
    x = umin32(x, __builtin_amdgcn_update_dpp(I, x, 0x114, 0xf, 0xf, false));
    x = umin32(x, __builtin_amdgcn_update_dpp(I, x, 0x118, 0xf, 0xf, false));
    x = umin32(x, __builtin_amdgcn_update_dpp(I, x, 0x142, 0xa, 0xf, false));
    x = umin32(x, __builtin_amdgcn_update_dpp(I, x, 0x143, 0xc, 0xf, false));
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(x), 63));
}

__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x)
{
    x = umax32(x, __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false));
    x = umax32(x, __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false));
    x = umax32(x, __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false));
    x = umax32(x, __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false));
    x = umax32(x, __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false));
    x = umax32(x, __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false));
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(x), 63));
}

__device__ __forceinline__ uint64_t lanemask_lt()
{
    uint32_t t = lane_id();
    return t == 0 ? 0ull : (~0ull >> (64u - t));
}

// ---- wave histogram of small keys -----------------------------------------
// C copies laid out [bin][C]; lane t adds into copy t % C, so lanes that share
// a bin hit C different banks (64/C lanes per address at worst) instead of one
// address 256 times: same-address LDS atomics serialise (measured 110 conflict
// cycles per block with a single copy).  Scratch: NBINS*C u32, 16-B aligned.
template <uint32_t C, uint32_t NBINS>
struct WaveHist
{
    static constexpr uint32_t kU32 = NBINS * C;

    __device__ __forceinline__ static void zero(uint32_t * h, uint32_t t)
    {
        for (uint32_t i = t; i < kU32 / 4u; i += 64u)
            reinterpret_cast<u32x4 *>(h)[i] = u32x4{0u, 0u, 0u, 0u};
    }

    __device__ __forceinline__ static void add(uint32_t * h, uint32_t bin, uint32_t t)
    {
        atomicAdd(&h[bin * C + (t & (C - 1u))], 1u);
    }

    // count of `bin` (bins >= NBINS read as 0)
    __device__ __forceinline__ static uint32_t get(const uint32_t * h, uint32_t bin)
    {
        if (bin >= NBINS)
            return 0u;
        const u32x4 * p = reinterpret_cast<const u32x4 *>(h + bin * C);
        u32x4 s = p[0];
#pragma unroll
        for (uint32_t i = 1; i < C / 4u; ++i)
            s += p[i];
        return (s.x + s.y) + (s.z + s.w);
    }
};

// ---- buffer loads: OOB lanes read zeros (no fault, no slack required) -----
// Descriptor inputs are forced through readfirstlane so the compiler can
// prove the SRD wave-uniform (otherwise every buffer op is wrapped in a
// readfirstlane "waterfall" loop, cdna_hip_programming.md T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void * base, uint32_t nbytes)
{
    const uint64_t b = uni64(reinterpret_cast<uint64_t>(base));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(b), static_cast<short>(0),
                                             static_cast<int>(uni(nbytes)), 0x00020000);
}

__device__ __forceinline__ u32x4 buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(off), 0, 0);
}

// 16 bytes at base+off where only [0, avail) of base is readable.  Raw buffer
// loads range-check the whole 16-byte access (a straddling load returns
// zeros), so the single chunk that straddles the end is read byte by byte.
__device__ __forceinline__ u32x4 load16_guarded(const uint8_t * base, __amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t avail)
{
    if (off + 16u <= avail)
        return buf_load16(r, off);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (uint32_t i = 0; i < 16u; ++i)
        if (off + i < avail)
            w[i >> 2] |= static_cast<uint32_t>(base[off + i]) << (8u * (i & 3u));
    return u32x4{w[0], w[1], w[2], w[3]};
}

} // namespace tpf::dev
