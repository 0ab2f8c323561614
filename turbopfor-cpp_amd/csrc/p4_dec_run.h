// p4_dec_run.h -- per-wave run machinery shared by the 256v32 decode kernels
// (p4_dec256v32.hip, p4_d1chain.hip): the run's control plane held in vector
// lanes, the register-chunk loads and the LDS staging of one block.
#pragma once

#include "p4_block32.h"

namespace tpf::dev
{

constexpr uint32_t kSlotBytes = 2304 + 64;
constexpr uint32_t kRunDefault = 16; // blocks per wave (<= 62: lanes >= n hold "no block")

// ctl word bits
constexpr uint32_t kCtlSpan = 0xFFFu;    // bytes the fast path stages (0: none)
constexpr uint32_t kCtlShift = 12;       // [12,16): block start inside its 16-aligned chunk
constexpr uint32_t kCtlSlow = 1u << 16;  // > 2 KB or straddles the stream end: guarded loads
constexpr uint32_t kCtlTwo = 1u << 17;   // second 1 KB half present
constexpr uint32_t kCtlBig = 1u << 18;   // ONE layout: bytes past the first 1 KB, loaded at staging

struct Chunk
{
    u32x4 a, b; // bytes [0,1024) and [1024,2048) of the 16-aligned block image
};

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t lane)
{
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(lane)));
}

// POL (A/B knob): bit 0 = non-temporal loads (measured -4%), bit 1 =
// non-temporal stores (measured +2.5%), bit 2 = block order, bit 3 = "sc1 nt"
// stores through a run descriptor (round 2: +1-2.5% over bit 1, default).
template <uint32_t POL>
__device__ __forceinline__ u32x4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(off), 0, (POL & 1u) ? 2 : 0);
}

// 16-byte store through a buffer descriptor with cache policy "sc1 nt"
// (aux: bit 1 nt, bit 4 sc1): streamed output that is not kept in the XCD's L2
__device__ __forceinline__ void st16_run(__amdgpu_buffer_rsrc_t r, uint32_t off, const u32x4 & v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, r, static_cast<int>(off), 0, 18);
}

template <uint32_t POL>
__device__ __forceinline__ void st16(u32x4 * p, const u32x4 & v)
{
    if constexpr ((POL & 2u) != 0u)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// Control plane of a run of up to 62 blocks, lane j = the run's j-th block:
// the run's offsets arrive with one vector load and every per-block quantity
// (chunk base, span, byte offset inside the chunk, expected length) is
// computed once in VALU and fetched per block with v_readlane.  The scalar
// unit is shared by the CU's four SIMDs; per-block 64-bit address arithmetic
// on it was the measured limiter before this layout.
// ONE: one 16-byte load per lane per block in flight (the block's first
// 1 KB; the rest of a larger block is loaded when it is staged), so twice as
// many blocks fit in flight in the same registers.
// Length check of a run without per-block scalar work: lane jj keeps the
// byte count block jj consumed (one v_cndmask per block); after the run one
// compare against the plane's expected lengths and a ballot give the blocks
// whose parse disagrees with their offsets.  (The per-block form -- readlane,
// scalar compare, 64-bit mask update -- put ~5 more SALU instructions on
// every block.)
struct UsedLanes
{
    uint32_t v = 0u;
    __device__ __forceinline__ void put(uint32_t used, uint32_t jj, uint32_t t) { v = t == jj ? used : v; }
    __device__ __forceinline__ uint64_t bad(uint32_t len, bool valid) const { return __ballot(valid && v != len); }
};

template <uint32_t SLOT, bool ONE = false>
struct RunPlaneT
{
    uint32_t ctl;        // kCtl* bits
    uint32_t len;        // expected byte length (0xFFFFFFFF: implausible offsets)
    uint32_t cblo, cbhi; // 16-aligned chunk base address
    uint32_t span;       // bytes to stage
    uint32_t avail;      // readable bytes from the chunk base (stream end)

    // A block whose offsets do not lie inside the stream (o <= e <= in_bytes)
    // loads nothing -- whatever the offset values, no descriptor is based
    // outside the stream -- and is reported by the length check (len =
    // 0xFFFFFFFF).  (Round 5: a caller passing a 2-entry offset array for
    // 3,200 blocks made the decoder read garbage offsets and fault.)
    __device__ __forceinline__ void init(uint64_t in_base, uint64_t in_end, uint64_t o, uint64_t e, bool valid)
    {
        const bool inb = valid && e >= o && e <= in_end - in_base;
        const uint64_t ab = in_base + (inb ? o : 0ull);
        const uint64_t cb = ab & ~15ull;
        span = inb ? static_cast<uint32_t>(min_u64(sub_sat(in_base + e, cb), SLOT - 64)) : 0u;
        avail = inb ? static_cast<uint32_t>(min_u64(sub_sat(in_end, cb), SLOT)) : 0u;
        const bool slow = inb && ((!ONE && span > 2048u) || span + 16u > avail);
        ctl = (slow ? 0u : span) | ((static_cast<uint32_t>(ab) & 15u) << kCtlShift) | (slow ? kCtlSlow : 0u)
            | (!ONE && !slow && span > 1024u ? kCtlTwo : 0u) | (ONE && !slow && span > 1024u ? kCtlBig : 0u);
        len = (inb && e - o < 0x10000ull) ? static_cast<uint32_t>(e - o) : 0xFFFFFFFFu;
        cblo = static_cast<uint32_t>(cb);
        cbhi = static_cast<uint32_t>(cb >> 32);
    }

    // Two unconditional 16-byte loads per lane (block jj's bytes [0,2048));
    // lanes past the block, and blocks jj >= n (ctl 0), get an out-of-range
    // offset: zeros, no memory traffic, and the same vmcnt pattern on every path.
    template <uint32_t POL>
    __device__ __forceinline__ void issue(Chunk & c, uint32_t jj, uint32_t t) const
    {
        const uint32_t cw = rl(ctl, jj);
        const uint64_t base = (static_cast<uint64_t>(rl(cbhi, jj)) << 32) | rl(cblo, jj);
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const void *>(base), SLOT);
        const uint32_t fspan = cw & kCtlSpan;
        c.a = ld16<POL>(rs, 16u * t < fspan ? 16u * t : 0x80000000u);
        if constexpr (!ONE)
            c.b = ld16<POL>(rs, 1024u + 16u * t < fspan ? 1024u + 16u * t : 0x80000000u);
    }

    // First 4 bytes of block jj (wave-uniform), from the load registers:
    // lane 0 holds chunk bytes 0..15, lane 1 bytes 16..31.  Slow-path blocks
    // (staged by guarded loads) read them from the slot instead.
    __device__ __forceinline__ uint32_t head(const Chunk & c, uint32_t cw, const uint32_t * slot) const
    {
        const uint32_t s = (cw >> kCtlShift) & 15u;
        if (cw & kCtlSlow)
            return uni(lds_u32(slot, s));
        const uint32_t a0 = rl(c.a.x, 0), a1 = rl(c.a.y, 0), a2 = rl(c.a.z, 0), a3 = rl(c.a.w, 0), a4 = rl(c.a.x, 1);
        const uint32_t k = s >> 2;
        const uint32_t lo = k == 0 ? a0 : k == 1 ? a1 : k == 2 ? a2 : a3;
        const uint32_t hi = k == 0 ? a1 : k == 1 ? a2 : k == 2 ? a3 : a4;
        return uni(__builtin_amdgcn_alignbyte(hi, lo, s & 3u));
    }

    // Probe mode (no staging): the same extra loads of a big block, OR-ed.
    __device__ __forceinline__ u32x4 big_rest_or(uint32_t jj, uint32_t t) const
    {
        u32x4 acc{0u, 0u, 0u, 0u};
        const uint32_t cw = rl(ctl, jj);
        if (ONE && (cw & kCtlBig))
        {
            const uint32_t sp = cw & kCtlSpan;
            const uint64_t base = (static_cast<uint64_t>(rl(cbhi, jj)) << 32) | rl(cblo, jj);
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const void *>(base), SLOT);
            for (uint32_t x = 1024u + 16u * t; x < sp; x += 1024u)
                acc |= ld16<0>(rs, x);
        }
        return acc;
    }

    // Write block jj's chunk into the wave's LDS slot; returns its ctl word.
    __device__ __forceinline__ uint32_t stage(const Chunk & c, uint32_t jj, uint32_t * slot, uint32_t t) const
    {
        const uint32_t cw = rl(ctl, jj);
        reinterpret_cast<u32x4 *>(slot)[t] = c.a;
        if (!ONE && (cw & kCtlTwo))
            reinterpret_cast<u32x4 *>(slot)[64 + t] = c.b;
        if (ONE && (cw & kCtlBig))
        {
            // the rest of a block larger than 1 KB (inside the stream: plain loads)
            const uint32_t sp = cw & kCtlSpan;
            const uint64_t base = (static_cast<uint64_t>(rl(cbhi, jj)) << 32) | rl(cblo, jj);
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const void *>(base), SLOT);
            for (uint32_t x = 1024u + 16u * t; x < sp; x += 1024u)
                reinterpret_cast<u32x4 *>(slot)[x >> 4] = ld16<0>(rs, x);
        }
        if (cw & kCtlSlow)
        {
            // rare: > 2 KB units or the chunk straddling the end of the stream
            // (a raw buffer load that crosses num_records returns 0)
            const uint32_t sp = rl(span, jj), av = rl(avail, jj);
            const uint64_t base = (static_cast<uint64_t>(rl(cbhi, jj)) << 32) | rl(cblo, jj);
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const void *>(base), av);
            const uint8_t * bp = reinterpret_cast<const uint8_t *>(base);
            for (uint32_t x = 16u * t; x < sp; x += 1024u)
                reinterpret_cast<u32x4 *>(slot)[x >> 4] = load16_guarded(bp, rs, x, av);
        }
        wave_lds_sync();
        return cw;
    }
};

using RunPlane = RunPlaneT<kSlotBytes>;

} // namespace tpf::dev
