// p4_block32.h -- wave-level decode of one 32-bit P4 block staged in LDS.
//
// Restates, for the GPU, the per-block decoders of the reference:
//   p4Dec256v32   src/scalar/p4dec256v32_scalar.cpp:90-137   (modes below)
//   p4D1Dec256v32 src/scalar/p4d1dec256v32_scalar.cpp:198-268
//   p4Dec128v32   src/scalar/p4dec128v32_scalar.cpp          (L = 4 lanes)
// Header byte h: (h&0xC0)==0xC0 constant; (h&0x40)==0 plain / bitmap patch
// (h&0x80 plus bx byte); else vbyte exceptions (xn byte).
//
// Work split inside the wave: lane t owns the four consecutive values
// 4t..4t+3 of a 256-value block, i.e. lanes 4(t&1)..4(t&1)+3 of interleave
// group g = t>>1.  The four values share one lane-bit offset g*b, so the lane
// reads the 16-byte word group k = g*b/32 and k+1 (5 aligned dwords each,
// realigned with v_alignbyte) and funnel-shifts with v_alignbit.
#pragma once

#include "tpf_device.h"

namespace tpf::dev
{

// Scratch per wave: 256 u32 exception values by position + 256 u32 temp.
constexpr uint32_t kWaveScratchU32 = 512;

// Unpack 4 values of lane t from the 256v32 (L=8) base layout at byte p.
__device__ __forceinline__ u32x4 unpack256v32_lane(const uint32_t * lds, uint32_t p, uint32_t b, uint32_t t)
{
    const uint32_t g = t >> 1;
    const uint32_t o = g * b;
    const uint32_t pos = p + 32u * (o >> 5) + 16u * (t & 1u);
    const uint32_t sh = o & 31u;
    const uint32_t m = p & 3u;
    const uint32_t q = pos >> 2;
    const uint32_t d0 = lds[q], d1 = lds[q + 1], d2 = lds[q + 2], d3 = lds[q + 3], d4 = lds[q + 4];
    const uint32_t e0 = lds[q + 8], e1 = lds[q + 9], e2 = lds[q + 10], e3 = lds[q + 11], e4 = lds[q + 12];
    const uint32_t msk = mask32(b);
    u32x4 v;
    v.x = __builtin_amdgcn_alignbit(__builtin_amdgcn_alignbyte(e1, e0, m), __builtin_amdgcn_alignbyte(d1, d0, m), sh) & msk;
    v.y = __builtin_amdgcn_alignbit(__builtin_amdgcn_alignbyte(e2, e1, m), __builtin_amdgcn_alignbyte(d2, d1, m), sh) & msk;
    v.z = __builtin_amdgcn_alignbit(__builtin_amdgcn_alignbyte(e3, e2, m), __builtin_amdgcn_alignbyte(d3, d2, m), sh) & msk;
    v.w = __builtin_amdgcn_alignbit(__builtin_amdgcn_alignbyte(e4, e3, m), __builtin_amdgcn_alignbyte(d4, d3, m), sh) & msk;
    return v;
}

__device__ __forceinline__ uint32_t comp(const u32x4 & v, uint32_t j)
{
    return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}

__device__ __forceinline__ void or_comp(u32x4 & v, uint32_t j, uint32_t x)
{
    if (j == 0)
        v.x |= x;
    else if (j == 1)
        v.y |= x;
    else if (j == 2)
        v.z |= x;
    else
        v.w |= x;
}

// Bitmap-patch exceptions (p4Dec256PayloadBitmap, p4dec256v32_scalar.cpp:10-66):
// 32-byte bitmap at bm_pos, then the xn exception high parts as ONE horizontal
// LSB-first bx-bit stream (bitunpack32Scalar), then the base payload.  Lane t
// owns values 4t..4t+3, i.e. bits 4(t&7)..4(t&7)+3 of bitmap dword t>>3: it
// reads that one dword, and its rank among the exceptions is the popcount of
// the dwords before (one wave scan) plus the bits below its own.  This
// replaces the serial ctz loop of the reference.
struct BitmapInfo
{
    uint32_t my;     // this lane's 4 bitmap bits
    uint32_t before; // exceptions at positions < 4t
    uint32_t xn;     // total (wave-uniform)
};

__device__ __forceinline__ BitmapInfo read_bitmap256(uint32_t w, uint32_t t)
{
    BitmapInfo bi;
    const uint32_t sh = 4u * (t & 7u);
    bi.my = (w >> sh) & 0xFu;
    const uint32_t pcd = __builtin_popcount(w);
    const uint32_t incl = wave_incl_scan((t & 7u) == 0u ? pcd : 0u);
    bi.before = incl - pcd + __builtin_popcount(w & ((1u << sh) - 1u));
    bi.xn = uni(__builtin_amdgcn_readlane(incl, 63));
    return bi;
}

__device__ __forceinline__ void patch_bitmap256(const uint32_t * lds, const BitmapInfo & bi, uint32_t xs, uint32_t bx,
                                                uint32_t b, uint32_t t, u32x4 & v)
{
    // Branch-free: with ~10% exceptions every one of the four bit positions is
    // set in some lane of almost every block, so per-bit `if`s would execute
    // anyway and only add exec-mask (SALU) work.  A lane without the bit reads
    // a harmless in-slot word and masks it out.
    const uint32_t my = bi.my;
    const uint32_t bp = xs * 8u + bi.before * bx;
    const uint32_t r1 = my & 1u, r2 = __builtin_popcount(my & 3u), r3 = __builtin_popcount(my & 7u);
    const uint32_t e0 = lds_bits(lds, bp, bx), e1 = lds_bits(lds, bp + r1 * bx, bx);
    const uint32_t e2 = lds_bits(lds, bp + r2 * bx, bx), e3 = lds_bits(lds, bp + r3 * bx, bx);
    v.x |= (my & 1u) ? shl32(e0, b) : 0u;
    v.y |= (my & 2u) ? shl32(e1, b) : 0u;
    v.z |= (my & 4u) ? shl32(e2, b) : 0u;
    v.w |= (my & 8u) ? shl32(e3, b) : 0u;
}

// ds_bpermute: value of x in lane `lane` (lane taken mod 64).
__device__ __forceinline__ uint32_t bperm(uint32_t x, uint32_t lane)
{
    return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(lane << 2), static_cast<int>(x)));
}

// Start positions of consecutive variable-length values inside a 64-byte
// window, without a serial walk.  nxt = t + len(byte t) is "the next start if
// t is one"; J_i = nxt applied 2^i times, stopping at the first position
// >= 64 (binary lifting, 5 ds_bpermute), then lane k composes the J_i of the
// bits of k starting from sp (6 ds_bpermute).  Returns p_k = position of the
// k-th value from sp (>= 64: beyond the window, the smallest such = end of the
// window's last value).
__device__ __forceinline__ uint32_t window_starts(uint32_t nxt, uint32_t sp, uint32_t t)
{
    uint32_t J[6];
    J[0] = nxt;
#pragma unroll
    for (int i = 1; i < 6; ++i)
    {
        const uint32_t x = J[i - 1];
        const uint32_t r = bperm(J[i - 1], x);
        J[i] = x >= 64u ? x : r;
    }
    uint32_t p = sp;
#pragma unroll
    for (int i = 0; i < 6; ++i)
    {
        const uint32_t r = bperm(J[i], p);
        const uint32_t q = p >= 64u ? p : r;
        p = ((t >> i) & 1u) ? q : p;
    }
    return p;
}

// vbyte exceptions (p4dec256v32_scalar.cpp:123-136; vbDec32 p4_scalar_internal.cpp:215-237,
// vbGet32Inline p4_scalar_internal.h:589-625).  V starts at v0: either
// 0xFF + 4*xn raw LE words, or xn vbytes whose lengths are decided by their
// marker byte.  The compressed stream is split in 64-byte windows: each lane
// classifies one byte, ballots give 64-bit length masks and a wave-uniform
// (SALU) chain walk finds the value starts; each start lane decodes its value.
// Exception values are OR-ed into scr[pos] (ds_or, so duplicate positions
// behave like the reference's sequential |=).  Returns the byte position just
// past the position list.
__device__ __forceinline__ uint32_t vbyte_exceptions(const uint32_t * lds, uint32_t v0, uint32_t xn, uint32_t * scr,
                                                     uint32_t t)
{
    uint32_t * tmp = scr + 256;
    reinterpret_cast<u32x4 *>(scr)[t] = u32x4{0u, 0u, 0u, 0u};
    wave_lds_sync();
    const uint32_t first = uni(lds_byte(lds, v0));
    uint32_t vend;
    if (first == 0xFFu)
    {
        const uint32_t pbase = v0 + 1u + 4u * xn;
        for (uint32_t k = t; k < xn; k += kWave)
        {
            const uint32_t val = lds_u32(lds, v0 + 1u + 4u * k);
            const uint32_t pos = lds_byte(lds, pbase + k);
            atomicOr(&scr[pos], val);
        }
        vend = pbase;
    }
    else
    {
        uint32_t c = v0, sp = 0, found = 0;
        vend = v0;
        while (found < xn)
        {
            const uint32_t by0 = lds_byte(lds, c + t);
            const uint32_t len0 = by0 < 0x9Cu ? 1u : by0 < 0xDCu ? 2u : by0 < 0xFCu ? 3u : by0 == 0xFCu ? 4u : 5u;
            const uint32_t p = window_starts(t + len0, sp, t);
            const uint32_t m = static_cast<uint32_t>(__builtin_popcountll(__ballot(p < 64u)));
            const uint32_t cnt = min(m, xn - found);
            // end of value k (exact, may pass 64).  The permute must run in
            // every lane: ds_bpermute reads 0 from a lane that is inactive.
            const uint32_t pn = bperm(t + len0, p);
            const uint32_t pe = p < 64u ? pn : p;
            if (t < cnt)
            {
                const uint32_t by = lds_byte(lds, c + p);
                const uint32_t d = lds_u32(lds, c + p + 1u);
                const uint32_t v2 = ((by - 0x9Cu) << 8) + (d & 0xFFu) + 156u;
                const uint32_t v3 = (d & 0xFFFFu) + ((by - 0xDCu) << 16) + 16540u;
                const uint32_t val = by < 0x9Cu ? by : by < 0xDCu ? v2 : by < 0xFCu ? v3 : by == 0xFCu ? (d & 0xFFFFFFu) : d;
                tmp[(found + t) & 255u] = val;
            }
            const uint32_t e_last = uni(__builtin_amdgcn_readlane(pe, cnt - 1u));
            found += cnt;
            vend = c + e_last;
            sp = e_last >= 64u ? e_last - 64u : e_last;
            c += e_last >= 64u ? 64u : 0u;
        }
        wave_lds_sync();
        for (uint32_t k = t; k < xn; k += kWave)
        {
            const uint32_t pos = lds_byte(lds, vend + k);
            atomicOr(&scr[pos], tmp[k]);
        }
    }
    wave_lds_sync();
    return vend + xn;
}

// Decode one 256v32 block at LDS byte s.  Returns consumed bytes (uniform).
// hw: the block's first 4 bytes (header byte, bx / xn byte), wave-uniform,
// taken by the caller from the load registers so the mode is known without
// an LDS round trip.  The lane's bitmap dword is read before the mode
// branch (a harmless in-slot read for other modes) so that a bitmap block
// needs one LDS round trip before its unpack instead of two.
__device__ __forceinline__ uint32_t decode_block256v32(const uint32_t * lds, uint32_t s, uint32_t hw, uint32_t * scr, uint32_t t,
                                                       u32x4 & v)
{
    const uint32_t wbm = lds_u32(lds, s + 2u + 4u * (t >> 3));
    const uint32_t h = hw & 0xFFu, x1 = (hw >> 8) & 0xFFu;
    if ((h & 0xC0u) == 0xC0u)
    {
        const uint32_t b = h & 0x3Fu;
        uint32_t c = lds_u32(lds, s + 1u);
        if (b < 32u)
            c &= mask32(b);
        v = u32x4{c, c, c, c};
        return 1u + ((b + 7u) >> 3);
    }
    if ((h & 0x40u) == 0u)
    {
        const uint32_t hdr = (h & 0x80u) ? 2u : 1u;
        const uint32_t bx = (h & 0x80u) ? min(x1, 32u) : 0u;
        const uint32_t b = min(h & 0x7Fu, 32u);
        const uint32_t bad = ((h & 0x7Fu) > 32u || ((h & 0x80u) && x1 > 32u)) ? kWidthBad : 0u;
        if (bx == 0u)
        {
            v = unpack256v32_lane(lds, s + hdr, b, t);
            return (hdr + 32u * b) | bad;
        }
        const BitmapInfo bi = read_bitmap256(wbm, t);
        const uint32_t xs = s + 34u;
        const uint32_t xbytes = (bi.xn * bx + 7u) >> 3;
        v = unpack256v32_lane(lds, xs + xbytes, b, t);
        patch_bitmap256(lds, bi, xs, bx, b, t, v);
        return (34u + xbytes + 32u * b) | bad;
    }
    const uint32_t b = min(h & 0x3Fu, 32u);
    const uint32_t bad = (h & 0x3Fu) > 32u ? kWidthBad : 0u;
    const uint32_t xn = x1;
    v = unpack256v32_lane(lds, s + 2u, b, t);
    const uint32_t end = vbyte_exceptions(lds, s + 2u + 32u * b, xn, scr, t);
    const u32x4 ex = reinterpret_cast<const u32x4 *>(scr)[t];
    v.x |= shl32(ex.x, b);
    v.y |= shl32(ex.y, b);
    v.z |= shl32(ex.z, b);
    v.w |= shl32(ex.w, b);
    return (end - s) | bad;
}

// Delta-1 (applyDelta1_256, p4d1dec256v32_scalar.cpp:39-50): inclusive scan
// of v[i]+1 seeded with start, mod 2^32.  Per lane serial over its 4 values,
// wave scan (DPP) over the 64 lane totals.  Returns the block's last value.
__device__ __forceinline__ uint32_t apply_delta1_256(u32x4 & v, uint32_t start)
{
    const uint32_t a0 = v.x + 1u;
    const uint32_t a1 = a0 + v.y + 1u;
    const uint32_t a2 = a1 + v.z + 1u;
    const uint32_t a3 = a2 + v.w + 1u;
    const uint32_t incl = wave_incl_scan(a3);
    const uint32_t base = start + incl - a3;
    v = u32x4{base + a0, base + a1, base + a2, base + a3};
    return start + __builtin_amdgcn_readlane(incl, 63);
}

} // namespace tpf::dev
