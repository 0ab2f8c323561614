// p4_enc32.h -- wave-level pieces of the 32-bit P4 encoder (one block per
// wave, lane t owns values 4t..4t+3).
//
// Restates for the GPU:
//   p4Bits32     src/scalar/p4_scalar_internal.cpp:270-387 (cost model)
//   writeHeader  src/scalar/p4_scalar_internal.cpp:409-429
//   p4Enc256v32  src/scalar/p4enc256v32_scalar.cpp:49-235 (payloads)
//   vbEnc32      src/scalar/p4_scalar_internal.cpp:47-89, :163-197
//   deltaEnc1    src/scalar/p4_scalar_internal.h:711-719
//
// The reference walks base widths b = max-1 .. 0 serially, carrying the
// exception count and a vbyte-size accumulator.  Both have closed forms:
//   ec(b)    = sum_{c>b} cnt[c]
//   vbsum(b) = sum_{c>b} (cnt[c] + cnt[c+7] + 2cnt[c+15] + 3cnt[c+19] + 4cnt[c+25])
// so lane b evaluates candidate b in parallel (suffix sums by wave scan) and
// one wave min-reduction picks the first minimum in the reference's order
// (plain first, then descending b; patching preferred over vbyte on ties).
#pragma once

#include "tpf_device.h"

namespace tpf::dev
{

struct Plan32
{
    uint32_t b;    // base bit width
    uint32_t bx;   // 0 plain, 1..32 bitmap patch bits, 33 vbyte, 34 constant
    uint32_t size; // exact encoded byte size
    uint32_t xn;   // exception count
    uint32_t raw;  // vbyte: 1 if the 0xFF raw escape is used
};

__device__ __forceinline__ uint32_t bw32(uint32_t x) { return x ? 32u - __builtin_clz(x) : 0u; }

// vbPut32 byte length (p4_scalar_internal.cpp:47-89)
__device__ __forceinline__ uint32_t vblen32(uint32_t x)
{
    return x < 156u ? 1u : x < 16540u ? 2u : x < 2113692u ? 3u : x <= 0xFFFFFFu ? 4u : 5u;
}

// hist: per-wave LDS scratch of >= 64 u32.
__device__ __forceinline__ Plan32 plan_block256(const u32x4 & v, uint32_t * hist, uint32_t t)
{
    Plan32 P;
    const uint32_t orv = uni(wave_or(v.x | v.y | v.z | v.w));
    if (orv == 0u)
    {
        P.b = 0;
        P.bx = 0;
        P.size = 1;
        P.xn = 0;
        P.raw = 0;
        return P;
    }
    const uint32_t maxb = bw32(orv);
    const uint32_t first = __builtin_amdgcn_readlane(v.x, 0);
    const uint32_t eqc = wave_sum((v.x == first) + (v.y == first) + (v.z == first) + (v.w == first));
    if (eqc == 256u)
    {
        P.b = maxb;
        P.bx = 34;
        P.size = 1u + ((maxb + 7u) >> 3);
        P.xn = 0;
        P.raw = 0;
        return P;
    }
    hist[t] = 0u;
    wave_lds_sync();
    atomicAdd(&hist[bw32(v.x)], 1u);
    atomicAdd(&hist[bw32(v.y)], 1u);
    atomicAdd(&hist[bw32(v.z)], 1u);
    atomicAdd(&hist[bw32(v.w)], 1u);
    wave_lds_sync();
    const uint32_t cnt = hist[t]; // lane c holds cnt[c] (0 for c > 32)
    auto at = [&](uint32_t c) -> uint32_t {
        uint32_t x = static_cast<uint32_t>(__shfl(static_cast<int>(cnt), static_cast<int>(c & 63u), 64));
        return c < 64u ? x : 0u;
    };
    const uint32_t vbacc = at(t + 7u) + 2u * at(t + 15u) + 3u * at(t + 19u) + 4u * at(t + 25u);
    const uint32_t a = cnt, bsum = cnt + vbacc;
    const uint32_t pa = wave_incl_scan(a), pb = wave_incl_scan(bsum);
    const uint32_t ta = __builtin_amdgcn_readlane(pa, 63), tb = __builtin_amdgcn_readlane(pb, 63);
    const uint32_t ec = ta - pa;    // sum_{c > t} cnt[c]
    const uint32_t vbsum = tb - pb; // sum_{c > t} (cnt[c] + vbacc[c])
    uint32_t key = 0xFFFFFFFFu;
    if (t < maxb)
    {
        const uint32_t vsz = 32u * t + 2u + ec + vbsum;
        const uint32_t psz = 32u * t + 2u + 32u + ((ec * (maxb - t) + 7u) >> 3);
        const uint32_t cost = psz <= vsz ? psz : vsz;
        const uint32_t kind = psz <= vsz ? 0u : 1u;
        key = (cost << 8) | ((maxb - t) << 1) | kind;
    }
    else if (t == maxb)
    {
        key = ((32u * maxb + 1u) << 8); // plain: order 0
    }
    key = uni(wave_min(key));
    const uint32_t order = (key >> 1) & 127u;
    const uint32_t kind = key & 1u;
    P.b = maxb - order;
    if (order == 0u)
    {
        P.bx = 0;
        P.size = 1u + 32u * maxb;
        P.xn = 0;
        P.raw = 0;
        return P;
    }
    const uint32_t b = P.b;
    const uint32_t m = mask32(b);
    const uint32_t xn = wave_sum((v.x > m) + (v.y > m) + (v.z > m) + (v.w > m));
    P.xn = xn;
    if (kind == 0u)
    {
        P.bx = maxb - b;
        P.size = 34u + ((xn * P.bx + 7u) >> 3) + 32u * b;
        P.raw = 0;
    }
    else
    {
        P.bx = 33;
        const uint32_t sl = (v.x > m ? vblen32(v.x >> b) : 0u) + (v.y > m ? vblen32(v.y >> b) : 0u)
            + (v.z > m ? vblen32(v.z >> b) : 0u) + (v.w > m ? vblen32(v.w >> b) : 0u);
        const uint32_t sumlen = wave_sum(sl);
        P.raw = (sumlen + 32u > 4u * xn) ? 1u : 0u;
        const uint32_t vsize = P.raw ? 1u + 4u * xn : sumlen;
        P.size = 2u + 32u * b + vsize + xn;
    }
    return P;
}

// OR nb (<= 32) bits of val (already < 2^nb) at bit position bp of an LDS image.
__device__ __forceinline__ void or_bits(uint32_t * img, uint32_t bp, uint32_t val, uint32_t nb)
{
    if (nb == 0u || val == 0u)
        return;
    const uint32_t q = bp >> 5, sh = bp & 31u;
    atomicOr(&img[q], val << sh);
    if (sh + nb > 32u)
        atomicOr(&img[q + 1], val >> (32u - sh));
}

// Scatter the 4 values of lane t into the 256v32 base layout at byte p.
__device__ __forceinline__ void pack256v32_lane(uint32_t * img, uint32_t p, uint32_t b, uint32_t t, const u32x4 & v)
{
    if (b == 0u)
        return;
    const uint32_t m = mask32(b);
    const uint32_t g = t >> 1;
    const uint32_t o = g * b;
    const uint32_t k = o >> 5, sh = o & 31u;
    const uint32_t lane0 = 4u * (t & 1u);
    const uint32_t vals[4] = {v.x & m, v.y & m, v.z & m, v.w & m};
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
    {
        const uint32_t l = lane0 + j;
        const uint32_t lo_byte = p + 32u * k + 4u * l;
        const uint32_t x = vals[j];
        const uint32_t lo_bits = min(b, 32u - sh);
        or_bits(img, lo_byte * 8u + sh, x & mask32(lo_bits), lo_bits);
        if (b > lo_bits)
            or_bits(img, (lo_byte + 32u) * 8u, x >> lo_bits, b - lo_bits);
    }
}

// Build the encoded block in the LDS image (zeroed, image byte 0 == block
// byte 0 shifted by `phase` bytes).  Returns nothing; size is P.size.
__device__ __forceinline__ void emit_block256(uint32_t * img, uint32_t phase, const Plan32 & P, const u32x4 & v, uint32_t t)
{
    const uint32_t b = P.b;
    const uint32_t s = phase; // byte position of the header in the image
    if (P.bx == 0u)
    {
        if (t == 0)
            or_bits(img, s * 8u, b, 8);
        pack256v32_lane(img, s + 1u, b, t, v);
        return;
    }
    if (P.bx == 34u)
    {
        // constant block (p4enc256v32_scalar.cpp:183-190): ceil(b/8) value bytes
        if (t == 0)
        {
            or_bits(img, s * 8u, 0xC0u | b, 8);
            or_bits(img, (s + 1u) * 8u, v.x & mask32(b), b);
        }
        return;
    }
    const uint32_t m = mask32(b);
    const uint32_t f0 = v.x > m, f1 = v.y > m, f2 = v.z > m, f3 = v.w > m;
    const uint32_t my = f0 | (f1 << 1) | (f2 << 2) | (f3 << 3);
    const uint32_t cnt = f0 + f1 + f2 + f3;
    const uint32_t incl = wave_incl_scan(cnt);
    const uint32_t before = incl - cnt; // exceptions in elements < 4t
    const u32x4 base = u32x4{v.x & m, v.y & m, v.z & m, v.w & m};
    const uint32_t ex[4] = {v.x >> (b & 31u), v.y >> (b & 31u), v.z >> (b & 31u), v.w >> (b & 31u)};
    if (P.bx <= 32u)
    {
        // [0x80|b][bx][bitmap 32B][xn*bx bits horizontal][256v32 base]
        if (t == 0)
        {
            or_bits(img, s * 8u, 0x80u | b, 8);
            or_bits(img, (s + 1u) * 8u, P.bx, 8);
        }
        or_bits(img, (s + 2u) * 8u + 4u * t, my, 4);
        const uint32_t xs = (s + 34u) * 8u;
        uint32_t k = before;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            if ((my >> j) & 1u)
            {
                or_bits(img, xs + k * P.bx, ex[j], P.bx);
                ++k;
            }
        pack256v32_lane(img, s + 34u + ((P.xn * P.bx + 7u) >> 3), b, t, base);
        return;
    }
    // vbyte: [0x40|b][xn][256v32 base][V][positions]
    if (t == 0)
    {
        or_bits(img, s * 8u, 0x40u | b, 8);
        or_bits(img, (s + 1u) * 8u, P.xn, 8);
    }
    pack256v32_lane(img, s + 2u, b, t, base);
    const uint32_t v0 = s + 2u + 32u * b;
    if (P.raw)
    {
        if (t == 0)
            or_bits(img, v0 * 8u, 0xFFu, 8);
        uint32_t k = before;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            if ((my >> j) & 1u)
            {
                or_bits(img, (v0 + 1u + 4u * k) * 8u, ex[j], 32);
                or_bits(img, (v0 + 1u + 4u * P.xn + k) * 8u, 4u * t + j, 8);
                ++k;
            }
        return;
    }
    uint32_t len[4];
    uint32_t mylen = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
    {
        len[j] = ((my >> j) & 1u) ? vblen32(ex[j]) : 0u;
        mylen += len[j];
    }
    const uint32_t lincl = wave_incl_scan(mylen);
    const uint32_t vtotal = __builtin_amdgcn_readlane(lincl, 63);
    uint32_t pos = v0 + lincl - mylen;
    uint32_t k = before;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
    {
        if (!((my >> j) & 1u))
            continue;
        const uint32_t x = ex[j];
        const uint32_t bp = pos * 8u;
        if (x < 156u)
            or_bits(img, bp, x, 8);
        else if (x < 16540u)
        {
            const uint32_t d = x - 156u;
            or_bits(img, bp, (0x9Cu + (d >> 8)) | ((d & 0xFFu) << 8), 16);
        }
        else if (x < 2113692u)
        {
            const uint32_t d = x - 16540u;
            or_bits(img, bp, (0xDCu + (d >> 16)) | ((d & 0xFFFFu) << 8), 24);
        }
        else if (x <= 0xFFFFFFu)
            or_bits(img, bp, 0xFCu | (x << 8), 32);
        else
        {
            or_bits(img, bp, 0xFDu, 8);
            or_bits(img, bp + 8u, x, 32);
        }
        or_bits(img, (v0 + vtotal + k) * 8u, 4u * t + j, 8);
        pos += len[j];
        ++k;
    }
}

} // namespace tpf::dev
