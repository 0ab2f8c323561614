// p4_dsum64_lanes.h -- phase A of the chained 64-bit delta-1 decode with ONE
// LANE PER UNIT (round 4): the delta total sum(v + 1) mod 2^64 of a 128v64 /
// 256v64 D1 unit (applyDelta1 of p4D1Dec128v64, reference
// src/scalar/p4d1dec128v64_scalar.cpp:157-251; a 256v64 unit is two blocks,
// p4d1dec256v64_scalar.cpp:15-32) computed without decoding it -- the 64-bit
// counterpart of p4_dsum_lanes.h, whose digit-sum table and reasoning it
// reuses.
//
// A 128v64 block with b <= 32 stores its base payload in the 128v32 layout
// (bitpack128v64_scalar.cpp:38-104): 4 interleaved streams of 32 values (the
// pair swap permutes elements, which a sum does not see), so the per-stream-
// word SWAR sums of p4_dsum_lanes.h apply with 4 dwords per stream word; the
// partial sums are carried in 64 bits (128 values of up to 32 bits).
// Exceptions add (sum of exceptions) << b mod 2^64.  The lane path takes
// constant blocks, plain / bitmap / vbyte blocks with b <= 32, bitmap
// exceptions up to 64 bits, raw and compressed vbyte64 exceptions whose
// positions strictly increase and stay below 128; it declines a unit whose
// parse does not use exactly its offsets' bytes.  Every declined unit is
// decoded exactly by the wave decoder (decode_block128v64 + sum): horizontal
// 64-bit payloads (b > 32), repeated positions (the reference ORs them), and
// malformed blocks, whose length error it reports like the plain decode.
#pragma once

#include "p4_dsum_lanes.h"
#include "p4_generic.h"

namespace tpf::dev
{

// Base payload sum of one lane's 128v32-layout block (4 streams of b dwords)
// at LDS byte pay, 64-bit exact; P pre levels, L levels (as base_sum_lanes).
template <uint32_t P, uint32_t L, uint32_t LIM>
__device__ __forceinline__ uint64_t base_sum4_lanes(const uint32_t * w, uint32_t pay, uint32_t b, bool on, uint32_t bmax,
                                                    const uint32_t * row)
{
    const uint32_t meta = row[15];
    const uint32_t c32 = meta & 0xFFu, pre = (meta >> 12) & 15u, T = meta >> 16;
    uint32_t PA[P > 0 ? P : 1], PB[P > 0 ? P : 1], QA[L > 0 ? L : 1], QB[L > 0 ? L : 1], W[L > 0 ? L : 1];
#pragma unroll
    for (uint32_t l = 0; l < L; ++l)
    {
        const uint32_t a = row[l], bb = row[5 + l];
        W[l] = row[10 + l];
        if (l < P)
        {
            PA[l] = l < pre ? a : 0xFFFFFFFFu;
            PB[l] = l < pre ? bb : 0u;
        }
        QA[l] = l >= pre ? a : 0xFFFFFFFFu;
        QB[l] = l >= pre ? bb : 0u;
    }
    const uint32_t m = pay & 3u;
    uint32_t q = min(pay, LIM) >> 2;
    uint32_t phi = 0u;
    uint64_t bs = 0ull;
    for (uint32_t k = 0; k < bmax; ++k)
    {
        const uint32_t s = phi ? b - phi : 0u;
        uint32_t d[5];
#pragma unroll
        for (uint32_t l = 0; l < 5u; ++l)
            d[l] = w[q + l];
        // the 4 folded dwords summed in 64 bits (base_sum_lanes, round 5)
        uint64_t firsts = 0ull, acc = 0ull;
#pragma unroll
        for (uint32_t l = 0; l < 4u; ++l)
        {
            const uint32_t x = __builtin_amdgcn_alignbyte(d[l + 1], d[l], m);
            firsts += __builtin_amdgcn_ubfe(x, 0u, s);
            uint32_t z = x >> s;
#pragma unroll
            for (uint32_t lv = 0; lv < P; ++lv)
                z = (z & PA[lv]) + ((z >> W[lv]) & PB[lv]);
            acc += z;
        }
        uint32_t lo = __builtin_amdgcn_ubfe(static_cast<uint32_t>(acc), 0u, T);
        const uint64_t hi = acc >> T;
#pragma unroll
        for (uint32_t lv = (P < 1u ? P : 1u); lv < L; ++lv)
            lo = (lo & QA[lv]) + ((lo >> W[lv]) & QB[lv]);
        bs += on && k < b ? (firsts << phi) + lo + hi : 0ull;
        q = min(q + 4u, LIM / 4u);
        phi += c32;
        phi = phi >= b ? phi - b : phi;
    }
    return bs;
}

// vbGet64Inline's value (p4_scalar_internal.h:638-670) from its marker m and
// the 8 bytes after it, D
__device__ __forceinline__ uint64_t vb64_value(uint32_t m, uint64_t D)
{
    const uint32_t d = static_cast<uint32_t>(D);
    const uint32_t v2 = ((m - 0x98u) << 8) + (d & 0xFFu) + 152u;
    const uint32_t v3 = (d & 0xFFFFu) + ((m - 0xD8u) << 16) + 16536u;
    const uint32_t nb = m - 0xF8u + 3u; // m >= 0xF8: 3..8 value bytes
    const uint64_t vl = nb >= 8u ? D : (D & ((1ull << (8u * (nb & 7u))) - 1ull));
    return m < 0x98u ? m : m < 0xD8u ? v2 : m < 0xF8u ? v3 : vl;
}

// Sum of one lane's 128v64 block at LDS byte p (act: the lane has a block
// there).  Returns the block's byte length (wild for declined lanes); ok is
// cleared when the lane path does not take the block.
template <uint32_t LIM>
__device__ __forceinline__ uint32_t dsum_block128v64_lanes(const uint32_t * w, uint32_t p, bool act, const uint32_t * tab, bool & ok,
                                                          uint64_t & sum)
{
    const uint32_t hw = wu32<LIM>(w, p);
    const uint32_t h = hw & 0xFFu, x1 = (hw >> 8) & 0xFFu;
    const bool is_const = (h & 0xC0u) == 0xC0u;
    const bool is_vb = (h & 0xC0u) == 0x40u;
    const bool is_pb = (h & 0x40u) == 0u;
    const bool is_bm = is_pb && (h & 0x80u) != 0u;
    const uint32_t braw = is_pb ? (h & 0x7Fu) : (h & 0x3Fu);
    const uint32_t b = braw == 63u ? 64u : braw;
    ok = ok && act && (is_const || b <= 32u) && !(is_bm && (x1 == 0u || x1 > 64u));
    uint64_t exsum = 0ull;
    uint32_t len = 1u, pay = p + 1u;

    // constant block: ceil(b/8) value bytes; 128 * (c + 1)
    const uint64_t cv = lds_u64(w, min(p + 1u, LIM)) & mask64d(b);

    // bitmap: [0x80|b][bx][bitmap 16 B][xn * bx bits horizontal][base]
    if (__ballot(ok && is_bm) != 0ull)
    {
        uint32_t pc = 0u;
#pragma unroll
        for (uint32_t i = 0; i < 4u; ++i)
            pc += __builtin_popcount(wu32<LIM>(w, p + 2u + 4u * i));
        const uint32_t bx = min(x1, 64u);
        const uint32_t xbytes = (pc * bx + 7u) >> 3;
        const bool on = ok && is_bm;
        const uint32_t kmax = uni(wave_max_u32(on ? pc : 0u));
        const uint32_t xs = (p + 18u) * 8u;
        if (__ballot(on && bx > 32u) == 0ull)
        {
            // every lane's exceptions fit 32 bits (round 6; the C3-as-u64 list:
            // bx <= 12): one funnel read per exception -- lds_bits64's per-lane
            // width tests cost two exec-mask sections per exception
            for (uint32_t k = 0; k < kmax; ++k)
            {
                const uint32_t v = lds_bits(w, min(xs + k * bx, LIM * 8u), bx);
                exsum += on && k < pc ? v : 0u;
            }
        }
        else
        {
            for (uint32_t k = 0; k < kmax; ++k)
            {
                const uint64_t v = lds_bits64(w, min(xs + k * bx, LIM * 8u), bx);
                exsum += on && k < pc ? v : 0ull;
            }
        }
        len = is_bm ? 18u + xbytes + 16u * b : len;
        pay = is_bm ? p + 18u + xbytes : pay;
    }
    len = (is_pb && !is_bm) ? 1u + 16u * b : len;
    len = is_const ? 1u + ((b + 7u) >> 3) : len;

    // vbyte: [0x40|b][xn][base 16b][V][xn positions]; raw escape 0xFF + 8 xn LE words
    const uint32_t xn = is_vb ? x1 : 0u;
    ok = ok && (!is_vb || (xn != 0u && xn < 128u));
    const uint32_t v0 = p + 2u + 16u * b;
    const bool raw = is_vb && wbyte<LIM>(w, v0) == 0xFFu;
    const bool comp = is_vb && !raw;
    uint32_t vend = v0 + 1u + 8u * xn;
    if (__ballot(ok && raw) != 0ull)
    {
        const bool on = ok && raw;
        const uint32_t kmax = uni(wave_max_u32(on ? xn : 0u));
        for (uint32_t k = 0; k < kmax; ++k)
        {
            const uint64_t v = lds_u64(w, min(v0 + 1u + 8u * k, LIM));
            exsum += on && k < xn ? v : 0ull;
        }
    }
    if (__ballot(ok && comp) != 0ull)
    {
        // the lane's own marker walk (vbGet64Inline, p4_scalar_internal.h:638-670),
        // two values per step (round 6; the 32-bit phase A's general walk): 24
        // bytes from 6 aligned dwords, realigned to a[0..4] = bytes c..c+19;
        // value 1 at offset 0, value 2 at value 1's length when that is <= 4
        // (its 9 bytes then lie in a[0..4]; a longer first value takes the
        // step alone).  One value per step cost 0.33 ms of the 1.45 ms phase A
        // on the C3 64-bit list (r6h ablation).
        const bool on = ok && comp;
        uint32_t c = v0, k = 0u;
        while (__ballot(on && k < xn) != 0ull)
        {
            const uint32_t cc = min(c, LIM);
            const uint32_t q = cc >> 2, m = cc & 3u;
            uint32_t d[6], a[5];
#pragma unroll
            for (uint32_t u = 0; u < 6u; ++u)
                d[u] = w[q + u];
#pragma unroll
            for (uint32_t u = 0; u < 5u; ++u)
                a[u] = __builtin_amdgcn_alignbyte(d[u + 1], d[u], m);
            const bool s1 = on && k < xn;
            const uint32_t by1 = a[0] & 0xFFu;
            const uint32_t l1 = vbyte_len<true>(by1);
            const uint64_t D1 = (static_cast<uint64_t>(__builtin_amdgcn_alignbyte(a[2], a[1], 1u)) << 32) |
                                __builtin_amdgcn_alignbyte(a[1], a[0], 1u);
            exsum += s1 ? vb64_value(by1, D1) : 0ull;
            const bool hi1 = l1 >= 4u;
            const uint32_t x0 = hi1 ? a[1] : a[0], x1 = hi1 ? a[2] : a[1], x2 = hi1 ? a[3] : a[2], x3 = hi1 ? a[4] : a[3];
            const uint32_t r = l1 & 3u;
            const uint32_t xw = __builtin_amdgcn_alignbyte(x1, x0, r), yw = __builtin_amdgcn_alignbyte(x2, x1, r),
                           zw = __builtin_amdgcn_alignbyte(x3, x2, r);
            const uint32_t by2 = xw & 0xFFu;
            const uint64_t D2 = (static_cast<uint64_t>(__builtin_amdgcn_alignbyte(zw, yw, 1u)) << 32) | __builtin_amdgcn_alignbyte(yw, xw, 1u);
            const bool s2v = s1 && k + 1u < xn && l1 <= 4u;
            exsum += s2v ? vb64_value(by2, D2) : 0ull;
            c += s1 ? l1 + (s2v ? vbyte_len<true>(by2) : 0u) : 0u;
            k += s1 ? (s2v ? 2u : 1u) : 0u;
        }
        vend = comp ? c : vend;
    }
    pay = is_vb ? p + 2u : pay;
    // positions: strictly increasing (the reference ORs repeated ones) and < 128
    if (__ballot(ok && is_vb) != 0ull)
    {
        // 16 positions per step from 5 aligned dwords (round 6, as the 32-bit
        // phase A; one LDS byte read per position before)
        const bool on = ok && is_vb;
        const uint32_t kmax = uni(wave_max_u32(on ? xn : 0u));
        const uint32_t m = vend & 3u;
        uint32_t prev = 0u;
        bool inc = true;
        for (uint32_t k0 = 0; k0 < kmax; k0 += 16u)
        {
            const uint32_t q = min(vend + k0, LIM) >> 2;
            uint32_t d[5];
#pragma unroll
            for (uint32_t u = 0; u < 5u; ++u)
                d[u] = w[q + u];
#pragma unroll
            for (uint32_t u = 0; u < 16u; ++u)
            {
                const uint32_t a = __builtin_amdgcn_alignbyte(d[(u >> 2) + 1], d[u >> 2], m);
                const uint32_t pos = __builtin_amdgcn_ubfe(a, 8u * (u & 3u), 8u) + 1u; // 1..256: the first compares against 0
                inc = inc && (!(on && k0 + u < xn) || (pos > prev && pos <= 128u));
                prev = pos;
            }
        }
        ok = ok && (!is_vb || inc);
        len = is_vb ? vend + xn - p : len;
    }

    // base payload (b <= 32: four streams of b dwords); the fold depth per wave as in dsum_lanes
    const bool on = ok && !is_const && b != 0u;
    const uint32_t bmax = uni(wave_max_u32(on ? b : 0u));
    const uint32_t lmax = uni(wave_max_u32(on ? sum_levels(tab, b) : 0u));
    const uint32_t pmax = uni(wave_max_u32(on ? sum_pre(tab, b) : 0u));
    uint64_t bs = 0ull;
    if (bmax != 0u)
    {
        const uint32_t * row = tab + (on ? b : 0u) * kSumTabRow;
        const uint32_t key = pmax * 8u + lmax;
        if (key == 1u * 8u + 3u)
            bs = base_sum4_lanes<1, 3, LIM>(w, pay, b, on, bmax, row);
        else if (key == 1u * 8u + 2u)
            bs = base_sum4_lanes<1, 2, LIM>(w, pay, b, on, bmax, row);
        else if (key == 1u * 8u + 1u)
            bs = base_sum4_lanes<1, 1, LIM>(w, pay, b, on, bmax, row);
        else if (key == 2u * 8u + 4u)
            bs = base_sum4_lanes<2, 4, LIM>(w, pay, b, on, bmax, row);
        else if (key == 3u * 8u + 5u)
            bs = base_sum4_lanes<3, 5, LIM>(w, pay, b, on, bmax, row);
        else
            bs = base_sum4_lanes<0, 0, LIM>(w, pay, b, on, bmax, row); // every lane b = 32
    }
    sum = is_const ? 128ull * (cv + 1ull) : bs + 128ull + shl64(exsum, b);
    return len;
}

// Delta total of one lane's unit of NB 128v64 blocks at LDS byte p whose
// offsets give len bytes; false: the lane path declines the unit.
template <uint32_t NB, uint32_t LIM>
__device__ __forceinline__ bool dsum64_lanes(const uint32_t * w, uint32_t p, uint32_t len, bool act, const uint32_t * tab, uint64_t & sum)
{
    bool ok = act;
    uint64_t total = 0ull;
    uint32_t pos = p;
#pragma unroll
    for (uint32_t u = 0; u < NB; ++u)
    {
        uint64_t s = 0ull;
        const uint32_t l = dsum_block128v64_lanes<LIM>(w, min(pos, LIM), act, tab, ok, s);
        total += s;
        pos += l;
    }
    sum = total;
    return ok && pos - p == len;
}

} // namespace tpf::dev
