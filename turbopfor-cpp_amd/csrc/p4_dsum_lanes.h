// p4_dsum_lanes.h -- phase A of the chained delta-1 decode with ONE LANE PER
// BLOCK: the delta total of a 256v32 D1 block (the sum of v[i] + 1 over its
// 256 values, mod 2^32: applyDelta1_256, reference
// src/scalar/p4d1dec256v32_scalar.cpp:39-50) computed without decoding it.
//
// Why a lane per block (round 3): the wave-per-block phase A of rounds 1-2
// (stage the block in LDS, unpack 4 values per lane, wave sums) issued ~181
// wave-cycles per block -- header, staging, unpack and reductions paid once
// per 256 values -- and ran at 1.37 ms per 10M C3 blocks, compute-bound
// (DESIGN.md 4.3).  Here a wave stages the bytes of a 64-block run into LDS
// with coalesced 16-byte loads and then every lane parses its own block from
// LDS the way the reference's scalar decoder walks it, so one wave
// instruction advances 64 blocks.
//
// The block sum needs no unpacking: with b-bit values the base payload is 8
// interleaved streams of 32 values each (stream l = dwords 8k + l), and a
// payload dword of stream word k holds stream bits [32k, 32k + 32): its first
// s = (b - phi) mod b bits are the top of a value that started in word k-1
// (value bits phi.. with phi = 32k mod b), the rest are whole values from bit
// 0 (the last one possibly cut).  So
//     sum of a dword = (x & mask(s)) << phi  +  digit sum of (x >> s) in base 2^b
// and the digit sum is a SWAR fold: level l adds the upper half of every
// 2^(l+1)*b-bit slot to its lower half (masks per width from an LDS table).
// Exceptions add (sum of exceptions) << b (a shift left distributes mod 2^32).
//
// Exactness: the fast path mirrors the decoder's parse (p4_block32.h
// decode_block256v32, the same clamps of b and bx) and takes a block only if
// its parse consumes exactly its offsets' bytes and, for vbyte exceptions,
// its positions strictly increase.  Every other block -- duplicate positions
// (the reference ORs them: p4d1dec256v32_scalar.cpp:260), a length that
// disagrees with the offsets, a block larger than the staging window --
// goes to the wave decoder (decode_block256v32 + wave sum), which is exact
// by construction and reports length errors exactly as the plain decode does.
#pragma once

#include "p4_dec_run.h"

namespace tpf::dev
{

#ifndef TPF_DSUM_RUN
#define TPF_DSUM_RUN 64
#endif
constexpr uint32_t kLaneRun = TPF_DSUM_RUN; // blocks per wave run: lane j = block first + j (16 | kLaneRun <= 64)

// Per-width row of the SWAR digit-sum table (b = 0..32, 16 dwords each):
// [0,5) keep masks A_l, [5,10) add masks B_l, [10,15) shifts w_l = b << l,
// [15] = (32 mod b) | (levels << 8).  Level l < levels: A_l = B_l = the low
// w_l bits of every 2*w_l-bit slot; levels beyond: A_l = ~0, B_l = 0 (no-op).
constexpr uint32_t kSumTabRow = 16;

__device__ __forceinline__ void build_sum_row(uint32_t * row, uint32_t b)
{
    uint32_t levels = 0;
    if (b >= 1u && b < 32u)
    {
        const uint32_t fields = (32u + b - 1u) / b;
        while ((1u << levels) < fields)
            ++levels;
    }
    for (uint32_t l = 0; l < 5u; ++l)
    {
        if (l < levels)
        {
            const uint32_t w = b << l;
            uint32_t a = 0u;
            for (uint32_t j = 0; j * 2u * w < 32u; ++j)
                a |= mask32(w) << (j * 2u * w);
            row[l] = a;
            row[5 + l] = a;
            row[10 + l] = w;
        }
        else
        {
            row[l] = 0xFFFFFFFFu;
            row[5 + l] = 0u;
            row[10 + l] = 0u;
        }
    }
    row[15] = (b ? 32u % b : 0u) | (levels << 8);
}

__device__ __forceinline__ uint32_t sum_levels(const uint32_t * tab, uint32_t b) { return tab[b * kSumTabRow + 15u] >> 8; }

// Byte / unaligned u32 at LDS byte position pos, the position clamped to the
// wave's window (lanes without a block, or a malformed header, compute wild
// positions; their results are discarded, their reads must stay in bounds).
template <uint32_t LIM>
__device__ __forceinline__ uint32_t wbyte(const uint32_t * w, uint32_t pos)
{
    return lds_byte(w, min(pos, LIM));
}
template <uint32_t LIM>
__device__ __forceinline__ uint32_t wu32(const uint32_t * w, uint32_t pos)
{
    return lds_u32(w, min(pos, LIM));
}

// SIMT form of the lane-serial block sum: every loop runs the wave's maximum
// trip count with per-lane predicated accumulation (v_cndmask), so the wave
// executes one instruction stream with no divergent branches -- divergent
// per-lane loops cost exec-mask bookkeeping on the CU-shared scalar unit on
// every iteration (measured: the first, branchy form of this kernel spent
// more time in SALU exec-mask code than in the sums).
//   w: the wave's LDS window (LIM = last readable byte position),
//   p: the block's byte position in it, len: its length by the offsets,
//   act: the lane has a block to sum.
// Returns ok (sum valid); lanes with !ok go to the wave decoder.
template <uint32_t LIM>
__device__ __forceinline__ bool dsum_lanes(const uint32_t * w, uint32_t p, uint32_t len, bool act, const uint32_t * tab, uint32_t & sum)
{
    const uint32_t hw = wu32<LIM>(w, p);
    const uint32_t h = hw & 0xFFu, x1 = (hw >> 8) & 0xFFu;
    const bool is_const = (h & 0xC0u) == 0xC0u;
    const bool is_vb = (h & 0xC0u) == 0x40u;
    const bool is_pb = (h & 0x40u) == 0u;
    const uint32_t bx = is_pb && (h & 0x80u) ? min(x1, 32u) : 0u;
    const bool is_bm = is_pb && bx != 0u;
    const uint32_t hdr = (h & 0x80u) ? 2u : 1u;
    uint32_t b = is_const ? 0u : is_vb ? min(h & 0x3Fu, 32u) : min(h & 0x7Fu, 32u);
    bool ok = act;
    uint32_t exsum = 0u, xn = is_vb ? x1 : 0u, pay = p + hdr;

    // constant block (p4d1dec256v32_scalar.cpp:212-229): 256 * (c + 1)
    const uint32_t cb = h & 0x3Fu;
    const uint32_t cv = wu32<LIM>(w, p + 1u) & (cb < 32u ? mask32(cb) : 0xFFFFFFFFu);
    const bool const_ok = 1u + ((cb + 7u) >> 3) == len;

    // bitmap exceptions (p4Dec256PayloadBitmap, p4dec256v32_scalar.cpp:10-66):
    // xn = popcount of the 32-byte bitmap, the exceptions ONE horizontal
    // LSB-first bx-bit stream after it
    if (__ballot(ok && is_bm) != 0ull)
    {
        uint32_t pc = 0u;
#pragma unroll
        for (uint32_t i = 0; i < 8u; ++i)
            pc += __builtin_popcount(wu32<LIM>(w, p + 2u + 4u * i));
        const uint32_t xbytes = (pc * bx + 7u) >> 3;
        xn = is_bm ? pc : xn;
        pay = is_bm ? p + 34u + xbytes : pay;
        ok = ok && (!is_bm || 34u + xbytes + 32u * b == len);
        const bool on = ok && is_bm;
        const uint32_t kmax = uni(wave_max_u32(on ? pc : 0u));
        const uint32_t xs = (p + 34u) * 8u;
        for (uint32_t k = 0; k < kmax; ++k)
        {
            const uint32_t bp = min(xs + k * bx, LIM * 8u);
            const uint32_t v = lds_bits(w, bp, bx);
            exsum += on && k < pc ? v : 0u;
        }
    }
    ok = ok && (!is_pb || is_bm || hdr + 32u * b == len);
    ok = ok && (!is_const || const_ok);

    // vbyte exceptions (p4dec256v32_scalar.cpp:123-136, vbDec32
    // p4_scalar_internal.cpp:215-237): raw escape 0xFF + 4*xn LE words, or
    // xn vbytes; then the xn position bytes
    ok = ok && (!is_vb || xn != 0u); // never emitted; its length depends on a byte past the payload
    const uint32_t v0 = p + 2u + 32u * b;
    const bool raw = is_vb && wbyte<LIM>(w, v0) == 0xFFu;
    const bool comp = is_vb && !raw;
    uint32_t vend = v0 + 1u + 4u * xn;
    if (__ballot(ok && raw) != 0ull)
    {
        // 8 values per step from 9 aligned dwords: one LDS round trip per step
        ok = ok && (!raw || vend + xn - p == len);
        const bool on = ok && raw;
        const uint32_t kmax = uni(wave_max_u32(on ? xn : 0u));
        const uint32_t a0 = v0 + 1u;
        const uint32_t m = a0 & 3u;
        for (uint32_t k0 = 0; k0 < kmax; k0 += 8u)
        {
            const uint32_t q = min(a0 + 4u * k0, LIM) >> 2;
            uint32_t d[9];
#pragma unroll
            for (uint32_t u = 0; u < 9u; ++u)
                d[u] = w[q + u];
#pragma unroll
            for (uint32_t u = 0; u < 8u; ++u)
                exsum += on && k0 + u < xn ? __builtin_amdgcn_alignbyte(d[u + 1], d[u], m) : 0u;
        }
    }
    if (__ballot(ok && comp) != 0ull)
    {
        // The marker chain is serial; each step reads 24 bytes at c (7 aligned
        // dwords, realigned to a[0..5] = bytes c..c+23) and decodes up to four
        // values starting at window offsets <= 15 from registers, so an LDS
        // round trip serves several values (C3: ~2 bytes per value).
        const bool on = ok && comp;
        const uint32_t lim = p + len;
        const uint32_t kmax = uni(wave_max_u32(on ? xn : 0u));
        uint32_t c = v0, k = 0u;
        bool inb = true;
        for (;;)
        {
            if (__ballot(on && k < xn) == 0ull)
                break;
            const uint32_t q = min(c, LIM) >> 2, m = c & 3u;
            uint32_t d[7], a[6];
#pragma unroll
            for (uint32_t u = 0; u < 7u; ++u)
                d[u] = w[q + u];
#pragma unroll
            for (uint32_t u = 0; u < 6u; ++u)
                a[u] = __builtin_amdgcn_alignbyte(d[u + 1], d[u], m);
            uint32_t o = 0u;
#pragma unroll
            for (uint32_t v = 0; v < 4u; ++v)
            {
                // x = bytes o..o+3, y = bytes o+4..o+7 (a value is taken only at o <= 15)
                const uint32_t oc = min(o, 15u);
                const uint32_t i = oc >> 2, r = oc & 3u;
                const uint32_t l0 = i == 0u ? a[0] : i == 1u ? a[1] : i == 2u ? a[2] : a[3];
                const uint32_t l1 = i == 0u ? a[1] : i == 1u ? a[2] : i == 2u ? a[3] : a[4];
                const uint32_t l2 = i == 0u ? a[2] : i == 1u ? a[3] : i == 2u ? a[4] : a[5];
                const uint32_t x = __builtin_amdgcn_alignbyte(l1, l0, r);
                const uint32_t y = __builtin_amdgcn_alignbyte(l2, l1, r);
                // vbGet32Inline (p4_scalar_internal.h:589-625)
                const uint32_t by = x & 0xFFu;
                const uint32_t dd = __builtin_amdgcn_alignbyte(y, x, 1u);
                const uint32_t v2 = ((by - 0x9Cu) << 8) + (dd & 0xFFu) + 156u;
                const uint32_t v3 = (dd & 0xFFFFu) + ((by - 0xDCu) << 16) + 16540u;
                const uint32_t val = by < 0x9Cu ? by : by < 0xDCu ? v2 : by < 0xFCu ? v3 : by == 0xFCu ? (dd & 0xFFFFFFu) : dd;
                const uint32_t l = by < 0x9Cu ? 1u : by < 0xDCu ? 2u : by < 0xFCu ? 3u : by == 0xFCu ? 4u : 5u;
                const bool step = on && k < xn && o <= 15u;
                inb = inb && (!step || c + o < lim);
                exsum += step ? val : 0u;
                o += step ? l : 0u;
                k += step ? 1u : 0u;
            }
            c += o;
            // a lane whose walk left its block stops (it is declined below)
            if (!inb)
                k = xn;
        }
        (void)kmax;
        vend = comp ? c : vend;
        ok = ok && (!comp || (inb && vend + xn - p == len));
    }
    pay = is_vb ? p + 2u : pay;
    // positions must strictly increase for the sum to be exact: the
    // reference ORs exceptions that share a position (patch loop
    // p4d1dec256v32_scalar.cpp:260); the wave decoder takes those blocks.
    // 16 positions per step from 5 aligned dwords.
    if (__ballot(ok && is_vb) != 0ull)
    {
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
                inc = inc && (!(on && k0 + u < xn) || pos > prev);
                prev = pos;
            }
        }
        ok = ok && (!is_vb || inc);
    }

    // base payload: per stream word k the 8 dwords share phi = 32k mod b
    const bool on = ok && b != 0u;
    const uint32_t bmax = uni(wave_max_u32(on ? b : 0u));
    const uint32_t lmax = uni(wave_max_u32(on ? sum_levels(tab, b) : 0u));
    uint32_t bs = 0u;
    if (bmax != 0u)
    {
        const uint32_t * row = tab + (on ? b : 0u) * kSumTabRow;
        uint32_t A[5], B[5], W[5];
#pragma unroll
        for (uint32_t l = 0; l < 5u; ++l)
        {
            A[l] = row[l];
            B[l] = row[5 + l];
            W[l] = row[10 + l];
        }
        const uint32_t c32 = row[15] & 0xFFu;
        const uint32_t m = pay & 3u;
        uint32_t q = min(pay, LIM) >> 2;
        uint32_t prev = w[q];
        uint32_t phi = 0u;
        for (uint32_t k = 0; k < bmax; ++k)
        {
            const uint32_t s = phi ? b - phi : 0u;
            uint32_t firsts = 0u, zs = 0u;
#pragma unroll
            for (uint32_t l = 0; l < 8u; ++l)
            {
                const uint32_t cur = w[q + 1u + l];
                const uint32_t x = __builtin_amdgcn_alignbyte(cur, prev, m);
                prev = cur;
                firsts += __builtin_amdgcn_ubfe(x, 0u, s);
                uint32_t z = x >> s;
#pragma unroll
                for (uint32_t lv = 0; lv < 5u; ++lv)
                    if (lv < lmax)
                        z = (z & A[lv]) + ((z >> W[lv]) & B[lv]);
                zs += z;
            }
            bs += on && k < b ? (firsts << phi) + zs : 0u;
            q = min(q + 8u, LIM / 4u);
            phi += c32;
            phi = phi >= b ? phi - b : phi;
        }
    }
    sum = is_const ? 256u * (cv + 1u) : bs + 256u + shl32(exsum, b);
    return ok;
}

} // namespace tpf::dev
