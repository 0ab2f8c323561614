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

constexpr uint32_t kLaneRun = 64; // blocks per wave run: lane j = block first + j (16 | kLaneRun <= 64)

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
    // pre levels P: folded per dword before the 8 dwords of a stream word
    // are added (slots of S = b << P bits then hold sums of 8 dwords: needs
    // S - b - P >= 3, so P = 3 / 2 / 2 / 1 for b = 1 / 2 / 3 / >= 4); the
    // top slot [T, 32) may be cut by bit 32, so it is split off and added as
    // a plain integer (T = start of the slot holding bit 31)
    const uint32_t pre = min(b == 1u ? 3u : b <= 3u ? 2u : 1u, levels);
    const uint32_t S = b ? b << pre : 32u;
    const uint32_t T = S >= 32u ? 0u : S * (31u / S);
    row[15] = (b ? 32u % b : 0u) | (levels << 8) | (pre << 12) | (T << 16);
}

__device__ __forceinline__ uint32_t sum_levels(const uint32_t * tab, uint32_t b) { return (tab[b * kSumTabRow + 15u] >> 8) & 15u; }
__device__ __forceinline__ uint32_t sum_pre(const uint32_t * tab, uint32_t b) { return (tab[b * kSumTabRow + 15u] >> 12) & 15u; }

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
// vbGet32Inline (p4_scalar_internal.h:589-625): byte length and value of a
// vbyte whose marker is `by` and whose next four bytes are `d`.
__device__ __forceinline__ uint32_t vb_len32(uint32_t by)
{
    return by < 0x9Cu ? 1u : by < 0xDCu ? 2u : by < 0xFCu ? 3u : by == 0xFCu ? 4u : 5u;
}
__device__ __forceinline__ uint32_t vb_val32(uint32_t by, uint32_t d)
{
    const uint32_t v2 = ((by - 0x9Cu) << 8) + (d & 0xFFu) + 156u;
    const uint32_t v3 = (d & 0xFFFFu) + ((by - 0xDCu) << 16) + 16540u;
    return by < 0x9Cu ? by : by < 0xDCu ? v2 : by < 0xFCu ? v3 : by == 0xFCu ? (d & 0xFFFFFFu) : d;
}

// Base payload sum of one lane's block (see dsum_lanes): P pre levels per
// dword, L levels in all (per-lane rows whose own counts are smaller hold
// no-op masks for the extra levels).
template <uint32_t P, uint32_t L, uint32_t LIM>
__device__ __forceinline__ uint32_t base_sum_lanes(const uint32_t * w, uint32_t pay, uint32_t b, bool on, uint32_t bmax,
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
    uint32_t phi = 0u, bs = 0u;
    uint32_t d[9];
    d[0] = w[q];
    for (uint32_t k = 0; k < bmax; ++k)
    {
        const uint32_t s = phi ? b - phi : 0u;
        // d[0] is the previous word's d[8] (the same dword: q advances by 8
        // and a valid lane's q is never clamped)
#pragma unroll
        for (uint32_t l = 1; l < 9u; ++l)
            d[l] = w[q + l];
        // the 8 folded dwords summed in 64 bits (one add with carry each,
        // round 5): slots below T cannot carry into T, so the low T bits
        // are their sums and the bits from T up the cut top slots' sum
        uint32_t firsts = 0u;
        uint64_t acc = 0ull;
#pragma unroll
        for (uint32_t l = 0; l < 8u; ++l)
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
        const uint32_t hi = static_cast<uint32_t>(acc >> T);
        // levels pre..L-1 of each lane: a lane narrower in pre than the
        // wave's P (e.g. b = 6 beside b = 2) still needs levels pre..P-1
        // here, so the loop starts at the smallest pre any b < 32 has (1);
        // QA/QB are no-ops below each lane's own pre
#pragma unroll
        for (uint32_t lv = (P < 1u ? P : 1u); lv < L; ++lv)
            lo = (lo & QA[lv]) + ((lo >> W[lv]) & QB[lv]);
        bs += on && k < b ? (firsts << phi) + lo + hi : 0u;
        q = min(q + 8u, LIM / 4u);
        d[0] = d[8];
        phi += c32;
        phi = phi >= b ? phi - b : phi;
    }
    return bs;
}

#ifndef TPF_DSUM_ABLATE
#define TPF_DSUM_ABLATE 0 // measurement builds only (p4_dec256v32.hip): 1 base payload, 2 compressed vbyte, 4 raw vbyte, 8 positions
#endif
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
    // a width field outside 32 bits: the wave decoder flags it (kWidthBad)
    bool ok = act && !(is_vb && (h & 0x3Fu) > 32u) && !(is_pb && ((h & 0x7Fu) > 32u || ((h & 0x80u) && x1 > 32u)));
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
    if ((TPF_DSUM_ABLATE & 4) == 0 && __ballot(ok && raw) != 0ull)
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
    if ((TPF_DSUM_ABLATE & 2) == 0 && __ballot(ok && comp) != 0ull)
    {
        // Fast path, no serial marker chain: when every value is 1 or 2 bytes
        // (markers < 0xDC; C3's compressed blocks are all of this kind) the
        // markers of the region follow from the bytes alone.  With A = bytes
        // in [0x9C, 0xDC) (2-byte markers if they are markers), byte k is a
        // marker iff byte k-1 is not a marker in A; inside a maximal run of A
        // bytes the markers alternate from the run's first byte, so they are
        // the run's bytes of the start's parity, and the byte after a run is
        // a marker iff the run's last byte is not.  Runs starting at even
        // offsets are found with one add (A + their start bytes clears them
        // by carry), all on 0xFF/0x00 byte masks, four bytes per dword.
        // The region's length comes from the offsets (len - header - base -
        // xn position bytes); the parse is taken only if it has xn values
        // that use exactly those bytes, with no marker >= 0xDC.  Sum of the
        // values = bytes + 255 * (2-byte markers) - (0x9C*256 - 156) * n2.
        const uint32_t hl = 2u + 32u * b;
        const uint32_t lr = len - hl - xn;
        bool fast = ok && comp && len >= hl + xn && lr >= xn && lr <= 64u;
        if (__ballot(fast) != 0ull)
        {
            // Round 6: the region's dwords q0 .. q0 + 16 (lr <= 64 bytes
            // from byte m0 < 4 of dword q0) are read from one base pointer
            // clamped once to QF, so that every read stays inside the wave's
            // window ((LIM + 36) / 4 dwords); a valid lane's region ends
            // inside [0, WB) = [0, LIM - 28), so its base is never clamped.
            // The byte mask is one 64-bit shift, the carry between dwords two
            // 32-bit adds, and the markers are counted by popcounts of whole
            // 0xFF bytes (8 per marker).
            constexpr uint32_t QF = (LIM + 36u) / 4u - 17u;
            const uint32_t jmax = uni(wave_max_u32(fast ? (lr + 3u) >> 2 : 0u));
            const uint32_t * wq = w + min(v0 >> 2, QF);
            const uint32_t m0 = v0 & 3u, e8 = 8u * lr;
            uint32_t dprev = wq[0];
            uint32_t aprev = 0u, mprev = 0u, cin = 0u, tsum = 0u, s2 = 0u, nm8 = 0u, n28 = 0u, bad = 0u;
#pragma unroll
            for (uint32_t j = 0; j < 16u; ++j)
            {
                if (j >= jmax)
                    break;
                const uint32_t dn = wq[j + 1u];
                const uint32_t x = __builtin_amdgcn_alignbyte(dn, dprev, m0); // region bytes 4j..4j+3
                dprev = dn;
                // the bytes of x inside the region: the low min(lr - 4j, 4) (clamped at 0)
                const uint32_t sh = min(e8 > 32u * j ? e8 - 32u * j : 0u, 32u);
                const uint32_t rm = static_cast<uint32_t>((0xFFFFFFFFull << sh) >> 32);
                const uint32_t hi = x & 0x80808080u, y = x & 0x7F7F7F7Fu;
                const uint32_t gedc = (y + 0x24242424u) & hi;                     // bytes >= 0xDC (bit 7)
                const uint32_t a80 = (y + 0x64646464u) & hi & ~gedc;              // bytes in [0x9C, 0xDC)
                const uint32_t am = a80 | (a80 - (a80 >> 7));                     // as 0xFF bytes
                const uint32_t sha = __builtin_amdgcn_alignbyte(am, aprev, 3u);   // A of byte k-1
                aprev = am;
                uint32_t c1, c2;
                const uint32_t xs0 = __builtin_addc(am, (am & ~sha) & 0x00010001u, 0u, &c1);
                const uint32_t xs = __builtin_addc(xs0, 0u, cin, &c2);
                cin = c1 | c2;
                const uint32_t re = am & ~xs;                                     // runs starting at even offsets
                const uint32_t mr = (re & 0x00FF00FFu) | (am & ~re & 0xFF00FF00u); // markers inside runs
                const uint32_t shm = __builtin_amdgcn_alignbyte(mr, mprev, 3u);
                mprev = mr;
                const uint32_t mk = (mr | ~(am | shm)) & rm;                     // every marker, as 0xFF bytes
                const uint32_t ma = mk & am;                                      // the 2-byte markers
                tsum = __builtin_amdgcn_sad_u8(x & rm, 0u, tsum);
                s2 = __builtin_amdgcn_sad_u8(x & ma, 0u, s2);
                nm8 += __builtin_popcount(mk);
                n28 += __builtin_popcount(ma);
                bad |= mk & gedc;
            }
            // xn values (markers) in exactly lr bytes: n1 + n2 = xn, n1 + 2 n2 = lr
            fast = fast && bad == 0u && nm8 == 8u * xn && 8u * xn + n28 == 8u * lr;
            exsum += fast ? tsum + 255u * s2 - 39780u * (n28 >> 3) : 0u;
        }
        // The general walk (any vbyte lengths) for the other lanes.  The
        // marker chain is serial: each step reads 20 bytes at c (5 aligned
        // dwords, realigned to a[0..3] = bytes c..c+15) and decodes two
        // values: the first at offset 0, the second at the first one's
        // length (1..5: a one-level select).
        const bool on = ok && comp && !fast;
        const uint32_t lim = p + len;
        uint32_t c = v0, k = 0u;
        bool inb = true;
        while (__ballot(on && k < xn) != 0ull)
        {
            const uint32_t q = min(c, LIM) >> 2, m = c & 3u;
            uint32_t d[5], a[4];
#pragma unroll
            for (uint32_t u = 0; u < 5u; ++u)
                d[u] = w[q + u];
#pragma unroll
            for (uint32_t u = 0; u < 4u; ++u)
                a[u] = __builtin_amdgcn_alignbyte(d[u + 1], d[u], m);
            // value 1 at offset 0: marker a0 & 0xFF, data bytes 1..4
            const uint32_t by1 = a[0] & 0xFFu;
            const uint32_t dd1 = __builtin_amdgcn_alignbyte(a[1], a[0], 1u);
            const uint32_t l1 = vb_len32(by1);
            const bool s1 = on && k < xn;
            inb = inb && (!s1 || c < lim);
            exsum += s1 ? vb_val32(by1, dd1) : 0u;
            // value 2 at offset l1 (1..5): bytes l1..l1+7 from a[i..i+2], i = l1 >> 2
            const bool hi1 = l1 >= 4u;
            const uint32_t x0 = hi1 ? a[1] : a[0], x1 = hi1 ? a[2] : a[1], x2 = hi1 ? a[3] : a[2];
            const uint32_t r = l1 & 3u;
            const uint32_t xw = __builtin_amdgcn_alignbyte(x1, x0, r), yw = __builtin_amdgcn_alignbyte(x2, x1, r);
            const uint32_t by2 = xw & 0xFFu;
            const uint32_t dd2 = __builtin_amdgcn_alignbyte(yw, xw, 1u);
            const bool s2v = s1 && k + 1u < xn;
            inb = inb && (!s2v || c + l1 < lim);
            exsum += s2v ? vb_val32(by2, dd2) : 0u;
            const uint32_t adv = s1 ? l1 + (s2v ? vb_len32(by2) : 0u) : 0u;
            c += adv;
            k += s1 ? (s2v ? 2u : 1u) : 0u;
            // a lane whose walk left its block stops (it is declined below)
            k = inb ? k : xn;
        }
        vend = comp ? (fast ? v0 + lr : c) : vend;
        ok = ok && (!comp || fast || (inb && vend + xn - p == len));
    }
    pay = is_vb ? p + 2u : pay;
    // positions must strictly increase for the sum to be exact: the
    // reference ORs exceptions that share a position (patch loop
    // p4d1dec256v32_scalar.cpp:260); the wave decoder takes those blocks.
    // 16 positions per step from 5 aligned dwords.
    if ((TPF_DSUM_ABLATE & 8) == 0 && __ballot(ok && is_vb) != 0ull)
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

    // base payload: per stream word k the 8 dwords share phi = 32k mod b.
    // Per dword: the first piece (x & mask(s)) << phi is summed raw; the rest
    // z = x >> s (whole fields from bit 0) is folded `pre` SWAR levels, its
    // top slot split off; the 8 dwords' folded parts are added, and the sum
    // folded the remaining levels once per stream word (the fold is linear
    // while no slot overflows: see build_sum_row).  The level counts are
    // template parameters: a wave's (max pre, max levels) is always that of
    // its narrowest block, so six instantiations cover every wave, and the
    // fold runs exactly its levels (with run-time counts the compiler
    // if-converts every possible level into selects: 243 VALU per stream
    // word instead of ~110 at b = 6).
    const bool on = ok && b != 0u;
    const uint32_t bmax = uni(wave_max_u32(on ? b : 0u));
    const uint32_t lmax = uni(wave_max_u32(on ? sum_levels(tab, b) : 0u));
    const uint32_t pmax = uni(wave_max_u32(on ? sum_pre(tab, b) : 0u));
    uint32_t bs = 0u;
    if ((TPF_DSUM_ABLATE & 1) == 0 && bmax != 0u)
    {
        const uint32_t * row = tab + (on ? b : 0u) * kSumTabRow;
        const uint32_t key = pmax * 8u + lmax;
        if (key == 1u * 8u + 3u)
            bs = base_sum_lanes<1, 3, LIM>(w, pay, b, on, bmax, row);
        else if (key == 1u * 8u + 2u)
            bs = base_sum_lanes<1, 2, LIM>(w, pay, b, on, bmax, row);
        else if (key == 1u * 8u + 1u)
            bs = base_sum_lanes<1, 1, LIM>(w, pay, b, on, bmax, row);
        else if (key == 2u * 8u + 4u)
            bs = base_sum_lanes<2, 4, LIM>(w, pay, b, on, bmax, row);
        else if (key == 3u * 8u + 5u)
            bs = base_sum_lanes<3, 5, LIM>(w, pay, b, on, bmax, row);
        else
            bs = base_sum_lanes<0, 0, LIM>(w, pay, b, on, bmax, row); // every lane b = 32
    }
    sum = is_const ? 256u * (cv + 1u) : bs + 256u + shl32(exsum, b);
    return ok;
}

} // namespace tpf::dev
