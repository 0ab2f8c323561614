// p4_generic.h -- wave-level P4 block codec for every format of the
// reference's include/turbopfor.h other than the specialised 256v32 hot path:
//
//   Fmt::H32    p4Enc32/p4Dec32       horizontal base, n = 1..256
//                (src/scalar/p4enc32.cpp:201-217, p4dec32.cpp:70-142)
//   Fmt::V128   p4Enc128v32/p4Dec128v32  4-lane interleave, 128 values
//                (src/scalar/bitpack128v32_scalar.cpp:57-231, p4dec128v32_scalar.cpp)
//   Fmt::V256   p4Enc256v32/p4Dec256v32 for n != 256 (per-block API)
//   Fmt::H64    p4Enc64/p4Dec64       horizontal 64-bit base (p4enc64.cpp, p4dec64.cpp)
//   Fmt::V128X64 p4Enc128v64/p4Dec128v64 hybrid: b<=32 -> 128v32 layout of the
//                pair-swapped low halves, b>32 -> horizontal 64-bit
//                (bitpack128v64_scalar.cpp:38-104, p4d1dec128v64_scalar.cpp:157-375)
//   (256v64 = two consecutive V128X64 blocks, p4enc256v64_scalar.cpp:15-30)
//
// One block per wave; lane t owns elements e = t + 64*j (j = 0..3), so the
// bitmap rank of element e is popc(words before j) + popc(word j & lanes<t).
#pragma once

#include "p4_block32.h"

namespace tpf::dev
{

enum class Fmt : int
{
    H32 = 0,
    V128 = 1,
    V256 = 2,
    H64 = 3,
    V128X64 = 4,
};

template <Fmt F>
struct FmtTraits
{
    static constexpr bool wide = (F == Fmt::H64 || F == Fmt::V128X64);
    static constexpr uint32_t W = wide ? 64u : 32u;
    static constexpr uint32_t N = F == Fmt::V256 ? 256u : (F == Fmt::V128 || F == Fmt::V128X64) ? 128u : 0u; // 0: n
    using T = typename std::conditional<wide, uint64_t, uint32_t>::type;
};

__device__ __forceinline__ uint64_t mask64d(uint32_t b) { return b >= 64u ? ~0ull : ((1ull << b) - 1ull); }
__device__ __forceinline__ uint64_t shl64(uint64_t v, uint32_t b) { return b >= 64u ? 0ull : (v << b); }
__device__ __forceinline__ uint32_t pad8d(uint32_t bits) { return (bits + 7u) >> 3; }

// up to 64 bits at bit position bp
__device__ __forceinline__ uint64_t lds_bits64(const uint32_t * w, uint32_t bp, uint32_t nb)
{
    if (nb == 0u)
        return 0ull;
    const uint64_t lo = lds_bits(w, bp, nb < 32u ? nb : 32u);
    if (nb <= 32u)
        return lo;
    return lo | (static_cast<uint64_t>(lds_bits(w, bp + 32u, nb - 32u)) << 32);
}

__device__ __forceinline__ uint64_t lds_u64(const uint32_t * w, uint32_t pos)
{
    return static_cast<uint64_t>(lds_u32(w, pos)) | (static_cast<uint64_t>(lds_u32(w, pos + 4u)) << 32);
}

// Base payload bytes for n values at width b.
template <Fmt F>
__device__ __forceinline__ uint32_t base_bytes(uint32_t n, uint32_t b)
{
    if constexpr (F == Fmt::H32 || F == Fmt::H64)
        return pad8d(n * b);
    else if constexpr (F == Fmt::V256)
        return 32u * b;
    else
        return 16u * b; // V128, V128X64 (b<=32: 128v32; b>32: pad8(128*b) == 16*b)
}

// Element e of the base payload at byte P, width b.
template <Fmt F>
__device__ __forceinline__ typename FmtTraits<F>::T base_elem(const uint32_t * lds, uint32_t P, uint32_t b, uint32_t e)
{
    if constexpr (F == Fmt::H32)
        return lds_bits(lds, P * 8u + e * b, b);
    else if constexpr (F == Fmt::H64)
        return lds_bits64(lds, P * 8u + e * b, b);
    else
    {
        constexpr uint32_t L = F == Fmt::V256 ? 8u : 4u;
        if constexpr (F == Fmt::V128X64)
        {
            if (b > 32u)
                return lds_bits64(lds, P * 8u + e * b, b);
            e ^= 2u; // IP32 pair swap (bitpack128v64_scalar.cpp:50-56 / :91-97)
        }
        const uint32_t l = e % L, g = e / L;
        const uint32_t o = g * b;
        const uint32_t pos = P + 4u * L * (o >> 5) + 4u * l;
        const uint32_t w0 = lds_u32(lds, pos);
        const uint32_t w1 = lds_u32(lds, pos + 4u * L);
        return __builtin_amdgcn_alignbit(w1, w0, o & 31u) & mask32(b);
    }
}

// vbyte value at byte position c (marker already known): 32-bit markers
// (vbGet32Inline, p4_scalar_internal.h:589-625) or 64-bit markers
// (vbGet64Inline, :638-670).  Returns the value, *len = bytes consumed.
// 64-bit markers: the 1-3 byte forms by selects, only the long form behind a
// branch (round 5: C3 64-bit lists +3.4%, per-unit starts +4%,
// profiles/r5ai_vbyte64_ab.txt).
template <bool Wide>
__device__ __forceinline__ uint64_t vbyte_value(const uint32_t * lds, uint32_t c, uint32_t m)
{
    if constexpr (!Wide)
    {
        const uint32_t d = lds_u32(lds, c + 1u);
        if (m < 0x9Cu)
            return m;
        if (m < 0xDCu)
            return ((m - 0x9Cu) << 8) + (d & 0xFFu) + 156u;
        if (m < 0xFCu)
            return (d & 0xFFFFu) + ((m - 0xDCu) << 16) + 16540u;
        if (m == 0xFCu)
            return d & 0xFFFFFFu;
        return d;
    }
    else
    {
        const uint32_t d = lds_u32(lds, c + 1u);
        const uint32_t v2 = ((m - 0x98u) << 8) + (d & 0xFFu) + 152u;
        const uint32_t v3 = (d & 0xFFFFu) + ((m - 0xD8u) << 16) + 16536u;
        uint64_t r = m < 0x98u ? m : m < 0xD8u ? v2 : v3;
        if (m >= 0xF8u)
        {
            const uint32_t nb = m - 0xF8u + 3u;
            const uint64_t x = lds_u64(lds, c + 1u);
            r = nb >= 8u ? x : (x & ((1ull << (8u * nb)) - 1ull));
        }
        return r;
    }
}

template <bool Wide>
__device__ __forceinline__ uint32_t vbyte_len(uint32_t m)
{
    if constexpr (!Wide)
        return m < 0x9Cu ? 1u : m < 0xDCu ? 2u : m < 0xFCu ? 3u : m == 0xFCu ? 4u : 5u;
    else
        return m < 0x98u ? 1u : m < 0xD8u ? 2u : m < 0xF8u ? 3u : (m - 0xF8u + 4u);
}

// vbyte exceptions into scr[pos] (T per position, zeroed here).  Same
// 64-byte window parse as vbyte_exceptions in p4_block32.h, generic width.
// NPOS: scratch entries of scr and of tmp (256; 128 for the 128-value 64-bit
// blocks, whose valid positions and exception counts are < 128: a malformed
// position past them is dropped and flagged with kWidthBad)
// The 64-bit vbyte scratch is cleared by one 16-byte store per lane instead
// of two 8-byte stores (round 4, profiles/r4y_d64_ab.txt: C3 64-bit lists
// +2.5%, C4's 64-bit leg level).
template <bool Wide, uint32_t NPOS = 256>
__device__ __forceinline__ uint32_t vbyte_exceptions_g(const uint32_t * lds, uint32_t v0, uint32_t xn,
                                                       typename std::conditional<Wide, uint64_t, uint32_t>::type * scr,
                                                       typename std::conditional<Wide, uint64_t, uint32_t>::type * tmp,
                                                       uint32_t t)
{
    using T = typename std::conditional<Wide, uint64_t, uint32_t>::type;
    static_assert(NPOS == 128u || NPOS == 256u, "scratch of 128 or 256 positions");
    constexpr uint32_t PM = NPOS - 1u;
    // one 16-byte store per lane clears the 64-bit decoder's 1 KB scr
    // (16-byte aligned: k_dec128v64w's scratch, k_dsum128v64_lanes' window)
    if constexpr (Wide && NPOS == 128u)
    {
        typedef uint32_t z4 __attribute__((ext_vector_type(4)));
        reinterpret_cast<z4 *>(scr)[t] = z4{0u, 0u, 0u, 0u};
    }
    else
        for (uint32_t i = t; i < NPOS; i += 64u)
            scr[i] = 0;
    wave_lds_sync();
    const uint32_t first = uni(lds_byte(lds, v0));
    uint32_t vend;
    bool badpos = false;
    constexpr uint32_t ES = Wide ? 8u : 4u;
    if (first == 0xFFu)
    {
        const uint32_t pbase = v0 + 1u + ES * xn;
        for (uint32_t k = t; k < xn; k += 64u)
        {
            const T val = Wide ? static_cast<T>(lds_u64(lds, v0 + 1u + ES * k)) : static_cast<T>(lds_u32(lds, v0 + 1u + ES * k));
            const uint32_t pos = lds_byte(lds, pbase + k);
            badpos |= pos > PM;
            if (pos <= PM)
                atomicOr(&scr[pos], val);
        }
        vend = pbase;
    }
    else
    {
        // value starts by binary lifting (window_starts, p4_block32.h)
        uint32_t c = v0, sp = 0, found = 0;
        vend = v0;
        while (found < xn)
        {
            const uint32_t nxt = t + vbyte_len<Wide>(lds_byte(lds, c + t));
            const uint32_t p = window_starts(nxt, sp, t);
            const uint32_t m = static_cast<uint32_t>(__builtin_popcountll(__ballot(p < 64u)));
            const uint32_t cnt = min(m, xn - found);
            const uint32_t pn = bperm(nxt, p); // every lane: bpermute reads 0 from inactive lanes
            const uint32_t pe = p < 64u ? pn : p;
            if (t < cnt)
                tmp[(found + t) & PM] = static_cast<T>(vbyte_value<Wide>(lds, c + p, lds_byte(lds, c + p)));
            const uint32_t e_last = uni(__builtin_amdgcn_readlane(pe, cnt - 1u));
            found += cnt;
            vend = c + e_last;
            sp = e_last >= 64u ? e_last - 64u : e_last;
            c += e_last >= 64u ? 64u : 0u;
        }
        wave_lds_sync();
        for (uint32_t k = t; k < xn; k += 64u)
        {
            const uint32_t pos = lds_byte(lds, vend + k);
            badpos |= pos > PM;
            if (pos <= PM)
                atomicOr(&scr[pos], tmp[k & PM]);
        }
    }
    wave_lds_sync();
    // a position past the block (only possible with NPOS 128) is dropped, not
    // aliased into a real element, and flags the block like a bad width
    // (the reference writes it past the 128 values it unpacks)
    return (vend + xn) | ((NPOS < 256u && __builtin_amdgcn_ballot_w64(badpos) != 0ull) ? kWidthBad : 0u);
}

// Decode one block of format F (n values) staged at LDS byte s.  v[j] gets
// element t + 64j.  Returns consumed bytes.  *cmode = 1 for a constant block
// (the reference then writes only n values, otherwise the layout's full N).
template <Fmt F>
__device__ __forceinline__ uint32_t decode_block_g(const uint32_t * lds, uint32_t s, uint32_t n, void * scr_v,
                                                   uint32_t t, typename FmtTraits<F>::T v[4], uint32_t * cmode)
{
    using Tr = FmtTraits<F>;
    using T = typename Tr::T;
    constexpr bool wide = Tr::wide;
    constexpr uint32_t W = Tr::W;
    const uint32_t NE = Tr::N ? Tr::N : n; // elements the base payload holds
    T * scr = static_cast<T *>(scr_v);
    const uint32_t h = uni(lds_byte(lds, s));
    *cmode = 0;
    if ((h & 0xC0u) == 0xC0u)
    {
        uint32_t b = h & 0x3Fu;
        if (wide && b == 63u)
            b = 64u;
        const uint32_t cbad = (F == Fmt::H32 && b > 32u) ? kWidthBad : 0u; // framing.cpp: undefined in p4dec32.cpp:100-116
        T c;
        if constexpr (wide)
            c = static_cast<T>(lds_u64(lds, s + 1u) & mask64d(b));
        else
            c = static_cast<T>(lds_u32(lds, s + 1u) & mask32(b));
#pragma unroll
        for (int j = 0; j < 4; ++j)
            v[j] = c;
        *cmode = 1;
        return (1u + ((b + 7u) >> 3)) | cbad;
    }
    uint32_t b, bx = 0, hdr, xn = 0, P, xs = 0, wbad = 0;
    const bool vb = (h & 0x40u) != 0u;
    uint64_t bm[4] = {0, 0, 0, 0};
    uint32_t pc[4] = {0, 0, 0, 0};
    if (!vb)
    {
        hdr = (h & 0x80u) ? 2u : 1u;
        const uint32_t bxr = (h & 0x80u) ? uni(lds_byte(lds, s + 1u)) : 0u;
        bx = min(bxr, W);
        b = h & 0x7Fu;
        if (wide && b == 63u)
            b = 64u;
        wbad = (b > W || bxr > W) ? kWidthBad : 0u;
        b = min(b, W);
        if (bx == 0u)
            P = s + hdr;
        else
        {
            const uint32_t words = (n + 63u) >> 6;
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u)
            {
                uint64_t w = u < words ? lds_u64(lds, s + 2u + 8u * u) : 0ull;
                if (u == words - 1u && (n & 63u))
                    w &= (1ull << (n & 63u)) - 1ull;
                bm[u] = w;
                pc[u] = __builtin_popcountll(w);
                xn += pc[u];
            }
            xs = s + 2u + pad8d(n);
            P = xs + pad8d(xn * bx);
        }
    }
    else
    {
        hdr = 2u;
        b = h & 0x3Fu;
        if (wide && b == 63u)
            b = 64u;
        wbad = b > W ? kWidthBad : 0u;
        b = min(b, W);
        xn = uni(lds_byte(lds, s + 1u));
        P = s + 2u;
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
    {
        const uint32_t e = t + 64u * j;
        v[j] = (e < NE && b) ? base_elem<F>(lds, P, b, e) : T(0);
    }
    const uint32_t bb = base_bytes<F>(NE, b);
    if (!vb)
    {
        if (bx == 0u)
            return (hdr + bb) | wbad;
        uint32_t before = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
        {
            if ((bm[j] >> t) & 1ull)
            {
                const uint32_t k = before + __builtin_popcountll(bm[j] & lanemask_lt());
                const T ex = static_cast<T>(lds_bits64(lds, xs * 8u + k * bx, bx));
                if constexpr (wide)
                    v[j] |= shl64(ex, b);
                else
                    v[j] |= shl32(static_cast<uint32_t>(ex), b);
            }
            before += pc[j];
        }
        return ((xs - s) + pad8d(xn * bx) + bb) | wbad;
    }
    T * tmp = scr + 256;
    const uint32_t end = vbyte_exceptions_g<wide>(lds, P + bb, xn, scr, tmp, t);
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
    {
        const uint32_t e = t + 64u * j;
        const T ex = scr[e & 255u];
        if constexpr (wide)
            v[j] |= shl64(ex, b);
        else
            v[j] |= shl32(static_cast<uint32_t>(ex), b);
    }
    return (end - s) | wbad;
}

// Delta-1 over elements e < n in order (applyDelta1_*): out[e] = start +
// sum_{i<=e}(v[i]+1).  Returns the value of element n-1.
template <class T>
__device__ __forceinline__ T delta1_g(T v[4], uint32_t n, T start, uint32_t t)
{
    T carry = start;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
    {
        const uint32_t e = t + 64u * j;
        T x = e < n ? T(v[j] + 1u) : T(0);
        T incl;
        if constexpr (sizeof(T) == 8)
            incl = wave_incl_scan64(x);
        else
            incl = wave_incl_scan(x);
        if (e < n)
            v[j] = carry + incl;
        T tot;
        if constexpr (sizeof(T) == 8)
            tot = readlane_u64(incl, 63);
        else
            tot = __builtin_amdgcn_readlane(incl, 63);
        carry += tot;
    }
    return carry;
}

// deltaEnc1 (p4_scalar_internal.h:711-719) over elements e < n in order.
template <class T>
__device__ __forceinline__ void delta_enc_g(T v[4], T prev0, uint32_t n, uint32_t t)
{
    T d[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
    {
        T prev;
        if constexpr (sizeof(T) == 8)
        {
            // lane t-1's value by DPP wave_shr:1 (lane 0: the previous row's last)
            const uint64_t p0 = j == 0 ? static_cast<uint64_t>(prev0) : readlane_u64(v[j - 1], 63);
            const uint32_t lo = wave_shr1(static_cast<uint32_t>(v[j]), static_cast<uint32_t>(p0));
            const uint32_t hi = wave_shr1(static_cast<uint32_t>(v[j] >> 32), static_cast<uint32_t>(p0 >> 32));
            prev = (static_cast<uint64_t>(hi) << 32) | lo;
        }
        else
        {
            const uint32_t p0 = j == 0 ? static_cast<uint32_t>(prev0) : __builtin_amdgcn_readlane(v[j - 1], 63);
            prev = wave_shr1(static_cast<uint32_t>(v[j]), p0);
        }
        d[j] = (t + 64u * j < n) ? T(v[j] - prev - 1u) : T(0);
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
        v[j] = d[j];
}

} // namespace tpf::dev

// ============================================================== encoder
#include "p4_enc32.h"

namespace tpf::dev
{

struct PlanG
{
    uint32_t b, bx, size, xn, raw;
};

__device__ __forceinline__ uint32_t bw64d(uint64_t x) { return x ? 64u - static_cast<uint32_t>(__builtin_clzll(x)) : 0u; }

// vbPut64 byte length (p4_scalar_internal.cpp:447-476)
__device__ __forceinline__ uint32_t vblen64(uint64_t x)
{
    // selects on the range tests, not a ?: chain (which compiled into exec-mask branches)
    const uint32_t small = 1u + (x >= 152u) + (x >= 16536u);
    return __builtin_unpredictable(x >= 2113688u) ? 1u + ((bw64d(x) + 7u) >> 3) : small;
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t x)
{
    return (static_cast<uint64_t>(wave_or(static_cast<uint32_t>(x >> 32))) << 32) | wave_or(static_cast<uint32_t>(x));
}

__device__ __forceinline__ uint64_t readlane64(uint64_t x, uint32_t l)
{
    return readlane_u64(x, l);
}

// p4Bits32 / p4Bits64 (p4_scalar_internal.cpp:270-387, :538-652) evaluated
// across lanes (see p4_enc32.h for the closed forms), plus the exact size of
// the chosen encoding.  hist: per-wave LDS scratch of kPlanGHistU32 u32.
using PlanGHist = WaveHist<4, 68>; // bit widths 0..64 (lane t reads bin t < 64, plus bin 64)
constexpr uint32_t kPlanGHistU32 = PlanGHist::kU32;
template <Fmt F>
__device__ __forceinline__ PlanG plan_block_g(const typename FmtTraits<F>::T v[4], uint32_t n, uint32_t * hist, uint32_t t)
{
    using Tr = FmtTraits<F>;
    constexpr uint32_t W = Tr::W;
    constexpr bool wide = Tr::wide;
    const uint32_t NE = Tr::N ? Tr::N : n;
    PlanG P{0, 0, 1, 0, 0};
    const uint64_t first = wide ? readlane64(static_cast<uint64_t>(v[0]), 0)
                                : static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(v[0])), 0));
    // constant block (all zero: the plain b = 0 block): a ballot, not a wave reduction
    bool same = true;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
        same = same && (t + 64u * j >= n || static_cast<uint64_t>(v[j]) == first);
    if (__builtin_amdgcn_ballot_w64(!same) == 0ull)
    {
        if (first == 0ull)
        {
            P.size = 1u + base_bytes<F>(NE, 0);
            return P;
        }
        const uint32_t cb = wide ? bw64d(first) : bw32(static_cast<uint32_t>(first));
        P.b = cb;
        P.bx = W + 2u;
        P.size = 1u + ((cb + 7u) >> 3);
        return P;
    }
    PlanGHist::zero(hist, t);
    wave_lds_sync();
    uint32_t cnt, cnt64;
    if constexpr (!wide)
    {
        // 32-bit values: bins keyed by v_ffbh_u32 + 1 (= 33 - bw, 0 for 0), as plan_block256
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            if (64u * j < n)
                PlanGHist::add(hist, t + 64u * j < n ? ffbh1(static_cast<uint32_t>(v[j])) : 67u, t);
        wave_lds_sync();
        cnt = PlanGHist::get(hist, t == 0u ? 0u : (t <= 32u ? 33u - t : 68u));
        cnt64 = 0u;
    }
    else
    {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            if (t + 64u * j < n)
                PlanGHist::add(hist, bw64d(v[j]), t);
        wave_lds_sync();
        cnt = PlanGHist::get(hist, t);
        cnt64 = uni(PlanGHist::get(hist, 64));
    }
    wave_lds_sync();
    // the block's bit width: the highest width with a count (lane c holds
    // cnt[c]; a ballot and a scalar bit scan instead of a wave OR reduction
    // of the values, round 5); not all zero, so some width >= 1 has a count
    const uint32_t maxb = cnt64 != 0u ? 64u : 63u - static_cast<uint32_t>(__builtin_clzll(__builtin_amdgcn_ballot_w64(cnt != 0u)));
    uint32_t ec, vbsum;
    if constexpr (!wide)
    {
        // as plan_block256: suffix sums S(k), the shifted ones through LDS
        const uint32_t incl = wave_incl_scan(cnt);
        ec = __builtin_amdgcn_readlane(incl, 63) - incl; // sum_{c > t} cnt[c]; 0 for lanes >= 32
        hist[t] = ec;
        wave_lds_sync();
        vbsum = ec + hist[t + 7u] + 2u * hist[t + 15u] + 3u * hist[t + 19u] + 4u * hist[t + 25u]; // lanes t > 38: unused
        wave_lds_sync();
    }
    else
    {
        // cnt[c] for c = t+7, t+15, t+19, t+25 back through the histogram's
        // LDS (cnt[64] = cnt64, zeros past it; the bins were read above):
        // one store and four reads at immediate offsets instead of four
        // ds_bpermute with their address and range selects (round 5)
        hist[t] = cnt;
        if (t < 25u)
            hist[64u + t] = t == 0u ? cnt64 : 0u;
        wave_lds_sync();
        const uint32_t vbacc = hist[t + 7u] + 2u * hist[t + 15u] + 3u * hist[t + 19u] + 4u * hist[t + 25u];
        wave_lds_sync();
        // both suffix sums in one scan (cnt <= 256 low half, cnt + vbacc <= 11*256 high half)
        const uint32_t pab = wave_incl_scan(cnt | ((cnt + vbacc) << 16));
        const uint32_t tab = __builtin_amdgcn_readlane(pab, 63);
        ec = (tab & 0xFFFFu) - (pab & 0xFFFFu) + cnt64;
        vbsum = (tab >> 16) - (pab >> 16) + cnt64;
    }
    uint32_t key = 0xFFFFFFFFu;
    const uint32_t bmp = pad8d(n);
    if (t < maxb)
    {
        const uint32_t vsz = pad8d(n * t) + 2u + ec + vbsum;
        const uint32_t psz = pad8d(n * t) + 2u + bmp + pad8d(ec * (maxb - t));
        const uint32_t cost = psz <= vsz ? psz : vsz;
        key = (cost << 8) | ((maxb - t) << 1) | (psz <= vsz ? 0u : 1u);
    }
    uint32_t kmin = uni(wave_min(key));
    const uint32_t plain_key = (pad8d(n * maxb) + 1u) << 8;
    if (plain_key <= kmin)
        kmin = plain_key;
    const uint32_t order = (kmin >> 1) & 127u;
    uint32_t b = maxb - order;
    if (order == 0u || (wide && b == 63u))
    {
        if (wide && b == 63u)
            b = 64u; // 63->64 quirk (p4_scalar_internal.cpp:645-649)
        P.b = b;
        P.bx = 0;
        P.size = 1u + base_bytes<F>(NE, b);
        return P;
    }
    P.b = b;
    if ((kmin & 1u) == 0u)
    {
        // bitmap patch: xn = ec(b), already in lane b (b <= 63 here)
        const uint32_t xn = uni(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(ec), static_cast<int>(b))));
        P.xn = xn;
        P.bx = maxb - b;
        P.size = 2u + bmp + pad8d(xn * P.bx) + base_bytes<F>(NE, b);
        return P;
    }
    uint32_t xn, sumlen;
    if constexpr (!wide)
    {
        // exception count and vbyte bytes by ballot popcounts per vblen32
        // threshold of y = x >> b (see plan_block256); b < maxb <= 32
        uint32_t y[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            y[j] = t + 64u * j < n ? static_cast<uint32_t>(v[j]) >> b : 0u;
        auto count_ge = [&](uint32_t T) -> uint32_t {
            uint32_t c = 0u;
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (64u * j < n)
                    c += static_cast<uint32_t>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(y[j] >= T)));
            return c;
        };
        xn = uni(count_ge(1u));
        sumlen = uni(xn + count_ge(156u) + count_ge(16540u) + count_ge(2113692u) + count_ge(0x1000000u));
    }
    else
    {
        const uint64_t m = mask64d(b);
        uint32_t xc = 0, sl = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            if (t + 64u * j < n && static_cast<uint64_t>(v[j]) > m)
            {
                ++xc;
                sl += vblen64(static_cast<uint64_t>(v[j]) >> b);
            }
        const uint32_t xs_tot = wave_sum(xc | (sl << 16)); // count | vbyte bytes (<= 9*256)
        xn = xs_tot & 0xFFFFu;
        sumlen = xs_tot >> 16;
    }
    P.xn = xn;
    P.bx = W + 1u;
    constexpr uint32_t ES = W / 8u;
    P.raw = (sumlen + 32u > ES * xn) ? 1u : 0u;
    P.size = 2u + base_bytes<F>(NE, b) + (P.raw ? 1u + ES * xn : sumlen) + xn;
    return P;
}

__device__ __forceinline__ void or_bits64(uint32_t * img, uint32_t bp, uint64_t val, uint32_t nb)
{
    if (nb == 0u)
        return;
    val &= mask64d(nb);
    const uint32_t lo = nb < 32u ? nb : 32u;
    or_bits(img, bp, static_cast<uint32_t>(val), lo);
    if (nb > 32u)
        or_bits(img, bp + 32u, static_cast<uint32_t>(val >> 32), nb - 32u);
}

// Scatter element e (value x < 2^b) into the base payload at byte P.
template <Fmt F>
__device__ __forceinline__ void pack_elem(uint32_t * img, uint32_t P, uint32_t b, uint32_t e, uint64_t x)
{
    if (b == 0u)
        return;
    if constexpr (F == Fmt::H32 || F == Fmt::H64)
    {
        or_bits64(img, P * 8u + e * b, x, b);
    }
    else
    {
        constexpr uint32_t L = F == Fmt::V256 ? 8u : 4u;
        if constexpr (F == Fmt::V128X64)
        {
            if (b > 32u)
            {
                or_bits64(img, P * 8u + e * b, x, b);
                return;
            }
            e ^= 2u;
        }
        const uint32_t l = e % L, g = e / L;
        const uint32_t o = g * b;
        const uint32_t k = o >> 5, sh = o & 31u;
        const uint32_t lo_byte = P + 4u * L * k + 4u * l;
        const uint32_t lo_bits = min(b, 32u - sh);
        const uint32_t xv = static_cast<uint32_t>(x);
        or_bits(img, lo_byte * 8u + sh, xv & mask32(lo_bits), lo_bits);
        if (b > lo_bits)
            or_bits(img, (lo_byte + 4u * L) * 8u, xv >> lo_bits, b - lo_bits);
    }
}

// Emit the block (header + payload) into the zeroed LDS image at byte s.
template <Fmt F>
__device__ __forceinline__ void emit_block_g(uint32_t * img, uint32_t s, const PlanG & P, const typename FmtTraits<F>::T v[4],
                                             uint32_t n, uint32_t t)
{
    using Tr = FmtTraits<F>;
    constexpr uint32_t W = Tr::W;
    constexpr bool wide = Tr::wide;
    const uint32_t NE = Tr::N ? Tr::N : n;
    const uint32_t b = P.b;
    (void)sizeof(typename Tr::T);
    const uint32_t bh = (wide && b >= 64u) ? 63u : b;
    if (P.bx == 0u)
    {
        if (t == 0)
            or_bits(img, s * 8u, bh, 8);
        const uint64_t m = mask64d(b);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            if (t + 64u * j < NE)
                pack_elem<F>(img, s + 1u, b, t + 64u * j, static_cast<uint64_t>(v[j]) & m);
        return;
    }
    if (P.bx == W + 2u)
    {
        if (t == 0)
        {
            or_bits(img, s * 8u, 0xC0u | bh, 8);
            or_bits64(img, (s + 1u) * 8u, static_cast<uint64_t>(v[0]) & mask64d(b), b);
        }
        return;
    }
    const uint64_t m = mask64d(b);
    uint32_t fl[4];
    uint64_t bal[4];
    uint32_t rowc[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
    {
        fl[j] = (t + 64u * j < n && static_cast<uint64_t>(v[j]) > m) ? 1u : 0u;
        bal[j] = __ballot(fl[j]);
        rowc[j] = __builtin_popcountll(bal[j]);
    }
    const uint32_t PB = (P.bx <= W) ? s + 2u + pad8d(n) + pad8d(P.xn * P.bx) : s + 2u;
    if (t == 0)
        or_bits(img, s * 8u, ((P.bx <= W) ? 0x80u : 0x40u) | bh, 8);
    // base values (exceptions keep their low b bits)
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
        if (t + 64u * j < NE)
            pack_elem<F>(img, PB, b, t + 64u * j, (t + 64u * j < n) ? (static_cast<uint64_t>(v[j]) & m) : 0ull);
    if (P.bx <= W)
    {
        if (t == 0)
        {
            or_bits(img, (s + 1u) * 8u, P.bx, 8);
            const uint32_t words = (n + 63u) >> 6;
            for (uint32_t j = 0; j < words; ++j)
                or_bits64(img, (s + 2u) * 8u + 64u * j, bal[j], min(64u, n - 64u * j));
        }
        const uint32_t xs = (s + 2u + pad8d(n)) * 8u;
        uint32_t before = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
        {
            if (fl[j])
            {
                const uint32_t k = before + __builtin_popcountll(bal[j] & lanemask_lt());
                or_bits64(img, xs + k * P.bx, static_cast<uint64_t>(v[j]) >> b, P.bx);
            }
            before += rowc[j];
        }
        return;
    }
    // vbyte: [xn][base][V][positions]
    if (t == 0)
        or_bits(img, (s + 1u) * 8u, P.xn, 8);
    const uint32_t v0 = PB + base_bytes<F>(NE, b);
    constexpr uint32_t ES = W / 8u;
    if (P.raw)
    {
        if (t == 0)
            or_bits(img, v0 * 8u, 0xFFu, 8);
        uint32_t before = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
        {
            if (fl[j])
            {
                const uint32_t k = before + __builtin_popcountll(bal[j] & lanemask_lt());
                or_bits64(img, (v0 + 1u + ES * k) * 8u, static_cast<uint64_t>(v[j]) >> b, W);
                or_bits(img, (v0 + 1u + ES * P.xn + k) * 8u, t + 64u * j, 8);
            }
            before += rowc[j];
        }
        return;
    }
    // compressed: byte offsets by scan of lengths in element order
    uint32_t carry = 0, before = 0;
    uint32_t vtot = 0;
    uint32_t lens[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
    {
        const uint64_t ex = static_cast<uint64_t>(v[j]) >> b;
        lens[j] = fl[j] ? (wide ? vblen64(ex) : vblen32(static_cast<uint32_t>(ex))) : 0u;
        vtot += wave_sum(lens[j]);
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
    {
        const uint32_t incl = wave_incl_scan(lens[j]);
        if (fl[j])
        {
            const uint32_t k = before + __builtin_popcountll(bal[j] & lanemask_lt());
            const uint32_t pos = v0 + carry + incl - lens[j];
            const uint64_t x = static_cast<uint64_t>(v[j]) >> b;
            const uint32_t bp = pos * 8u;
            if constexpr (!wide)
            {
                const uint32_t xx = static_cast<uint32_t>(x);
                if (xx < 156u)
                    or_bits(img, bp, xx, 8);
                else if (xx < 16540u)
                {
                    const uint32_t d = xx - 156u;
                    or_bits(img, bp, (0x9Cu + (d >> 8)) | ((d & 0xFFu) << 8), 16);
                }
                else if (xx < 2113692u)
                {
                    const uint32_t d = xx - 16540u;
                    or_bits(img, bp, (0xDCu + (d >> 16)) | ((d & 0xFFFFu) << 8), 24);
                }
                else if (xx <= 0xFFFFFFu)
                    or_bits(img, bp, 0xFCu | (xx << 8), 32);
                else
                {
                    or_bits(img, bp, 0xFDu, 8);
                    or_bits(img, bp + 8u, xx, 32);
                }
            }
            else
            {
                if (x < 152u)
                    or_bits(img, bp, static_cast<uint32_t>(x), 8);
                else if (x < 16536u)
                {
                    const uint32_t d = static_cast<uint32_t>(x) - 152u;
                    or_bits(img, bp, (0x98u + (d >> 8)) | ((d & 0xFFu) << 8), 16);
                }
                else if (x < 2113688u)
                {
                    const uint32_t d = static_cast<uint32_t>(x) - 16536u;
                    or_bits(img, bp, (0xD8u + (d >> 16)) | ((d & 0xFFFFu) << 8), 24);
                }
                else
                {
                    const uint32_t nb = (bw64d(x) + 7u) >> 3;
                    or_bits(img, bp, 0xF8u + (nb - 3u), 8);
                    or_bits64(img, bp + 8u, x, 8u * nb);
                }
            }
            or_bits(img, (v0 + vtot + k) * 8u, t + 64u * j, 8);
        }
        carry += __builtin_amdgcn_readlane(incl, 63);
        before += rowc[j];
    }
}

} // namespace tpf::dev
