// p4_enc256v64.hip -- batch encode of 128v64 / 256v64 P4 blocks (p4Enc128v64,
// p4Enc256v64 and their D1 variants; reference
// src/scalar/p4enc128v64_scalar.cpp:51-224, p4enc256v64_scalar.cpp:15-30,
// p4d1enc256v64_scalar.cpp) on gfx950.
//
// Same three launches as the 256v32 encoder (p4_enc256v32.hip): plan (cost
// model + exact sizes) -> exclusive scan of unit sizes -> write.  A unit is
// one reference call: one 128v64 block (NB = 1) or the two 128v64 blocks of a
// 256v64 call (NB = 2).  Lane t owns values 2t, 2t+1 of each 128-value block:
// one 16-byte load per lane per block, the layout of k_dec128v64w.
// Each block is built in its own LDS image whose dword phase puts the base
// payload on a dword (a 256v64 unit's second block starts at an arbitrary
// byte), then copied out in whole 16-byte chunks, the chunk a block ends in
// carried into the next block of the run (RunCopyB, p4_enc32.h).
#include "p4_scan.h"

#include "p4_generic.h"
#include "tpf_kernels.h"

namespace tpf::dev
{

constexpr uint32_t kEnc64Run = 16;    // units per wave run
constexpr uint32_t kEnc64NC = 3;      // units in flight per wave
constexpr uint32_t kImg64U32 = 592;   // block image: 4..7 lead + block (<= 2150 B) + slack
constexpr uint32_t kVal64U32 = 128;   // staged low halves (b <= 32 base packing)
constexpr int kEnc64PolPlan = 2;      // plan pass value loads: nontemporal (+1.5-3%, r5s)

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t rl32w64(uint32_t v, uint32_t lane)
{
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(lane)));
}

struct Chunk64
{
    u32x4 a, b; // blocks 0 and 1 of the unit, lane t = values 2t, 2t+1
};

__device__ __forceinline__ void split2(const u32x4 & c, uint64_t & x0, uint64_t & x1)
{
    x0 = (static_cast<uint64_t>(c.y) << 32) | c.x;
    x1 = (static_cast<uint64_t>(c.w) << 32) | c.z;
}

// deltaEnc1 (p4_scalar_internal.h:711-719) over one 128-value block:
// d[e] = x[e] - x[e-1] - 1 with x[-1] = prev.
__device__ __forceinline__ void delta_encode64(uint64_t & x0, uint64_t & x1, uint64_t prev, uint32_t t)
{
    // x1 of lane t-1, lane 0: prev (two DPP wave_shr:1, no ds_bpermute)
    const uint64_t p = (static_cast<uint64_t>(wave_shr1(static_cast<uint32_t>(x1 >> 32), static_cast<uint32_t>(prev >> 32))) << 32) |
                       wave_shr1(static_cast<uint32_t>(x1), static_cast<uint32_t>(prev));
    (void)t;
    const uint64_t d0 = x0 - p - 1u, d1 = x1 - x0 - 1u;
    x0 = d0;
    x1 = d1;
}

// Plan word of one block: b | bx << 7 | xn << 14 | raw << 22 (23 bits).
__device__ __forceinline__ uint32_t plan64_word(const PlanG & P) { return P.b | (P.bx << 7) | (P.xn << 14) | (P.raw << 22); }

__device__ __forceinline__ PlanG plan_block128v64(uint64_t x0, uint64_t x1, uint32_t * hist, uint32_t t)
{
    const uint64_t v[4] = {x0, x1, 0ull, 0ull}; // element order is irrelevant to the cost model
    return plan_block_g<Fmt::V128X64>(v, 128u, hist, t);
}

// OR a lane's one or two consecutive nb-bit values a, b (b = 0 for one;
// both < 2^nb, 1 <= nb <= 64) into the image's bit stream at `bit` (five
// dwords at most).  No branches (round 4, as or_run in p4_enc32.h): the pair
// as 128 bits (b shifted by nb in two steps so that 64 shifts it out), the
// lane's bit offset applied with 64-bit shifts, a wave-uniform store bound.
__device__ __forceinline__ void or_pair64(uint32_t * img, uint32_t bit, uint64_t a, uint64_t b, uint32_t nb)
{
    const uint64_t lo = a | ((b << (nb - 1u)) << 1);
    const uint64_t hi = b >> (64u - nb);
    const uint32_t sh = bit & 31u, q = bit >> 5;
    uint32_t w[5];
    w[0] = static_cast<uint32_t>(lo) << sh;
    w[1] = static_cast<uint32_t>((lo << sh) >> 32);
    w[2] = static_cast<uint32_t>((((hi << 32) | (lo >> 32)) << sh) >> 32);
    w[3] = static_cast<uint32_t>((hi << sh) >> 32);
    w[4] = static_cast<uint32_t>(((hi >> 32) << sh) >> 32);
    const uint32_t maxw = (62u + 2u * nb) >> 5;
#pragma unroll
    for (uint32_t i = 0; i < 5; ++i)
        if (i < maxw)
            atomicOr(&img[q + i], w[i]);
}

// or_pair64 with the store count decided by nested wave-uniform tests of nb
// ((62 + 2 nb) >> 5 dwords at most; round 6: the unrolled `i < maxw` bound
// compiled into four compares per call)
__device__ __forceinline__ void or_pair64n(uint32_t * img, uint32_t bit, uint64_t a, uint64_t b, uint32_t nb)
{
    const uint64_t lo = a | ((b << (nb - 1u)) << 1);
    const uint64_t hi = b >> (64u - nb);
    const uint32_t sh = bit & 31u, q = bit >> 5;
    atomicOr(&img[q], static_cast<uint32_t>(lo) << sh);
    atomicOr(&img[q + 1u], static_cast<uint32_t>((lo << sh) >> 32));
    if (nb > 1u)
    {
        atomicOr(&img[q + 2u], static_cast<uint32_t>((((hi << 32) | (lo >> 32)) << sh) >> 32));
        if (nb > 17u)
        {
            atomicOr(&img[q + 3u], static_cast<uint32_t>((hi << sh) >> 32));
            if (nb > 33u)
                atomicOr(&img[q + 4u], static_cast<uint32_t>(((hi >> 32) << sh) >> 32));
        }
    }
}

// Layout of one 128v64 block from its plan word (plan64_word), size, output
// byte rel (relative to the run's 16-byte aligned output base) and the run's
// lead (round 6, as enc_geo in p4_enc32.h): bh = the header's width (64 is
// stored as 63), sb / pw = image byte of the block / dword of its base
// payload, hdr = header bytes 0 | 1 << 8, v0 = the vbyte area.
struct EncGeo64
{
    uint32_t b, bh, bx, xn, raw, sb, pw, hdr, v0;
    CopyGeo c;
};

__device__ __forceinline__ EncGeo64 enc_geo64(uint32_t w, uint32_t size, uint32_t rel, uint32_t lead)
{
    EncGeo64 G;
    G.b = w & 0x7Fu;
    G.bx = (w >> 7) & 0x7Fu;
    G.xn = (w >> 14) & 0xFFu;
    G.raw = (w >> 22) & 1u;
    G.bh = G.b >= 64u ? 63u : G.b;
    const bool bmp = G.bx != 0u && G.bx <= 64u, cst = G.bx == 66u;
    const uint32_t xbytes = bmp ? ((G.xn * G.bx + 7u) >> 3) : 0u;
    const uint32_t po = G.bx == 0u ? 1u : (bmp ? 18u + xbytes : 2u); // payload offset in the block
    G.sb = cst ? kImgLead : kImgLead + ((4u - (po & 3u)) & 3u);
    G.pw = (G.sb + po) >> 2;
    G.hdr = G.bx == 0u ? G.bh : (bmp ? ((0x80u | G.bh) | (G.bx << 8)) : (cst ? (0xC0u | G.bh) : ((0x40u | G.bh) | (G.xn << 8))));
    G.v0 = G.sb + 2u + 16u * G.b;
    G.c = copy_geo(G.sb, size, rel, lead, kImg64U32);
    return G;
}

// Build one 128v64 block (p4Enc128v64 = writeHeader64 + p4Enc128v64Payload)
// in the zeroed image from its layout G.  Round 6: the header, constant,
// bitmap and raw-marker bytes are stored from every lane (unowned lanes to
// their scratch bytes), not in single-lane exec-mask sections.
__device__ __forceinline__ void emit_block128v64_g(uint32_t * img, uint32_t * val, const EncGeo64 & G, uint64_t x0, uint64_t x1,
                                                   uint32_t t)
{
    uint8_t * const ib = reinterpret_cast<uint8_t *>(img);
    const uint32_t b = G.b;
    const uint32_t trash_at = static_cast<uint32_t>(reinterpret_cast<uint8_t *>(val + 2u * t) - ib);
    auto put = [&](bool own, uint32_t at, uint32_t k, uint32_t byte) {
        ib[__builtin_unpredictable(own) ? at : trash_at + (k & 7u)] = static_cast<uint8_t>(byte);
    };
    if (G.bx == 66u)
    {
        // constant block: header, ceil(b/8) bytes of element 0
        const uint64_t c = readlane_u64(x0, 0) & mask64d(b);
        put(t <= ((b + 7u) >> 3), kImgLead + t, 0u, t == 0u ? G.hdr : static_cast<uint32_t>(c >> (8u * ((t - 1u) & 7u))));
        return;
    }
    const uint32_t sb = G.sb, pw = G.pw;
    const uint64_t m = mask64d(b);
    const uint64_t m0 = x0 & m, m1 = x1 & m;
    const uint32_t f0 = x0 > m, f1 = x1 > m;
    // header bytes 0 and 1 from lanes 0 and 1 (a plain block's byte 1 is a
    // payload byte: 0 here, OR-ed below)
    put(t < 2u, sb + t, 0u, G.hdr >> (8u * (t & 1u)));
    // base payload (bitpack128v64Scalar, bitpack128v64_scalar.cpp:38-104)
    if (b != 0u && b <= 32u)
    {
        // 128v32 layout of the pair-swapped low halves: column l, group g holds
        // element (4g + l) ^ 2.  Lane t < 32 ORs a run of groups 4r..4r+3 of
        // column l = t >> 3 (so at most 8 lanes share a dword).
        reinterpret_cast<uint64_t *>(val)[t] = (static_cast<uint64_t>(static_cast<uint32_t>(m1)) << 32) | static_cast<uint32_t>(m0);
        wave_lds_sync();
        if (t < 32u)
        {
            const uint32_t l = t >> 3, r = t & 7u;
            uint32_t x[4];
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i)
                x[i] = val[(4u * (4u * r + i) + l) ^ 2u];
            or_run4(img, pw + l, 4u, 4u * r * b, x, b);
        }
        wave_lds_sync(); // val is scratch below
    }
    else if (b > 32u)
    {
        // horizontal 64-bit stream: values 2t, 2t+1 are consecutive
        or_pair64n(img, pw * 32u + 2u * t * b, m0, m1, b);
    }
    if (G.bx == 0u)
        return;
    const uint64_t B0 = __ballot(f0), B1 = __ballot(f1);
    const uint32_t cnt = f0 + f1;
    const uint32_t before = static_cast<uint32_t>(__builtin_popcountll(B0 & lanemask_lt()) + __builtin_popcountll(B1 & lanemask_lt()));
    const uint64_t e0 = b >= 64u ? 0ull : (x0 >> b), e1 = b >= 64u ? 0ull : (x1 >> b);
    if (G.bx <= 64u)
    {
        // [0x80|b][bx][bitmap 16 B][xn * bx bits][base]: bitmap byte k holds
        // elements 8k..8k+7, i.e. lanes 4k..4k+3 (x0 on even bits, x1 on odd)
        const uint32_t k = t & 15u;
        uint32_t n0 = static_cast<uint32_t>(B0 >> (4u * k)) & 15u, n1 = static_cast<uint32_t>(B1 >> (4u * k)) & 15u;
        n0 = (n0 | (n0 << 2)) & 0x33u;
        n0 = (n0 | (n0 << 1)) & 0x55u;
        n1 = (n1 | (n1 << 2)) & 0x33u;
        n1 = (n1 | (n1 << 1)) & 0x55u;
        put(t < 16u, sb + 2u + k, 0u, n0 | (n1 << 1));
        const uint64_t mx = mask64d(G.bx);
        if (cnt != 0u) // lanes without exceptions share `before` with a neighbour: no zero ORs
            or_pair64n(img, (sb + 18u) * 8u + before * G.bx, (f0 ? e0 : e1) & mx, cnt > 1u ? (e1 & mx) : 0ull, G.bx);
        return;
    }
    // vbyte: [0x40|b][xn][base 16b][V][positions]
    const uint32_t v0 = G.v0;
    if (G.raw)
    {
        // 0xFF, xn raw LE u64, xn position bytes
        const uint32_t a0 = v0 + 1u + 8u * before, a1 = a0 + 8u * f0;
#pragma unroll
        for (uint32_t k = 0; k < 8u; ++k)
        {
            put(f0, a0 + k, k, static_cast<uint32_t>(e0 >> (8u * k)));
            put(f1, a1 + k, k, static_cast<uint32_t>(e1 >> (8u * k)));
        }
        const uint32_t pp = v0 + 1u + 8u * G.xn + before;
        put(f0, pp, 0u, 2u * t);
        put(f1, pp + f0, 1u, 2u * t + 1u);
        put(t == 0u, v0, 2u, 0xFFu);
        return;
    }
    // vbPut64 (p4_scalar_internal.cpp:447-476): marker byte, then up to 8 bytes
    const uint32_t l0 = f0 ? vblen64(e0) : 0u, l1 = f1 ? vblen64(e1) : 0u;
    const uint32_t lincl = wave_incl_scan(l0 + l1);
    const uint32_t vtot = __builtin_amdgcn_readlane(lincl, 63);
    const uint32_t pos = v0 + lincl - l0 - l1;
    auto vbput = [&](bool own, uint32_t at, uint64_t x, uint32_t L) {
        const bool g1 = x >= 152u, g2 = x >= 16536u, g3 = x >= 2113688u;
        const uint32_t d2 = static_cast<uint32_t>(x) - 152u, d3 = static_cast<uint32_t>(x) - 16536u;
        const uint32_t mk3 = 0xF8u + (L - 1u) - 3u;
        const uint32_t mk12 = __builtin_unpredictable(g2) ? 0xD8u + (d3 >> 16) : 0x98u + (d2 >> 8);
        const uint32_t mk = __builtin_unpredictable(g3) ? mk3 : (__builtin_unpredictable(g1) ? mk12 : static_cast<uint32_t>(x));
        const uint64_t tail = __builtin_unpredictable(g3) ? x : (__builtin_unpredictable(g2) ? (d3 & 0xFFFFu) : (d2 & 0xFFu));
        put(own, at, 0u, mk);
#pragma unroll
        for (uint32_t k = 1; k < 9u; ++k)
            put(own && k < L, at + k, k, static_cast<uint32_t>(tail >> (8u * (k - 1u))));
    };
    vbput(f0, pos, e0, l0);
    vbput(f1, pos + l0, e1, l1);
    put(f0, v0 + vtot + before, 0u, 2u * t);
    put(f1, v0 + vtot + before + f0, 1u, 2u * t + 1u);
}

// A wave's run of up to kEnc64Run consecutive units (NB blocks of 128 u64);
// POL: cache policy of the value loads (buffer-load aux bits).
template <uint32_t NB, int POL = 0>
struct EncRun64
{
    uint64_t first;
    uint32_t n;
    __amdgpu_buffer_rsrc_t rs;

    __device__ __forceinline__ bool init(const uint64_t * in, uint64_t nunits, uint32_t wv)
    {
        first = (static_cast<uint64_t>(blockIdx.x) * 4u + wv) * kEnc64Run;
        if (first >= nunits)
            return false;
        n = static_cast<uint32_t>(min_u64(kEnc64Run, nunits - first));
        rs = make_rsrc(in + first * (128u * NB), n * 1024u * NB);
        return true;
    }

    __device__ __forceinline__ void load(Chunk64 & c, uint32_t jj, uint32_t t) const
    {
        c.a = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(jj * 1024u * NB + 16u * t), 0, POL);
        if constexpr (NB == 2)
            c.b = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(jj * 2048u + 1024u + 16u * t), 0, POL);
    }

    // value preceding unit first+t (lanes t < n): the given starts, or for one
    // chained list the last value of the previous unit
    __device__ __forceinline__ uint64_t start_lane(const uint64_t * in, const uint64_t * starts, uint64_t start0, uint32_t t) const
    {
        if (t >= n)
            return 0ull;
        const uint64_t u = first + t;
        if (starts)
            return starts[u];
        return u == 0 ? start0 : in[u * (128u * NB) - 1u];
    }

    // body(chunk, jj) for jj = 0..n-1 with kEnc64NC units in flight
    template <class Body>
    __device__ __forceinline__ void walk(uint32_t t, Body && body) const
    {
        Chunk64 C[kEnc64NC];
#pragma unroll
        for (uint32_t u = 0; u + 1 < kEnc64NC; ++u)
            load(C[u], u, t);
        bool more = true;
        for (uint32_t j = 0; more; j += kEnc64NC)
        {
#pragma unroll
            for (uint32_t u = 0; u < kEnc64NC; ++u)
            {
                if (more)
                {
                    load(C[(u + kEnc64NC - 1) % kEnc64NC], j + u + kEnc64NC - 1, t);
                    body(C[u], j + u);
                    more = j + u + 1 < n;
                }
            }
        }
    }
};

// The unit's blocks as (x0, x1) pairs after optional delta coding.
template <uint32_t NB, bool D1>
__device__ __forceinline__ void unit_values(const Chunk64 & c, uint64_t start, uint32_t t, uint64_t (&x)[2][2])
{
    split2(c.a, x[0][0], x[0][1]);
    if constexpr (NB == 2)
        split2(c.b, x[1][0], x[1][1]);
    if constexpr (D1)
    {
        const uint64_t last0 = readlane_u64(x[0][1], 63); // element 127, before coding
        delta_encode64(x[0][0], x[0][1], start, t);
        if constexpr (NB == 2)
            delta_encode64(x[1][0], x[1][1], last0, t);
    }
}

template <uint32_t NB, bool D1>
__global__ __launch_bounds__(256) void k_enc128v64_plan(const uint64_t * __restrict in, uint64_t nunits,
                                                        const uint64_t * __restrict starts, uint64_t start0,
                                                        uint64_t * __restrict sizes, uint64_t * __restrict plan,
                                                        uint32_t * __restrict run_tot)
{
    __shared__ __attribute__((aligned(16))) uint32_t hist[4][kPlanGHistU32];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    EncRun64<NB, kEnc64PolPlan> R;
    if (!R.init(in, nunits, wv))
        return;
    const uint64_t stv = D1 ? R.start_lane(in, starts, start0, t) : 0ull;
    uint32_t szv = 0u;
    uint64_t pwv = 0ull; // lane j: unit first+j
    R.walk(t, [&](const Chunk64 & c, uint32_t jj) {
        uint64_t x[2][2];
        unit_values<NB, D1>(c, D1 ? readlane_u64(stv, jj) : 0ull, t, x);
        const PlanG P0 = plan_block128v64(x[0][0], x[0][1], hist[wv], t);
        uint32_t size = P0.size;
        uint64_t w = plan64_word(P0);
        if constexpr (NB == 2)
        {
            const PlanG P1 = plan_block128v64(x[1][0], x[1][1], hist[wv], t);
            size += P1.size;
            w |= (static_cast<uint64_t>(plan64_word(P1)) << 23) | (static_cast<uint64_t>(P0.size) << 46);
        }
        szv = t == jj ? size : szv;
        pwv = t == jj ? w : pwv;
    });
    if (t < R.n)
    {
        sizes[R.first + t] = szv;
        plan[R.first + t] = pwv;
    }
    publish_run_total(run_tot, R.first / kEnc64Run, t < R.n ? szv : 0u, t);
}

template <uint32_t NB, bool D1>
__global__ __launch_bounds__(256) void k_enc128v64_write(const uint64_t * __restrict in, uint64_t nunits,
                                                         const uint64_t * __restrict starts, uint64_t start0,
                                                         uint64_t * __restrict off, const uint64_t * __restrict plan,
                                                         const uint64_t * __restrict run_pre, const uint64_t * __restrict run_tile,
                                                         uint8_t * __restrict out, uint64_t out_cap)
{
    __shared__ __attribute__((aligned(16))) uint32_t img_all[4][kImg64U32];
    __shared__ __attribute__((aligned(16))) uint32_t val_all[4][kVal64U32];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t * img = img_all[wv];
    EncRun64<NB> R;
    if (!R.init(in, nunits, wv))
        return;
    const uint64_t stv = D1 ? R.start_lane(in, starts, start0, t) : 0ull;
    uint64_t ov, ev;
    run_offsets(off, R.first, R.n, run_base(run_pre, run_tile, R.first / kEnc64Run), t, ov, ev);
    const uint32_t szv = static_cast<uint32_t>(ev - ov);
    const uint64_t pwv = t < R.n ? plan[R.first + t] : 0ull;
    const uint64_t out_base = reinterpret_cast<uint64_t>(out);
    (void)out_cap; // tpf_enc_batch requires out_cap >= tpf_enc_bound: no chunk passes the stream's end
    zero_image(img, kImg64U32 / 4u, t);
    wave_lds_sync();
    // the run's output through one descriptor based at its first byte rounded
    // down to 16, 32-bit offsets (RunCopyB, p4_enc32.h; round 6)
    const uint64_t ab = out_base + ov;
    const uint64_t A = readlane_u64(ab, 0) & ~15ull;
    const uint32_t rel = static_cast<uint32_t>(ab - A);
    const uint32_t lead = rl32w64(rel, 0); // < 16
    const uint32_t rel_end = rl32w64(rel + szv, R.n - 1u);
    RunCopyB rc;
    rc.rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(A), static_cast<short>(0), static_cast<int>(rel_end), 0x00020000);
    uint32_t * const val = val_all[wv];
    const uint32_t trash_at = static_cast<uint32_t>(reinterpret_cast<uint8_t *>(val + 2u * t) - reinterpret_cast<uint8_t *>(img));
    R.walk(t, [&](const Chunk64 & c, uint32_t jj) {
        uint64_t x[2][2];
        unit_values<NB, D1>(c, D1 ? readlane_u64(stv, jj) : 0ull, t, x);
        const uint32_t urel = rl32w64(rel, jj), usize = rl32w64(szv, jj);
        const uint64_t w = readlane_u64(pwv, jj);
        const uint32_t size0 = NB == 2 ? static_cast<uint32_t>(w >> 46) : usize;
#pragma unroll
        for (uint32_t u = 0; u < NB; ++u)
        {
            const uint32_t size = u == 0 ? size0 : usize - size0;
            const uint32_t brel = urel + (u == 0 ? 0u : size0);
            const EncGeo64 G = enc_geo64(static_cast<uint32_t>(w >> (23u * u)) & 0x7FFFFFu, size, brel, lead);
            emit_block128v64_g(img, val, G, x[u][0], x[u][1], t);
            wave_lds_sync();
            // the block that completes the run's partial first chunk stores its bytes [lead, 16)
            rc.put(img, G.c, lead != 0u && brel < 16u && brel + size >= 16u, lead, trash_at, t);
            wave_lds_sync();
            zero_image_n(img, G.c.n16, t); // only [0, sb + size) can be non-zero
            wave_lds_sync();
        }
    });
    rc.flush_tail(rel_end, lead, t);
}

} // namespace tpf::dev

namespace tpf
{

size_t enc128v64_workspace(uint64_t nunits)
{
    return ((nunits * 8u + 255u) & ~size_t(255)) + RunScanWs<uint64_t>::bytes((nunits + dev::kEnc64Run - 1u) / dev::kEnc64Run);
}

namespace
{
template <uint32_t NB, bool D1>
hipError_t enc64_launch(const uint64_t * in, uint64_t nunits, const uint64_t * starts, uint64_t start0, uint8_t * out,
                        uint64_t out_cap, uint64_t * off, void * ws, size_t ws_bytes, hipStream_t s)
{
    if (ws_bytes < enc128v64_workspace(nunits))
        return hipErrorInvalidValue;
    auto * plan = static_cast<uint64_t *>(ws);
    const size_t plan_bytes = (nunits * 8u + 255u) & ~size_t(255);
    const uint64_t nruns = (nunits + dev::kEnc64Run - 1u) / dev::kEnc64Run;
    const RunScanWs<uint64_t> rs = RunScanWs<uint64_t>::carve(static_cast<uint8_t *>(ws) + plan_bytes, nruns);
    const uint64_t per_wg = 4ull * dev::kEnc64Run;
    const uint32_t grid = static_cast<uint32_t>((nunits + per_wg - 1) / per_wg);
    hipLaunchKernelGGL((dev::k_enc128v64_plan<NB, D1>), dim3(grid), dim3(256), 0, s, in, nunits, starts, start0, off, plan, rs.tot);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return e;
    e = launch_run_scan_u64(rs.tot, nruns, rs.pre, rs.tile, off + nunits, s);
    if (e != hipSuccess)
        return e;
    hipLaunchKernelGGL((dev::k_enc128v64_write<NB, D1>), dim3(grid), dim3(256), 0, s, in, nunits, starts, start0, off, plan, rs.pre,
                       rs.tile, out, out_cap);
    return hipGetLastError();
}
} // namespace

hipError_t launch_enc128v64(uint32_t nb, const uint64_t * in, uint64_t nunits, bool d1, const uint64_t * starts, uint64_t start0,
                            uint8_t * out, uint64_t out_cap, uint64_t * off, void * ws, size_t ws_bytes, hipStream_t s)
{
    if (nunits == 0)
        return fill_u32(off, 0u, 2, s);
    if (nunits + 1 > 0x7FFFFFFFull)
        return hipErrorInvalidValue;
    if (nb == 2u)
        return d1 ? enc64_launch<2, true>(in, nunits, starts, start0, out, out_cap, off, ws, ws_bytes, s)
                  : enc64_launch<2, false>(in, nunits, starts, start0, out, out_cap, off, ws, ws_bytes, s);
    return d1 ? enc64_launch<1, true>(in, nunits, starts, start0, out, out_cap, off, ws, ws_bytes, s)
              : enc64_launch<1, false>(in, nunits, starts, start0, out, out_cap, off, ws, ws_bytes, s);
}

} // namespace tpf
