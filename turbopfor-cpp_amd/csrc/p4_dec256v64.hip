// p4_dec256v64.hip -- batch decode of 128v64 / 256v64 P4 blocks (p4Dec128v64,
// p4Dec256v64 and their D1 variants, reference
// src/scalar/p4d1dec128v64_scalar.cpp:157-375, p4d1dec256v64_scalar.cpp:15-49)
// on gfx950, with the run pipeline of the 256v32 hot path (p4_dec_run.h).
//
// A unit is one reference call: one 128v64 block (NB = 1) or the pair of
// 128v64 blocks of a 256v64 call (NB = 2); offsets are per unit, so the second
// block starts where the first one's parse ends.  Lane t owns the two
// consecutive values 2t, 2t+1 of each 128-value block and writes them with
// one 16-byte store (1 KB per block per wave, fully coalesced).
// Base payload (bitunpack128v64Scalar, bitpack128v64_scalar.cpp:78-104):
//   b <= 32: the 128v32 layout (4 interleaved lanes) of the pair-swapped low
//            halves, element e at 128v32 index e ^ 2.  Elements 2t and 2t+1
//            land in columns (t&1 ? 0 : 2) and +1 of group t>>1: one bit
//            offset, two adjacent dwords per 16-byte word group;
//   b >  32: a horizontal LSB-first 64-bit stream.
// Header b = 63 means 64 (p4_scalar_internal.cpp:645-649).
#include "p4_dec_run.h"
#include "p4_dsum64_lanes.h"
#include "p4_generic.h"
#include "p4_scan.h"
#include "tpf_kernels.h"

namespace tpf::dev
{

// Worst-case unit: two vbyte-mode blocks with raw escape (2 + 16*62 + 1 + 8*128
// + 128 = 2147 B each), staged from a 16-aligned chunk base.
constexpr uint32_t kSlot64 = 4352 + 64;

// Values 2t, 2t+1 of the 128v64 base payload at LDS byte p, width b.
__device__ __forceinline__ void unpack128v64_lane(const uint32_t * lds, uint32_t p, uint32_t b, uint32_t t, uint64_t & x0,
                                                  uint64_t & x1)
{
    if (b <= 32u)
    {
        const uint32_t o = (t >> 1) * b;
        const uint32_t pos = p + 16u * (o >> 5) + ((t & 1u) ? 0u : 8u);
        const uint32_t sh = o & 31u, m = p & 3u, q = pos >> 2;
        const uint32_t d0 = lds[q], d1 = lds[q + 1], d2 = lds[q + 2];
        const uint32_t e0 = lds[q + 4], e1 = lds[q + 5], e2 = lds[q + 6];
        const uint32_t msk = mask32(b);
        x0 = __builtin_amdgcn_alignbit(__builtin_amdgcn_alignbyte(e1, e0, m), __builtin_amdgcn_alignbyte(d1, d0, m), sh) & msk;
        x1 = __builtin_amdgcn_alignbit(__builtin_amdgcn_alignbyte(e2, e1, m), __builtin_amdgcn_alignbyte(d2, d1, m), sh) & msk;
    }
    else
    {
        const uint32_t bp = p * 8u + 2u * t * b;
        x0 = lds_bits64(lds, bp, b);
        x1 = lds_bits64(lds, bp + b, b);
    }
}

// vbyte scratch of a 128-value block: positions and exception counts < 128
// (round 4: 2 KB per wave instead of 4, one more workgroup per CU)
#ifndef TPF_D64_POS
#define TPF_D64_POS 128
#endif
constexpr uint32_t kPos64 = TPF_D64_POS;

// Decode one 128v64 block at LDS byte s into lane t's values 2t, 2t+1.
// Returns the consumed bytes (wave-uniform).  scr: 2 * kPos64 u64 per wave.
// hw: the block's first 4 bytes when the caller has them in registers
// (wave-uniform), ~0u to read them from LDS.
__device__ __forceinline__ uint32_t decode_block128v64(const uint32_t * lds, uint32_t s, uint64_t * scr, uint32_t t, uint64_t & x0,
                                                       uint64_t & x1, uint32_t hwin = ~0u)
{
    const uint32_t hw = hwin != ~0u ? hwin : uni(lds_u32(lds, s));
    const uint32_t h = hw & 0xFFu, x1b = (hw >> 8) & 0xFFu;
    if ((h & 0xC0u) == 0xC0u)
    {
        uint32_t b = h & 0x3Fu;
        if (b == 63u)
            b = 64u;
        const uint64_t c = lds_u64(lds, s + 1u) & mask64d(b);
        x0 = x1 = c;
        return 1u + ((b + 7u) >> 3);
    }
    if ((h & 0x40u) == 0u)
    {
        const uint32_t hdr = (h & 0x80u) ? 2u : 1u;
        const uint32_t bx = (h & 0x80u) ? min(x1b, 64u) : 0u;
        uint32_t b = h & 0x7Fu;
        if (b == 63u)
            b = 64u;
        const uint32_t bad = (b > 64u || ((h & 0x80u) && x1b > 64u)) ? kWidthBad : 0u;
        b = min(b, 64u);
        if (bx == 0u)
        {
            unpack128v64_lane(lds, s + hdr, b, t, x0, x1);
            return (hdr + 16u * b) | bad;
        }
        // 128-bit bitmap at s+2: lane t's bits 2t, 2t+1 sit in dword t>>4;
        // rank = popcount of the dwords before (lanes 0,16,32,48 each bring
        // one dword into a wave scan) + the bits below 2t in its own dword.
        const uint32_t w = lds_u32(lds, s + 2u + 4u * (t >> 4));
        const uint32_t sh = (2u * t) & 31u;
        const uint32_t my = (w >> sh) & 3u;
        const uint32_t pcd = __builtin_popcount(w);
        const uint32_t incl = wave_incl_scan((t & 15u) == 0u ? pcd : 0u);
        const uint32_t before = incl - pcd + __builtin_popcount(w & ((1u << sh) - 1u));
        const uint32_t xn = uni(__builtin_amdgcn_readlane(incl, 63));
        const uint32_t xs = s + 18u;
        const uint32_t xbytes = (xn * bx + 7u) >> 3;
        unpack128v64_lane(lds, xs + xbytes, b, t, x0, x1);
        const uint64_t ex0 = lds_bits64(lds, xs * 8u + before * bx, bx);
        const uint64_t ex1 = lds_bits64(lds, xs * 8u + (before + (my & 1u)) * bx, bx);
        x0 |= (my & 1u) ? shl64(ex0, b) : 0ull;
        x1 |= (my & 2u) ? shl64(ex1, b) : 0ull;
        return (18u + xbytes + 16u * b) | bad;
    }
    uint32_t b = h & 0x3Fu;
    if (b == 63u)
        b = 64u;
    unpack128v64_lane(lds, s + 2u, b, t, x0, x1);
    const uint32_t end = vbyte_exceptions_g<true, kPos64>(lds, s + 2u + 16u * b, x1b, scr, scr + kPos64, t);
    x0 |= shl64(scr[2u * t], b);
    x1 |= shl64(scr[2u * t + 1u], b);
    return end - s;
}

// Delta-1 over the block (applyDelta1 of p4D1Dec128v64): inclusive scan of
// v + 1 from start, mod 2^64.  Returns the block's last value.
__device__ __forceinline__ uint64_t delta1_128v64(uint64_t & x0, uint64_t & x1, uint64_t start)
{
    const uint64_t a0 = x0 + 1u, a1 = a0 + x1 + 1u;
    const uint64_t incl = wave_incl_scan64(a1);
    const uint64_t base = start + incl - a1;
    x0 = base + a0;
    x1 = base + a1;
    return start + readlane_u64(incl, 63);
}

// Start handling of a run (the 32-bit decoder's StartMode, p4_dec256v32.hip):
//   None    p4Dec128v64 / p4Dec256v64
//   PerUnit p4D1Dec*v64 with the start of unit i = starts[i]
//   Prefix  one chained list (round 4): start of unit i = base + the unit sums
//           before it (phase A below + the run scan, p4_scan.h), so a chained
//           list decodes with only its initial start
//   Sum     phase A of the chained decode: each unit's delta total
//           sum(v + 1) mod 2^64 (decoded, not stored) and one total per run
//   Probe   measurement only: the same loads and stores with the decoding
//           removed (the 256v32 decoder's Probe mode), the data-movement
//           ceiling of the pipeline on a given stream
enum class Start64 : int
{
    None = 0,
    PerUnit = 1,
    Prefix = 2,
    Sum = 3,
    Probe = 4,
};

struct Dec64Args
{
    const uint8_t * in;
    uint64_t in_bytes;
    const uint64_t * off;
    uint64_t nunits;
    uint64_t * out;
    const uint64_t * starts;          // PerUnit: starts; Prefix: phase A's unit sums
    uint64_t base;                    // Prefix: the value preceding unit 0
    uint64_t * sums;                  // Sum: unit sums
    uint64_t * run_tot;               // Sum: one total per run
    const uint64_t * run_pre;         // Prefix: run scan
    const uint64_t * run_tile;        // Prefix: run scan
    unsigned long long * err;
};

constexpr uint32_t kRun64 = 16; // units per wave run (both phases: a Prefix run is a Sum run)

// output store policy (A/B knob): 0 = nt, 1 = sc1 nt through a run descriptor
#ifndef TPF_D64_SC1NT
#define TPF_D64_SC1NT 0
#endif
template <uint32_t NB, Start64 SM>
// pipeline (A/B knobs): units in flight, one 16-byte load per lane per unit
// (the 256v32 hot path's ONE layout: the rest of a unit larger than 1 KB is
// loaded at staging) or two, and the waves per SIMD the launch bounds ask for.
// Round-4 A/B on C4 (profiles/r4f_d64_time.log): ONE + 4 in flight + 6 waves
// 457 G int64/s, ONE + 6 in flight 456, 4 in flight alone 448, the earlier
// TWO + 3 + 4 waves 445.
// first block's header from the load registers instead of LDS (A/B knob;
// round 4, profiles/r4y_d64_ab.txt: level on C4, -0.5..-2% on C3 64-bit lists)
#ifndef TPF_D64_HEAD
#define TPF_D64_HEAD 0
#endif
#ifndef TPF_D64_NC
#define TPF_D64_NC 4
#endif
#ifndef TPF_D64_ONE
#define TPF_D64_ONE 1
#endif
#ifndef TPF_D64_MINW
#define TPF_D64_MINW 6
#endif
__global__ __launch_bounds__(256, TPF_D64_MINW) void k_dec128v64w(const Dec64Args A)
{
    constexpr uint32_t kRun = kRun64, NC = TPF_D64_NC;
    constexpr bool D1 = SM == Start64::PerUnit || SM == Start64::Prefix;
    const uint8_t * in = A.in;
    const uint64_t in_bytes = A.in_bytes, nunits = A.nunits;
    const uint64_t * off = A.off;
    uint64_t * out = A.out;
    unsigned long long * err = A.err;
    __shared__ uint32_t slots[4][kSlot64 / 4];
    __shared__ __attribute__((aligned(16))) uint64_t scratch[4][2 * kPos64];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t * slot = slots[wv];
    uint64_t * scr = scratch[wv];
    const uint64_t in_base = reinterpret_cast<uint64_t>(in);
    const uint64_t first = (static_cast<uint64_t>(blockIdx.x) * 4u + wv) * kRun;
    if (first >= nunits)
        return;
    const uint32_t n = static_cast<uint32_t>(min_u64(kRun, nunits - first));

    const bool valid = t < n;
    const uint64_t unit = first + t;
    const uint64_t o = valid ? off[unit] : 0ull;
    const uint64_t e = valid ? off[unit + 1u] : 0ull;
    RunPlaneT<kSlot64, TPF_D64_ONE != 0> P;
    P.init(in_base, in_base + in_bytes, o, e, valid);
    uint64_t startv = 0ull;
    if constexpr (SM == Start64::PerUnit)
        startv = valid ? A.starts[unit] : 0ull;
    if constexpr (SM == Start64::Prefix)
    {
        // lane t: base + the run's base + the sums of the run's units before first+t
        const uint64_t sv = valid ? A.starts[unit] : 0ull;
        startv = A.base + run_base(A.run_pre, A.run_tile, first / kRun) + (wave_incl_scan64(sv) - sv);
    }
    uint64_t sumv = 0ull; // Sum: lane jj = unit first+jj's delta total
    UsedLanes usedv;
    uint64_t * const out_run = out + first * (128u * NB);
#if TPF_D64_SC1NT
    const __amdgpu_buffer_rsrc_t ors = make_rsrc(out_run, n * NB * 1024u);
#endif

    auto consume = [&](const Chunk & c, uint32_t jj) {
        if constexpr (SM == Start64::Probe)
        {
            // the unit's loads (the rest of a unit over 1 KB too), NB 1 KB stores
            typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
            const u32x4 a = c.a | (TPF_D64_ONE ? P.big_rest_or(jj, t) : c.b);
            const u64x2 x{(static_cast<uint64_t>(a.y) << 32) | a.x, (static_cast<uint64_t>(a.w) << 32) | a.z};
#pragma unroll
            for (uint32_t u = 0; u < NB; ++u)
                __builtin_nontemporal_store(x, reinterpret_cast<u64x2 *>(out_run + (jj * NB + u) * 128u) + t);
            return;
        }
        const uint32_t ctl = P.stage(c, jj, slot, t);
        uint32_t s = (ctl >> kCtlShift) & 15u;
        const uint32_t s0 = s;
        uint64_t carry = D1 ? readlane_u64(startv, jj) : 0ull;
        uint64_t usum = 0ull;
        uint32_t wbad = 0u;
#pragma unroll
        for (uint32_t u = 0; u < NB; ++u)
        {
            uint64_t x0, x1;
#if TPF_D64_HEAD
            // the first block's header from the load registers (the 256v32 path's head())
            const uint32_t used = decode_block128v64(slot, s, scr, t, x0, x1, u == 0 ? P.head(c, ctl, slot) : ~0u);
#else
            const uint32_t used = decode_block128v64(slot, s, scr, t, x0, x1);
#endif
            s += used & ~kWidthBad; // a flagged first block: the second is still parsed in the slot
            wbad |= used & kWidthBad;
            if constexpr (SM == Start64::Sum)
            {
                usum += readlane_u64(wave_incl_scan64(x0 + x1 + 2ull), 63);
                wave_lds_sync();
                continue;
            }
            if constexpr (D1)
                carry = delta1_128v64(x0, x1, carry);
#if TPF_D64_SC1NT
            // "sc1 nt" through the run's descriptor (the hot path's policy for whole 1 KB lines)
            st16_run(ors, (jj * NB + u) * 1024u + 16u * t,
                     u32x4{static_cast<uint32_t>(x0), static_cast<uint32_t>(x0 >> 32), static_cast<uint32_t>(x1), static_cast<uint32_t>(x1 >> 32)});
#else
            typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
            __builtin_nontemporal_store(u64x2{x0, x1}, reinterpret_cast<u64x2 *>(out_run + (jj * NB + u) * 128u) + t);
#endif
            wave_lds_sync();
        }
        usedv.put((s - s0) | wbad, jj, t);
        if constexpr (SM == Start64::Sum)
            sumv = t == jj ? usum : sumv;
    };

    Chunk C[NC];
#pragma unroll
    for (uint32_t u = 0; u + 1 < NC; ++u)
        P.template issue<0>(C[u], u, t);
    bool more = true;
    for (uint32_t j = 0; more; j += NC)
    {
#pragma unroll
        for (uint32_t u = 0; u < NC; ++u)
        {
            if (more)
            {
                P.template issue<0>(C[(u + NC - 1) % NC], j + u + NC - 1, t);
                consume(C[u], j + u);
                more = j + u + 1 < n;
            }
        }
    }
    if constexpr (SM == Start64::Sum)
    {
        if (valid)
            A.sums[unit] = sumv;
        const uint64_t rt = readlane_u64(wave_incl_scan64(valid ? sumv : 0ull), 63);
        if (t == 0)
            A.run_tot[first / kRun] = rt;
    }
    if constexpr (SM == Start64::Probe)
        return;
    const uint64_t badmask = usedv.bad(P.len, valid);
    if (err != nullptr && t == 0 && badmask != 0u)
        atomicMin(err, static_cast<unsigned long long>(first + __builtin_ctzll(badmask)));
}


// Phase A of the chained 64-bit decode, one LANE per unit (round 4,
// p4_dsum64_lanes.h): the 32-bit phase A's scheme (k_dsum256v32_lanes,
// p4_dec256v32.hip) -- a wave stages a 64-unit run's bytes into its LDS
// window with coalesced 16-byte loads, in passes of at most WB bytes from the
// first unit not yet summed, every lane sums its unit from LDS, and the units
// the lane path declines go through the wave decoder one at a time --
// writing each unit's u64 total and one total per 16-unit run (phase B's
// runs, k_dec128v64w<Prefix>) for the u64 run scan.
constexpr uint32_t kLaneRun64 = 64;

struct Dsum64Run
{
    uint64_t first = 0, o = 0, e = 0, rend = 0;
    uint32_t n = 0, len = 0;
    bool valid = false, fb = false, done = true;

    __device__ __forceinline__ void load(const Dec64Args & A, uint64_t run, uint32_t t, uint32_t wb)
    {
        first = run * kLaneRun64;
        n = static_cast<uint32_t>(min_u64(kLaneRun64, A.nunits - first));
        valid = t < n;
        o = valid ? A.off[first + t] : 0ull;
        e = valid ? A.off[first + t + 1u] : 0ull;
        len = (e >= o && e - o < 0x10000ull) ? static_cast<uint32_t>(e - o) : 0xFFFFFFFFu;
        fb = valid && (len > wb - 32u || e > A.in_bytes);
        done = !valid || fb;
        rend = readlane_u64(e, n - 1u);
    }
};

template <uint32_t WB>
__device__ __forceinline__ bool dsum64_pass(const Dec64Args & A, const Dsum64Run & R, uint64_t & wbase, uint32_t & span, uint32_t & avail)
{
    const uint64_t pend = __ballot(!R.done);
    if (pend == 0ull)
        return false;
    const uint32_t lead = static_cast<uint32_t>(__builtin_ctzll(pend));
    const uint64_t ws = readlane_u64(R.o, lead);
    const uint64_t we = readlane_u64(R.e, lead);
    wbase = ws & ~15ull;
    span = static_cast<uint32_t>(min_u64(wbase + WB, R.rend > we ? R.rend : we) - wbase);
    avail = static_cast<uint32_t>(min_u64(sub_sat(A.in_bytes, wbase), WB));
    return true;
}

// Sum over each 16-lane row (u64 mod 2^64), valid in the row's last lane:
// three 32-bit DPP row scans of 16-bit pieces and the high word.
__device__ __forceinline__ uint64_t row16_sum64(uint64_t x)
{
    auto rs = [](uint32_t v) {
        v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false); // row_shr:1
        v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false); // row_shr:2
        v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false); // row_shr:4
        v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false); // row_shr:8
        return v;
    };
    const uint32_t sh = rs(static_cast<uint32_t>(x >> 32));
    const uint32_t sm = rs(static_cast<uint32_t>(x >> 16) & 0xFFFFu);
    const uint32_t sl = rs(static_cast<uint32_t>(x) & 0xFFFFu);
    return (static_cast<uint64_t>(sh) << 32) + (static_cast<uint64_t>(sm) << 16) + sl;
}

template <uint32_t WB>
constexpr uint32_t kDsum64Lim = WB + 28u;
static_assert(kDsum64Lim<16384u> / 4u + 5u <= (16384u + 64u) / 4u, "clamped phase-A reads stay in the wave's window");

template <uint32_t NB, uint32_t WB>
__global__ __launch_bounds__(256, 2) void k_dsum128v64_lanes(const Dec64Args A)
{
    static_assert(WB % 1024u == 0u && WB + 64u >= kSlot64 + 16u * kPos64, "the window also hosts the fallback's slot and scratch");
    constexpr uint32_t NL = WB / 1024u;
    constexpr uint32_t LIM = kDsum64Lim<WB>;
    __shared__ uint32_t tab[33 * kSumTabRow];
    __shared__ __attribute__((aligned(16))) uint32_t win_all[4][(WB + 64u) / 4u];
    if (threadIdx.x < 33u)
        build_sum_row(tab + threadIdx.x * kSumTabRow, threadIdx.x);
    __syncthreads();
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint64_t nruns = (A.nunits + kLaneRun64 - 1u) / kLaneRun64;
    const uint64_t nruns16 = (A.nunits + kRun64 - 1u) / kRun64;
    const uint64_t rstride = static_cast<uint64_t>(gridDim.x) * 4u;
    uint64_t run = static_cast<uint64_t>(blockIdx.x) * 4u + wv;
    if (run >= nruns)
        return;
    uint32_t * win = win_all[wv];
    const uint64_t in_base = reinterpret_cast<uint64_t>(A.in);
    const uint64_t in_end = in_base + A.in_bytes;

    u32x4 r[NL];
    uint64_t wbase = 0;
    uint32_t span = 0, avail = 0;
    auto issue = [&]() {
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(A.in + wbase, avail);
#pragma unroll
        for (uint32_t i = 0; i < NL; ++i)
        {
            const uint32_t x = 16u * t + 1024u * i;
            r[i] = buf_load16(rs, x < span ? x : 0x80000000u);
        }
    };

    Dsum64Run cur;
    cur.load(A, run, t, WB);
    uint64_t sumv = 0ull;
    dsum64_pass<WB>(A, cur, wbase, span, avail);
    issue();
    for (;;)
    {
        const uint64_t pbase = wbase;
        const uint32_t pspan = span;
#pragma unroll
        for (uint32_t i = 0; i < NL; ++i)
        {
            const uint32_t x = 16u * t + 1024u * i;
            if (x < pspan)
                reinterpret_cast<u32x4 *>(win)[x >> 4] = r[i];
        }
        {
            const uint32_t xs = avail & ~15u;
            if (xs < pspan && (avail & 15u) != 0u && t == ((xs >> 4) & 63u))
                reinterpret_cast<u32x4 *>(win)[xs >> 4] = load16_guarded(A.in + pbase, make_rsrc(A.in + pbase, avail), xs, avail);
        }
        wave_lds_sync();
        const bool in_win = !cur.done && cur.o >= pbase && cur.e <= pbase + pspan;
        cur.done = cur.done || in_win;
        Dsum64Run nxt;
        bool run_end = false, last = false;
        if (!dsum64_pass<WB>(A, cur, wbase, span, avail))
        {
            run_end = true;
            const uint64_t nrun = run + rstride;
            last = nrun >= nruns;
            if (!last)
            {
                nxt.load(A, nrun, t, WB);
                if (!dsum64_pass<WB>(A, nxt, wbase, span, avail))
                    span = 0u;
            }
            else
                span = 0u;
        }
        if (span != 0u)
            issue();
        const uint32_t p = in_win ? static_cast<uint32_t>(cur.o - pbase) : 0u;
        uint64_t s = 0ull;
        const bool ok = dsum64_lanes<NB, LIM>(win, p, cur.len, in_win, tab, s);
        sumv = in_win ? s : sumv;
        cur.fb = cur.fb || (in_win && !ok);
        if (!run_end)
        {
            wave_lds_sync();
            continue;
        }
        wave_lds_sync();
        // declined units, one at a time through the wave decoder (exact)
        uint64_t fbm = __ballot(cur.fb);
        uint64_t badmask = 0ull;
        uint32_t * slot = win;
        uint64_t * scr = reinterpret_cast<uint64_t *>(win + kSlot64 / 4u);
        while (fbm != 0ull)
        {
            const uint32_t j = static_cast<uint32_t>(__builtin_ctzll(fbm));
            fbm &= fbm - 1ull;
            const uint64_t ab = in_base + readlane_u64(cur.o, j);
            const uint64_t cb = ab & ~15ull;
            const uint32_t sp = static_cast<uint32_t>(min_u64(sub_sat(in_base + readlane_u64(cur.e, j), cb), kSlot64 - 64u));
            const uint32_t av = static_cast<uint32_t>(min_u64(sub_sat(in_end, cb), kSlot64));
            const __amdgpu_buffer_rsrc_t rb = make_rsrc(reinterpret_cast<const void *>(cb), av);
            for (uint32_t x = 16u * t; x < sp; x += 1024u)
                reinterpret_cast<u32x4 *>(slot)[x >> 4] = load16_guarded(reinterpret_cast<const uint8_t *>(cb), rb, x, av);
            wave_lds_sync();
            uint32_t sb = static_cast<uint32_t>(ab & 15u);
            const uint32_t s0 = sb;
            uint64_t usum = 0ull;
            uint32_t wbad = 0u;
#pragma unroll
            for (uint32_t u = 0; u < NB; ++u)
            {
                uint64_t x0, x1;
                const uint32_t used = decode_block128v64(slot, min(sb, kSlot64 - 64u), scr, t, x0, x1);
                sb += used & ~kWidthBad;
                wbad |= used & kWidthBad;
                usum += readlane_u64(wave_incl_scan64(x0 + x1 + 2ull), 63);
                wave_lds_sync();
            }
            sumv = t == j ? usum : sumv;
            if (((sb - s0) | wbad) != rl(cur.len, j))
                badmask |= 1ull << j;
            wave_lds_sync();
        }
        if (cur.valid)
            A.sums[cur.first + t] = sumv;
        // one total per 16-unit run (phase B's runs)
        const uint64_t rt = row16_sum64(cur.valid ? sumv : 0ull);
        const uint64_t r16 = cur.first / kRun64 + (t >> 4);
        if ((t & 15u) == 15u && r16 < nruns16)
            A.run_tot[r16] = rt;
        if (A.err != nullptr && t == 0 && badmask != 0ull)
            atomicMin(A.err, static_cast<unsigned long long>(cur.first + __builtin_ctzll(badmask)));
        if (last)
            break;
        run += rstride;
        cur = nxt;
        sumv = 0ull;
        if (span == 0u)
        {
            wbase = 0;
            avail = 0;
        }
    }
}

} // namespace tpf::dev

namespace tpf
{

namespace
{
template <dev::Start64 SM>
hipError_t launch64(uint32_t nb, const dev::Dec64Args & A, hipStream_t s)
{
    const uint32_t grid = static_cast<uint32_t>((A.nunits + 4u * dev::kRun64 - 1u) / (4u * dev::kRun64));
    if (nb == 2u)
        hipLaunchKernelGGL((dev::k_dec128v64w<2, SM>), dim3(grid), dim3(256), 0, s, A);
    else
        hipLaunchKernelGGL((dev::k_dec128v64w<1, SM>), dim3(grid), dim3(256), 0, s, A);
    return hipGetLastError();
}

uint64_t runs64(uint64_t nunits) { return (nunits + dev::kRun64 - 1u) / dev::kRun64; }
size_t al256(size_t x) { return (x + 255u) & ~size_t(255); }

// workspace of the chained decode: unit sums (u64), then the run scan over
// u64 run totals: totals, in-tile prefixes, tile totals
struct Chain64Ws
{
    uint64_t * sums, * tot, * pre, * tile;
    static size_t bytes(uint64_t nunits)
    {
        const uint64_t r = runs64(nunits);
        return al256(8u * nunits) + al256(8u * r) + al256(8u * r) + al256(8u * RunScanWs<uint64_t>::tiles(r)) + 256u;
    }
    static Chain64Ws carve(void * ws, uint64_t nunits)
    {
        const uint64_t r = runs64(nunits);
        auto * p = static_cast<uint8_t *>(ws);
        Chain64Ws w;
        w.sums = reinterpret_cast<uint64_t *>(p);
        p += al256(8u * nunits);
        w.tot = reinterpret_cast<uint64_t *>(p);
        p += al256(8u * r);
        w.pre = reinterpret_cast<uint64_t *>(p);
        p += al256(8u * r);
        w.tile = reinterpret_cast<uint64_t *>(p);
        return w;
    }
};
} // namespace

// fmt 128v64 (nb = 1) or 256v64 (nb = 2), n == 128 * nb values per unit.
hipError_t launch_dec128v64(uint32_t nb, const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nunits,
                            uint64_t * out, const uint64_t * starts, unsigned long long * err, hipStream_t s)
{
    if (nunits == 0)
        return hipSuccess;
    dev::Dec64Args A{in, in_bytes, off, nunits, out, starts, 0ull, nullptr, nullptr, nullptr, nullptr, err};
    return starts ? launch64<dev::Start64::PerUnit>(nb, A, s) : launch64<dev::Start64::None>(nb, A, s);
}

// Measurement only: k_dec128v64w's loads and stores without the decoding.
hipError_t launch_probe128v64(uint32_t nb, const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nunits, uint64_t * out,
                              hipStream_t s)
{
    if (nunits == 0)
        return hipSuccess;
    dev::Dec64Args A{in, in_bytes, off, nunits, out, nullptr, 0ull, nullptr, nullptr, nullptr, nullptr, nullptr};
    return launch64<dev::Start64::Probe>(nb, A, s);
}

// Chained delta-1 decode of a 64-bit list (128v64 / 256v64 units chained the
// way reference callers chain p4D1Enc256v64, README.md:116-123; inside a
// 256v64 unit the second block already starts from the first's last value,
// p4d1dec256v64_scalar.cpp:15-32).  Phase A: every unit's delta total and one
// total per 16-unit run, then the run scan (u64, mod 2^64); phase B decodes
// with start(i) = base + the totals before i.
size_t d1chain64_workspace(uint64_t nunits) { return Chain64Ws::bytes(nunits); }

// phase A: lane per unit (k_dsum128v64_lanes) or the decoder's Sum mode (A/B knob)
#ifndef TPF_D64_LANESUM
#define TPF_D64_LANESUM 1
#endif

hipError_t launch_d1chain64_sums(uint32_t nb, const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nunits, void * ws,
                                 size_t ws_bytes, uint64_t * total, unsigned long long * err, hipStream_t s)
{
    if (nunits == 0)
        return total ? fill_u32(total, 0u, 2, s) : hipSuccess;
    if (ws_bytes < d1chain64_workspace(nunits))
        return hipErrorInvalidValue;
    const Chain64Ws w = Chain64Ws::carve(ws, nunits);
    dev::Dec64Args A{in, in_bytes, off, nunits, nullptr, nullptr, 0ull, w.sums, w.tot, nullptr, nullptr, err};
#if TPF_D64_LANESUM
    // lane-per-unit phase A (round 4), grid-stride over 64-unit runs, two
    // workgroups per CU (the LDS windows admit two)
    constexpr uint64_t per_wg = 4ull * dev::kLaneRun64;
    const uint64_t wgs = std::min<uint64_t>((nunits + per_wg - 1) / per_wg, grid_cap(s, 2));
    if (nb == 2u)
        hipLaunchKernelGGL((dev::k_dsum128v64_lanes<2, 16384>), dim3(static_cast<uint32_t>(wgs)), dim3(256), 0, s, A);
    else
        hipLaunchKernelGGL((dev::k_dsum128v64_lanes<1, 16384>), dim3(static_cast<uint32_t>(wgs)), dim3(256), 0, s, A);
    hipError_t e = hipGetLastError();
#else
    hipError_t e = launch64<dev::Start64::Sum>(nb, A, s);
#endif
    if (e != hipSuccess)
        return e;
    return launch_run_scan_u64t(w.tot, runs64(nunits), w.pre, w.tile, total, s);
}

hipError_t launch_d1chain64_decode(uint32_t nb, const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nunits,
                                   uint64_t * out, const void * ws, uint64_t base, unsigned long long * err, hipStream_t s)
{
    if (nunits == 0)
        return hipSuccess;
    const Chain64Ws w = Chain64Ws::carve(const_cast<void *>(ws), nunits);
    dev::Dec64Args A{in, in_bytes, off, nunits, out, w.sums, base, nullptr, nullptr, w.pre, w.tile, err};
    return launch64<dev::Start64::Prefix>(nb, A, s);
}

} // namespace tpf
