// p4_dec256v64.h -- the batch decode kernel of 128v64 / 256v64 P4 blocks (p4Dec128v64,
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
// Launched by the library (p4_dec256v64.hip) and, in its data-movement Probe
// mode only, by the measurement library (measure/tpf_measure.hip).
#pragma once

#include "p4_dec_run.h"
#include "p4_generic.h"
#include "p4_scan.h"

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
constexpr uint32_t kPos64 = 128;

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
    // every lane's pair total below 2^26 (posting lists: small gaps): the
    // 64-lane inclusive scan stays below 2^32, so one 32-bit DPP scan does
    // instead of the three of wave_incl_scan64 (wave-uniform test, round 5)
    const uint64_t incl = __builtin_amdgcn_ballot_w64(a1 >= (1ull << 26)) == 0ull
                              ? static_cast<uint64_t>(wave_incl_scan(static_cast<uint32_t>(a1)))
                              : wave_incl_scan64(a1);
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
//   (3 was Sum, the chained decode's first phase A: now k_dsum128v64_lanes)
//   Probe   measurement only: the same loads and stores with the decoding
//           removed (the 256v32 decoder's Probe mode), the data-movement
//           ceiling of the pipeline on a given stream
enum class Start64 : int
{
    None = 0,
    PerUnit = 1,
    Prefix = 2,
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
    uint64_t * sums;                  // phase A (k_dsum128v64_lanes): unit sums
    uint64_t * run_tot;               // phase A: one total per run
    const uint64_t * run_pre;         // Prefix: run scan
    const uint64_t * run_tile;        // Prefix: run scan
    unsigned long long * err;
};

constexpr uint32_t kRun64 = 16; // units per wave run (phase A publishes one total per 16 units)

// Pipeline: one 16-byte load per lane per unit (the 256v32 hot path's ONE
// layout: the rest of a unit larger than 1 KB is loaded at staging), kNC64
// units in flight, launch bounds for 6 waves per SIMD.  Round-4 A/B on C4
// (profiles/r4f_d64_time.log): ONE + 4 in flight + 6 waves 457 G int64/s,
// ONE + 6 in flight 456, 4 in flight alone 448, the earlier two loads per unit
// + 3 in flight + 4 waves 445.  Measured and not kept (profiles/r4w, r4y):
// "sc1 nt" output stores through a run descriptor (neutral), the first
// block's header from the load registers (level on C4, -0.5..-2% on C3
// 64-bit lists).
constexpr uint32_t kNC64 = 4;
template <uint32_t NB, Start64 SM>
__global__ __launch_bounds__(256, 6) void k_dec128v64w(const Dec64Args A)
{
    constexpr uint32_t kRun = kRun64, NC = kNC64;
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
    RunPlaneT<kSlot64, true> P;
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
    UsedLanes usedv;
    uint64_t * const out_run = out + first * (128u * NB);

    auto consume = [&](const Chunk & c, uint32_t jj) {
        if constexpr (SM == Start64::Probe)
        {
            // the unit's loads (the rest of a unit over 1 KB too), NB 1 KB stores
            typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
            const u32x4 a = c.a | P.big_rest_or(jj, t);
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
        uint32_t wbad = 0u;
#pragma unroll
        for (uint32_t u = 0; u < NB; ++u)
        {
            uint64_t x0, x1;
            const uint32_t used = decode_block128v64(slot, s, scr, t, x0, x1);
            s += used & ~kWidthBad; // a flagged first block: the second is still parsed in the slot
            wbad |= used & kWidthBad;
            if constexpr (D1)
                carry = delta1_128v64(x0, x1, carry);
            typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
            __builtin_nontemporal_store(u64x2{x0, x1}, reinterpret_cast<u64x2 *>(out_run + (jj * NB + u) * 128u) + t);
            wave_lds_sync();
        }
        usedv.put((s - s0) | wbad, jj, t);
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
    if constexpr (SM == Start64::Probe)
        return;
    const uint64_t badmask = usedv.bad(P.len, valid);
    if (err != nullptr && t == 0 && badmask != 0u)
        atomicMin(err, static_cast<unsigned long long>(first + __builtin_ctzll(badmask)));
}

} // namespace tpf::dev
