// p4_dec256v32.h -- the 256v32 decode kernel (k_dec256v32w) of the hot path:
// p4Dec256v32 / p4D1Dec256v32 (reference src/scalar/p4dec256v32_scalar.cpp:
// 90-137 and p4d1dec256v32_scalar.cpp:198-268).  Launched by the library
// (p4_dec256v32.hip) and, in its data-movement Probe mode only, by the
// measurement library (measure/tpf_measure.hip).
//
// Design notes (measured on MI355X): a first version staged
// tiles of 8 consecutive blocks per workgroup with one coalesced sweep and
// __syncthreads; it was latency-bound (one tile in flight per workgroup,
// 39% of HBM peak).  The kernel below runs every wave independently with a
// software pipeline and no workgroup barrier.
#pragma once

#include "p4_dec_run.h"
#include "p4_dsum_lanes.h"
#include "p4_scan.h"

namespace tpf::dev
{

// blocks per run of the chained decode's phase A (k_dsum256v32_lanes): one
// run sum each for the run scan; phase B's 16-block runs nest in them
constexpr uint32_t kSumRun = kLaneRun;

enum class StartMode : int
{
    None = 0,     // p4Dec256v32
    PerBlock = 1, // p4D1Dec256v32, start of block i = starts[i]
    Prefix = 2,   // chained list: start of block i = base + sum of the block sums before i (run scan, p4_scan.h)
    // 3 was SumOnly (phase A of the chained decode): now k_dsum256v32_lanes
    Probe = 4,    // measurement only: same loads and stores, no decode (data-movement ceiling)
};

struct DecArgs
{
    const uint8_t * in;
    uint64_t in_bytes;
    const uint64_t * off;
    uint64_t nblocks;
    uint32_t * out;
    const uint32_t * starts; // PerBlock: starts; Prefix: the block sums of phase A
    uint32_t base;           // Prefix: value preceding block 0
    uint32_t * sums;         // k_dsum256v32w: block sums
    unsigned long long * err;
    uint32_t * run_tot = nullptr;        // k_dsum256v32w: one sum per wave run
    const uint32_t * run_pre = nullptr;  // Prefix: run scan (p4_scan.h)
    const uint32_t * run_tile = nullptr; // Prefix: run scan (p4_scan.h)
};

// ---------------------------------------------------------------------------
// Wave-independent kernel: every wave owns a private LDS slot and decodes a
// contiguous run of kRun blocks with a software pipeline: while block j is
// decoded, the bytes of the next NC-1 blocks are in flight.  Default launch
// (ONE): one unconditional 16-byte buffer load per lane per block (its first
// 1 KB; a bigger block's rest is loaded at staging), NC = 6; without ONE:
// two loads per block (a 2 KB window), NC = 3.  The NC register chunks
// rotate (loop unrolled by NC) so no in-flight load result is ever copied
// (a copy forces s_waitcnt vmcnt(0)).  No workgroup barriers at all.  The
// run's control plane lives in vector lanes (RunPlaneT, p4_dec_run.h).
// Measured and kept: runs of 16 (8: same, 32..62:
// -2..-5%), 7 waves/SIMD; ONE/NC=6 beat two loads/NC=3 by 1-2% (C2) and
// 2-6% (C3); deeper pipelines lose occupancy.
// GB != 0 (round 4; chosen per launch since round 5, launch_mode): the pipeline moves GROUPS of
// consecutive blocks whose bytes fit one GB-byte window from the first
// block's 16-aligned start (one ballot per group: block ends ascend) instead
// of single blocks, so a wave keeps ~NC KB of reads in flight whatever the
// block size (a 166-byte bw-1 block uses 11 of 64 lanes of its own load);
// a group of one block larger than the window takes the big-block path.
template <StartMode SM, uint32_t kRun, uint32_t POL = 2, uint32_t NC = 3, int MINW = 7, bool ONE = false, uint32_t GB = 0>
__global__ __launch_bounds__(256, MINW) void k_dec256v32w(const DecArgs A)
{
    __shared__ uint32_t slots[4][kSlotBytes / 4];
    __shared__ uint32_t scratch[4][kWaveScratchU32];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint64_t wg = blockIdx.x;
    uint32_t * slot = slots[wv];
    uint32_t * scr = scratch[wv];
    const uint64_t in_base = reinterpret_cast<uint64_t>(A.in);
    const uint64_t in_end = in_base + A.in_bytes;

    // POL bit 2: the workgroup's 4*kRun blocks are dealt to its waves
    // round-robin (block first + stride*j) instead of in contiguous runs.
    constexpr uint32_t stride = (POL & 4u) ? 4u : 1u;
    const uint64_t first = (POL & 4u) ? wg * 4u * kRun + wv : (wg * 4u + wv) * kRun;
    if (first >= A.nblocks)
        return;
    const uint32_t n = static_cast<uint32_t>(min_u64(kRun, (A.nblocks - first + stride - 1u) / stride));

    // ---- per-run control plane, lane j = block first+j ---------------------
    const bool valid = t < n;
    const uint64_t blk = first + stride * t;
    const uint64_t o = valid ? A.off[blk] : 0ull;
    const uint64_t e = valid ? A.off[blk + 1u] : 0ull;
    RunPlaneT<kSlotBytes, ONE> P;
    // groups (GB != 0): lane g = group g (first block, block count); the plane holds groups
    uint32_t gfb = 0u, gcnt = 0u, ng = n, blen = 0u, ablo = 0u;
    if constexpr (GB != 0u)
    {
        static_assert(ONE && stride == 1u && kRun <= 64u && GB <= 1024u, "groups: one load per lane, contiguous runs");
        blen = (e >= o && e <= A.in_bytes && e - o < 0x10000ull) ? static_cast<uint32_t>(e - o) : 0xFFFFFFFFu;
        const uint64_t ab = in_base + o;
        ablo = static_cast<uint32_t>(ab);
        ng = 0u;
        for (uint32_t j = 0; j < n;)
        {
            const uint64_t cb = readlane_u64(ab, j) & ~15ull;
            const uint64_t fit = __ballot(valid && t >= j && e >= o && e <= A.in_bytes && in_base + e <= cb + GB) >> j;
            uint32_t c = static_cast<uint32_t>(__builtin_ctzll(~fit)); // consecutive fitting blocks from j
            c = c == 0u ? 1u : c;                                      // a big (or implausible) block alone
            gfb = t == ng ? j : gfb;
            gcnt = t == ng ? c : gcnt;
            ++ng;
            j += c;
        }
        const bool gvalid = t < ng;
        const uint32_t l0 = gfb & 63u, l1 = (gfb + gcnt - 1u) & 63u;
        const uint64_t go = (static_cast<uint64_t>(static_cast<uint32_t>(__shfl(static_cast<int>(static_cast<uint32_t>(o >> 32)), static_cast<int>(l0), 64))) << 32)
                            | static_cast<uint32_t>(__shfl(static_cast<int>(static_cast<uint32_t>(o)), static_cast<int>(l0), 64));
        const uint64_t ge = (static_cast<uint64_t>(static_cast<uint32_t>(__shfl(static_cast<int>(static_cast<uint32_t>(e >> 32)), static_cast<int>(l1), 64))) << 32)
                            | static_cast<uint32_t>(__shfl(static_cast<int>(static_cast<uint32_t>(e)), static_cast<int>(l1), 64));
        P.init(in_base, in_end, gvalid ? go : 0ull, gvalid ? ge : 0ull, gvalid);
    }
    else
        P.init(in_base, in_end, o, e, valid);
    uint32_t startv = 0u;
    if constexpr (SM == StartMode::PerBlock)
        startv = valid ? A.starts[blk] : 0u;
    if constexpr (SM == StartMode::Prefix)
    {
        // base + the base of phase A's kSumRun-block run holding this one +
        // the sums of that run's blocks before each block (mod 2^32): lanes
        // 0..kSumRun-1 scan the run's block sums, lane t takes entry k + t
        static_assert(kSumRun % kRun == 0 && kSumRun <= 64 && (POL & 4u) == 0u, "prefix runs nest in phase A's runs");
        const uint64_t f = first / kSumRun * kSumRun;
        const uint32_t k = static_cast<uint32_t>(first - f);
        const uint32_t sv = (t < kSumRun && f + t < A.nblocks) ? A.starts[f + t] : 0u;
        const uint32_t ex = wave_incl_scan(sv) - sv;
        startv = A.base + run_base(A.run_pre, A.run_tile, first / kSumRun)
                 + static_cast<uint32_t>(__shfl(static_cast<int>(ex), static_cast<int>((k + t) & 63u), 64));
    }
    uint32_t * const out_run = A.out + first * 256u;
    // POL bit 3: the run's output through one buffer descriptor, stored
    // "sc1 nt" (streamed and not kept in the XCD's L2): 1-2.5% over nt alone
    // on every stream shape (scripts/dec_variants.hip)
    const __amdgpu_buffer_rsrc_t ors = make_rsrc(out_run, (POL & 8u) && out_run ? n * stride * 1024u : 0u);
    auto put = [&](uint32_t jj, const u32x4 & v) {
        if constexpr ((POL & 8u) != 0u)
            st16_run(ors, jj * stride * 1024u + 16u * t, v);
        else
            st16<POL>(reinterpret_cast<u32x4 *>(out_run + jj * stride * 256u) + t, v);
    };
    // per-block scalar length check: the lane-held form (UsedLanes) costs one
    // more VGPR, which at 7 waves/SIMD made the PerBlock/Prefix modes spill
    // (12 B/lane of scratch: C3 WRITE_SIZE +3%)
    uint64_t badmask = 0u;

    auto issue = [&](Chunk & c, uint32_t jj) { P.template issue<POL>(c, jj, t); };
    auto consume = [&](const Chunk & c, uint32_t jj) {
        if constexpr (GB != 0u)
        {
            // group jj: its blocks decoded one after another from the staged window
            const uint32_t fb = rl(gfb, jj), cnt = rl(gcnt, jj);
            if constexpr (SM == StartMode::Probe)
            {
                const u32x4 x = c.a | P.big_rest_or(jj, t);
                for (uint32_t k = 0; k < cnt; ++k)
                    put(fb + k, x);
                return;
            }
            P.stage(c, jj, slot, t);
            const uint32_t cblo = rl(P.cblo, jj);
            for (uint32_t k = 0; k < cnt; ++k)
            {
                const uint32_t b = fb + k;
                const uint32_t sb = rl(ablo, b) - cblo; // the block's start inside the window
                u32x4 v;
                const uint32_t used = decode_block256v32(slot, sb, uni(lds_u32(slot, sb)), scr, t, v);
                if constexpr (SM == StartMode::PerBlock || SM == StartMode::Prefix)
                    apply_delta1_256(v, rl(startv, b));
                put(b, v);
                wave_lds_sync();
                if (used != rl(blen, b))
                    badmask |= 1ull << b;
            }
            return;
        }
        if constexpr (SM == StartMode::Probe)
        {
            put(jj, ONE ? (c.a | P.big_rest_or(jj, t)) : (c.a | c.b));
            return;
        }
        const uint32_t ctl = P.stage(c, jj, slot, t);
        u32x4 v;
        const uint32_t used = decode_block256v32(slot, (ctl >> kCtlShift) & 15u, P.head(c, ctl, slot), scr, t, v);
        if constexpr (SM == StartMode::PerBlock || SM == StartMode::Prefix)
            apply_delta1_256(v, rl(startv, jj));
        put(jj, v);
        wave_lds_sync();
        if (used != rl(P.len, jj))
            badmask |= 1ull << jj;
    };

    // NC register chunks rotate (loop unrolled by NC, no copies): while block
    // j is decoded, blocks j+1 .. j+NC-1 are in flight.
    auto run_pass = [&]() {
        Chunk C[NC];
#pragma unroll
        for (uint32_t u = 0; u + 1 < NC; ++u)
            issue(C[u], u);
        bool more = true;
        for (uint32_t j = 0; more; j += NC)
        {
#pragma unroll
            for (uint32_t u = 0; u < NC; ++u)
            {
                if (more)
                {
                    issue(C[(u + NC - 1) % NC], j + u + NC - 1);
                    consume(C[u], j + u);
                    more = j + u + 1 < ng;
                }
            }
        }
    };
    run_pass();
    if (A.err != nullptr && t == 0 && badmask != 0u)
        atomicMin(A.err, static_cast<unsigned long long>(first + stride * __builtin_ctzll(badmask)));
}

// The launch configuration of the library (p4_dec256v32.hip), shared with
// the measurement library's Probe launch so the probe moves data exactly as
// the decoder does.  "sc1 nt" output stores through a run descriptor (POL 8,
// round 2; non-temporal alone was POL 2), one 16-byte load per lane per block
// with six blocks in flight, 7 waves per SIMD (C2 899 -> 906, C3 1080 -> 1106
// G int32/s vs two loads per block with three in flight).
constexpr uint32_t kDecPol = 2 | 8;
constexpr uint32_t kDecNC = 6;
constexpr int kDecMinW = 7;

// Grouped loads (round 5: chosen per launch).  A stream of
// small blocks moves 1 KB GROUPS of consecutive blocks through the pipeline
// (GB = 1024) instead of one block per load: round 4's A/B per bit width
// (profiles/r4e_dec_groups.txt, 10M blocks each) had it 7% faster at 166-194
// B per block (bw 1-2), 2% at 252 B (bw 4), level at 367 B (bw 8) and 3-4%
// slower at 482-636 B (bw 12-17): two blocks sharing a window decode one after
// the other inside one pipeline slot.  So a plain-decode launch whose blocks
// average under kGroupMeanBytes takes the grouped kernel, every other launch
// (C2's mix averages 607 B) the single-block pipeline.  Both are exact on any
// stream: a block larger than the window is a group of one.  (The delta-1
// modes keep the single-block pipeline: their grouped form spills at 7
// waves/SIMD.)
constexpr uint64_t kGroupMeanBytes = 300;
__host__ __device__ constexpr bool dec_grouped(uint64_t in_bytes, uint64_t nblocks) { return in_bytes < kGroupMeanBytes * nblocks; }

} // namespace tpf::dev
