// p4_dec256v32.hip -- batch decode of 256v32 P4 blocks (p4Dec256v32 /
// p4D1Dec256v32, reference src/scalar/p4dec256v32_scalar.cpp:90-137 and
// p4d1dec256v32_scalar.cpp:198-268) on gfx950: the hot path.
//
// Design notes (measured on MI355X): a first version staged
// tiles of 8 consecutive blocks per workgroup with one coalesced sweep and
// __syncthreads; it was latency-bound (one tile in flight per workgroup,
// 39% of HBM peak).  The kernel below runs every wave independently with a
// software pipeline and no workgroup barrier.
#include "p4_dec_run.h"
#include "p4_dsum_lanes.h"
#include "tpf_kernels.h"

#include "p4_scan.h"

#ifndef TPF_DSUM_WINDOW
#define TPF_DSUM_WINDOW 16384
#endif

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
        blen = (e >= o && e - o < 0x10000ull) ? static_cast<uint32_t>(e - o) : 0xFFFFFFFFu;
        const uint64_t ab = in_base + o;
        ablo = static_cast<uint32_t>(ab);
        ng = 0u;
        for (uint32_t j = 0; j < n;)
        {
            const uint64_t cb = readlane_u64(ab, j) & ~15ull;
            const uint64_t fit = __ballot(valid && t >= j && e >= o && in_base + e <= cb + GB) >> j;
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

// Phase A of the chained decode (round 3): the block delta sums of 64-block
// runs, one lane per block (p4_dsum_lanes.h), one sum per run for the run
// scan.  A wave stages a run's bytes into its LDS window with coalesced
// 16-byte loads -- in passes of at most WB bytes starting at the first block
// not yet summed, each pass summing every block that lies wholly inside it --
// and the blocks the lane path declines go through the wave decoder one at a
// time.  Waves walk the runs grid-stride and load the NEXT pass (the same
// run's next window, or the next run's first) into registers while they sum
// the current one, so the loads of one pass overlap the arithmetic of the
// previous (measured without that overlap: staging alone 0.46 ms, staging +
// sums 1.30 ms per 10M C3 blocks).  Phase B's 16-block runs nest in the
// 64-block runs.
#ifdef TPF_DSUM_COUNT
__device__ unsigned long long g_dsum_count[2]; // blocks sent to the wave decoder, staging passes
#endif

// One 64-block run of phase A as lanes see it.
struct DsumRun
{
    uint64_t first = 0, o = 0, e = 0, rend = 0;
    uint32_t n = 0, len = 0;
    bool valid = false, fb = false, done = true;

    __device__ __forceinline__ void load(const DecArgs & A, uint64_t run, uint32_t t, uint32_t wb)
    {
        first = run * kLaneRun;
        n = static_cast<uint32_t>(min_u64(kLaneRun, A.nblocks - first));
        valid = t < n;
        o = valid ? A.off[first + t] : 0ull;
        e = valid ? A.off[first + t + 1u] : 0ull;
        len = (e >= o && e - o < 0x10000ull) ? static_cast<uint32_t>(e - o) : 0xFFFFFFFFu;
        // blocks larger than a window (or with implausible offsets) go to the wave decoder
        fb = valid && (len > wb - 32u || e > A.in_bytes);
        done = !valid || fb;
        // end of the run's bytes: a pass never stages past it, so neighbouring
        // runs do not re-read each other's bytes (offsets ascend in a valid stream)
        rend = readlane_u64(e, n - 1u);
    }
};

// The next staging pass of run R: [wbase, wbase + span) starting at the first
// block not yet summed (it always fits); false when every block is done.
template <uint32_t WB>
__device__ __forceinline__ bool dsum_pass(const DecArgs & A, const DsumRun & R, uint64_t & wbase, uint32_t & span, uint32_t & avail)
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

// Last LDS byte position dsum_lanes may clamp to: its widest read is 9
// dwords from a clamped position (base_sum_lanes, the raw-vbyte loop), and
// the wave's window holds (WB + 64) / 4 dwords, so clamped reads stay inside
// the wave's own window (WB + 40 let them run 3 dwords into the
// next wave's).  Valid blocks lie inside [0, WB) and never reach the clamp.
template <uint32_t WB>
constexpr uint32_t kDsumLim = WB + 28u;
static_assert(kDsumLim<16384u> / 4u + 9u <= (16384u + 64u) / 4u, "clamped phase-A reads stay in the wave's window");

#ifndef TPF_DSUM_WAVES
#define TPF_DSUM_WAVES 2
#endif
template <uint32_t WB>
__global__ __launch_bounds__(256, TPF_DSUM_WAVES) void k_dsum256v32_lanes(const DecArgs A)
{
    static_assert(WB % 1024u == 0u && WB + 64u >= kSlotBytes + 4u * kWaveScratchU32, "the window also hosts the fallback's slot and scratch");
    constexpr uint32_t NL = WB / 1024u; // 16-byte loads per lane per pass
    __shared__ uint32_t tab[33 * kSumTabRow];
    __shared__ __attribute__((aligned(16))) uint32_t win_all[4][(WB + 64u) / 4u];
    if (threadIdx.x < 33u)
        build_sum_row(tab + threadIdx.x * kSumTabRow, threadIdx.x);
    __syncthreads();
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint64_t nruns = (A.nblocks + kLaneRun - 1u) / kLaneRun;
    const uint64_t rstride = static_cast<uint64_t>(gridDim.x) * 4u;
    uint64_t run = static_cast<uint64_t>(blockIdx.x) * 4u + wv;
    if (run >= nruns)
        return;
    uint32_t * win = win_all[wv];
    const uint64_t in_base = reinterpret_cast<uint64_t>(A.in);
    const uint64_t in_end = in_base + A.in_bytes;

    // the pass in flight: its loads land in r[]
    u32x4 r[NL];
    uint64_t wbase = 0;
    uint32_t span = 0, avail = 0;
    auto issue = [&]() {
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(A.in + wbase, avail);
#pragma unroll
        for (uint32_t i = 0; i < NL; ++i)
        {
            // unconditional: chunks past the span get an out-of-range offset
            // (zeros, no traffic); a chunk straddling the end of the stream
            // reads zeros and is patched byte-wise when staged
            const uint32_t x = 16u * t + 1024u * i;
            r[i] = buf_load16(rs, x < span ? x : 0x80000000u);
        }
    };

    DsumRun cur;
    cur.load(A, run, t, WB);
    uint32_t sumv = 0u;
    dsum_pass<WB>(A, cur, wbase, span, avail); // the lead lane of a fresh run is pending or every lane declined
    issue();
    for (;;)
    {
        // ---- stage the pass in flight
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
                reinterpret_cast<u32x4 *>(win)[xs >> 4] =
                    load16_guarded(A.in + pbase, make_rsrc(A.in + pbase, avail), xs, avail);
        }
        wave_lds_sync();
#ifdef TPF_DSUM_COUNT
        if (t == 0)
            atomicAdd(&g_dsum_count[1], 1ull);
#endif
        const bool in_win = !cur.done && cur.o >= pbase && cur.e <= pbase + pspan;
        cur.done = cur.done || in_win;
        // ---- put the next pass in flight: the same run's next window, or the next run's first
        DsumRun nxt;
        bool run_end = false, last = false;
        if (!dsum_pass<WB>(A, cur, wbase, span, avail))
        {
            run_end = true;
            const uint64_t nrun = run + rstride;
            last = nrun >= nruns;
            if (!last)
            {
                nxt.load(A, nrun, t, WB);
                if (!dsum_pass<WB>(A, nxt, wbase, span, avail))
                    span = 0u; // every block of that run declined: nothing to stage
            }
            else
                span = 0u;
        }
        if (span != 0u)
            issue();
        // ---- sum the staged pass
        const uint32_t p = in_win ? static_cast<uint32_t>(cur.o - pbase) : 0u;
        uint32_t s = 0u;
#ifdef TPF_DSUM_STAGEONLY // measurement builds only (scripts/chain_phase_probe.py)
        const bool ok = true;
#else
        const bool ok = dsum_lanes<kDsumLim<WB>>(win, p, cur.len, in_win, tab, s);
#endif
        sumv = in_win ? s : sumv;
        cur.fb = cur.fb || (in_win && !ok);
        if (!run_end)
        {
            wave_lds_sync(); // the window is restaged next
            continue;
        }
        wave_lds_sync();
        // ---- the run is summed: the declined blocks, one at a time through
        // the wave decoder (exact: duplicate vbyte positions OR, as in the
        // reference, and the plain decode's length check); the next pass is in
        // registers, so the window is free
        uint64_t fbm = __ballot(cur.fb);
#ifdef TPF_DSUM_COUNT
        if (t == 0)
            atomicAdd(&g_dsum_count[0], static_cast<unsigned long long>(__builtin_popcountll(fbm)));
#endif
#ifdef TPF_DSUM_NOFB
        fbm = 0ull;
#endif
        uint64_t badmask = 0ull;
        uint32_t * slot = win;
        uint32_t * scr = win + kSlotBytes / 4u;
        while (fbm != 0ull)
        {
            const uint32_t j = static_cast<uint32_t>(__builtin_ctzll(fbm));
            fbm &= fbm - 1ull;
            const uint64_t ab = in_base + readlane_u64(cur.o, j);
            const uint64_t cb = ab & ~15ull;
            // the plain decode stages at most kSlotBytes - 64 bytes of a block (RunPlaneT)
            const uint32_t sp = static_cast<uint32_t>(min_u64(sub_sat(in_base + readlane_u64(cur.e, j), cb), kSlotBytes - 64u));
            const uint32_t av = static_cast<uint32_t>(min_u64(sub_sat(in_end, cb), kSlotBytes));
            const __amdgpu_buffer_rsrc_t rb = make_rsrc(reinterpret_cast<const void *>(cb), av);
            for (uint32_t x = 16u * t; x < sp; x += 1024u)
                reinterpret_cast<u32x4 *>(slot)[x >> 4] = load16_guarded(reinterpret_cast<const uint8_t *>(cb), rb, x, av);
            wave_lds_sync();
            const uint32_t sb = static_cast<uint32_t>(ab & 15u);
            u32x4 v;
            const uint32_t used = decode_block256v32(slot, sb, uni(lds_u32(slot, sb)), scr, t, v);
            const uint32_t sm = wave_sum(v.x + v.y + v.z + v.w + 4u);
            sumv = t == j ? sm : sumv;
            if (used != rl(cur.len, j))
                badmask |= 1ull << j;
            wave_lds_sync();
        }
        if (cur.valid)
            A.sums[cur.first + t] = sumv;
        publish_run_total(A.run_tot, cur.first / kLaneRun, cur.valid ? sumv : 0u, t);
        if (A.err != nullptr && t == 0 && badmask != 0ull)
            atomicMin(A.err, static_cast<unsigned long long>(cur.first + __builtin_ctzll(badmask)));
        if (last)
            break;
        run += rstride;
        cur = nxt;
        sumv = 0u;
        if (span == 0u)
        {
            // the new run has nothing to stage (all declined): an empty pass
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
// The measured best of the A/B knobs, fixed (no environment switch on the
// product path): "sc1 nt" output stores through a run descriptor (POL 8,
// round 2; non-temporal alone was POL 2), contiguous runs,
// one 16-byte load per lane per block with six blocks in flight (ONE / NC 6),
// 7 waves per SIMD.  (C2 899 -> 906, C3 1080 -> 1106 G int32/s vs two loads
// per block with three in flight)
// load / store cache policy of the decode (POL bits of ld16 / st16, p4_dec_run.h)
#ifndef TPF_DEC_POL
#define TPF_DEC_POL (2 | 8)
#endif
// Grouped loads (round 5: chosen per launch).  A stream of
// small blocks moves 1 KB GROUPS of consecutive blocks through the pipeline
// (GB = 1024) instead of one block per load: round 4's A/B per bit width
// (profiles/r4e_dec_groups.txt, 10M blocks each) had it 7% faster at 166-194
// B per block (bw 1-2), 2% at 252 B (bw 4), level at 367 B (bw 8) and 3-4%
// slower at 482-636 B (bw 12-17): two blocks sharing a window decode one after
// the other inside one pipeline slot.  So a launch whose blocks average under
// kGroupMeanBytes takes the grouped kernel, every other launch (C2's mix
// averages 607 B) the single-block pipeline.  Both are exact on any stream: a
// block larger than the window is a group of one.
constexpr uint64_t kGroupMeanBytes = 300;
template <dev::StartMode SM>
hipError_t launch_mode(const dev::DecArgs & A, hipStream_t stream)
{
    constexpr uint32_t run = dev::kRunDefault;
    constexpr uint64_t per_wg = 4ull * run;
    const uint32_t grid = static_cast<uint32_t>((A.nblocks + per_wg - 1) / per_wg);
    // (plain decode only: the delta-1 modes' grouped form spills at 7 waves/SIMD)
    if ((SM == dev::StartMode::None || SM == dev::StartMode::Probe) && A.in_bytes < kGroupMeanBytes * A.nblocks)
        hipLaunchKernelGGL((dev::k_dec256v32w<SM, run, TPF_DEC_POL, 6, 7, true, (SM == dev::StartMode::None || SM == dev::StartMode::Probe) ? 1024u : 0u>),
                           dim3(grid), dim3(256), 0, stream, A);
    else
        hipLaunchKernelGGL((dev::k_dec256v32w<SM, run, TPF_DEC_POL, 6, 7, true, 0>), dim3(grid), dim3(256), 0, stream, A);
    return hipGetLastError();
}
} // namespace

hipError_t launch_probe256v32(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t * out,
                              hipStream_t stream)
{
    if (nblocks == 0)
        return hipSuccess;
    const dev::DecArgs A{in, in_bytes, off, nblocks, out, nullptr, 0u, nullptr, nullptr};
    return launch_mode<dev::StartMode::Probe>(A, stream);
}

hipError_t launch_dec256v32(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t * out,
                            const uint32_t * starts, unsigned long long * err, hipStream_t stream)
{
    if (nblocks == 0)
        return hipSuccess;
    const dev::DecArgs A{in, in_bytes, off, nblocks, out, starts, 0u, nullptr, err};
    return starts ? launch_mode<dev::StartMode::PerBlock>(A, stream) : launch_mode<dev::StartMode::None>(A, stream);
}

// Chained delta-1: phase A computes every block's sum of
// (v+1) and one sum per 16-block wave run, the run sums are scanned
// (p4_scan.h, mod 2^32); phase B decodes with start(i) = base + the run's
// base + the sums of the run's blocks before i.  A shard of a multi-GPU list
// runs A, exchanges its total with the other ranks, then B with its base.
// Workspace: block sums (u32) + the run scan.
namespace
{
// workspace carve count (both phases carve the same layout; phase A scans
// only its nblocks / kSumRun run sums)
uint64_t chain_runs(uint64_t nblocks) { return (nblocks + dev::kRunDefault - 1u) / dev::kRunDefault; }
size_t al256(size_t x) { return (x + 255u) & ~size_t(255); }
} // namespace

// LDS staging window per wave of phase A (bytes)
constexpr uint32_t kDsumWindow = TPF_DSUM_WINDOW;
constexpr uint32_t kDsumWgPerCu = (160u * 1024u) / (4u * (kDsumWindow + 64u) + 33u * 64u);

size_t d1chain_workspace(uint64_t nblocks) { return al256(nblocks * 4u) + RunScanWs<uint32_t>::bytes(chain_runs(nblocks)); }

hipError_t launch_d1chain_sums(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, void * ws, size_t ws_bytes,
                               uint32_t * total, unsigned long long * err, hipStream_t stream)
{
    if (nblocks == 0)
        return total ? fill_u32(total, 0u, 1, stream) : hipSuccess;
    if (nblocks > 0x7FFFFFFFull || ws_bytes < d1chain_workspace(nblocks))
        return hipErrorInvalidValue;
    auto * sums = static_cast<uint32_t *>(ws);
    const RunScanWs<uint32_t> rs = RunScanWs<uint32_t>::carve(static_cast<uint8_t *>(ws) + al256(nblocks * 4u), chain_runs(nblocks));
    dev::DecArgs A{in, in_bytes, off, nblocks, nullptr, nullptr, 0u, sums, err};
    A.run_tot = rs.tot;
    // grid-stride over the runs: two workgroups per CU (the LDS windows admit two)
    constexpr uint64_t per_wg = 4ull * dev::kSumRun;
    const uint64_t wgs = std::min<uint64_t>((nblocks + per_wg - 1) / per_wg, grid_cap(stream, kDsumWgPerCu));
    hipLaunchKernelGGL((dev::k_dsum256v32_lanes<kDsumWindow>), dim3(static_cast<uint32_t>(wgs)), dim3(256), 0, stream, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return e;
    return launch_run_scan_u32(rs.tot, (nblocks + dev::kSumRun - 1u) / dev::kSumRun, rs.pre, rs.tile, total, stream);
}

hipError_t launch_d1chain_decode(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t * out,
                                 const void * ws, uint32_t base, unsigned long long * err, hipStream_t stream)
{
    if (nblocks == 0)
        return hipSuccess;
    const auto * sums = static_cast<const uint32_t *>(ws);
    const RunScanWs<uint32_t> rs =
        RunScanWs<uint32_t>::carve(const_cast<uint8_t *>(static_cast<const uint8_t *>(ws)) + al256(nblocks * 4u), chain_runs(nblocks));
    dev::DecArgs A{in, in_bytes, off, nblocks, out, sums, base, nullptr, err};
    A.run_pre = rs.pre;
    A.run_tile = rs.tile;
    return launch_mode<dev::StartMode::Prefix>(A, stream);
}

#ifdef TPF_DSUM_COUNT
extern "C" int tpf_dsum_counters(unsigned long long * out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(dev::g_dsum_count), 16) == hipSuccess ? 0 : 1;
}
#endif

} // namespace tpf
