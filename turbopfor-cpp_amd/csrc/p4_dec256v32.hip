// p4_dec256v32.hip -- launches of the 256v32 decode kernel (p4_dec256v32.h)
// and the chained delta-1 decode: phase A
// (k_dsum256v32_lanes, p4_dsum_lanes.h), the run scan, phase B.
#include "p4_dec256v32.h"
#include "tpf_kernels.h"

#include "p4_scan.h"

// Phase-A ablation (measurement builds only, scripts/chain_phase_probe.py;
// the library is built with 0): TPF_DSUM_ABLATE bits 1 / 2 / 4 / 8 skip the
// base-payload sums / compressed vbyte / raw vbyte / position checks
// (p4_dsum_lanes.h), 16 stages only, 32 sends no block to the wave decoder,
// 64 counts the fallback blocks and staging passes (tpf_dsum_counters).
#ifndef TPF_DSUM_ABLATE
#define TPF_DSUM_ABLATE 0
#endif

namespace tpf::dev
{

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
#if TPF_DSUM_ABLATE & 64
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

template <uint32_t WB>
__global__ __launch_bounds__(256, 2) void k_dsum256v32_lanes(const DecArgs A)
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
        // unconditional (round 6): chunks past the span hold the zeros their
        // out-of-range loads returned, and no block summed from this pass
        // reaches them (a per-chunk test cost an exec-mask branch per chunk)
#pragma unroll
        for (uint32_t i = 0; i < NL; ++i)
            reinterpret_cast<u32x4 *>(win)[(16u * t + 1024u * i) >> 4] = r[i];
        {
            const uint32_t xs = avail & ~15u;
            if (xs < pspan && (avail & 15u) != 0u && t == ((xs >> 4) & 63u))
                reinterpret_cast<u32x4 *>(win)[xs >> 4] =
                    load16_guarded(A.in + pbase, make_rsrc(A.in + pbase, avail), xs, avail);
        }
        wave_lds_sync();
#if TPF_DSUM_ABLATE & 64
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
#if TPF_DSUM_ABLATE & 16
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
#if TPF_DSUM_ABLATE & 64
        if (t == 0)
            atomicAdd(&g_dsum_count[0], static_cast<unsigned long long>(__builtin_popcountll(fbm)));
#endif
#if TPF_DSUM_ABLATE & 32
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
template <dev::StartMode SM>
hipError_t launch_mode(const dev::DecArgs & A, hipStream_t stream)
{
    constexpr uint32_t run = dev::kRunDefault;
    constexpr uint64_t per_wg = 4ull * run;
    const uint32_t grid = static_cast<uint32_t>((A.nblocks + per_wg - 1) / per_wg);
    // (plain decode only: the delta-1 modes' grouped form spills at 7 waves/SIMD)
    using dev::kDecPol, dev::kDecNC, dev::kDecMinW;
    if (SM == dev::StartMode::None && dev::dec_grouped(A.in_bytes, A.nblocks))
        hipLaunchKernelGGL((dev::k_dec256v32w<SM, run, kDecPol, kDecNC, kDecMinW, true, SM == dev::StartMode::None ? 1024u : 0u>),
                           dim3(grid), dim3(256), 0, stream, A);
    else
        hipLaunchKernelGGL((dev::k_dec256v32w<SM, run, kDecPol, kDecNC, kDecMinW, true, 0>), dim3(grid), dim3(256), 0, stream, A);
    return hipGetLastError();
}
} // namespace

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
constexpr uint32_t kDsumWindow = 16384;
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

#if TPF_DSUM_ABLATE & 64
extern "C" int tpf_dsum_counters(unsigned long long * out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(dev::g_dsum_count), 16) == hipSuccess ? 0 : 1;
}
#endif

} // namespace tpf
