// p4_dec256v64.hip -- launches of the 128v64 / 256v64 decode kernel
// (p4_dec256v64.h) and the chained 64-bit delta-1 decode: phase A one lane
// per unit (k_dsum128v64_lanes, p4_dsum64_lanes.h), the u64 run scan, phase B.
#include "p4_dec256v64.h"
#include "p4_dsum64_lanes.h"
#include "tpf_kernels.h"

namespace tpf::dev
{

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
static_assert(kDsum64Lim<16384u> / 4u + 6u <= (16384u + 64u) / 4u, "clamped phase-A reads stay in the wave's window");

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
        // unconditional (round 6, as k_dsum256v32_lanes): chunks past the
        // span hold the zeros their out-of-range loads returned
#pragma unroll
        for (uint32_t i = 0; i < NL; ++i)
            reinterpret_cast<u32x4 *>(win)[(16u * t + 1024u * i) >> 4] = r[i];
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

// Chained delta-1 decode of a 64-bit list (128v64 / 256v64 units chained the
// way reference callers chain p4D1Enc256v64, README.md:116-123; inside a
// 256v64 unit the second block already starts from the first's last value,
// p4d1dec256v64_scalar.cpp:15-32).  Phase A: every unit's delta total and one
// total per 16-unit run, then the run scan (u64, mod 2^64); phase B decodes
// with start(i) = base + the totals before i.
size_t d1chain64_workspace(uint64_t nunits) { return Chain64Ws::bytes(nunits); }

hipError_t launch_d1chain64_sums(uint32_t nb, const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nunits, void * ws,
                                 size_t ws_bytes, uint64_t * total, unsigned long long * err, hipStream_t s)
{
    if (nunits == 0)
        return total ? fill_u32(total, 0u, 2, s) : hipSuccess;
    if (ws_bytes < d1chain64_workspace(nunits))
        return hipErrorInvalidValue;
    const Chain64Ws w = Chain64Ws::carve(ws, nunits);
    dev::Dec64Args A{in, in_bytes, off, nunits, nullptr, nullptr, 0ull, w.sums, w.tot, nullptr, nullptr, err};
    // lane-per-unit phase A (round 4; the decoder's Sum mode before it:
    // 4.69 -> 1.53 ms per 10M units), grid-stride over 64-unit runs, two
    // workgroups per CU (the LDS windows admit two)
    constexpr uint64_t per_wg = 4ull * dev::kLaneRun64;
    const uint64_t wgs = std::min<uint64_t>((nunits + per_wg - 1) / per_wg, grid_cap(s, 2));
    if (nb == 2u)
        hipLaunchKernelGGL((dev::k_dsum128v64_lanes<2, 16384>), dim3(static_cast<uint32_t>(wgs)), dim3(256), 0, s, A);
    else
        hipLaunchKernelGGL((dev::k_dsum128v64_lanes<1, 16384>), dim3(static_cast<uint32_t>(wgs)), dim3(256), 0, s, A);
    hipError_t e = hipGetLastError();
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
