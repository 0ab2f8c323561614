// p4_enc256v32.h -- the 256v32 two-pass encoder (p4Enc256v32 /
// p4D1Enc256v32, reference src/scalar/p4enc256v32_scalar.cpp:216-235 and
// p4d1enc256v32_scalar.cpp:7-15) on gfx950: device code and its launch
// sequence, shared by the library (p4_enc256v32.hip) and the measurement
// library (measure/tpf_measure.hip: the pass probes and forced paths).
//
// Four launches:
//   1. plan  : one wave per block evaluates p4Bits32 (parallel cost model,
//              p4_enc32.h) and the exact encoded size -> d_off[i], plan word,
//              and one byte total per 16-block wave run.
//   2,3. run scan (p4_scan.h): exclusive prefix of the run totals only (two
//              small kernels over 1/16 of the entries; a library device scan
//              over every block's size cost 0.08 ms per 10M blocks).
//   4. write : rebuilds its run's offsets (run base + wave scan of the
//              sizes) and writes them to d_off; one wave per block scatters
//              header, bitmap / exceptions / base payload / vbytes into a
//              zeroed LDS image whose dword phase matches the destination,
//              then streams it out with dword stores (byte stores only on the
//              two edge dwords shared with the neighbouring blocks).
// Both kernels walk runs of 16 consecutive blocks per wave with the values of
// the next two blocks in flight (the first version loaded one block per loop
// iteration and waited for it: 5.0 and 5.4 ms per 10M blocks, latency-bound).
//
// PROBE (measurement only, instantiated by measure/tpf_measure.hip -- the
// output is NOT a valid stream): 1 = plan kernel with the cost model replaced
// by a wave OR, 2 = write kernel copying the staged values instead of
// building blocks; same loads and stores, so they time each pass's
// data-movement ceiling (profiles/archive/r1/r1_v4_enc_probe.txt).
#pragma once

#include "p4_scan.h"

#include "p4_enc32.h"
#include "tpf_kernels.h"

namespace tpf::dev
{

constexpr uint32_t kImgU32 = kImgU32Max; // dwords per wave image: 4..7 lead + block (<= 2276 B) + slack, 16-B multiple
constexpr uint32_t kEncRun = 16;  // blocks per wave run (the workspace is sized for it)
// D1 encodes (posting lists: small blocks) run 32 blocks per wave: C3 D1
// encode +2%, while the plain C4 mix loses 0.8% with 32 (r5ab)
constexpr uint32_t kEncRunD1 = 32;
// value chunks in flight per wave (NC: blocks j+1 .. j+NC-1 while j is
// encoded).  Measured and not kept: 2 / 4 / 6 in flight, nt or
// sc1 value loads, nt interior stores, dword copy-out.
constexpr uint32_t kEncNCPlan = 3;
constexpr uint32_t kEncNCWrite = 3;

// deltaEnc1 (p4_scalar_internal.h:711-719): d[i] = in[i] - in[i-1] - 1, in[-1] = start.
__device__ __forceinline__ u32x4 delta_encode(const u32x4 & v, uint32_t start, uint32_t t)
{
    const uint32_t prev = wave_shr1(v.w, start);
    (void)t;
    return u32x4{v.x - prev - 1u, v.y - v.x - 1u, v.z - v.y - 1u, v.w - v.z - 1u};
}

__device__ __forceinline__ uint32_t plan_word(const Plan32 & P)
{
    return P.b | (P.bx << 8) | (P.xn << 16) | (P.raw << 25);
}

__device__ __forceinline__ Plan32 unplan(uint32_t w, uint32_t size)
{
    Plan32 P;
    P.b = w & 0xFFu;
    P.bx = (w >> 8) & 0xFFu;
    P.xn = (w >> 16) & 0x1FFu;
    P.raw = (w >> 25) & 1u;
    P.size = size;
    return P;
}

// A wave's run of up to kEncRun consecutive blocks of 256 values.  Values
// arrive through a buffer descriptor over exactly the run's n KB, so the
// pipelined loads of blocks >= n return zeros without memory traffic and
// every path has the same vmcnt pattern (see RunPlane, p4_dec_run.h).
// POL: cache policy of the value loads (buffer-load aux bits)
template <int POL = 0>
struct EncRunT
{
    uint64_t first;
    uint32_t n;
    __amdgpu_buffer_rsrc_t rs;

    __device__ __forceinline__ bool init(const uint32_t * in, uint64_t nblocks, uint32_t wv)
    {
        return init_at(in, nblocks, (static_cast<uint64_t>(blockIdx.x) * 4u + wv) * kEncRun, kEncRun);
    }

    // run of up to nmax (<= 64) blocks from block `at`
    __device__ __forceinline__ bool init_at(const uint32_t * in, uint64_t nblocks, uint64_t at, uint32_t nmax)
    {
        first = at;
        if (first >= nblocks)
        {
            n = 0;
            return false;
        }
        n = static_cast<uint32_t>(min_u64(nmax, nblocks - first));
        rs = make_rsrc(in + first * 256u, n * 1024u);
        return true;
    }

    __device__ __forceinline__ u32x4 load(uint32_t jj, uint32_t t) const
    {
        return __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(jj * 1024u + 16u * t), 0, POL);
    }

    // Start value of block first+t for delta-1 (lanes t < n): the given
    // starts, or for one chained list the last value of the previous block.
    __device__ __forceinline__ uint32_t start_lane(const uint32_t * in, const uint32_t * starts, uint32_t start0,
                                                    uint32_t t) const
    {
        if (t >= n)
            return 0u;
        const uint64_t blk = first + t;
        if (starts)
            return starts[blk];
        return blk == 0 ? start0 : in[blk * 256u - 1u];
    }

    // Pipelined walk: body(v, jj) for jj = 0..n-1 with NC blocks in flight.
    template <uint32_t NC, class Body>
    __device__ __forceinline__ void walk(uint32_t t, Body && body) const
    {
        u32x4 C[NC];
#pragma unroll
        for (uint32_t u = 0; u + 1 < NC; ++u)
            C[u] = load(u, t);
        bool more = true;
        for (uint32_t j = 0; more; j += NC)
        {
#pragma unroll
            for (uint32_t u = 0; u < NC; ++u)
            {
                if (more)
                {
                    C[(u + NC - 1) % NC] = load(j + u + NC - 1, t);
                    body(C[u], j + u);
                    more = j + u + 1 < n;
                }
            }
        }
    }
};

using EncRun = EncRunT<0>;
constexpr int kEncPolPlan = 2;  // plan pass value loads: nontemporal (C3 D1 encode +1.6%, C4 level; the write pass loses with it, r5r)
constexpr int kEncPolWrite = 0; // write pass value loads

__device__ __forceinline__ uint32_t rl32(uint32_t v, uint32_t lane)
{
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(lane)));
}

// Plan a run: lane j of (szv, pwv) = size and plan word of block R.first+j.
template <bool D1, int PROBE = 0, class Run>
__device__ __forceinline__ void plan_run(const Run & R, const uint32_t * in, const uint32_t * starts, uint32_t start0,
                                         uint32_t * hist, uint32_t t, uint32_t & szv, uint32_t & pwv)
{
    const uint32_t stv = D1 ? R.start_lane(in, starts, start0, t) : 0u;
    szv = 0u;
    pwv = 0u;
    R.template walk<kEncNCPlan>(t, [&](u32x4 v, uint32_t jj) {
        if constexpr (D1)
            v = delta_encode(v, rl32(stv, jj), t);
        Plan32 P;
        if constexpr (PROBE == 1)
        {
            P.b = bw32(uni(wave_or(v.x | v.y | v.z | v.w)));
            P.bx = 0;
            P.size = 1 + 32 * P.b;
            P.xn = 0;
            P.raw = 0;
        }
        else
            P = plan_block256(v, hist, t);
        szv = t == jj ? P.size : szv;
        pwv = t == jj ? plan_word(P) : pwv;
    });
}

// Write a run: lane j of (szv, pwv, ov) = size, plan word and byte offset of
// block R.first+j.  img: the wave's zeroed LDS image (left zeroed).  Round 6:
// each block's layout from enc_geo, single-lane steps without exec masks,
// the copy-out through one buffer descriptor per run (RunCopyB; p4_enc32.h).
template <bool D1, int PROBE = 0, class Run>
__device__ __forceinline__ void write_run(const Run & R, const uint32_t * in, const uint32_t * starts, uint32_t start0,
                                          uint32_t szv, uint32_t pwv, uint64_t ov, uint32_t * img, uint32_t * val,
                                          uint64_t out_base, uint64_t cap_end, uint32_t t)
{
    const uint32_t stv = D1 ? R.start_lane(in, starts, start0, t) : 0u;
    if constexpr (PROBE == 2)
    {
        R.template walk<kEncNCWrite>(t, [&](u32x4 v, uint32_t jj) {
            const uint32_t size = rl32(szv, jj);
            const uint64_t dst = out_base + readlane_u64(ov, jj);
            reinterpret_cast<u32x4 *>(img)[4 + t] = v;
            wave_lds_sync();
            copy_out_image16(img, kImgLead, dst, size, cap_end, t);
            wave_lds_sync();
            zero_image(img, kImgU32 / 4u, t);
            wave_lds_sync();
        });
        return;
    }
    (void)cap_end; // the batch entry points require out_cap >= the bound: no chunk passes the stream's end
    // the run's output through one descriptor based at its first byte rounded down to 16
    const uint64_t ab = out_base + ov;
    const uint64_t A = readlane_u64(ab, 0) & ~15ull;
    const uint32_t rel = static_cast<uint32_t>(ab - A);
    const uint32_t lead = rl32(rel, 0); // < 16
    const uint32_t rel_end = rl32(rel + szv, R.n - 1u);
    RunCopyB rc;
    rc.rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(A), static_cast<short>(0), static_cast<int>(rel_end), 0x00020000);
    // the block that completes the run's partial first chunk stores its bytes [lead, 16)
    const uint64_t flush = __builtin_amdgcn_ballot_w64(t < R.n && lead != 0u && rel < 16u && rel + szv >= 16u);
    const uint32_t trash_at = static_cast<uint32_t>(reinterpret_cast<uint8_t *>(val + kEncTrash + t) - reinterpret_cast<uint8_t *>(img));
    R.template walk<kEncNCWrite>(t, [&](u32x4 v, uint32_t jj) {
        if constexpr (D1)
            v = delta_encode(v, rl32(stv, jj), t);
        // the layout from three values read per block (the plan word, size and
        // output byte), derived on the scalar unit: eighteen v_readlane of a
        // full run plane cost more VALU cycles and 19 VGPRs (6 waves per SIMD
        // instead of 7) than the scalar derivation (r6d)
        const EncGeo G = enc_geo(rl32(pwv, jj), rl32(szv, jj), rl32(rel, jj), lead);
        emit_block256_g<true>(img, val, G, v, t);
        wave_lds_sync();
        rc.put(img, G.c, (flush >> jj) & 1u, lead, trash_at, t);
        wave_lds_sync();
        zero_image_n(img, G.c.n16, t); // only [0, sb + size) can be non-zero
        wave_lds_sync();
    });
    rc.flush_tail(rel_end, lead, t);
}

// ---- two-pass encoder (plan -> run scan -> write): the production path ---
// The plan pass leaves each block's size in off[block] and one total per
// wave run; p4_scan.h scans only the run totals; the write pass rebuilds the
// offsets of its run from the run base and its sizes and writes them back.

template <bool D1, int PROBE = 0, uint32_t RUN = kEncRun>
__global__ __launch_bounds__(256) void k_enc256v32_plan(const uint32_t * __restrict in, uint64_t nblocks,
                                                         const uint32_t * __restrict starts, uint32_t start0,
                                                         uint64_t * __restrict sizes, uint32_t * __restrict plan,
                                                         uint32_t * __restrict run_tot)
{
    __shared__ __attribute__((aligned(16))) uint32_t hist[4][kPlanHistU32];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    for (uint64_t g = blockIdx.x;; g += gridDim.x)
    {
        EncRunT<kEncPolPlan> R;
        if (!R.init_at(in, nblocks, (g * 4u + wv) * RUN, RUN))
            return;
        uint32_t szv, pwv; // lane j: block first+j
        plan_run<D1, PROBE>(R, in, starts, start0, hist[wv], t, szv, pwv);
        if (t < R.n)
        {
            sizes[R.first + t] = szv;
            plan[R.first + t] = pwv;
        }
        publish_run_total(run_tot, R.first / RUN, t < R.n ? szv : 0u, t);
    }
}

template <bool D1, int PROBE = 0, uint32_t RUN = kEncRun>
__global__ __launch_bounds__(256) void k_enc256v32_write(const uint32_t * __restrict in, uint64_t nblocks,
                                                          const uint32_t * __restrict starts, uint32_t start0,
                                                          uint64_t * __restrict off, const uint32_t * __restrict plan,
                                                          const uint64_t * __restrict run_pre, const uint64_t * __restrict run_tile,
                                                          uint8_t * __restrict out, uint64_t out_cap)
{
    __shared__ __attribute__((aligned(16))) uint32_t img_all[4][kImgU32];
    __shared__ __attribute__((aligned(16))) uint32_t val_all[4][kEncValU32];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t * img = img_all[wv];
    zero_image(img, kImgU32 / 4u, t);
    wave_lds_sync();
    const uint64_t out_base = reinterpret_cast<uint64_t>(out);
    for (uint64_t g = blockIdx.x;; g += gridDim.x)
    {
        EncRunT<kEncPolWrite> R;
        if (!R.init_at(in, nblocks, (g * 4u + wv) * RUN, RUN))
            return;
        // lane j: destination offset (64-bit), size and plan of block first+j
        uint64_t ov, ev;
        run_offsets(off, R.first, R.n, run_base(run_pre, run_tile, R.first / RUN), t, ov, ev);
        const uint32_t szv = static_cast<uint32_t>(ev - ov);
        const uint32_t pwv = t < R.n ? plan[R.first + t] : 0u;
        write_run<D1, PROBE>(R, in, starts, start0, szv, pwv, ov, img, val_all[wv], out_base, out_base + out_cap, t);
    }
}

} // namespace tpf::dev

namespace tpf::enc256
{

inline size_t al256(size_t x) { return (x + 255u) & ~size_t(255); }

inline uint64_t enc_runs(uint64_t nblocks, uint32_t run = dev::kEncRun) { return (nblocks + run - 1u) / run; }

// two-pass encoder workspace: plan words + the run scan (p4_scan.h)
inline size_t twopass_workspace(uint64_t nblocks) { return al256(nblocks * 4u) + RunScanWs<uint64_t>::bytes(enc_runs(nblocks)); }

// plan -> run scan -> write.  PP / PW: PROBE of the plan / write kernel (0 =
// production; the probes are instantiated only by the measurement library,
// measure/tpf_measure.hip).
template <int PP, int PW>
hipError_t launch_twopass(const uint32_t * in, uint64_t nblocks, const uint32_t * starts, uint32_t start0, bool d1, uint8_t * out,
                          uint64_t out_cap, uint64_t * off, void * ws, hipStream_t stream)
{
    uint32_t * plan = static_cast<uint32_t *>(ws);
    constexpr uint32_t RD = dev::kEncRunD1;
    const uint32_t run = d1 ? RD : dev::kEncRun;
    const uint64_t nruns = enc_runs(nblocks, run); // <= enc_runs(nblocks): fits the workspace
    const RunScanWs<uint64_t> rs = RunScanWs<uint64_t>::carve(static_cast<uint8_t *>(ws) + al256(nblocks * 4u), nruns);
    const uint64_t per_wg = 4ull * run;
    const uint32_t grid = static_cast<uint32_t>((nblocks + per_wg - 1) / per_wg);
    if constexpr (PP != 0)
    {
        if (d1)
            return hipErrorInvalidValue; // the plan probe measures the plain encoder only
    }
    // (the write probe runs after the real plan pass in either mode: with d1
    // it copies the staged values into the D1 blocks' sizes, the data
    // movement of the D1 write pass, round 6)
    if (d1)
        hipLaunchKernelGGL((dev::k_enc256v32_plan<true, 0, RD>), dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off,
                           plan, rs.tot);
    else
        hipLaunchKernelGGL((dev::k_enc256v32_plan<false, PP>), dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan,
                           rs.tot);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return e;
    e = launch_run_scan_u64(rs.tot, nruns, rs.pre, rs.tile, off + nblocks, stream);
    if (e != hipSuccess)
        return e;
    if (d1)
        hipLaunchKernelGGL((dev::k_enc256v32_write<true, PW, RD>), dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off,
                           plan, rs.pre, rs.tile, out, out_cap);
    else
        hipLaunchKernelGGL((dev::k_enc256v32_write<false, PW>), dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan,
                           rs.pre, rs.tile, out, out_cap);
    return hipGetLastError();
}

} // namespace tpf::enc256
