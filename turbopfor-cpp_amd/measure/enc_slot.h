// enc_slot.h -- the slot encoder (round 5, measured and NOT adopted; part of
// the measurement library only, measure/tpf_measure.hip mode 4 / 5).
//
// VERDICT r4 asked for a 256v32 encoder that reads the values once: plan
// and build every block of a wave run in one kernel, stream the run's blocks
// back to back into the run's own slot of a workspace, scan the run totals,
// then move each run's bytes to its place with a compaction kernel.  Traffic
// per block 1024 + 3S against 2048 + S for the two-pass encoder.  A/B on one
// box (profiles/r5b_enc_slot_ab.txt, HIP events, 10M blocks): C3 D1 encode
// 456-458 G int32/s (fused plan/build scans; 444-445 without) against 497-499
// for the two-pass encoder; C4 encode 380-383 against 503-505.  The encode
// is bound by the issue of its plan and build work, not by the second read of
// the values: planning and building in one kernel saved ~0.5 ms of the two
// passes' 5.1 ms and the compaction added ~1 ms.
#pragma once

#include "../csrc/p4_enc256v32.h"

namespace tpf::dev
{

// ---- slot encoder (round 5): the values are read ONCE -----------------------
// k_enc256v32_slot plans AND builds every block of its wave run (the plan is
// the write pass's input, so it never leaves the wave), and streams the run's
// blocks back to back into the run's own slot of the workspace: slot r holds
// run r's bytes from slot byte 0, whatever the global offset turns out to be.
// It leaves the block sizes in d_off and one total per run (as the plan pass
// does); the run scan gives every run's base; k_enc256v32_compact then moves
// each run's bytes from its slot to out[base..) and writes the offsets.
// Traffic per block: 1024 + 3S (+ offsets) against 2048 + S for the two-pass
// encoder -- less whenever the blocks average S < 512 B (posting lists:
// S ~ 248 B).  Slots are sized for the worst case (every block plain at
// b = 32: 16 x 1025 B), so the workspace is ~1.03x the input.
constexpr uint32_t kSlotRunBytes = 16512; // >= 16 x 1025, a multiple of 128

template <bool D1, bool FUSE>
__global__ __launch_bounds__(256) void k_enc256v32_slot(const uint32_t * __restrict in, uint64_t nblocks,
                                                         const uint32_t * __restrict starts, uint32_t start0,
                                                         uint64_t * __restrict sizes, uint32_t * __restrict run_tot,
                                                         uint8_t * __restrict slots)
{
    __shared__ __attribute__((aligned(16))) uint32_t img_all[4][kImgU32];
    __shared__ __attribute__((aligned(16))) uint32_t val_all[4][kEncValU32];
    static_assert(kPlanHistU32 + 32u <= kEncValU32, "the plan's histogram lives in the staging area");
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t * img = img_all[wv];
    uint32_t * val = val_all[wv];
    zero_image(img, kImgU32 / 4u, t);
    wave_lds_sync();
    for (uint64_t g = blockIdx.x;; g += gridDim.x)
    {
        EncRun R;
        if (!R.init_at(in, nblocks, (g * 4u + wv) * kEncRun, kEncRun))
            return;
        const uint32_t stv = D1 ? R.start_lane(in, starts, start0, t) : 0u;
        const uint64_t slot = reinterpret_cast<uint64_t>(slots) + (R.first / kEncRun) * kSlotRunBytes;
        uint32_t szv = 0u, pos = 0u;
        R.template walk<kEncNCWrite>(t, [&](u32x4 v, uint32_t jj) {
            if constexpr (D1)
                v = delta_encode(v, rl32(stv, jj), t);
            // the histogram (plan) and the staged values (build) share `val`:
            // the plan has read its bins back before the build stages values
            VbPre pre;
            const Plan32 P = plan_block256<FUSE>(v, val, t, &pre);
            wave_lds_sync();
            const uint32_t sb = emit_block256<true, FUSE>(img, val, P, v, t, &pre);
            wave_lds_sync();
            copy_out_image16(img, sb, slot + pos, P.size, ~0ull, t);
            wave_lds_sync();
            zero_image(img, min((sb + P.size + 15u) >> 4, kImgU32 / 4u), t);
            wave_lds_sync();
            szv = t == jj ? P.size : szv;
            pos += P.size;
        });
        if (t < R.n)
            sizes[R.first + t] = szv;
        if (t == 0)
            run_tot[R.first / kEncRun] = pos;
    }
}

// Move run r's bytes [0, T) from its slot to out[base, base + T) (T = the
// run's total, base = its scanned offset) and write its blocks' offsets.  One
// wave per run: the 16-byte chunks that lie wholly inside the run's range are
// 16-byte stores of realigned slot bytes (two aligned loads and v_alignbyte
// per lane), the partial chunks at both ends, shared with the neighbouring
// runs, byte stores.
__global__ __launch_bounds__(256) void k_enc256v32_compact(const uint8_t * __restrict slots, uint64_t nblocks,
                                                            uint64_t * __restrict off, const uint32_t * __restrict run_tot,
                                                            const uint64_t * __restrict run_pre, const uint64_t * __restrict run_tile,
                                                            uint8_t * __restrict out, uint64_t out_cap)
{
    typedef __attribute__((address_space(1))) uint8_t gu8;
    typedef __attribute__((address_space(1))) u32x4 gu32x4;
    const uint32_t t = threadIdx.x & 63u;
    const uint64_t r = static_cast<uint64_t>(blockIdx.x) * 4u + uni(threadIdx.x >> 6);
    const uint64_t first = r * kEncRun;
    if (first >= nblocks)
        return;
    const uint32_t n = static_cast<uint32_t>(min_u64(kEncRun, nblocks - first));
    const uint64_t base = uni64(run_base(run_pre, run_tile, r));
    uint64_t ov, ev;
    run_offsets(off, first, n, base, t, ov, ev);
    const uint32_t T = uni(run_tot[r]);
    const uint64_t end = base + T;
    const uint8_t * src = slots + r * kSlotRunBytes;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(src, kSlotRunBytes);
    gu8 * const o = (gu8 *)out;
    if (end <= out_cap)
    {
        const uint64_t c0 = (base + 15u) >> 4, c1 = end >> 4; // whole chunks [c0, c1)
        const uint32_t q = static_cast<uint32_t>(16u * c0 - base); // slot byte of chunk c0 (0..15)
        const uint32_t qa = q & ~3u, qs = q & 3u;
        const uint32_t nc = c1 > c0 ? static_cast<uint32_t>(c1 - c0) : 0u;
        // four chunks per lane in flight: the loads of a step are issued
        // together (a chunk past the run reads as zeros from an out-of-range
        // offset: no traffic), then realigned and stored
        constexpr uint32_t U = 4;
        for (uint32_t k0 = 0; k0 < nc; k0 += 64u * U)
        {
            u32x4 a[U];
            uint32_t e[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u)
            {
                // slot bytes [q + 16k, q + 16k + 16): dwords from qa + 16k, five of them
                const uint32_t k = k0 + 64u * u + t;
                const int at = k < nc ? static_cast<int>(qa + 16u * k) : static_cast<int>(0x80000000u);
                a[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, at, 0, 0);
                e[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, at + 16, 0, 0);
            }
#pragma unroll
            for (uint32_t u = 0; u < U; ++u)
            {
                const uint32_t k = k0 + 64u * u + t;
                const u32x4 c = u32x4{__builtin_amdgcn_alignbyte(a[u].y, a[u].x, qs), __builtin_amdgcn_alignbyte(a[u].z, a[u].y, qs),
                                      __builtin_amdgcn_alignbyte(a[u].w, a[u].z, qs), __builtin_amdgcn_alignbyte(e[u], a[u].w, qs)};
                if (k < nc)
                    *(gu32x4 *)(o + 16u * (c0 + k)) = c;
            }
        }
        // partial chunks: head bytes [base, 16 c0), tail bytes [16 c1, end)
        const uint64_t g = t < 16u ? base + t : 16u * c1 + (t - 16u);
        const bool on = t < 16u ? (g < 16u * c0 && g < end) : (t < 32u && g >= base && g >= 16u * c0 && g < end);
        if (on)
            o[g] = src[g - base];
    }
    else
    {
        for (uint32_t i = t; i < T; i += 64u)
            if (base + i < out_cap)
                o[base + i] = src[i];
    }
}

} // namespace tpf::dev

namespace tpf::enc256
{

// slot encoder workspace: the two-pass workspace (run scan) + one slot per run
inline size_t slot_workspace(uint64_t nblocks) { return twopass_workspace(nblocks) + al256(enc_runs(nblocks) * dev::kSlotRunBytes); }

// plan+build into slots -> run scan -> compact
template <bool FUSE = true>
inline hipError_t launch_slot(const uint32_t * in, uint64_t nblocks, const uint32_t * starts, uint32_t start0, bool d1, uint8_t * out,
                              uint64_t out_cap, uint64_t * off, void * ws, hipStream_t stream)
{
    const uint64_t nruns = enc_runs(nblocks);
    const RunScanWs<uint64_t> rs = RunScanWs<uint64_t>::carve(static_cast<uint8_t *>(ws) + al256(nblocks * 4u), nruns);
    uint8_t * slots = static_cast<uint8_t *>(ws) + twopass_workspace(nblocks);
    const uint64_t per_wg = 4ull * dev::kEncRun;
    const uint32_t grid = static_cast<uint32_t>((nblocks + per_wg - 1) / per_wg);
    if (d1)
        hipLaunchKernelGGL((dev::k_enc256v32_slot<true, FUSE>), dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, rs.tot,
                           slots);
    else
        hipLaunchKernelGGL((dev::k_enc256v32_slot<false, FUSE>), dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, rs.tot,
                           slots);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return e;
    e = launch_run_scan_u64(rs.tot, nruns, rs.pre, rs.tile, off + nblocks, stream);
    if (e != hipSuccess)
        return e;
    hipLaunchKernelGGL(dev::k_enc256v32_compact, dim3(static_cast<uint32_t>((nruns + 3) / 4)), dim3(256), 0, stream, slots, nblocks, off,
                       rs.tot, rs.pre, rs.tile, out, out_cap);
    return hipGetLastError();
}

} // namespace tpf::enc256
