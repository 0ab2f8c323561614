// dec_groups.hip -- measurement tool (not part of the library): the 256v32
// decode with GROUPED loads, timed against the product kernel on the same
// streams by scripts/dec_groups.py (small blocks are bound by
// the per-block load pipeline).
//
// The product kernel issues one 16-byte load per lane per BLOCK, six blocks in
// flight; a 166-byte block (bw 1) uses 11 of the 64 lanes, so a wave has only
// ~1 KB of reads in flight and bw 1-6 run ~15% under the loads-first probe of
// scripts/hbm_probe2.hip.  Here a wave's run is cut into GROUPS of consecutive
// blocks whose bytes fit one 1 KB window from the first block's 16-aligned
// start (one ballot per group: block ends ascend), and the pipeline moves
// groups instead of blocks: one full-width load per group, NC groups in flight,
// so the bytes in flight no longer shrink with the block size.  A group of one
// block larger than the window takes the product's big-block path (the rest
// loaded at staging).  Blocks are decoded from the staged window by the same
// wave decoder (p4_block32.h).  PROBE: the same loads and stores, no decode.
// Build: scripts/build_variants.sh
#include "p4_dec_run.h"

namespace tpf::dev
{

struct GArgs
{
    const uint8_t * in;
    uint64_t in_bytes;
    const uint64_t * off;
    uint64_t nblocks;
    uint32_t * out;
    unsigned long long * err;
};

template <uint32_t RUN, uint32_t NC, int MINW, bool PROBE>
__global__ __launch_bounds__(256, MINW) void k_decg(const GArgs A)
{
    static_assert(RUN <= 64, "a run's blocks and groups live in lanes");
    __shared__ uint32_t slots[4][kSlotBytes / 4];
    __shared__ uint32_t scratch[4][kWaveScratchU32];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t * slot = slots[wv];
    uint32_t * scr = scratch[wv];
    const uint64_t in_base = reinterpret_cast<uint64_t>(A.in);
    const uint64_t in_end = in_base + A.in_bytes;
    const uint64_t first = (static_cast<uint64_t>(blockIdx.x) * 4u + wv) * RUN;
    if (first >= A.nblocks)
        return;
    const uint32_t n = static_cast<uint32_t>(min_u64(RUN, A.nblocks - first));
    const bool valid = t < n;
    const uint64_t o = valid ? A.off[first + t] : 0ull;
    const uint64_t e = valid ? A.off[first + t + 1u] : 0ull;
    const uint32_t len = (e >= o && e - o < 0x10000ull) ? static_cast<uint32_t>(e - o) : 0xFFFFFFFFu;
    // the window of a group: 1 KB from its first block's 16-aligned start
    // (ends past it: the group's last block is alone and big, or the offsets are implausible)
    const uint64_t ab = in_base + o;
    // ---- groups: lane g = group g (first block, block count)
    uint32_t gfb = 0u, gcnt = 0u, ng = 0u;
    for (uint32_t j = 0; j < n;)
    {
        const uint64_t cb = readlane_u64(ab, j) & ~15ull;
        // blocks j.. whose end lies inside the window (a prefix: ends ascend in a valid stream)
        const uint64_t fit = __ballot(valid && t >= j && in_base + e <= cb + 1024u && e >= o);
        const uint64_t above = fit >> j;
        uint32_t c = static_cast<uint32_t>(__builtin_ctzll(~above)); // consecutive fitting blocks from j
        c = c == 0u ? 1u : c;                                        // a big (or implausible) block alone
        gfb = t == ng ? j : gfb;
        gcnt = t == ng ? c : gcnt;
        ++ng;
        j += c;
    }
    const bool gvalid = t < ng;
    const uint32_t glast = gfb + gcnt - 1u;
    auto shfl64 = [](uint64_t x, uint32_t lane) {
        const uint32_t lo = static_cast<uint32_t>(__shfl(static_cast<int>(static_cast<uint32_t>(x)), static_cast<int>(lane & 63u), 64));
        const uint32_t hi = static_cast<uint32_t>(__shfl(static_cast<int>(static_cast<uint32_t>(x >> 32)), static_cast<int>(lane & 63u), 64));
        return (static_cast<uint64_t>(hi) << 32) | lo;
    };
    const uint64_t go = shfl64(o, gfb), ge = shfl64(e, glast);
    RunPlaneT<kSlotBytes, true> P;
    P.init(in_base, in_end, gvalid ? go : 0ull, gvalid ? ge : 0ull, gvalid);

    uint32_t * const out_run = A.out + first * 256u;
    const __amdgpu_buffer_rsrc_t ors = make_rsrc(out_run, n * 1024u);
    uint64_t badmask = 0u;
    auto consume = [&](const Chunk & c, uint32_t g) {
        const uint32_t fb = rl(gfb, g), cnt = rl(gcnt, g);
        if constexpr (PROBE)
        {
            const u32x4 x = c.a | P.big_rest_or(g, t);
            for (uint32_t k = 0; k < cnt; ++k)
                st16_run(ors, (fb + k) * 1024u + 16u * t, x);
            return;
        }
        const uint32_t ctl = P.stage(c, g, slot, t);
        const uint32_t cblo = rl(P.cblo, g);
        (void)ctl;
        for (uint32_t k = 0; k < cnt; ++k)
        {
            const uint32_t b = fb + k;
            const uint32_t s = rl(static_cast<uint32_t>(ab), b) - cblo; // block start inside the window
            u32x4 v;
            const uint32_t used = decode_block256v32(slot, s, uni(lds_u32(slot, s)), scr, t, v);
            st16_run(ors, b * 1024u + 16u * t, v);
            wave_lds_sync();
            if (used != rl(len, b))
                badmask |= 1ull << b;
        }
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
                more = j + u + 1 < ng;
            }
        }
    }
    if (A.err != nullptr && t == 0 && badmask != 0u)
        atomicMin(A.err, static_cast<unsigned long long>(first + __builtin_ctzll(badmask)));
}

template <uint32_t RUN, uint32_t NC, int MINW, bool PROBE>
int launch_g(const GArgs & A, hipStream_t s)
{
    const uint32_t grid = static_cast<uint32_t>((A.nblocks + 4u * RUN - 1u) / (4u * RUN));
    hipLaunchKernelGGL((k_decg<RUN, NC, MINW, PROBE>), dim3(grid), dim3(256), 0, s, A);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace tpf::dev

// variant ids: 0 RUN16 NC6 W7, 1 RUN32 NC6 W7, 2 RUN64 NC6 W7, 3 RUN32 NC4 W8, 4 RUN64 NC8 W6, 5 RUN32 NC8 W6
extern "C" int decgrp_launch(int var, int probe, const void * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, void * out,
                             unsigned long long * err, void * stream)
{
    using namespace tpf::dev;
    const GArgs A{static_cast<const uint8_t *>(in), in_bytes, off, nblocks, static_cast<uint32_t *>(out), err};
    const hipStream_t s = static_cast<hipStream_t>(stream);
    if (nblocks == 0)
        return 0;
    switch (var * 2 + (probe ? 1 : 0))
    {
        case 0: return launch_g<16, 6, 7, false>(A, s);
        case 1: return launch_g<16, 6, 7, true>(A, s);
        case 2: return launch_g<32, 6, 7, false>(A, s);
        case 3: return launch_g<32, 6, 7, true>(A, s);
        case 4: return launch_g<64, 6, 7, false>(A, s);
        case 5: return launch_g<64, 6, 7, true>(A, s);
        case 6: return launch_g<32, 4, 8, false>(A, s);
        case 7: return launch_g<32, 4, 8, true>(A, s);
        case 8: return launch_g<64, 8, 6, false>(A, s);
        case 9: return launch_g<64, 8, 6, true>(A, s);
        case 10: return launch_g<32, 8, 6, false>(A, s);
        case 11: return launch_g<32, 8, 6, true>(A, s);
        default: return -2;
    }
}
