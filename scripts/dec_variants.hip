// dec_variants.hip -- measurement tool (not part of the library): variants of
// the 256v32 decode kernel's work dealing, timed against the product kernel
// on the same streams by scripts/dec_variants.py.  Same block machinery
// (p4_dec_run.h / p4_block32.h); only which blocks a wave owns changes.
//   DEAL 0: contiguous 16-block runs per wave (the product's layout)
//   DEAL 1: a workgroup's 64 blocks dealt round-robin to its 4 waves
//   DEAL 2: global stride: wave g owns blocks g + W*j (W = number of waves),
//           so the resident waves write one contiguous window at a time
//   DEAL 3: contiguous runs, workgroups remapped so each XCD takes one
//           contiguous range of the stream (dispatch deals WGs round-robin)
//   DEAL 4: global stride with 32 blocks per wave
//   DEAL 5: contiguous runs, workgroups remapped in chunks of 8K: XCD x
//           takes WGs [x*K, (x+1)*K) of each chunk (XCD-contiguous pieces of
//           K workgroups, all XCDs moving through the stream together)
//   DEAL 13..17 (python ids): contiguous runs, output stored by a buffer store
//           with cache-policy aux 0 (plain) / 2 (nt) / 16 (sc1) / 17 (sc0 sc1)
//           / 18 (sc1 nt); 18, 19: 3 (sc0 nt) / 19 (sc0 sc1 nt)
// PROBE: the same loads and stores with the decoding removed.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 -shared -fPIC
//        -I turbopfor-cpp_amd/csrc -o scripts/libdecvar.so scripts/dec_variants.hip
#include "p4_dec_run.h"

namespace tpf::dev
{

// Delta total of one 256v32 D1 block without decoding it: the block's last
// value minus its start = sum over i of (v[i] + 1) mod 2^32 (applyDelta1_256,
// p4d1dec256v32_scalar.cpp:39-50).  Exceptions add (sum of ex) << b (a shift
// left is a multiplication by 2^b, which distributes mod 2^32), so no
// exception needs its position: no bitmap ranking, no position bytes, no
// scatter.  Returns the sum (wave-uniform); `used` = consumed bytes.
// Round 2's phase A block sum, kept here for the round-2 phase-A variants
// (the library replaced it in round 3: it ADDS exceptions sharing a vbyte
// position where the reference ORs them; p4_dsum_lanes.h).
__device__ __forceinline__ uint32_t dsum_block256v32(const uint32_t * lds, uint32_t s, uint32_t t, uint32_t & used)
{
    const uint32_t hw = uni(lds_u32(lds, s));
    const uint32_t h = hw & 0xFFu, x1 = (hw >> 8) & 0xFFu;
    if ((h & 0xC0u) == 0xC0u)
    {
        const uint32_t b = h & 0x3Fu;
        uint32_t c = uni(lds_u32(lds, s + 1u));
        if (b < 32u)
            c &= mask32(b);
        used = 1u + ((b + 7u) >> 3);
        return 256u * (c + 1u);
    }
    uint32_t exsum = 0u, b, p;
    if ((h & 0x40u) == 0u)
    {
        const uint32_t hdr = (h & 0x80u) ? 2u : 1u;
        const uint32_t bx = (h & 0x80u) ? min(x1, 32u) : 0u;
        b = min(h & 0x7Fu, 32u);
        p = s + hdr;
        if (bx != 0u)
        {
            // xn = popcount of the 256-bit bitmap (lane t reads word t & 7)
            const uint32_t pc = __builtin_popcount(lds_u32(lds, s + 2u + 4u * (t & 7u)));
            const uint32_t xn = wave_sum((t < 8u) ? pc : 0u);
            const uint32_t xs = s + 34u;
            // uniform trip count, predicated adds: a divergent per-lane loop
            // costs exec-mask (SALU) work every block, and this pass is bound
            // by its scalar issue (SQ_INSTS_SALU); lanes past xn
            // read in-slot bytes and add nothing
            for (uint32_t k0 = 0; k0 < xn; k0 += kWave)
            {
                const uint32_t x = lds_bits(lds, xs * 8u + (k0 + t) * bx, bx);
                exsum += k0 + t < xn ? x : 0u;
            }
            p = xs + ((xn * bx + 7u) >> 3);
        }
        used = p + 32u * b - s;
    }
    else
    {
        b = min(h & 0x3Fu, 32u);
        const uint32_t xn = x1;
        p = s + 2u;
        const uint32_t v0 = p + 32u * b;
        const uint32_t first = uni(lds_byte(lds, v0));
        uint32_t vend;
        if (first == 0xFFu)
        {
            for (uint32_t k0 = 0; k0 < xn; k0 += kWave)
            {
                const uint32_t x = lds_u32(lds, v0 + 1u + 4u * (k0 + t));
                exsum += k0 + t < xn ? x : 0u;
            }
            vend = v0 + 1u + 4u * xn;
        }
        else
        {
            // the window walk of vbyte_exceptions, summing instead of storing
            uint32_t c = v0, sp = 0, found = 0;
            vend = v0;
            while (found < xn)
            {
                const uint32_t by0 = lds_byte(lds, c + t);
                const uint32_t len0 = by0 < 0x9Cu ? 1u : by0 < 0xDCu ? 2u : by0 < 0xFCu ? 3u : by0 == 0xFCu ? 4u : 5u;
                const uint32_t q = window_starts(t + len0, sp, t);
                const uint32_t m = static_cast<uint32_t>(__builtin_popcountll(__ballot(q < 64u)));
                const uint32_t cnt = min(m, xn - found);
                const uint32_t qn = bperm(t + len0, q);
                const uint32_t qe = q < 64u ? qn : q;
                {
                    // every lane decodes (q <= 68: in-slot bytes), lanes >= cnt add nothing
                    const uint32_t by = lds_byte(lds, c + q);
                    const uint32_t d = lds_u32(lds, c + q + 1u);
                    const uint32_t v2 = ((by - 0x9Cu) << 8) + (d & 0xFFu) + 156u;
                    const uint32_t v3 = (d & 0xFFFFu) + ((by - 0xDCu) << 16) + 16540u;
                    const uint32_t val = by < 0x9Cu ? by : by < 0xDCu ? v2 : by < 0xFCu ? v3 : by == 0xFCu ? (d & 0xFFFFFFu) : d;
                    exsum += t < cnt ? val : 0u;
                }
                const uint32_t e_last = uni(__builtin_amdgcn_readlane(qe, cnt - 1u));
                found += cnt;
                vend = c + e_last;
                sp = e_last >= 64u ? e_last - 64u : e_last;
                c += e_last >= 64u ? 64u : 0u;
            }
        }
        used = vend + xn - s;
    }
    const u32x4 v = unpack256v32_lane(lds, p, b, t);
    return wave_sum(v.x + v.y + v.z + v.w + 4u + shl32(exsum, b));
}



struct VArgs
{
    const uint8_t * in;
    uint64_t in_bytes;
    const uint64_t * off;
    uint64_t nblocks;
    uint32_t * out;
    uint64_t waves; // DEAL 2: total waves
    unsigned long long * err;
};

// ---- vbyte-path variants (VB template flag) -------------------------------
//   VB bit 0: raw-escape exceptions read speculatively with the first byte
//             (one LDS round trip less), accumulator cleared after use
//             instead of before (no zeroing pass per block)
//   VB bit 1: compressed windows with few values walked by a uniform
//             v_readlane chain (p += len[p]) instead of binary lifting over
//             ds_bpermute (11 dependent permutes per window)
template <uint32_t VB>
__device__ __forceinline__ uint32_t vbyte_exc_v(const uint32_t * lds, uint32_t v0, uint32_t xn, uint32_t * scr, uint32_t t,
                                               uint32_t first, uint32_t rv, uint32_t rp)
{
    uint32_t * tmp = scr + 256;
    if constexpr ((VB & 1u) == 0u)
    {
        reinterpret_cast<u32x4 *>(scr)[t] = u32x4{0u, 0u, 0u, 0u};
        wave_lds_sync();
    }
    uint32_t vend;
    if (first == 0xFFu)
    {
        const uint32_t pbase = v0 + 1u + 4u * xn;
        if constexpr ((VB & 1u) != 0u)
        {
            if (t < xn)
                atomicOr(&scr[rp], rv);
            for (uint32_t k = t + kWave; k < xn; k += kWave)
                atomicOr(&scr[lds_byte(lds, pbase + k)], lds_u32(lds, v0 + 1u + 4u * k));
        }
        else
        {
            for (uint32_t k = t; k < xn; k += kWave)
                atomicOr(&scr[lds_byte(lds, pbase + k)], lds_u32(lds, v0 + 1u + 4u * k));
        }
        vend = pbase;
    }
    else
    {
        uint32_t c = v0, sp = 0, found = 0;
        vend = v0;
        while (found < xn)
        {
            const uint32_t by0 = lds_byte(lds, c + t);
            const uint32_t len0 = by0 < 0x9Cu ? 1u : by0 < 0xDCu ? 2u : by0 < 0xFCu ? 3u : by0 == 0xFCu ? 4u : 5u;
            const uint32_t need = xn - found;
            uint32_t cnt, e_last;
            bool st;
            uint32_t rank;
            if ((VB & 2u) != 0u && need <= 24u)
            {
                uint64_t S = 0u;
                uint32_t p = sp;
                cnt = 0u;
                while (p < 64u && cnt < need)
                {
                    S |= 1ull << p;
                    p += rl(len0, p);
                    ++cnt;
                }
                e_last = p;
                st = (S >> t) & 1u;
                rank = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(S >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(S), 0u));
            }
            else
            {
                const uint32_t pk = window_starts(t + len0, sp, t);
                const uint32_t m = static_cast<uint32_t>(__builtin_popcountll(__ballot(pk < 64u)));
                cnt = min(m, need);
                const uint32_t pn = bperm(t + len0, pk);
                const uint32_t pe = pk < 64u ? pn : pk;
                e_last = uni(__builtin_amdgcn_readlane(pe, cnt - 1u));
                // express as "lane pk starts value t": decode in lane t at position pk
                st = t < cnt;
                rank = t;
                if (st)
                {
                    const uint32_t by = lds_byte(lds, c + pk);
                    const uint32_t d = lds_u32(lds, c + pk + 1u);
                    const uint32_t v2 = ((by - 0x9Cu) << 8) + (d & 0xFFu) + 156u;
                    const uint32_t v3 = (d & 0xFFFFu) + ((by - 0xDCu) << 16) + 16540u;
                    tmp[(found + t) & 255u] = by < 0x9Cu ? by : by < 0xDCu ? v2 : by < 0xFCu ? v3 : by == 0xFCu ? (d & 0xFFFFFFu) : d;
                }
                st = false;
            }
            if (st)
            {
                const uint32_t by = by0;
                const uint32_t d = lds_u32(lds, c + t + 1u);
                const uint32_t v2 = ((by - 0x9Cu) << 8) + (d & 0xFFu) + 156u;
                const uint32_t v3 = (d & 0xFFFFu) + ((by - 0xDCu) << 16) + 16540u;
                tmp[(found + rank) & 255u] = by < 0x9Cu ? by : by < 0xDCu ? v2 : by < 0xFCu ? v3 : by == 0xFCu ? (d & 0xFFFFFFu) : d;
            }
            found += cnt;
            vend = c + e_last;
            sp = e_last >= 64u ? e_last - 64u : e_last;
            c += e_last >= 64u ? 64u : 0u;
        }
        wave_lds_sync();
        for (uint32_t k = t; k < xn; k += kWave)
            atomicOr(&scr[lds_byte(lds, vend + k)], tmp[k]);
    }
    wave_lds_sync();
    return vend + xn;
}

template <uint32_t VB>
__device__ __forceinline__ uint32_t decode_block_v(const uint32_t * lds, uint32_t s, uint32_t hw, uint32_t * scr, uint32_t t, u32x4 & v)
{
    if constexpr (VB == 0u)
        return decode_block256v32(lds, s, hw, scr, t, v);
    const uint32_t h = hw & 0xFFu, x1 = (hw >> 8) & 0xFFu;
    if ((h & 0xC0u) != 0x40u)
        return decode_block256v32(lds, s, hw, scr, t, v);
    const uint32_t b = min(h & 0x3Fu, 32u);
    const uint32_t xn = x1;
    const uint32_t v0 = s + 2u + 32u * b;
    const uint32_t first = uni(lds_byte(lds, v0));
    uint32_t rv = 0u, rp = 0u;
    if constexpr ((VB & 1u) != 0u)
    {
        // raw-escape guess: value and position of exception t (in-slot bytes either way)
        rv = lds_u32(lds, v0 + 1u + 4u * t);
        rp = lds_byte(lds, v0 + 1u + 4u * xn + t);
    }
    v = unpack256v32_lane(lds, s + 2u, b, t);
    const uint32_t end = vbyte_exc_v<VB>(lds, v0, xn, scr, t, first, rv, rp);
    const u32x4 ex = reinterpret_cast<const u32x4 *>(scr)[t];
    if constexpr ((VB & 1u) != 0u)
        reinterpret_cast<u32x4 *>(scr)[t] = u32x4{0u, 0u, 0u, 0u};
    v.x |= shl32(ex.x, b);
    v.y |= shl32(ex.y, b);
    v.z |= shl32(ex.z, b);
    v.w |= shl32(ex.w, b);
    return end - s;
}

template <int DEAL, bool PROBE, uint32_t kRun = 16, uint32_t K = 1, uint32_t VB = 0, int STAUX = -1, uint32_t NC = 6, int MINW = 7>
__global__ __launch_bounds__(256, MINW) void k_var(const VArgs A)
{
    __shared__ uint32_t slots[4][kSlotBytes / 4];
    __shared__ uint32_t scratch[4][kWaveScratchU32];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint64_t wg = blockIdx.x;
    if constexpr (DEAL == 3)
    {
        const uint64_t G = gridDim.x, q = G / 8u, r = G % 8u, x = wg % 8u, k = wg / 8u;
        wg = x * q + (x < r ? x : r) + k;
    }
    if constexpr (DEAL == 5)
    {
        const uint64_t G = gridDim.x, base = wg / (8u * K) * (8u * K), Gc = min_u64(8u * K, G - base), i = wg - base;
        const uint64_t q = Gc / 8u, r = Gc % 8u, x = i % 8u, k = i / 8u;
        wg = base + x * q + (x < r ? x : r) + k;
    }
    uint32_t * slot = slots[wv];
    uint32_t * scr = scratch[wv];
    if constexpr ((VB & 1u) != 0u)
        reinterpret_cast<u32x4 *>(scr)[t] = u32x4{0u, 0u, 0u, 0u};
    const uint64_t in_base = reinterpret_cast<uint64_t>(A.in);
    const uint64_t in_end = in_base + A.in_bytes;

    uint64_t first, stride;
    if constexpr (DEAL == 1)
    {
        first = wg * 4u * kRun + wv;
        stride = 4u;
    }
    else if constexpr (DEAL == 2 || DEAL == 4)
    {
        first = wg * 4u + wv;
        stride = A.waves;
    }
    else
    {
        first = (wg * 4u + wv) * kRun;
        stride = 1u;
    }
    if (first >= A.nblocks || ((DEAL == 2 || DEAL == 4) && first >= A.waves))
        return;
    const uint32_t n = static_cast<uint32_t>(min_u64(kRun, (A.nblocks - first + stride - 1u) / stride));

    const bool valid = t < n;
    const uint64_t blk = first + stride * t;
    const uint64_t o = valid ? A.off[blk] : 0ull;
    const uint64_t e = valid ? A.off[blk + 1u] : 0ull;
    RunPlaneT<kSlotBytes, true> P;
    P.init(in_base, in_end, o, e, valid);
    uint32_t * const out_run = A.out + first * 256u;
    uint64_t badmask = 0u;
    // STAUX >= 0: output through a buffer store with that cache-policy aux
    // (bit 0 sc0, bit 1 nt, bit 4 sc1) instead of the product's nt store
    const __amdgpu_buffer_rsrc_t ors = make_rsrc(out_run, n * 1024u);
    auto store = [&](u32x4 * dst, uint32_t jj, const u32x4 & v) {
        if constexpr (STAUX < 0)
            st16<2>(dst, v);
        else
            __builtin_amdgcn_raw_buffer_store_b128(v, ors, static_cast<int>(jj * 1024u + 16u * t), 0, STAUX);
    };

    auto issue = [&](Chunk & c, uint32_t jj) { P.template issue<2>(c, jj, t); };
    auto consume = [&](const Chunk & c, uint32_t jj) {
        u32x4 * dst = reinterpret_cast<u32x4 *>(out_run + jj * stride * 256u) + t;
        if constexpr (PROBE)
        {
            store(dst, jj, c.a | P.big_rest_or(jj, t));
            return;
        }
        const uint32_t ctl = P.stage(c, jj, slot, t);
        u32x4 v;
        const uint32_t used = decode_block_v<VB>(slot, (ctl >> kCtlShift) & 15u, P.head(c, ctl, slot), scr, t, v);
        store(dst, jj, v);
        wave_lds_sync();
        if (used != rl(P.len, jj))
            badmask |= 1ull << jj;
    };
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
                more = j + u + 1 < n;
            }
        }
    }
    if (A.err != nullptr && t == 0 && badmask != 0u)
        atomicMin(A.err, static_cast<unsigned long long>(first + stride * __builtin_ctzll(badmask)));
}

template <int DEAL, bool PROBE, uint32_t K = 1, uint32_t VB = 0, int STAUX = -1>
int launch_var(const VArgs & A0, hipStream_t s)
{
    constexpr uint32_t kRun = DEAL == 4 ? 32u : 16u;
    VArgs A = A0;
    const uint64_t waves = (A.nblocks + kRun - 1u) / kRun;
    A.waves = waves;
    const uint32_t grid = static_cast<uint32_t>((waves + 3u) / 4u);
    hipLaunchKernelGGL((k_var<DEAL, PROBE, kRun, K, VB, STAUX>), dim3(grid), dim3(256), 0, s, A);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// sc1 nt stores with another pipeline depth / occupancy
template <uint32_t NC, int MINW, bool PROBE>
int launch_nc(const VArgs & A0, hipStream_t s)
{
    VArgs A = A0;
    const uint64_t waves = (A.nblocks + 15u) / 16u;
    A.waves = waves;
    const uint32_t grid = static_cast<uint32_t>((waves + 3u) / 4u);
    hipLaunchKernelGGL((k_var<0, PROBE, 16, 1, 0, 18, NC, MINW>), dim3(grid), dim3(256), 0, s, A);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// dsum_block256v32 (p4_block32.h) returning the lane's partial sum: the
// block sums are then reduced once per run (LDS transpose) instead of one
// wave reduction per block -- measurement of that reduction's cost
__device__ __forceinline__ uint32_t dsum_partial256v32(const uint32_t * lds, uint32_t s, uint32_t t, uint32_t & used)
{
    const uint32_t hw = uni(lds_u32(lds, s));
    const uint32_t h = hw & 0xFFu, x1 = (hw >> 8) & 0xFFu;
    if ((h & 0xC0u) == 0xC0u)
    {
        const uint32_t b = h & 0x3Fu;
        uint32_t c = uni(lds_u32(lds, s + 1u));
        if (b < 32u)
            c &= mask32(b);
        used = 1u + ((b + 7u) >> 3);
        return t == 0 ? 256u * (c + 1u) : 0u;
    }
    uint32_t exsum = 0u, b, p;
    if ((h & 0x40u) == 0u)
    {
        const uint32_t hdr = (h & 0x80u) ? 2u : 1u;
        const uint32_t bx = (h & 0x80u) ? min(x1, 32u) : 0u;
        b = min(h & 0x7Fu, 32u);
        p = s + hdr;
        if (bx != 0u)
        {
            // xn = popcount of the 256-bit bitmap (lane t reads word t & 7)
            const uint32_t pc = __builtin_popcount(lds_u32(lds, s + 2u + 4u * (t & 7u)));
            const uint32_t xn = wave_sum((t < 8u) ? pc : 0u);
            const uint32_t xs = s + 34u;
            // uniform trip count, predicated adds: a divergent per-lane loop
            // costs exec-mask (SALU) work every block, and this pass is bound
            // by its scalar issue (SQ_INSTS_SALU); lanes past xn
            // read in-slot bytes and add nothing
            for (uint32_t k0 = 0; k0 < xn; k0 += kWave)
            {
                const uint32_t x = lds_bits(lds, xs * 8u + (k0 + t) * bx, bx);
                exsum += k0 + t < xn ? x : 0u;
            }
            p = xs + ((xn * bx + 7u) >> 3);
        }
        used = p + 32u * b - s;
    }
    else
    {
        b = min(h & 0x3Fu, 32u);
        const uint32_t xn = x1;
        p = s + 2u;
        const uint32_t v0 = p + 32u * b;
        const uint32_t first = uni(lds_byte(lds, v0));
        uint32_t vend;
        if (first == 0xFFu)
        {
            for (uint32_t k0 = 0; k0 < xn; k0 += kWave)
            {
                const uint32_t x = lds_u32(lds, v0 + 1u + 4u * (k0 + t));
                exsum += k0 + t < xn ? x : 0u;
            }
            vend = v0 + 1u + 4u * xn;
        }
        else
        {
            // the window walk of vbyte_exceptions, summing instead of storing
            uint32_t c = v0, sp = 0, found = 0;
            vend = v0;
            while (found < xn)
            {
                const uint32_t by0 = lds_byte(lds, c + t);
                const uint32_t len0 = by0 < 0x9Cu ? 1u : by0 < 0xDCu ? 2u : by0 < 0xFCu ? 3u : by0 == 0xFCu ? 4u : 5u;
                const uint32_t q = window_starts(t + len0, sp, t);
                const uint32_t m = static_cast<uint32_t>(__builtin_popcountll(__ballot(q < 64u)));
                const uint32_t cnt = min(m, xn - found);
                const uint32_t qn = bperm(t + len0, q);
                const uint32_t qe = q < 64u ? qn : q;
                {
                    // every lane decodes (q <= 68: in-slot bytes), lanes >= cnt add nothing
                    const uint32_t by = lds_byte(lds, c + q);
                    const uint32_t d = lds_u32(lds, c + q + 1u);
                    const uint32_t v2 = ((by - 0x9Cu) << 8) + (d & 0xFFu) + 156u;
                    const uint32_t v3 = (d & 0xFFFFu) + ((by - 0xDCu) << 16) + 16540u;
                    const uint32_t val = by < 0x9Cu ? by : by < 0xDCu ? v2 : by < 0xFCu ? v3 : by == 0xFCu ? (d & 0xFFFFFFu) : d;
                    exsum += t < cnt ? val : 0u;
                }
                const uint32_t e_last = uni(__builtin_amdgcn_readlane(qe, cnt - 1u));
                found += cnt;
                vend = c + e_last;
                sp = e_last >= 64u ? e_last - 64u : e_last;
                c += e_last >= 64u ? 64u : 0u;
            }
        }
        used = vend + xn - s;
    }
    const u32x4 v = unpack256v32_lane(lds, p, b, t);
    return v.x + v.y + v.z + v.w + 4u + shl32(exsum, b);
}


// phase A with per-run reduction: lane t's partial of block j goes to
// part[j][t]; after the run lane j sums row j (64 words, 16 ds_read_b128)
template <uint32_t NC, int MINW, uint32_t kRun>
__global__ __launch_bounds__(256, MINW) void k_sum_deferred(const VArgs A)
{
    __shared__ uint32_t slots[4][kSlotBytes / 4];
    __shared__ __attribute__((aligned(16))) uint32_t part[4][kRun][64];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint64_t first = (static_cast<uint64_t>(blockIdx.x) * 4u + wv) * kRun;
    if (first >= A.nblocks)
        return;
    uint32_t * slot = slots[wv];
    const uint64_t in_base = reinterpret_cast<uint64_t>(A.in);
    const uint32_t n = static_cast<uint32_t>(min_u64(kRun, A.nblocks - first));
    const bool valid = t < n;
    const uint64_t o = valid ? A.off[first + t] : 0ull;
    const uint64_t e = valid ? A.off[first + t + 1u] : 0ull;
    RunPlaneT<kSlotBytes, true> P;
    P.init(in_base, in_base + A.in_bytes, o, e, valid);
    auto issue = [&](Chunk & c, uint32_t jj) { P.template issue<2>(c, jj, t); };
    auto consume = [&](const Chunk & c, uint32_t jj) {
        const uint32_t ctl = P.stage(c, jj, slot, t);
        uint32_t used;
        part[wv][jj][t] = dsum_partial256v32(slot, (ctl >> kCtlShift) & 15u, t, used);
        wave_lds_sync();
    };
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
                more = j + u + 1 < n;
            }
        }
    }
    uint32_t sm = 0u;
    if (valid)
    {
        const u32x4 * row = reinterpret_cast<const u32x4 *>(part[wv][t]);
#pragma unroll
        for (uint32_t i = 0; i < 16; ++i)
        {
            const u32x4 q = row[(i + t) & 15u]; // rotated start: lanes hit different banks
            sm += (q.x + q.y) + (q.z + q.w);
        }
        A.out[first + t] = sm;
    }
}

// ---- chained-D1 phase A (block delta sums) with another pipeline depth /
// occupancy / run length: sums[i] = the product's phase A block sum ----------
template <uint32_t NC, int MINW, uint32_t kRun>
__global__ __launch_bounds__(256, MINW) void k_sum(const VArgs A)
{
    __shared__ uint32_t slots[4][kSlotBytes / 4];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint64_t first = (static_cast<uint64_t>(blockIdx.x) * 4u + wv) * kRun;
    if (first >= A.nblocks)
        return;
    uint32_t * slot = slots[wv];
    const uint64_t in_base = reinterpret_cast<uint64_t>(A.in);
    const uint32_t n = static_cast<uint32_t>(min_u64(kRun, A.nblocks - first));
    const bool valid = t < n;
    const uint64_t o = valid ? A.off[first + t] : 0ull;
    const uint64_t e = valid ? A.off[first + t + 1u] : 0ull;
    RunPlaneT<kSlotBytes, true> P;
    P.init(in_base, in_base + A.in_bytes, o, e, valid);
    uint32_t sumv = 0u;
    auto issue = [&](Chunk & c, uint32_t jj) { P.template issue<2>(c, jj, t); };
    auto consume = [&](const Chunk & c, uint32_t jj) {
        const uint32_t ctl = P.stage(c, jj, slot, t);
        uint32_t used;
        const uint32_t sm = dsum_block256v32(slot, (ctl >> kCtlShift) & 15u, t, used);
        sumv = t == jj ? sm : sumv;
        wave_lds_sync();
    };
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
                more = j + u + 1 < n;
            }
        }
    }
    if (valid)
        A.out[first + t] = sumv;
}

template <uint32_t NC, int MINW, uint32_t kRun>
int launch_sum(const VArgs & A, hipStream_t s)
{
    const uint32_t grid = static_cast<uint32_t>((A.nblocks + 4u * kRun - 1u) / (4u * kRun));
    hipLaunchKernelGGL((k_sum<NC, MINW, kRun>), dim3(grid), dim3(256), 0, s, A);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <uint32_t NC, int MINW, uint32_t kRun>
int launch_sumd(const VArgs & A, hipStream_t s)
{
    const uint32_t grid = static_cast<uint32_t>((A.nblocks + 4u * kRun - 1u) / (4u * kRun));
    hipLaunchKernelGGL((k_sum_deferred<NC, MINW, kRun>), dim3(grid), dim3(256), 0, s, A);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace tpf::dev

// phase A variants: out = u32 block sums
extern "C" int decvar_sums(int v, const void * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, void * out, void * stream)
{
    using namespace tpf::dev;
    const VArgs A{static_cast<const uint8_t *>(in), in_bytes, off, nblocks, static_cast<uint32_t *>(out), 0u, nullptr};
    const hipStream_t s = static_cast<hipStream_t>(stream);
    if (nblocks == 0)
        return 0;
    switch (v)
    {
        case 0: return launch_sum<6, 7, 16>(A, s); // the product's configuration
        case 1: return launch_sum<4, 8, 16>(A, s);
        case 2: return launch_sum<3, 8, 16>(A, s);
        case 3: return launch_sum<8, 6, 16>(A, s);
        case 4: return launch_sum<6, 7, 32>(A, s);
        case 5: return launch_sum<4, 8, 32>(A, s);
        case 6: return launch_sum<2, 8, 16>(A, s);
        case 7: return launch_sum<12, 4, 16>(A, s);
        case 8: return launch_sumd<4, 8, 32>(A, s);
        case 9: return launch_sumd<4, 8, 16>(A, s);
        case 10: return launch_sumd<6, 7, 16>(A, s);
        default: return -2;
    }
}

extern "C" int decvar_launch(int deal, int probe, const void * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, void * out,
                             unsigned long long * err, void * stream)
{
    using namespace tpf::dev;
    const VArgs A{static_cast<const uint8_t *>(in), in_bytes, off, nblocks, static_cast<uint32_t *>(out), 0u, err};
    const hipStream_t s = static_cast<hipStream_t>(stream);
    if (nblocks == 0)
        return 0;
    switch (deal * 2 + (probe ? 1 : 0))
    {
        case 0: return launch_var<0, false>(A, s);
        case 1: return launch_var<0, true>(A, s);
        case 2: return launch_var<1, false>(A, s);
        case 3: return launch_var<1, true>(A, s);
        case 4: return launch_var<2, false>(A, s);
        case 5: return launch_var<2, true>(A, s);
        case 6: return launch_var<3, false>(A, s);
        case 7: return launch_var<3, true>(A, s);
        case 8: return launch_var<4, false>(A, s);
        case 9: return launch_var<4, true>(A, s);
        case 10: return launch_var<5, false, 2>(A, s);
        case 11: return launch_var<5, true, 2>(A, s);
        case 12: return launch_var<5, false, 8>(A, s);
        case 13: return launch_var<5, true, 8>(A, s);
        case 14: return launch_var<5, false, 32>(A, s);
        case 15: return launch_var<5, true, 32>(A, s);
        case 16: return launch_var<5, false, 128>(A, s);
        case 17: return launch_var<5, true, 128>(A, s);
        case 18: return launch_var<5, false, 512>(A, s);
        case 19: return launch_var<5, true, 512>(A, s);
        case 20: return launch_var<0, false, 1, 1>(A, s);
        case 22: return launch_var<0, false, 1, 2>(A, s);
        case 24: return launch_var<0, false, 1, 3>(A, s);
        case 26: return launch_var<0, false, 1, 0, 0>(A, s);
        case 27: return launch_var<0, true, 1, 0, 0>(A, s);
        case 28: return launch_var<0, false, 1, 0, 2>(A, s);
        case 29: return launch_var<0, true, 1, 0, 2>(A, s);
        case 30: return launch_var<0, false, 1, 0, 16>(A, s);
        case 31: return launch_var<0, true, 1, 0, 16>(A, s);
        case 32: return launch_var<0, false, 1, 0, 17>(A, s);
        case 33: return launch_var<0, true, 1, 0, 17>(A, s);
        case 34: return launch_var<0, false, 1, 0, 18>(A, s);
        case 35: return launch_var<0, true, 1, 0, 18>(A, s);
        case 36: return launch_var<0, false, 1, 0, 3>(A, s);
        case 37: return launch_var<0, true, 1, 0, 3>(A, s);
        case 38: return launch_var<0, false, 1, 0, 19>(A, s);
        case 39: return launch_var<0, true, 1, 0, 19>(A, s);
        case 40: return launch_nc<4, 8, false>(A, s);
        case 41: return launch_nc<4, 8, true>(A, s);
        case 42: return launch_nc<5, 8, false>(A, s);
        case 43: return launch_nc<5, 8, true>(A, s);
        case 44: return launch_nc<8, 5, false>(A, s);
        case 45: return launch_nc<8, 5, true>(A, s);
        case 46: return launch_nc<12, 4, false>(A, s);
        case 47: return launch_nc<12, 4, true>(A, s);
        case 48: return launch_nc<16, 4, false>(A, s);
        case 49: return launch_nc<16, 4, true>(A, s);
        case 50: return launch_nc<8, 4, false>(A, s);
        case 51: return launch_nc<8, 4, true>(A, s);
        default: return -2;
    }
}
