// c1_pair_variant.hip -- measurement record (not part of the library): the
// C1 decoder that puts two n <= 128 H32 blocks in one wave (one per 32-lane
// half).  Measured on MI355X against the product k_dec_gr (one block per
// wave) on the C1 stream: 560-563 G int32/s (NP 2), 568 (NP 3), 583-590
// (NP 4) vs 623 for k_dec_gr -- slower, so the library keeps k_dec_gr
// (DESIGN.md "C1").  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -shared -fPIC -I turbopfor-cpp_amd/csrc \
//         -o scripts/libc1pair.so scripts/c1_pair_variant.hip
#include "p4_scan.h"
#include "p4_dec_run.h"
#include "p4_generic.h"
#include "tpf_kernels.h"

namespace tpf::dev
{
// ---- p4Dec32 with n <= 128: two blocks per wave, one per 32-lane half ----
// C1 (BASELINE configs[0]) is n = 127: a one-block-per-wave decoder pays the
// per-block fixed cost -- staging wait, header, mode branches, length check
// (counters: 100 SALU / 24 branches / 41 VALU per 128-B block, 24% of
// wave-cycles issuing) -- for 508 B of output and leaves half the lanes
// without an element.  Here lanes 0-31 decode block 2q and lanes 32-63 block
// 2q+1 of a 32-block run (lane t owns elements (t & 31) + 32j, j < 4), every
// header quantity is per lane, so one instruction stream serves both blocks
// and a store instruction writes 128 B of each.  Plain, bitmap and constant
// blocks take this path; a block with vbyte exceptions is decoded by the
// whole wave (decode_block_g) as in k_dec_gr.
constexpr uint32_t kPRun = 32;       // blocks per wave run (16 pairs)
constexpr uint32_t kPairSlot = 1536; // staging bytes per block: an n <= 128 block is at most 1155 B (+ 15 phase)

// 32-lane inclusive scans (each half of the wave on its own): the wave scan
// without its last row_bcast:31 step.
__device__ __forceinline__ uint32_t half_incl_scan(uint32_t x)
{
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false); // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false); // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false); // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false); // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false); // row_bcast:15 (rows 1 and 3)
    return x;
}

// One H32 block (n <= 128) per lane half, staged at byte s of `lds`: v[j] =
// element (t & 31) + 32j.  Mirrors decode_block_g<H32> (p4_generic.h) for the
// constant, plain and bitmap modes (p4dec32.cpp:70-142); returns false for a
// vbyte block.  *used = consumed bytes.
__device__ __forceinline__ bool decode_half_h32(const uint32_t * lds, uint32_t s, uint32_t n, uint32_t lt, uint32_t v[4], uint32_t & used)
{
    const uint32_t hw = lds_u32(lds, s);
    const uint32_t h = hw & 0xFFu, x1 = (hw >> 8) & 0xFFu;
    if ((h & 0xC0u) == 0xC0u)
    {
        const uint32_t b = h & 0x3Fu;
        const uint32_t c = lds_u32(lds, s + 1u) & mask32(b);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            v[j] = c;
        used = 1u + ((b + 7u) >> 3);
        return true;
    }
    if (h & 0x40u)
        return false;
    const uint32_t hdr = (h & 0x80u) ? 2u : 1u;
    const uint32_t bx = (h & 0x80u) ? min(x1, 32u) : 0u;
    const uint32_t b = min(h & 0x7Fu, 32u);
    uint64_t bm0 = 0u, bm1 = 0u;
    uint32_t xn = 0u, xs = 0u, P = s + hdr;
    if (bx != 0u)
    {
        bm0 = lds_u64(lds, s + 2u);
        bm1 = n > 64u ? lds_u64(lds, s + 10u) : 0ull;
        if (n < 64u)
            bm0 &= (1ull << n) - 1ull;
        else if (n > 64u && n < 128u)
            bm1 &= (1ull << (n - 64u)) - 1ull;
        xn = __builtin_popcountll(bm0) + __builtin_popcountll(bm1);
        xs = s + 2u + pad8d(n);
        P = xs + pad8d(xn * bx);
    }
    const uint32_t pc0 = __builtin_popcountll(bm0);
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
    {
        const uint32_t e = lt + 32u * j;
        uint32_t x = (e < n && b) ? lds_bits(lds, P * 8u + e * b, b) : 0u;
        if (bx != 0u)
        {
            // rank of element e among the exceptions: set bitmap bits below e
            const uint32_t bit = e < 64u ? static_cast<uint32_t>(bm0 >> e) & 1u : static_cast<uint32_t>(bm1 >> (e - 64u)) & 1u;
            const uint32_t rank = e < 64u ? __builtin_popcountll(bm0 & ((1ull << e) - 1ull))
                                          : pc0 + __builtin_popcountll(bm1 & ((1ull << (e - 64u)) - 1ull));
            const uint32_t ex = lds_bits(lds, xs * 8u + rank * bx, bx);
            x |= (bit && e < n) ? shl32(ex, b) : 0u;
        }
        v[j] = x;
    }
    used = bx != 0u ? (xs - s) + pad8d(xn * bx) + pad8d(n * b) : hdr + pad8d(n * b);
    return true;
}

#ifndef TPF_PAIR_NP
#define TPF_PAIR_NP 2
#endif
#ifndef TPF_PAIR_MINW
#define TPF_PAIR_MINW 7
#endif
template <bool D1, uint32_t NP = TPF_PAIR_NP>
__global__ __launch_bounds__(256, TPF_PAIR_MINW) __attribute__((amdgpu_num_sgpr(80))) void k_dec_pair_h32(const uint8_t * __restrict in, uint64_t in_bytes, const uint64_t * __restrict off,
                                                      uint64_t nblocks, uint32_t n, uint32_t * __restrict out,
                                                      const uint32_t * __restrict starts, unsigned long long * __restrict err)
{
    __shared__ uint32_t slots[4][2][kPairSlot / 4];
    __shared__ uint32_t scratch[4][512];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint32_t half = t >> 5, lt = t & 31u;
    const uint64_t in_base = reinterpret_cast<uint64_t>(in);
    const uint64_t first = (static_cast<uint64_t>(blockIdx.x) * 4u + wv) * kPRun;
    if (first >= nblocks)
        return;
    const uint32_t nr = static_cast<uint32_t>(min_u64(kPRun, nblocks - first));
    const bool valid = t < nr;
    const uint64_t o = valid ? off[first + t] : 0ull;
    const uint64_t e = valid ? off[first + t + 1u] : 0ull;
    RunPlaneT<kPairSlot, true> P;
    P.init(in_base, in_base + in_bytes, o, e, valid);
    const uint32_t startv = (D1 && valid) ? starts[first + t] : 0u;
    uint32_t * const myslot = slots[wv][half];
    uint64_t badmask = 0u;

    auto consume = [&](const Chunk & ca, const Chunk & cb, uint32_t q) {
        const uint32_t ja = 2u * q, jb = ja + 1u;
        const uint32_t cwa = P.stage(ca, ja, slots[wv][0], t);
        const uint32_t cwb = jb < nr ? P.stage(cb, jb, slots[wv][1], t) : 0u;
        const uint32_t jj = ja + half;
        const bool act = jj < nr;
        const uint32_t s = ((half ? cwb : cwa) >> kCtlShift) & 15u;
        uint32_t v[4], used = 0u;
        const bool fast = decode_half_h32(myslot, s, n, lt, v, used);
        const uint32_t lenA = rl(P.len, ja), lenB = rl(P.len, jb);
        uint32_t * op = out + (first + jj) * n;
        if (fast && act)
        {
            if constexpr (D1)
            {
                uint32_t carry = half ? rl(startv, jb) : rl(startv, ja);
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                {
                    const uint32_t x = lt + 32u * j < n ? v[j] + 1u : 0u;
                    const uint32_t incl = half_incl_scan(x);
                    const uint32_t tot = half ? rl(incl, 63) : rl(incl, 31);
                    v[j] = carry + incl;
                    carry += tot;
                }
            }
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (lt + 32u * j < n)
                    __builtin_nontemporal_store(v[j], op + lt + 32u * j);
        }
        // a vbyte block: the whole wave decodes it (decode_block_g, as k_dec_gr)
        const uint64_t slow = __ballot(!fast && act);
#pragma unroll
        for (uint32_t hh = 0; hh < 2u; ++hh)
        {
            if ((slow >> (32u * hh)) & 0xFFFFFFFFull)
            {
                const uint32_t jh = ja + hh;
                uint32_t vv[4], cm;
                const uint32_t sh = ((hh ? cwb : cwa) >> kCtlShift) & 15u;
                const uint32_t uw = decode_block_g<Fmt::H32>(slots[wv][hh], sh, n, scratch[wv], t, vv, &cm);
                if constexpr (D1)
                    (void)delta1_g<uint32_t>(vv, n, rl(startv, jh), t);
                uint32_t * oh = out + (first + jh) * n;
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    if (t + 64u * j < n)
                        __builtin_nontemporal_store(vv[j], oh + t + 64u * j);
                used = half == hh ? uw : used;
                wave_lds_sync();
            }
        }
        wave_lds_sync();
        const uint64_t bad = __ballot(act && used != (half ? lenB : lenA));
        badmask |= ((bad & 0xFFFFFFFFull) ? 1ull << ja : 0ull) | ((bad >> 32) ? 1ull << jb : 0ull);
    };

    const uint32_t np = (nr + 1u) / 2u;
    Chunk CA[NP], CB[NP];
#pragma unroll
    for (uint32_t u = 0; u + 1 < NP; ++u)
    {
        P.template issue<0>(CA[u], 2u * u, t);
        P.template issue<0>(CB[u], 2u * u + 1u, t);
    }
    bool more = true;
    for (uint32_t q = 0; more; q += NP)
    {
#pragma unroll
        for (uint32_t u = 0; u < NP; ++u)
        {
            if (more)
            {
                const uint32_t nq = q + u + NP - 1u;
                P.template issue<0>(CA[(u + NP - 1) % NP], 2u * nq, t);
                P.template issue<0>(CB[(u + NP - 1) % NP], 2u * nq + 1u, t);
                consume(CA[u], CB[u], q + u);
                more = q + u + 1u < np;
            }
        }
    }
    if (err != nullptr && t == 0 && badmask != 0u)
        atomicMin(err, static_cast<unsigned long long>(first + __builtin_ctzll(badmask)));
}
} // namespace tpf::dev

extern "C" int c1pair_launch(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t n, uint32_t * out,
                             const uint32_t * starts, unsigned long long * err, hipStream_t s)
{
    const uint64_t per_wg2 = 4ull * tpf::dev::kPRun;
    const uint32_t g2 = static_cast<uint32_t>((nblocks + per_wg2 - 1) / per_wg2);
    if (starts)
        hipLaunchKernelGGL((tpf::dev::k_dec_pair_h32<true>), dim3(g2), dim3(256), 0, s, in, in_bytes, off, nblocks, n, out, starts, err);
    else
        hipLaunchKernelGGL((tpf::dev::k_dec_pair_h32<false>), dim3(g2), dim3(256), 0, s, in, in_bytes, off, nblocks, n, out,
                           static_cast<const uint32_t *>(nullptr), err);
    return static_cast<int>(hipGetLastError());
}
