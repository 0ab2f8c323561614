// p4_enc32.h -- wave-level pieces of the 32-bit P4 encoder (one block per
// wave, lane t owns values 4t..4t+3).
//
// Restates for the GPU:
//   p4Bits32     src/scalar/p4_scalar_internal.cpp:270-387 (cost model)
//   writeHeader  src/scalar/p4_scalar_internal.cpp:409-429
//   p4Enc256v32  src/scalar/p4enc256v32_scalar.cpp:49-235 (payloads)
//   vbEnc32      src/scalar/p4_scalar_internal.cpp:47-89, :163-197
//   deltaEnc1    src/scalar/p4_scalar_internal.h:711-719
//
// The reference walks base widths b = max-1 .. 0 serially, carrying the
// exception count and a vbyte-size accumulator.  Both have closed forms:
//   ec(b)    = sum_{c>b} cnt[c]
//   vbsum(b) = sum_{c>b} (cnt[c] + cnt[c+7] + 2cnt[c+15] + 3cnt[c+19] + 4cnt[c+25])
// so lane b evaluates candidate b in parallel (suffix sums by wave scan) and
// one wave min-reduction picks the first minimum in the reference's order
// (plain first, then descending b; patching preferred over vbyte on ties).
#pragma once

#include "tpf_device.h"

namespace tpf::dev
{

struct Plan32
{
    uint32_t b;    // base bit width
    uint32_t bx;   // 0 plain, 1..32 bitmap patch bits, 33 vbyte, 34 constant
    uint32_t size; // exact encoded byte size
    uint32_t xn;   // exception count
    uint32_t raw;  // vbyte: 1 if the 0xFF raw escape is used
};

__device__ __forceinline__ uint32_t bw32(uint32_t x) { return x ? 32u - __builtin_clz(x) : 0u; }

// vbPut32 byte length (p4_scalar_internal.cpp:47-89)
__device__ __forceinline__ uint32_t vblen32(uint32_t x)
{
    // a sum of compares, not a ?: chain (which compiled into exec-mask branches)
    return 1u + (x >= 156u) + (x >= 16540u) + (x >= 2113692u) + (x > 0xFFFFFFu);
}

// v_ffbh_u32(x) + 1: 0 for x == 0 (ffbh returns -1), else clz(x) + 1 = 33 - bw32(x)
__device__ __forceinline__ uint32_t ffbh1(uint32_t x)
{
    uint32_t r;
    asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
    return r + 1u;
}

// hist: per-wave LDS scratch of kPlanHistU32 u32 (16-byte aligned).
// 4 copies: the plan pass is bound by its LDS traffic as much as by conflicts
// (A/B, C4 encode: 16 copies 447-451 G int32/s, 32 copies 337, 8 copies 454,
// 4 copies 453-457; merging equal widths within a lane first: no gain)
using PlanHist = WaveHist<4, 36>; // bit widths 0..32
constexpr uint32_t kPlanHistU32 = PlanHist::kU32;
// A vbyte block's exception ranks and byte offsets, computed once by the
// plan and handed to the build (the slot encoder plans and builds in one
// wave: FUSE): lane t's exceptions are ranks before.. and their vbytes start
// at byte lbefore of the vbyte area; vtotal = the area's byte count.
struct VbPre
{
    uint32_t before = 0, lbefore = 0, vtotal = 0;
};

template <bool FUSE = false>
__device__ __forceinline__ Plan32 plan_block256(const u32x4 & v, uint32_t * hist, uint32_t t, VbPre * pre = nullptr)
{
    Plan32 P;
    const uint32_t first = __builtin_amdgcn_readlane(v.x, 0);
    // constant block: a ballot, not a wave reduction
    if (__builtin_amdgcn_ballot_w64(!((v.x == first) & (v.y == first) & (v.z == first) & (v.w == first))) == 0ull)
    {
        const uint32_t cb = bw32(first);
        P.b = cb;
        P.bx = first == 0u ? 0u : 34u; // all zero: the plain b = 0 block
        P.size = first == 0u ? 1u : 1u + ((cb + 7u) >> 3);
        P.xn = 0;
        P.raw = 0;
        return P;
    }
    PlanHist::zero(hist, t);
    wave_lds_sync();
    // bins keyed by v_ffbh_u32(x) + 1: 0 for x == 0, else 33 - bw32(x) -- two
    // VALU per value (ffbh, shift-add) instead of clz + zero select + address
    PlanHist::add(hist, ffbh1(v.x), t);
    PlanHist::add(hist, ffbh1(v.y), t);
    PlanHist::add(hist, ffbh1(v.z), t);
    PlanHist::add(hist, ffbh1(v.w), t);
    wave_lds_sync();
    const uint32_t cnt = PlanHist::get(hist, t == 0u ? 0u : (t <= 32u ? 33u - t : 64u)); // lane c: cnt[c] (0 for c > 32)
    wave_lds_sync();
    // the block's bit width: the highest width with a count (a ballot and a
    // scalar bit scan instead of a wave OR reduction of the values, round 5)
    const uint32_t maxb = 63u - static_cast<uint32_t>(__builtin_clzll(__builtin_amdgcn_ballot_w64(cnt != 0u)));
    // suffix sums S(k) = #values with bw > k, then
    // vbsum(b) = S(b) + S(b+7) + 2 S(b+15) + 3 S(b+19) + 4 S(b+25): the shifted
    // sums come back through the histogram's LDS (one write, two ds_read2)
    // instead of four bpermutes of cnt (the plan pass waits on its LDS pipe:
    // plan 1.982 -> 1.836 ms per 10M C4 blocks, round 3)
    const uint32_t incl = wave_incl_scan(cnt);
    const uint32_t ec = __builtin_amdgcn_readlane(incl, 63) - incl; // sum_{c > t} cnt[c]
    hist[t] = ec;                                                    // lanes >= 32 hold 0
    wave_lds_sync();
    const uint32_t vbsum = ec + hist[t + 7u] + 2u * hist[t + 15u] + 3u * hist[t + 19u] + 4u * hist[t + 25u]; // lanes t > 38: unused
    wave_lds_sync();
    uint32_t key = 0xFFFFFFFFu;
    if (t < maxb)
    {
        const uint32_t vsz = 32u * t + 2u + ec + vbsum;
        const uint32_t psz = 32u * t + 2u + 32u + ((ec * (maxb - t) + 7u) >> 3);
        const uint32_t cost = psz <= vsz ? psz : vsz;
        const uint32_t kind = psz <= vsz ? 0u : 1u;
        key = (cost << 8) | ((maxb - t) << 1) | kind;
    }
    else if (t == maxb)
    {
        key = ((32u * maxb + 1u) << 8); // plain: order 0
    }
    key = uni(wave_min(key));
    const uint32_t order = (key >> 1) & 127u;
    const uint32_t kind = key & 1u;
    P.b = maxb - order;
    if (order == 0u)
    {
        P.bx = 0;
        P.size = 1u + 32u * maxb;
        P.xn = 0;
        P.raw = 0;
        return P;
    }
    const uint32_t b = P.b;
    if (kind == 0u)
    {
        // bitmap patch: xn = ec(b), already in lane b (no second reduction;
        // A/B with the constant-test ballot: C4 encode 459-462 -> 463-466)
        const uint32_t xn = uni(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(ec), static_cast<int>(b))));
        P.xn = xn;
        P.bx = maxb - b;
        P.size = 34u + ((xn * P.bx + 7u) >> 3) + 32u * b;
        P.raw = 0;
        return P;
    }
    // vbyte: y = x >> b is non-zero exactly for the exceptions, and
    // vblen32(y) = 1 + [y >= 156] + [y >= 16540] + [y >= 2113692] + [y >= 2^24],
    // so the exception count and their vbyte bytes are ballot popcounts per
    // threshold (compares on the VALU, counts on the scalar unit) instead of a
    // per-value length under exec masks and a wave reduction
    const uint32_t y0 = v.x >> b, y1 = v.y >> b, y2 = v.z >> b, y3 = v.w >> b; // b < maxb <= 32
    if constexpr (FUSE)
    {
        // one wave scan of (exceptions, vbyte bytes) per lane gives the totals
        // here and the build's ranks and byte offsets (emit_block256<.., true>)
        const uint32_t f0 = y0 != 0u, f1 = y1 != 0u, f2 = y2 != 0u, f3 = y3 != 0u;
        const uint32_t mylen = (vblen32(y0) & (0u - f0)) + (vblen32(y1) & (0u - f1)) + (vblen32(y2) & (0u - f2)) + (vblen32(y3) & (0u - f3));
        const uint32_t mine = (f0 + f1 + f2 + f3) | (mylen << 16); // <= 256 exceptions, <= 1280 bytes: no carry between the halves
        const uint32_t incl = wave_incl_scan(mine);
        const uint32_t tot = uni(__builtin_amdgcn_readlane(incl, 63));
        const uint32_t xn = tot & 0xFFFFu, sumlen = tot >> 16;
        pre->before = (incl - mine) & 0xFFFFu;
        pre->lbefore = (incl - mine) >> 16;
        pre->vtotal = sumlen;
        P.xn = xn;
        P.bx = 33;
        P.raw = (sumlen + 32u > 4u * xn) ? 1u : 0u;
        P.size = 2u + 32u * b + (P.raw ? 1u + 4u * xn : sumlen) + xn;
        return P;
    }
    auto count_ge = [&](uint32_t T) -> uint32_t {
        return static_cast<uint32_t>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(y0 >= T))
                                     + __builtin_popcountll(__builtin_amdgcn_ballot_w64(y1 >= T))
                                     + __builtin_popcountll(__builtin_amdgcn_ballot_w64(y2 >= T))
                                     + __builtin_popcountll(__builtin_amdgcn_ballot_w64(y3 >= T)));
    };
    const uint32_t xn = uni(count_ge(1u));
    P.xn = xn;
    P.bx = 33;
    // y < 2^(maxb - b): the thresholds no y can reach are not counted (C3's
    // posting blocks: y < 2^12, two of five counts; round 5)
    const uint64_t ymax = (1ull << (maxb - b)) - 1ull;
    uint32_t sumlen = xn + count_ge(156u);
    if (ymax >= 16540u)
        sumlen += count_ge(16540u);
    if (ymax >= 2113692u)
        sumlen += count_ge(2113692u) + (ymax >= 0x1000000u ? count_ge(0x1000000u) : 0u);
    sumlen = uni(sumlen);
    P.raw = (sumlen + 32u > 4u * xn) ? 1u : 0u;
    const uint32_t vsize = P.raw ? 1u + 4u * xn : sumlen;
    P.size = 2u + 32u * b + vsize + xn;
    return P;
}

// OR nb (<= 32) bits of val (already < 2^nb) at bit position bp of an LDS image.
__device__ __forceinline__ void or_bits(uint32_t * img, uint32_t bp, uint32_t val, uint32_t nb)
{
    if (nb == 0u || val == 0u)
        return;
    const uint32_t q = bp >> 5, sh = bp & 31u;
    atomicOr(&img[q], val << sh);
    if (sh + nb > 32u)
        atomicOr(&img[q + 1], val >> (32u - sh));
}

// ---- block image construction (write pass) --------------------------------
// The image of one block is built in LDS so that its base payload starts on
// a dword: the block starts at image byte sb = kImgLead + s0, s0 in [0,3]
// chosen from the payload offset, and the copy-out shifts by bytes (v_alignbyte).
// Each lane ORs RUNS of up to four consecutive values of one bit stream
// (concatenated in registers first) into the image, so a dword receives few
// atomic ORs: for the base payload lane t = 8l + r takes column l's groups
// 4r..4r+3 (read back transposed from the staged values), for the bitmap
// exceptions its own exceptions, which are consecutive ranks.  The first
// version OR-ed every value separately (32 lanes into one dword at b = 1:
// 162 SALU + 51 LDS-conflict cycles per block); a per-dword gather variant
// was slower still (dependent LDS reads, 7.4 ms per 10M blocks).

// staged masked base values, element e at val_idx(e): with PAD, 4 dwords of
// padding after every 32 elements, so pack_base_runs' column reads (lane
// 8l + r reads element 32r + l + 8j, ds_read_b32 banks (a/4) % 32 per 32-lane
// half) land on 32 distinct banks instead of 8-way on 4 (A/B, C4 encode:
// 455-458 -> 460-464 G int32/s)
// + 64 trash dwords, one per lane, past the PAD layout (which ends at 284):
// bytes a lane does not own in the exception steps go to ITS OWN dword (a
// trash dword shared by lanes serialises their stores)
constexpr uint32_t kEncValU32 = 256 + 32 + 64;
constexpr uint32_t kEncTrash = 256 + 32;
template <bool PAD>
__device__ __forceinline__ uint32_t val_idx(uint32_t e)
{
    return PAD ? e + 4u * (e >> 5) : e;
}
// Block images start at byte kImgLead..kImgLead+3 (the payload lands on a
// dword); the 16-byte lead lets copy_out_image16 address the first chunk
// before the block without going below the image.
constexpr uint32_t kImgLead = 20;

// OR cnt (<= 4) consecutive nb-bit values x[] (each < 2^nb, x[j] = 0 for
// j >= cnt) into a bit stream at stream bit `bit`; stream dword i lives at
// img[dw0 + stride * i].  maxw: a wave-uniform bound on the dwords a run
// touches (extra dwords get OR 0), so the stores are not under divergent
// branches.  1 <= nb <= 32.
__device__ __forceinline__ void or_run(uint32_t * img, uint32_t dw0, uint32_t stride, uint32_t bit, const uint32_t x[4],
                                       uint32_t cnt, uint32_t nb, uint32_t maxw)
{
    uint32_t w[5];
    const uint32_t sh = bit & 31u, q = bit >> 5;
    // No branches (round 4): the run as two 64-bit pairs, the second shifted
    // by 2 nb (2..64, in two steps so that 64 shifts everything out), then
    // the lane's bit offset applied with 64-bit shifts (a shift by 0 needs no
    // special case).  The earlier form branched on the wave-uniform value
    // positions and on the per-lane shift; those branches cost the CU's one
    // scalar unit more than the stores they guarded (C3 D1 encode +7%, C4
    // encode +3%).
    (void)cnt;
    const uint64_t a = static_cast<uint64_t>(x[0]) | (static_cast<uint64_t>(x[1]) << nb);
    const uint64_t c = static_cast<uint64_t>(x[2]) | (static_cast<uint64_t>(x[3]) << nb);
    const uint32_t n2 = 2u * nb;
    const uint64_t lo = a | ((c << (n2 - 1u)) << 1);
    const uint64_t hi = c >> (64u - n2);
    const uint32_t d1 = static_cast<uint32_t>(lo >> 32), d2 = static_cast<uint32_t>(hi);
    w[0] = static_cast<uint32_t>(lo) << sh;
    w[1] = static_cast<uint32_t>((lo << sh) >> 32);
    w[2] = static_cast<uint32_t>((((static_cast<uint64_t>(d2) << 32) | d1) << sh) >> 32);
    w[3] = static_cast<uint32_t>((hi << sh) >> 32);
    w[4] = static_cast<uint32_t>(((hi >> 32) << sh) >> 32);
#pragma unroll
    for (uint32_t i = 0; i < 5; ++i)
        if (i < maxw)
            atomicOr(&img[dw0 + stride * (q + i)], w[i]);
}

// dwords a run of cnt <= 4 nb-bit values can touch at any bit alignment
__device__ __forceinline__ uint32_t run_maxw(uint32_t cnt, uint32_t nb) { return (31u + cnt * nb + 31u) >> 5; }

// Base payload (256v32 layout) at image dword pw from the staged values:
// word (k, l) at img[pw + 8k + l] holds bits [32k, 32k+32) of column l,
// whose g-th value is element 8g + l.
template <bool PAD>
__device__ __forceinline__ void pack_base_runs(uint32_t * img, uint32_t pw, const uint32_t * val, uint32_t b, uint32_t t)
{
    if (b == 0u)
        return;
    const uint32_t l = t >> 3, r = t & 7u;
    const uint32_t e = val_idx<PAD>(32u * r + l); // element of group 4r in column l
    const uint32_t x[4] = {val[e], val[e + 8u], val[e + 16u], val[e + 24u]};
    or_run(img, pw + l, 8u, 4u * r * b, x, 4u, b, run_maxw(4u, b));
}

// Build block image; returns sb (image byte of the block's first byte).
// v: lane t's values 4t..4t+3 (after delta coding), P: plan, val: scratch.
template <bool PAD = false, bool FUSE = false>
__device__ __forceinline__ uint32_t emit_block256(uint32_t * img, uint32_t * val, const Plan32 & P, const u32x4 & v,
                                                  uint32_t t, const VbPre * pre = nullptr)
{
    uint8_t * const ib = reinterpret_cast<uint8_t *>(img);
    const uint32_t b = P.b;
    if (P.bx == 34u)
    {
        // constant block (p4enc256v32_scalar.cpp:183-190): ceil(b/8) value bytes
        const uint32_t x = v.x & mask32(b);
        if (t == 0)
            ib[kImgLead] = static_cast<uint8_t>(0xC0u | b);
        if (t < ((b + 7u) >> 3))
            ib[kImgLead + 1u + t] = static_cast<uint8_t>(x >> (8u * t));
        return kImgLead;
    }
    const uint32_t m = mask32(b);
    const uint32_t xbytes = P.bx <= 32u ? ((P.xn * P.bx + 7u) >> 3) : 0u;
    const uint32_t po = P.bx == 0u ? 1u : (P.bx <= 32u ? 34u + xbytes : 2u); // payload offset in the block
    const uint32_t sb = kImgLead + ((4u - (po & 3u)) & 3u);
    const uint32_t pw = (sb + po) >> 2;
    *reinterpret_cast<u32x4 *>(val + val_idx<PAD>(4u * t)) = u32x4{v.x & m, v.y & m, v.z & m, v.w & m};
    if (P.bx == 0u)
    {
        if (t == 0)
            ib[sb] = static_cast<uint8_t>(b);
        wave_lds_sync();
        pack_base_runs<PAD>(img, pw, val, b, t);
        return sb;
    }
    const uint32_t f0 = v.x > m, f1 = v.y > m, f2 = v.z > m, f3 = v.w > m;
    const uint32_t my = f0 | (f1 << 1) | (f2 << 2) | (f3 << 3);
    const uint32_t cnt = f0 + f1 + f2 + f3;
    // exceptions in elements < 4t (a fused vbyte plan scanned them already)
    const uint32_t before = (FUSE && P.bx == 33u) ? pre->before : wave_incl_scan(cnt) - cnt;
    const uint32_t sh = b & 31u;
    const uint32_t ex[4] = {v.x >> sh, v.y >> sh, v.z >> sh, v.w >> sh};
    if (P.bx <= 32u)
    {
        // [0x80|b][bx][bitmap 32B][xn*bx bits horizontal][256v32 base]
        const uint32_t mynext = wave_shl1(my, 0u);
        if (t == 0)
        {
            ib[sb] = static_cast<uint8_t>(0x80u | b);
            ib[sb + 1u] = static_cast<uint8_t>(P.bx);
        }
        if ((t & 1u) == 0u)
            ib[sb + 2u + (t >> 1)] = static_cast<uint8_t>(my | (mynext << 4));
        wave_lds_sync();
        pack_base_runs<PAD>(img, pw, val, b, t);
        // this lane's exceptions are the consecutive ranks before..before+cnt-1
        // compact the flagged values to the front, in order (selects only)
        uint32_t xr[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 3; j >= 0; --j)
        {
            const bool fj = (my >> j) & 1u;
            xr[3] = fj ? xr[2] : xr[3];
            xr[2] = fj ? xr[1] : xr[2];
            xr[1] = fj ? xr[0] : xr[1];
            xr[0] = fj ? ex[j] : xr[0];
        }
        if (cnt != 0u) // lanes without exceptions share `before` with a neighbour: no zero ORs
            or_run(img, 0u, 1u, (sb + 34u) * 8u + before * P.bx, xr, cnt, P.bx, run_maxw(4u, P.bx));
        return sb;
    }
    // vbyte: [0x40|b][xn][256v32 base][V][positions]
    if (t == 0)
    {
        ib[sb] = static_cast<uint8_t>(0x40u | b);
        ib[sb + 1u] = static_cast<uint8_t>(P.xn);
    }
    wave_lds_sync();
    pack_base_runs<PAD>(img, pw, val, b, t);
    const uint32_t v0 = sb + 2u + 32u * b;
    // Exception emission (round 5), in two steps so that the per-exception
    // byte work runs once per 64 exceptions instead of once per exception a
    // lane holds (the wave's maximum, 2-3 steps on C3's posting blocks):
    //  1. the shifted values go to val[4t + j] in element order (one 16-byte
    //     store; `val` is free once pack_base_runs has read it, a wave's LDS
    //     operations complete in order) and the lane's i-th flagged element
    //     (lowest set bit of its flag mask) writes its position byte to rank
    //     before + i of the block's last xn bytes;
    //  2. lane r takes rank r: its position byte names its value; raw words
    //     at 4r, or vbytes at the exclusive wave scan of the lengths
    //     (p4_scalar_internal.cpp:47-89, :163-197).
    // Every lane stores in every step: what a lane does not own goes to its
    // own trash dword past the PAD layout, so the steps carry no exec-mask
    // sections (measured: element-order values with the positions OR-ed in
    // by every lane were 24% slower on C3 -- idle lanes' atomics on their
    // neighbours' dwords serialise).
    uint32_t * const trash = val + kEncTrash + t;
    const uint32_t trash_at = static_cast<uint32_t>(reinterpret_cast<uint8_t *>(trash) - ib); // (mod 2^32: LDS addresses are 32-bit)
    auto put = [&](bool own, uint32_t at, uint32_t byte) {
        ib[__builtin_unpredictable(own) ? at : trash_at] = static_cast<uint8_t>(byte);
    };
    const uint32_t mc = (__builtin_amdgcn_ballot_w64(cnt >= 1u) != 0u) + (__builtin_amdgcn_ballot_w64(cnt >= 2u) != 0u) +
                        (__builtin_amdgcn_ballot_w64(cnt >= 3u) != 0u) + (__builtin_amdgcn_ballot_w64(cnt >= 4u) != 0u);
    const uint32_t pbase = sb + P.size - P.xn; // the position bytes end the block
    *reinterpret_cast<u32x4 *>(val + 4u * t) = u32x4{ex[0], ex[1], ex[2], ex[3]};
    uint32_t rem = my;
#pragma unroll
    for (uint32_t i = 0; i < 4u; ++i)
        if (i < mc)
        {
            const bool on = rem != 0u;
            const uint32_t j = on ? static_cast<uint32_t>(__builtin_ctz(rem)) : 0u;
            rem &= rem - 1u;
            put(on, pbase + before + i, 4u * t + j);
        }
    wave_lds_sync();
    auto rank_value = [&](uint32_t r) { return val[ib[pbase + min(r, P.xn - 1u)]]; };
    if (P.raw)
    {
        // 0xFF, xn raw LE words, the positions
        if (t == 0)
            ib[v0] = 0xFFu;
        for (uint32_t c = 0; c < P.xn; c += 64u)
        {
            const uint32_t r = c + t;
            const bool on = r < P.xn;
            const uint32_t x = rank_value(r), A = v0 + 1u + 4u * r;
            put(on, A, x);
            put(on, A + 1u, x >> 8);
            put(on, A + 2u, x >> 16);
            put(on, A + 3u, x >> 24);
        }
        return sb;
    }
    uint32_t vb = v0; // byte of the chunk's first vbyte
    for (uint32_t c = 0; c < P.xn; c += 64u)
    {
        const uint32_t r = c + t;
        const bool on = r < P.xn;
        const uint32_t x = rank_value(r);
        const uint32_t d2 = x - 156u;
        const bool g1 = x >= 156u;
        if (__builtin_amdgcn_ballot_w64(on && x >= 16540u) == 0ull)
        {
            // every value of the chunk takes 1 or 2 bytes (posting-list
            // gaps: C3's blocks): no 3-5 byte forms (wave-uniform branch)
            const uint32_t L = on ? 1u + g1 : 0u;
            const uint32_t incl = wave_incl_scan(L);
            const uint32_t A = vb + incl - L;
            vb += __builtin_amdgcn_readlane(incl, 63);
            const uint32_t lo = __builtin_unpredictable(g1) ? (0x9Cu + (d2 >> 8)) | ((d2 & 0xFFu) << 8) : x;
            put(on, A, lo);
            put(L > 1u, A + 1u, lo >> 8);
            continue;
        }
        const uint32_t d3 = x - 16540u;
        const bool g2 = x >= 16540u, g3 = x >= 2113692u, g4 = x > 0xFFFFFFu;
        const uint32_t L = on ? 1u + g1 + g2 + g3 + g4 : 0u;
        const uint32_t incl = wave_incl_scan(L);
        const uint32_t A = vb + incl - L;
        vb += __builtin_amdgcn_readlane(incl, 63);
        // the value's first four bytes (the fifth, of a 5-byte value, is
        // x >> 24), selected by the range tests (an L == k chain compiled
        // into exec-mask branches)
        const uint32_t c2 = (0x9Cu + (d2 >> 8)) | ((d2 & 0xFFu) << 8);
        const uint32_t c3 = (0xDCu + (d3 >> 16)) | ((d3 & 0xFFFFu) << 8);
        const uint32_t c45 = (g4 ? 0xFDu : 0xFCu) | (x << 8);
        const uint32_t c23 = __builtin_unpredictable(g2) ? c3 : c2;
        const uint32_t c25 = __builtin_unpredictable(g3) ? c45 : c23;
        const uint32_t lo = __builtin_unpredictable(g1) ? c25 : x;
        put(on, A, lo);
        put(L > 1u, A + 1u, lo >> 8);
        put(L > 2u, A + 2u, lo >> 16);
        put(L > 3u, A + 3u, lo >> 24);
        put(L > 4u, A + 4u, x >> 24);
    }
    return sb;
}

// Copy a block built in an LDS image (block byte 0 at image byte sb >= 16)
// to dst (any alignment) with 16-byte stores: global chunk k of a16 = dst & ~15
// holds block bytes [16k - ph, 16k - ph + 16), ph = dst & 15, i.e. image
// bytes from base + 16k, base = sb - ph.  A full chunk costs 5 aligned
// ds_read_b32 + 4 v_alignbyte + one global_store_dwordx4 per lane (a 600-byte
// block: one store instruction instead of three dword stores); the partial
// first and last chunks, shared with the neighbouring blocks, are written
// byte by byte (lanes 0-15 and 16-31); a block crossing cap_end entirely byte
// by byte.
// Zero image u32x4 slots [0, n16) (a whole image: kImgU32 / 4).
__device__ __forceinline__ void zero_image(uint32_t * img, uint32_t n16, uint32_t t)
{
    for (uint32_t i = t; i < n16; i += 64u)
        reinterpret_cast<u32x4 *>(img)[i] = u32x4{0u, 0u, 0u, 0u};
}

__device__ __forceinline__ void copy_out_image16(const uint32_t * img, uint32_t sb, uint64_t dst, uint32_t size, uint64_t cap_end,
                                                 uint32_t t)
{
    const uint8_t * ib = reinterpret_cast<const uint8_t *>(img);
    const uint32_t ph = static_cast<uint32_t>(dst & 15u);
    const uint32_t base = sb - ph;
    // global address space: a pointer made from an integer is generic, and
    // flat stores also count against lgkmcnt, so every later LDS wait of
    // the wave would wait for these stores to reach memory
    typedef __attribute__((address_space(1))) uint8_t gu8;
    typedef __attribute__((address_space(1))) u32x4 gu32x4;
    gu8 * const a16 = (gu8 *)(dst & ~15ull);
    const uint32_t end = ph + size;
    if (dst + size <= cap_end)
    {
        const bool first_partial = ph != 0u || end < 16u;
        const uint32_t k_lo = first_partial ? 1u : 0u;
        const uint32_t k_hi = end >> 4; // chunks below k_hi end inside the block
        const uint32_t bs = base & 3u;
        for (uint32_t k = k_lo + t; k < k_hi; k += 64u)
        {
            const uint32_t q = (base >> 2) + 4u * k;
            const uint32_t w0 = img[q], w1 = img[q + 1], w2 = img[q + 2], w3 = img[q + 3], w4 = img[q + 4];
            const u32x4 c = u32x4{__builtin_amdgcn_alignbyte(w1, w0, bs), __builtin_amdgcn_alignbyte(w2, w1, bs),
                                  __builtin_amdgcn_alignbyte(w3, w2, bs), __builtin_amdgcn_alignbyte(w4, w3, bs)};
            *(gu32x4 *)(a16 + 16u * k) = c;
        }
        const uint32_t last = (end - 1u) >> 4; // chunk holding the block's last byte
        const uint32_t k = t < 16u ? 0u : last;
        const bool edge = ((t < 16u) & first_partial) | ((t >= 16u) & (t < 32u) & (last > 0u) & ((end & 15u) != 0u));
        const uint32_t gi = 16u * k + (t & 15u); // byte index from a16
        if (edge && gi >= ph && gi < end)
            a16[gi] = ib[base + gi];
    }
    else
    {
        for (uint32_t gi = ph + t; gi < end; gi += 64u)
            if (reinterpret_cast<uint64_t>(a16 + gi) < cap_end)
                a16[gi] = ib[base + gi];
    }
}


// Round 5's RunCopy (a run's blocks copied out in whole 16-byte chunks, the
// open chunk carried from block to block through lanes 0-15) became RunCopyB
// below in round 6: the same chunking, addressed through one buffer
// descriptor per run with the layout read per block.

// ---- round 6: the write pass with its scalar side cut ----------------------
// VERDICT r5 #1 read the D1 write pass's 136 SALU + 29 branches per block
// (against 141 VALU) as the CU's one scalar unit binding the pass: every block
// re-derived its layout (payload offset, image phase, header bytes, copy-out
// chunk range, 64-bit destination) with scalar arithmetic and wrapped each
// single-lane step in an exec-mask section.  Round 6 cut the scalar side:
//   * single-lane stores (headers, bitmap bytes, carried bytes, raw marker)
//     are stores from every lane, unowned lanes sent to their own trash dword
//     (LDS) or an out-of-range buffer offset (HBM: the store is dropped);
//   * the copy-out addresses a run's output through ONE buffer descriptor
//     with 32-bit offsets (RunCopyB), the chunk loop's stores need no mask;
//   * a block's layout comes from three values read per block (plan word,
//     size, output byte) by one closed-form derivation (enc_geo);
//   * the rank scatter, the vbyte loop and the base packing test their
//     bounds with nested wave-uniform branches (one test per C3 block).
// Measured (profiles/r6_enc_counters.txt, r6 A/B), per C3 block: this form
// issues 114 SALU + 128 VALU + 28.5 branches (round 5: 136 + 141 + 28.8); a
// first round-6 form with the layouts in a run plane of vector lanes, read
// with 18 v_readlane per block, issued 42 SALU + 144 VALU + 18.6 branches but
// needed 19 more VGPRs (6 instead of 7 waves per SIMD) and ran slower.  Both
// run the C3 write pass ~3% faster than round 5: the scalar unit was not
// what bound it.  The C4 write pass runs at the time of its own data-movement
// probe (the same loads and stores with the building removed: 3.13-3.19 vs
// 3.10-3.22 ms per 10M blocks), C3's 19-25% above the D1 probe.

// Buffer offset that the hardware range check drops (stores) / zeroes (loads).
constexpr uint32_t kOob = 0x80000000u;
// dwords of a write-pass block image (256v32 and 128v64: 4..7 lead bytes + a
// block of <= 2276 B + slack, a 16-byte multiple)
constexpr uint32_t kImgU32Max = 592;

// Copy-out layout of a block built at image byte sb (RunCopyB), from its
// size, its output byte rel relative to the run's 16-byte aligned output base
// and the run's lead (= the first block's rel: bytes of the open chunk that
// belong to the previous run).  ph: bytes of the open chunk before the block;
// base: image byte of that chunk; a16: its output offset; nfull: chunks the
// block completes; r: bytes of the chunk it leaves open (at image byte tb);
// kfirst: 1 when chunk 0 is the run's partial first chunk (byte stores);
// n16: image chunks to clear after the block.
struct CopyGeo
{
    uint32_t ph, base, a16, nfull, r, tb, kfirst, n16;
};

__device__ __forceinline__ CopyGeo copy_geo(uint32_t sb, uint32_t size, uint32_t rel, uint32_t lead, uint32_t img_u32)
{
    CopyGeo C;
    C.ph = rel & 15u;
    C.base = sb - C.ph;
    const uint32_t end = C.ph + size;
    C.nfull = end >> 4;
    C.r = end & 15u;
    C.tb = C.base + 16u * C.nfull;
    C.a16 = rel & ~15u;
    C.kfirst = (lead != 0u && rel < 16u) ? 1u : 0u;
    C.n16 = min((sb + size + 15u) >> 4, img_u32 / 4u);
    return C;
}

// Layout of one block.  sb: image byte of the block's first byte; pw: image
// dword of its base payload; hdr: header bytes 0 | 1 << 8 (byte 1 is 0 for a
// plain block: a payload byte, OR-ed afterwards); v0 / pbase: vbyte area /
// position bytes; c: copy-out.
struct EncGeo
{
    uint32_t b, m, bx, xn, raw, sb, pw, hdr, v0, pbase;
    CopyGeo c;
};

// Lane form: pwd = plan word (b | bx << 8 | xn << 16 | raw << 25), size =
// block bytes, rel = its output byte relative to the run's 16-byte aligned
// output base, lead = the run's first rel (bytes of the open chunk that
// belong to the previous run).
__device__ __forceinline__ EncGeo enc_geo(uint32_t pwd, uint32_t size, uint32_t rel, uint32_t lead)
{
    EncGeo G;
    G.b = pwd & 0xFFu;
    G.bx = (pwd >> 8) & 0xFFu;
    G.xn = (pwd >> 16) & 0x1FFu;
    G.raw = (pwd >> 25) & 1u;
    G.m = mask32(G.b);
    const bool bmp = G.bx != 0u && G.bx <= 32u, cst = G.bx == 34u;
    const uint32_t xbytes = bmp ? ((G.xn * G.bx + 7u) >> 3) : 0u;
    const uint32_t po = G.bx == 0u ? 1u : (bmp ? 34u + xbytes : 2u); // payload offset in the block
    G.sb = cst ? kImgLead : kImgLead + ((4u - (po & 3u)) & 3u);
    G.pw = (G.sb + po) >> 2;
    G.hdr = G.bx == 0u ? G.b : (bmp ? ((0x80u | G.b) | (G.bx << 8)) : (cst ? (0xC0u | G.b) : ((0x40u | G.b) | (G.xn << 8))));
    G.v0 = G.sb + 2u + 32u * G.b;
    G.pbase = G.sb + size - G.xn;
    G.c = copy_geo(G.sb, size, rel, lead, kImgU32Max);
    return G;
}

// OR a run of four nb-bit values (or_run's packing) with the store count
// decided by nested wave-uniform tests: a block of width <= 8 pays one test
// (or_run's unrolled `i < maxw` bound compiled into three compares).
__device__ __forceinline__ void or_run4(uint32_t * img, uint32_t dw0, uint32_t stride, uint32_t bit, const uint32_t x[4], uint32_t nb)
{
    const uint32_t sh = bit & 31u, q = bit >> 5;
    const uint64_t a = static_cast<uint64_t>(x[0]) | (static_cast<uint64_t>(x[1]) << nb);
    const uint64_t c = static_cast<uint64_t>(x[2]) | (static_cast<uint64_t>(x[3]) << nb);
    const uint32_t n2 = 2u * nb;
    const uint64_t lo = a | ((c << (n2 - 1u)) << 1);
    const uint64_t hi = c >> (64u - n2);
    const uint32_t d1 = static_cast<uint32_t>(lo >> 32), d2 = static_cast<uint32_t>(hi);
    atomicOr(&img[dw0 + stride * q], static_cast<uint32_t>(lo) << sh);
    atomicOr(&img[dw0 + stride * (q + 1u)], static_cast<uint32_t>((lo << sh) >> 32));
    if (nb > 8u) // (31 + 4 nb + 31) >> 5 dwords at most
    {
        atomicOr(&img[dw0 + stride * (q + 2u)], static_cast<uint32_t>((((static_cast<uint64_t>(d2) << 32) | d1) << sh) >> 32));
        if (nb > 16u)
        {
            atomicOr(&img[dw0 + stride * (q + 3u)], static_cast<uint32_t>((hi << sh) >> 32));
            if (nb > 24u)
                atomicOr(&img[dw0 + stride * (q + 4u)], static_cast<uint32_t>(((hi >> 32) << sh) >> 32));
        }
    }
}

template <bool PAD>
__device__ __forceinline__ void pack_base_runs4(uint32_t * img, uint32_t pw, const uint32_t * val, uint32_t b, uint32_t t)
{
    if (b == 0u)
        return;
    const uint32_t l = t >> 3, r = t & 7u;
    const uint32_t e = val_idx<PAD>(32u * r + l); // element of group 4r in column l
    const uint32_t x[4] = {val[e], val[e + 8u], val[e + 16u], val[e + 24u]};
    if (b <= 8u)
    {
        // the run's 4b <= 32 bits in one dword, placed by one 64-bit shift
        // (or_run4 builds two 64-bit pairs: ~9 VALU more per block; C3's
        // posting blocks have b <= 8)
        const uint32_t run = x[0] | (x[1] << b) | (x[2] << (2u * b)) | (x[3] << (3u * b));
        const uint32_t bit = 4u * r * b, q = bit >> 5;
        const uint64_t w = static_cast<uint64_t>(run) << (bit & 31u);
        atomicOr(&img[pw + l + 8u * q], static_cast<uint32_t>(w));
        atomicOr(&img[pw + l + 8u * (q + 1u)], static_cast<uint32_t>(w >> 32));
        return;
    }
    or_run4(img, pw + l, 8u, 4u * r * b, x, b);
}

// Build a block image from its uniform layout G (emit_block256's bytes:
// p4enc256v32_scalar.cpp:49-194, vbEnc32 p4_scalar_internal.cpp:47-89,
// :163-197), with no exec-mask section on the plain and vbyte paths.
template <bool PAD>
__device__ __forceinline__ void emit_block256_g(uint32_t * img, uint32_t * val, const EncGeo & G, const u32x4 & v, uint32_t t)
{
    uint8_t * const ib = reinterpret_cast<uint8_t *>(img);
    uint32_t * const trash = val + kEncTrash + t;
    const uint32_t trash_at = static_cast<uint32_t>(reinterpret_cast<uint8_t *>(trash) - ib); // (mod 2^32: LDS addresses are 32-bit)
    auto put = [&](bool own, uint32_t at, uint32_t byte) {
        ib[__builtin_unpredictable(own) ? at : trash_at] = static_cast<uint8_t>(byte);
    };
    const uint32_t b = G.b;
    if (G.bx == 34u)
    {
        // constant block (p4enc256v32_scalar.cpp:183-190): header, ceil(b/8) value bytes
        const uint32_t x = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v.x), 0)) & G.m;
        put(t <= ((b + 7u) >> 3), kImgLead + t, t == 0u ? G.hdr : x >> (8u * ((t - 1u) & 3u)));
        return;
    }
    // header bytes 0 and 1 from lanes 0 and 1 (a plain block's byte 1 is a
    // payload byte: 0 here, OR-ed below; the wave's LDS operations run in order)
    put(t < 2u, G.sb + t, G.hdr >> (8u * (t & 1u)));
    const uint32_t m = G.m;
    *reinterpret_cast<u32x4 *>(val + val_idx<PAD>(4u * t)) = u32x4{v.x & m, v.y & m, v.z & m, v.w & m};
    if (G.bx == 0u)
    {
        wave_lds_sync();
        pack_base_runs4<PAD>(img, G.pw, val, b, t);
        return;
    }
    const uint32_t f0 = v.x > m, f1 = v.y > m, f2 = v.z > m, f3 = v.w > m;
    const uint32_t my = f0 | (f1 << 1) | (f2 << 2) | (f3 << 3);
    const uint32_t cnt = f0 + f1 + f2 + f3;
    const uint32_t before = wave_incl_scan(cnt) - cnt; // exceptions in elements < 4t
    const uint32_t sh = b & 31u;
    const uint32_t ex[4] = {v.x >> sh, v.y >> sh, v.z >> sh, v.w >> sh};
    if (G.bx <= 32u)
    {
        // [0x80|b][bx][bitmap 32B][xn*bx bits horizontal][256v32 base]
        const uint32_t mynext = wave_shl1(my, 0u);
        put((t & 1u) == 0u, G.sb + 2u + (t >> 1), my | (mynext << 4));
        wave_lds_sync();
        pack_base_runs4<PAD>(img, G.pw, val, b, t);
        uint32_t xr[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 3; j >= 0; --j)
        {
            const bool fj = (my >> j) & 1u;
            xr[3] = fj ? xr[2] : xr[3];
            xr[2] = fj ? xr[1] : xr[2];
            xr[1] = fj ? xr[0] : xr[1];
            xr[0] = fj ? ex[j] : xr[0];
        }
        if (cnt != 0u) // lanes without exceptions share `before` with a neighbour: no zero ORs
            or_run4(img, 0u, 1u, (G.sb + 34u) * 8u + before * G.bx, xr, G.bx);
        return;
    }
    // vbyte: [0x40|b][xn][256v32 base][V][positions] -- emit_block256's two
    // steps (position bytes by rank, then one rank per lane)
    wave_lds_sync();
    pack_base_runs4<PAD>(img, G.pw, val, b, t);
    const uint32_t xn = G.xn, pbase = G.pbase, v0 = G.v0;
    *reinterpret_cast<u32x4 *>(val + 4u * t) = u32x4{ex[0], ex[1], ex[2], ex[3]};
    // the lane's i-th flagged element writes its position byte to rank
    // before + i: i = 0 from every lane, i >= 1 only when a lane holds that
    // many (two wave-uniform tests instead of a four-step maximum)
    uint32_t rem = my;
    auto scat = [&](uint32_t i) {
        const bool on = rem != 0u;
        const uint32_t j = on ? static_cast<uint32_t>(__builtin_ctz(rem)) : 0u;
        rem &= rem - 1u;
        put(on, pbase + before + i, 4u * t + j);
    };
    scat(0u);
    if (__builtin_amdgcn_ballot_w64(cnt >= 2u) != 0ull)
    {
        scat(1u);
        if (__builtin_amdgcn_ballot_w64(cnt >= 3u) != 0ull)
        {
            scat(2u);
            scat(3u);
        }
    }
    wave_lds_sync();
    auto rank_value = [&](uint32_t r) { return val[ib[pbase + min(r, xn - 1u)]]; };
    if (G.raw)
    {
        // 0xFF, xn raw LE words, the positions
        for (uint32_t c = 0; c < xn; c += 64u)
        {
            const uint32_t r = c + t;
            const bool on = r < xn;
            const uint32_t x = rank_value(r), A = v0 + 1u + 4u * r;
            put(on, A, x);
            put(on, A + 1u, x >> 8);
            put(on, A + 2u, x >> 16);
            put(on, A + 3u, x >> 24);
        }
        put(t == 0u, v0, 0xFFu); // after the words: lane 0's own bytes above went to [v0 + 1, v0 + 5)
        return;
    }
    uint32_t vb = v0; // byte of the chunk's first vbyte
    uint32_t c = 0;
    do // xn >= 1: the first 64 ranks without a loop test
    {
        const uint32_t r = c + t;
        const bool on = r < xn;
        const uint32_t x = rank_value(r);
        const uint32_t d2 = x - 156u;
        const bool g1 = x >= 156u;
        if (__builtin_amdgcn_ballot_w64(on && x >= 16540u) == 0ull)
        {
            // every value of the chunk takes 1 or 2 bytes (posting-list
            // gaps): rank r's first byte is at vb + r + the 2-byte values
            // before it -- a ballot and mbcnt, no wave scan (the ranks in use
            // are a prefix of the lanes)
            const uint64_t two = __builtin_amdgcn_ballot_w64(on && g1);
            const uint32_t A = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(two >> 32),
                                                         __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(two), vb + t));
            vb += min(xn - c, 64u) + static_cast<uint32_t>(__builtin_popcountll(two));
            const uint32_t lo = __builtin_unpredictable(g1) ? (0x9Cu + (d2 >> 8)) | ((d2 & 0xFFu) << 8) : x;
            put(on, A, lo);
            put(on && g1, A + 1u, lo >> 8);
        }
        else
        {
            const uint32_t d3 = x - 16540u;
            const bool g2 = x >= 16540u, g3 = x >= 2113692u, g4 = x > 0xFFFFFFu;
            const uint32_t L = on ? 1u + g1 + g2 + g3 + g4 : 0u;
            const uint32_t incl = wave_incl_scan(L);
            const uint32_t A = vb + incl - L;
            vb += __builtin_amdgcn_readlane(incl, 63);
            const uint32_t c2 = (0x9Cu + (d2 >> 8)) | ((d2 & 0xFFu) << 8);
            const uint32_t c3 = (0xDCu + (d3 >> 16)) | ((d3 & 0xFFFFu) << 8);
            const uint32_t c45 = (g4 ? 0xFDu : 0xFCu) | (x << 8);
            const uint32_t c23 = __builtin_unpredictable(g2) ? c3 : c2;
            const uint32_t c25 = __builtin_unpredictable(g3) ? c45 : c23;
            const uint32_t lo = __builtin_unpredictable(g1) ? c25 : x;
            put(on, A, lo);
            put(L > 1u, A + 1u, lo >> 8);
            put(L > 2u, A + 2u, lo >> 16);
            put(L > 3u, A + 3u, lo >> 24);
            put(L > 4u, A + 4u, x >> 24);
        }
        c += 64u;
    } while (c < xn);
}

// Clear image chunks [0, n16): one exec-masked store per lane, a loop only
// for images past 1 KB.
__device__ __forceinline__ void zero_image_n(uint32_t * img, uint32_t n16, uint32_t t)
{
    if (t < n16)
        reinterpret_cast<u32x4 *>(img)[t] = u32x4{0u, 0u, 0u, 0u};
    if (n16 > 64u)
        for (uint32_t i = 64u + t; i < n16; i += 64u)
            reinterpret_cast<u32x4 *>(img)[i] = u32x4{0u, 0u, 0u, 0u};
}

// Round 5's RunCopy with the block's copy-out layout (CopyGeo): the run's
// output is addressed through ONE buffer descriptor (base = the run's first
// output byte rounded down to 16, 32-bit offsets), the carried bytes placed
// from every lane (unowned lanes write their trash dword).  The run's partial
// first chunk (bytes [lead, 16) of chunk 0) is stored by the block that
// completes it (a wave-uniform flag) and the partial last chunk once after
// the run (flush_tail).
struct RunCopyB
{
    uint32_t carry = 0u; // lane t < r: byte t of the open output chunk
    __amdgpu_buffer_rsrc_t rs;

    __device__ __forceinline__ void put(uint32_t * img, const CopyGeo & G, bool flush_lead, uint32_t lead, uint32_t trash_at,
                                       uint32_t t)
    {
        uint8_t * ib = reinterpret_cast<uint8_t *>(img);
        // the carried bytes in front of the block (lanes t < lead carry zeros: never stored)
        ib[t < G.ph ? G.base + t : trash_at] = static_cast<uint8_t>(carry);
        wave_lds_sync();
        const uint32_t bs = G.base & 3u;
        for (uint32_t k0 = G.kfirst;; k0 += 64u)
        {
            // only the lanes with a chunk read the image: 64 lanes reading
            // 16-byte strided dwords conflict 4-way in the LDS banks (the
            // unmasked form: +27 conflict cycles per C3 block, -0.7% on C3
            // D1 encode and C4 encode, r6e)
            const uint32_t k = k0 + t;
            if (k < G.nfull)
            {
                const uint32_t q = (G.base >> 2) + 4u * k;
                const uint32_t w0 = img[q], w1 = img[q + 1], w2 = img[q + 2], w3 = img[q + 3], w4 = img[q + 4];
                const u32x4 c = u32x4{__builtin_amdgcn_alignbyte(w1, w0, bs), __builtin_amdgcn_alignbyte(w2, w1, bs),
                                      __builtin_amdgcn_alignbyte(w3, w2, bs), __builtin_amdgcn_alignbyte(w4, w3, bs)};
                __builtin_amdgcn_raw_buffer_store_b128(c, rs, static_cast<int>(G.a16 + 16u * k), 0, 0);
            }
            if (__builtin_expect(G.nfull <= k0 + 64u, 1)) // wave-uniform: chunks left?
                break;
        }
        if (flush_lead)
        {
            // the run's first chunk: bytes [lead, 16) are ours (G.a16 == 0 here)
            const uint32_t byte = ib[G.base + (t & 15u)];
            __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(byte), rs, static_cast<int>(t >= lead && t < 16u ? t : kOob), 0, 0);
        }
        const uint32_t nb = ib[G.tb + (t & 15u)];
        carry = t < G.r ? nb : 0u;
    }

    // after the run's last block: its partial last chunk (rel_end = the
    // run's end relative to the descriptor; the run's first chunk is shared
    // with the previous run when the whole run ends inside it)
    __device__ __forceinline__ void flush_tail(uint32_t rel_end, uint32_t lead, uint32_t t)
    {
        const uint32_t r = rel_end & 15u;
        const uint32_t lo = rel_end < 16u ? lead : 0u;
        __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(carry), rs,
                                             static_cast<int>(t >= lo && t < r ? (rel_end & ~15u) + t : kOob), 0, 0);
    }
};

} // namespace tpf::dev
