// p4_generic.hip -- batch kernels for the non-hot formats of include/turbopfor.h
// (32/64-bit horizontal, 128v32, 256v32 with n != 256) on gfx950; the
// 128v64/256v64 units are routed to p4_dec256v64.hip / p4_enc256v64.hip.
//
// Every wave owns a contiguous run of 16 blocks with the next blocks' bytes
// (or values) in flight.  Decode stages each block into a per-wave LDS slot
// (RunPlaneT, p4_dec_run.h) and runs decode_block_g (p4_generic.h); encode
// is the same three-pass scheme as the 256v32 encoder: plan pass -> exclusive
// scan -> write pass (LDS image copied out with dword stores and byte stores
// on the two shared edge dwords).
#include "p4_scan.h"

#include "p4_dec_run.h"
#include "p4_generic.h"
#include "tpf_kernels.h"

namespace tpf::dev
{

template <Fmt F, bool PAIR>
struct UnitGeom
{
    using T = typename FmtTraits<F>::T;
    static constexpr uint32_t kSlot = PAIR ? 4864u : 2432u; // staging / image bytes per wave
    __device__ static uint32_t nsub(uint32_t n) { return PAIR ? 128u : n; }
    __device__ static uint32_t per_unit(uint32_t n) // values per unit in the value arrays
    {
        return PAIR ? 256u : (FmtTraits<F>::N ? FmtTraits<F>::N : n);
    }
};

// Run-pipelined decode for the one-block units (H32, V128, V256 n != 256,
// H64): every wave owns a contiguous run of kGRun blocks, the run's
// control plane lives in vector lanes and the bytes of the next NC-1 blocks
// are in flight while one decodes (RunPlaneT, p4_dec_run.h -- the machinery
// of the 256v32 hot path).  The first version (one block per wave, grid
// stride: load, wait, decode) ran at 0.20 of HBM peak on p4Dec32 n=127
// batches (bench.py c1); 128v64/256v64 units use p4_dec256v64.hip.
constexpr uint32_t kGRun = 16;

template <Fmt F, bool D1, uint32_t NC = 4>
// SGPRs capped at 80 (a few spill to VGPR lanes): at 101 the scalar file
// (800 per SIMD, 16-register granules + 16) held the kernel to 6 waves per
// SIMD, one below its VGPR limit; C1 decode +4-5% (A/B on one box).
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_sgpr(80))) void k_dec_gr(const uint8_t * __restrict in, uint64_t in_bytes, const uint64_t * __restrict off,
                                                 uint64_t nblocks, uint32_t n, typename FmtTraits<F>::T * __restrict out,
                                                 const typename FmtTraits<F>::T * __restrict starts,
                                                 unsigned long long * __restrict err)
{
    using G = UnitGeom<F, false>;
    using T = typename FmtTraits<F>::T;
    __shared__ uint32_t slots[4][G::kSlot / 4];
    __shared__ T scratch[4][512];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t * slot = slots[wv];
    const uint64_t in_base = reinterpret_cast<uint64_t>(in);
    const uint64_t in_end = in_base + in_bytes;
    const uint32_t pu = G::per_unit(n);
    const uint32_t NE = FmtTraits<F>::N ? FmtTraits<F>::N : n;
    const uint64_t first = (static_cast<uint64_t>(blockIdx.x) * 4u + wv) * kGRun;
    if (first >= nblocks)
        return;
    const uint32_t nr = static_cast<uint32_t>(min_u64(kGRun, nblocks - first));
    const bool valid = t < nr;
    const uint64_t o = valid ? off[first + t] : 0ull;
    const uint64_t e = valid ? off[first + t + 1u] : 0ull;
    RunPlaneT<G::kSlot> P;
    P.init(in_base, in_end, o, e, valid);
    const T startv = (D1 && valid) ? starts[first + t] : T(0);
    uint64_t badmask = 0u;
    auto consume = [&](const Chunk & c, uint32_t jj) {
        const uint32_t ctl = P.stage(c, jj, slot, t);
        T v[4];
        uint32_t cm;
        const uint32_t used = decode_block_g<F>(slot, (ctl >> kCtlShift) & 15u, n, scratch[wv], t, v, &cm);
        if constexpr (D1)
        {
            T st;
            if constexpr (sizeof(T) == 8)
                st = readlane_u64(startv, jj);
            else
                st = rl(startv, jj);
            (void)delta1_g<T>(v, n, st, t);
        }
        const uint32_t lim = cm ? n : NE;
        T * op = out + (first + jj) * pu;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            if (t + 64u * j < lim)
                __builtin_nontemporal_store(v[j], op + t + 64u * j);
        wave_lds_sync();
        // per-block scalar check kept here: the lane-held form (UsedLanes,
        // p4_dec_run.h) measured -2.3% on C1 (A/B on one box)
        if (used != rl(P.len, jj))
            badmask |= 1ull << jj;
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
                more = j + u + 1 < nr;
            }
        }
    }
    if (err != nullptr && t == 0 && badmask != 0u)
        atomicMin(err, static_cast<unsigned long long>(first + __builtin_ctzll(badmask)));
}

// ---- p4Dec32 / p4D1Dec32 batches (n <= 256): windows staged whole ---------
// C1 (BASELINE configs[0]) is n = 127: 128-byte blocks for 508 B of output.
// k_dec_gr stages and parses every block on its own -- per block a run-plane
// lookup, a staging round trip and the header logic on the scalar unit
// (counters: 100 SALU, 24 branches, 41 VALU per block; the CU's one scalar
// unit bounds it).  Here a wave owns 64 consecutive blocks and stages a
// WINDOW of them at once: every block that ends inside kHWin bytes from the
// 16-aligned start of the first one, with full-wave 16-byte loads; then lane
// j parses block j's header in vector registers (mode, base width, payload
// offset, bitmap exception count, consumed bytes -- one instruction stream
// for the whole window) and the blocks are unpacked one after the other with
// a single v_readlane of the packed header word each.  Blocks with vbyte
// exceptions go through decode_block_g (p4_generic.h) from the same window.
// The length check is lane-held: one compare and one ballot per run.
// Reference: src/scalar/p4dec32.cpp:70-142 (p4Dec32), p4d1dec32.cpp.
constexpr uint32_t kHRun = 64;   // blocks per wave
// store cache policy of the values: default.  A block's 508 B start at any
// dword, so a store instruction covers parts of three 128-B lines: default
// write-back stores let L2 merge them (C1, A/B on one box: 900-907 G int32/s)
// where nt stores ran 632-659 and "sc1 nt" (write-through) 412-416.
constexpr uint32_t kHWin = 2560; // window staging bytes per wave (p4Enc32 blocks of n <= 256 values are about 1 KB at most)

// lane-parsed header word: [0,12) payload byte in the window (vbyte: block
// byte), [12,18) b, [18,20) kind, [20,26) bx
enum : uint32_t
{
    kH32Plain = 0,
    kH32Bitmap = 1,
    kH32Vbyte = 2,
    kH32Const = 3,
};

// bitmap words of an n-bit bitmap at window byte s (bits past n cleared)
__device__ __forceinline__ void h32_bitmap(const uint32_t * slot, uint32_t s, uint32_t n, uint64_t bm[4], uint32_t pc[4])
{
    const uint32_t words = (n + 63u) >> 6;
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u)
    {
        uint64_t w = u < words ? lds_u64(slot, s + 8u * u) : 0ull;
        if (u == words - 1u && (n & 63u))
            w &= (1ull << (n & 63u)) - 1ull;
        bm[u] = w;
        pc[u] = static_cast<uint32_t>(__builtin_popcountll(w));
    }
}

// EPL: elements per lane (n <= 64 EPL), a template so the element loops
// carry no per-block trip checks
template <bool D1, uint32_t EPL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_sgpr(80), amdgpu_waves_per_eu(8))) void k_dec_h32w(const uint8_t * __restrict in, uint64_t in_bytes, const uint64_t * __restrict off,
                                                   uint64_t nblocks, uint32_t n, uint32_t * __restrict out,
                                                   const uint32_t * __restrict starts, unsigned long long * __restrict err)
{
    __shared__ __attribute__((aligned(16))) uint32_t slots[4][kHWin / 4 + 4]; // +16 B: lds_u32 reads past a window's end
    __shared__ uint32_t scratch[4][512];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t * slot = slots[wv];
    const uint64_t first = (static_cast<uint64_t>(blockIdx.x) * 4u + wv) * kHRun;
    if (first >= nblocks)
        return;
    const uint32_t nr = static_cast<uint32_t>(min_u64(kHRun, nblocks - first));
    const bool valid = t < nr;
    const uint64_t o = valid ? off[first + t] : 0ull;
    const uint64_t e = valid ? off[first + t + 1u] : 0ull;
    // plausible blocks only: inside the stream and at most a window minus its phase
    const uint32_t len = (valid && e >= o && e <= in_bytes && e - o <= kHWin - 16u) ? static_cast<uint32_t>(e - o) : 0xFFFFFFFFu;
    const uint32_t startv = (D1 && valid) ? starts[first + t] : 0u;
    const uint64_t in_base = reinterpret_cast<uint64_t>(in);
    const __amdgpu_buffer_rsrc_t ors = make_rsrc(out + first * n, nr * n * 4u);
    uint32_t usedv = 0u; // lane j: bytes block j consumed
    // The window from the first plausible block at or after js: blocks
    // js.. up to the first one that is implausible or ends past kHWin bytes
    // from the window base (implausible blocks are skipped, left undecoded
    // and reported by the length check).
    auto find = [&](uint32_t & js, uint32_t & je, uint64_t & cb) {
        for (; js < nr; ++js)
        {
            cb = (in_base + readlane_u64(o, js)) & ~15ull;
            const uint64_t lim = cb - in_base + kHWin; // stream offset past the window
            const uint64_t stop = __ballot(t >= js && (!valid || len == 0xFFFFFFFFu || e > lim));
            je = stop ? static_cast<uint32_t>(__builtin_ctzll(stop)) : 64u;
            if (je != js)
                return;
        }
    };
    // the window's bytes into registers (lane t: bytes 16t + 1024k)
    u32x4 R[3];
    uint32_t span = 0u;
    auto issue = [&](uint32_t je, uint64_t cb) {
        span = static_cast<uint32_t>(in_base + readlane_u64(e, je - 1u) - cb);
        const uint32_t avail = static_cast<uint32_t>(min_u64(in_base + in_bytes - cb, kHWin));
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const void *>(cb), avail);
#pragma unroll
        for (uint32_t k = 0; k < 3; ++k)
        {
            const uint32_t x = 16u * t + 1024u * k;
            if (x < span && x + 16u > avail)
                R[k] = load16_guarded(reinterpret_cast<const uint8_t *>(cb), rs, x, avail); // straddles the stream end
            else
                R[k] = buf_load16(rs, x < span ? x : 0x80000000u);
        }
    };
    uint32_t js = 0, je = 0;
    uint64_t cb = 0;
    find(js, je, cb);
    if (js < nr)
        issue(je, cb);
    while (js < nr)
    {
#pragma unroll
        for (uint32_t k = 0; k < 3; ++k)
            if (16u * t + 1024u * k < span)
                reinterpret_cast<u32x4 *>(slot)[t + 64u * k] = R[k];
        wave_lds_sync();
        // the next window's loads fly while this one is decoded
        uint32_t js2 = je, je2 = 0;
        uint64_t cb2 = 0;
        find(js2, je2, cb2);
        if (js2 < nr)
            issue(je2, cb2);
        // lane j in [js, je): parse block j's header
        const bool inw = t >= js && t < je;
        const uint32_t s = inw ? static_cast<uint32_t>(in_base + o - cb) : 0u;
        const uint32_t hw = lds_u32(slot, s);
        const uint32_t h = hw & 0xFFu;
        uint32_t pk, cval = 0u, used = 0u;
        if ((h & 0xC0u) == 0xC0u)
        {
            const uint32_t b = h & 0x3Fu;
            cval = lds_u32(slot, s + 1u) & mask32(b);
            used = (1u + ((b + 7u) >> 3)) | (b > 32u ? kWidthBad : 0u);
            pk = (kH32Const << 18);
        }
        else if (h & 0x40u)
            pk = s | (kH32Vbyte << 18);
        else
        {
            const uint32_t b = min(h & 0x7Fu, 32u);
            const uint32_t bx = (h & 0x80u) ? min((hw >> 8) & 0xFFu, 32u) : 0u;
            uint32_t P = s + ((h & 0x80u) ? 2u : 1u), kind = kH32Plain;
            if (bx != 0u)
            {
                uint64_t bm[4];
                uint32_t pc[4];
                h32_bitmap(slot, s + 2u, n, bm, pc);
                const uint32_t xn = (pc[0] + pc[1]) + (pc[2] + pc[3]);
                P = s + 2u + pad8d(n) + pad8d(xn * bx);
                kind = kH32Bitmap;
            }
            used = ((P - s) + pad8d(n * b)) | (((h & 0x7Fu) > 32u || ((h & 0x80u) && ((hw >> 8) & 0xFFu) > 32u)) ? kWidthBad : 0u);
            pk = P | (b << 12) | (kind << 18) | (bx << 20);
        }
        usedv = inw ? used : usedv;
        for (uint32_t jj = js; jj < je; ++jj)
        {
            const uint32_t w = rl(pk, jj);
            const uint32_t kind = (w >> 18) & 3u;
            uint32_t v[4] = {0u, 0u, 0u, 0u};
            if (kind == kH32Vbyte)
            {
                uint32_t cm;
                const uint32_t u = decode_block_g<Fmt::H32>(slot, w & 0xFFFu, n, scratch[wv], t, v, &cm);
                usedv = t == jj ? u : usedv;
            }
            else if (kind == kH32Const)
            {
                const uint32_t c = rl(cval, jj);
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    v[j] = c;
            }
            else
            {
                const uint32_t P = w & 0xFFFu, b = (w >> 12) & 63u;
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                {
                    const uint32_t el = t + 64u * j;
                    // no per-element condition (it made two exec-mask sections per
                    // block): b = 0 reads mask 0, and values of elements past n go
                    // nowhere (their stores take an out-of-range offset); their LDS
                    // reads may run past this wave's window, which is harmless
                    if (j < EPL)
                        v[j] = lds_bits(slot, P * 8u + el * b, b);
                }
                if (kind == kH32Bitmap)
                {
                    // exceptions: bx-bit values after the bitmap, in element order
                    // (p4dec32.cpp:96-120); rank of element t + 64j from the bitmap
                    const uint32_t bx = (w >> 20) & 63u;
                    const uint32_t sb = uni(static_cast<uint32_t>(in_base + readlane_u64(o, jj) - cb));
                    uint64_t bm[4];
                    uint32_t pc[4];
                    h32_bitmap(slot, sb + 2u, n, bm, pc);
                    const uint32_t xs = sb + 2u + pad8d(n);
                    uint32_t before = 0;
#pragma unroll
                    for (uint32_t j = 0; j < 4; ++j)
                    {
                        if ((bm[j] >> t) & 1ull)
                        {
                            const uint32_t k = before + static_cast<uint32_t>(__builtin_popcountll(bm[j] & lanemask_lt()));
                            v[j] |= shl32(lds_bits(slot, xs * 8u + k * bx, bx), b);
                        }
                        before += pc[j];
                    }
                }
            }
            if constexpr (D1)
                (void)delta1_g<uint32_t>(v, n, rl(startv, jj), t);
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
            {
                const uint32_t el = t + 64u * j;
                if (j < EPL)
                    __builtin_amdgcn_raw_buffer_store_b32(v[j], ors, static_cast<int>(el < n ? (jj * n + el) * 4u : 0x80000000u), 0, 0);
            }
        }
        wave_lds_sync(); // the next window overwrites the slot
        js = js2;
        je = je2;
        cb = cb2;
    }
    const uint64_t bad = __ballot(valid && usedv != len);
    if (err != nullptr && t == 0 && bad != 0u)
        atomicMin(err, static_cast<unsigned long long>(first + __builtin_ctzll(bad)));
}

// ---- run-pipelined encode for the one-block units ------------------------
// Copy-out: a dword loop.  Copying a unit out with 16-byte stores and
// byte-store edges (copy_out_image16) instead: C1 encode, one box, 314 vs 342
// G int32/s for the dword loop -- not kept.
// Plan -> scan -> write as the 256v32 encoder; every wave owns a
// contiguous run of kGRun units whose values arrive through one buffer
// descriptor with the next NC-1 units in flight (the first version, one unit
// per wave: latency-bound, 169 G int32/s on p4Enc32 n=127 batches).
template <Fmt F>
struct EncRunG
{
    using T = typename FmtTraits<F>::T;
    uint64_t first;
    uint32_t nr, pu, NE, n;
    __amdgpu_buffer_rsrc_t rs;

    __device__ __forceinline__ bool init(const T * in, uint64_t nblocks, uint32_t wv, uint32_t n_values)
    {
        n = n_values;
        first = (static_cast<uint64_t>(blockIdx.x) * 4u + wv) * kGRun;
        if (first >= nblocks)
            return false;
        nr = static_cast<uint32_t>(min_u64(kGRun, nblocks - first));
        pu = UnitGeom<F, false>::per_unit(n);
        NE = FmtTraits<F>::N ? FmtTraits<F>::N : n;
        rs = make_rsrc(in + first * pu, nr * pu * static_cast<uint32_t>(sizeof(T)));
        return true;
    }

    // unit jj's elements t + 64j (zero past NE or past the run: out-of-range offsets)
    __device__ __forceinline__ void load(uint32_t jj, uint32_t t, T v[4]) const
    {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
        {
            const uint32_t e = t + 64u * j;
            const uint32_t o = (e < NE && jj < nr) ? (jj * pu + e) * static_cast<uint32_t>(sizeof(T)) : 0x80000000u;
            if constexpr (sizeof(T) == 8)
            {
                const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, static_cast<int>(o), 0, 0);
                v[j] = (static_cast<uint64_t>(x[1]) << 32) | x[0];
            }
            else
                v[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(o), 0, 0);
        }
    }

    // delta-1 start of unit first+t (lanes t < nr): the given starts, or for
    // one chained list the last value of the previous unit
    __device__ __forceinline__ T start_lane(const T * in, const T * starts, T start0, uint32_t t) const
    {
        if (t >= nr)
            return T(0);
        const uint64_t blk = first + t;
        if (starts)
            return starts[blk];
        // the previous unit's last real value: with n below the layout's
        // width (128v32/256v32/128v64 units) the slots after it are padding
        return blk == 0 ? start0 : in[(blk - 1u) * pu + n - 1u];
    }
};

template <class T>
struct Unit4
{
    T v[4];
};

// Plan pass (!WRITE): sizes into off[unit] and one byte total per wave run
// (run_tot); write pass: offsets rebuilt from the run scan (p4_scan.h).
template <Fmt F, bool D1, bool WRITE, uint32_t NC = 3>
__global__ __launch_bounds__(256) TPF_SGPR_ATTR void k_enc_gr(const typename FmtTraits<F>::T * __restrict in, uint64_t nblocks, uint32_t n,
                                                 const typename FmtTraits<F>::T * __restrict starts,
                                                 typename FmtTraits<F>::T start0, uint64_t * __restrict off,
                                                 uint32_t * __restrict plan, uint32_t * __restrict run_tot, const uint64_t * __restrict run_pre,
                                                 const uint64_t * __restrict run_tile, uint8_t * __restrict out, uint64_t out_cap)
{
    using G = UnitGeom<F, false>;
    using T = typename FmtTraits<F>::T;
    __shared__ __attribute__((aligned(16))) uint32_t imgs[WRITE ? 4 : 1][WRITE ? (G::kSlot / 4 + 8) : 1];
    __shared__ __attribute__((aligned(16))) uint32_t hist[WRITE ? 1 : 4][WRITE ? 4 : kPlanGHistU32]; // plan pass only
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    EncRunG<F> R;
    if (!R.init(in, nblocks, wv, n))
        return;
    const T stv = D1 ? R.start_lane(in, starts, start0, t) : T(0);
    uint32_t szv = 0u, pwv = 0u; // lane j: size and plan word of unit first+j
    uint32_t olo = 0u, ohi = 0u;
    if constexpr (WRITE)
    {
        pwv = t < R.nr ? plan[R.first + t] : 0u;
        uint64_t ov, ev;
        run_offsets(off, R.first, R.nr, run_base(run_pre, run_tile, R.first / kGRun), t, ov, ev);
        szv = static_cast<uint32_t>(ev - ov);
        olo = static_cast<uint32_t>(ov);
        ohi = static_cast<uint32_t>(ov >> 32);
    }
    const uint64_t out_base = reinterpret_cast<uint64_t>(out);
    const uint64_t cap_end = out_base + out_cap;
    uint32_t * img = imgs[wv];
    auto body = [&](Unit4<T> & U, uint32_t jj) {
        if constexpr (D1)
        {
            T st;
            if constexpr (sizeof(T) == 8)
                st = readlane_u64(stv, jj);
            else
                st = static_cast<T>(__builtin_amdgcn_readlane(static_cast<int>(stv), static_cast<int>(jj)));
            delta_enc_g<T>(U.v, st, n, t);
        }
        if constexpr (!WRITE)
        {
            const PlanG P = plan_block_g<F>(U.v, n, hist[wv], t);
            szv = t == jj ? P.size : szv;
            pwv = t == jj ? (P.b | (P.bx << 8) | (P.xn << 16) | (P.raw << 25)) : pwv;
        }
        else
        {
            // the plan pass's choice (b <= 64, bx <= 66, xn <= 256): not re-planned
            const uint32_t size = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(szv), static_cast<int>(jj)));
            const uint32_t pw = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(pwv), static_cast<int>(jj)));
            const PlanG P{pw & 0xFFu, (pw >> 8) & 0xFFu, size, (pw >> 16) & 0x1FFu, (pw >> 25) & 1u};
            const uint64_t o = (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(ohi), static_cast<int>(jj)))) << 32)
                             | static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(olo), static_cast<int>(jj)));
            const uint64_t dst = out_base + o;
            const uint32_t phase = static_cast<uint32_t>(dst & 3u);
            emit_block_g<F>(img, phase, P, U.v, n, t);
            wave_lds_sync();
            const uint64_t a0 = dst & ~3ull;
            const uint32_t end = phase + size;
            const uint32_t nd = (end + 3u) >> 2;
            // global address space (a pointer made from an integer is generic:
            // flat stores would also hold up the wave's LDS waits)
            typedef __attribute__((address_space(1))) uint32_t gu32;
            typedef __attribute__((address_space(1))) uint8_t gu8;
            for (uint32_t d = t; d < nd; d += 64u)
            {
                const uint64_t ga = a0 + 4u * d;
                const uint32_t w = img[d];
                const uint32_t lo = 4u * d, hi = lo + 4u;
                if (lo >= phase && hi <= end && ga + 4u <= cap_end)
                    *(gu32 *)ga = w;
                else
                    for (uint32_t x = 0; x < 4; ++x)
                    {
                        const uint32_t bi = lo + x;
                        if (bi >= phase && bi < end && ga + x < cap_end)
                            *(gu8 *)(ga + x) = static_cast<uint8_t>(w >> (8u * x));
                    }
            }
            wave_lds_sync();
            // only dwords [0, nd) can be non-zero: clear them for the next unit
            for (uint32_t d = t; d < nd; d += 64u)
                img[d] = 0u;
            wave_lds_sync();
        }
    };
    if constexpr (WRITE)
    {
        for (uint32_t i = t; i < G::kSlot / 4 + 8; i += 64u)
            img[i] = 0u;
        wave_lds_sync();
    }
    // NC units rotate in registers (loop unrolled by NC, no copies of
    // in-flight loads): while unit j is encoded, j+1 .. j+NC-1 are in flight.
    Unit4<T> C[NC];
#pragma unroll
    for (uint32_t u = 0; u + 1 < NC; ++u)
        R.load(u, t, C[u].v);
    bool more = true;
    for (uint32_t j = 0; more; j += NC)
    {
#pragma unroll
        for (uint32_t u = 0; u < NC; ++u)
        {
            if (more)
            {
                R.load(j + u + NC - 1, t, C[(u + NC - 1) % NC].v);
                body(C[u], j + u);
                more = j + u + 1 < R.nr;
            }
        }
    }
    if constexpr (!WRITE)
    {
        if (t < R.nr)
        {
            off[R.first + t] = szv;
            plan[R.first + t] = pwv;
        }
        publish_run_total(run_tot, R.first / kGRun, t < R.nr ? szv : 0u, t);
    }
}

} // namespace tpf::dev

namespace tpf
{

namespace
{

size_t plan_bytes(uint64_t nblocks) { return (nblocks * 4u + 255u) & ~size_t(255); }

template <dev::Fmt F>
hipError_t dec_fmt(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t n, void * out,
                   const void * starts, unsigned long long * err, hipStream_t s)
{
    using T = typename dev::FmtTraits<F>::T;
    const uint64_t per_wg = 4ull * dev::kGRun;
    const uint32_t g = static_cast<uint32_t>((nblocks + per_wg - 1) / per_wg);
    if (starts)
        hipLaunchKernelGGL((dev::k_dec_gr<F, true>), dim3(g), dim3(256), 0, s, in, in_bytes, off, nblocks, n, static_cast<T *>(out),
                           static_cast<const T *>(starts), err);
    else
        hipLaunchKernelGGL((dev::k_dec_gr<F, false>), dim3(g), dim3(256), 0, s, in, in_bytes, off, nblocks, n, static_cast<T *>(out),
                           static_cast<const T *>(nullptr), err);
    return hipGetLastError();
}

hipError_t dec_h32w(const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t n, uint32_t * out,
                    const uint32_t * starts, unsigned long long * err, hipStream_t s)
{
    const uint64_t per_wg = 4ull * dev::kHRun;
    const uint32_t g = static_cast<uint32_t>((nblocks + per_wg - 1) / per_wg);
    auto go = [&](auto d1, auto epl) {
        hipLaunchKernelGGL((dev::k_dec_h32w<decltype(d1)::value, decltype(epl)::value>), dim3(g), dim3(256), 0, s, in, in_bytes, off, nblocks,
                           n, out, starts, err);
    };
    using T1 = std::true_type;
    using F1 = std::false_type;
    using E1 = std::integral_constant<uint32_t, 1>;
    using E2 = std::integral_constant<uint32_t, 2>;
    using E4 = std::integral_constant<uint32_t, 4>;
    if (starts)
        n <= 64u ? go(T1{}, E1{}) : n <= 128u ? go(T1{}, E2{}) : go(T1{}, E4{});
    else
        n <= 64u ? go(F1{}, E1{}) : n <= 128u ? go(F1{}, E2{}) : go(F1{}, E4{});
    return hipGetLastError();
}

template <dev::Fmt F, bool D1>
hipError_t enc_fmt_d(const void * in, uint64_t nblocks, uint32_t n, const void * starts, uint64_t start0, uint8_t * out,
                     uint64_t out_cap, uint64_t * off, void * ws, size_t ws_bytes, hipStream_t s)
{
    using T = typename dev::FmtTraits<F>::T;
    const T * ip = static_cast<const T *>(in);
    const T * sp = static_cast<const T *>(starts);
    const uint64_t per_wg = 4ull * dev::kGRun;
    const uint32_t g = static_cast<uint32_t>((nblocks + per_wg - 1) / per_wg);
    const uint64_t nruns = (nblocks + dev::kGRun - 1u) / dev::kGRun;
    if (ws_bytes < generic_workspace(nblocks))
        return hipErrorInvalidValue;
    uint32_t * plan = static_cast<uint32_t *>(ws);
    const RunScanWs<uint64_t> rs = RunScanWs<uint64_t>::carve(static_cast<uint8_t *>(ws) + plan_bytes(nblocks), nruns);
    hipLaunchKernelGGL((dev::k_enc_gr<F, D1, false>), dim3(g), dim3(256), 0, s, ip, nblocks, n, sp, static_cast<T>(start0), off, plan,
                       rs.tot, nullptr, nullptr, out, out_cap);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return e;
    e = launch_run_scan_u64(rs.tot, nruns, rs.pre, rs.tile, off + nblocks, s);
    if (e != hipSuccess)
        return e;
    hipLaunchKernelGGL((dev::k_enc_gr<F, D1, true>), dim3(g), dim3(256), 0, s, ip, nblocks, n, sp, static_cast<T>(start0), off, plan,
                       nullptr, rs.pre, rs.tile, out, out_cap);
    return hipGetLastError();
}

template <dev::Fmt F>
hipError_t enc_fmt(const void * in, uint64_t nblocks, uint32_t n, bool d1, const void * starts, uint64_t start0, uint8_t * out,
                   uint64_t out_cap, uint64_t * off, void * ws, size_t ws_bytes, hipStream_t s)
{
    return d1 ? enc_fmt_d<F, true>(in, nblocks, n, starts, start0, out, out_cap, off, ws, ws_bytes, s)
              : enc_fmt_d<F, false>(in, nblocks, n, starts, start0, out, out_cap, off, ws, ws_bytes, s);
}

} // namespace

// plan words (one per unit, 256-B aligned) + the run scan
size_t generic_workspace(uint64_t nblocks) { return plan_bytes(nblocks) + RunScanWs<uint64_t>::bytes((nblocks + dev::kGRun - 1u) / dev::kGRun); }

hipError_t launch_dec_generic(int fmt, const uint8_t * in, uint64_t in_bytes, const uint64_t * off, uint64_t nblocks, uint32_t n,
                              void * out, const void * starts, unsigned long long * err, hipStream_t s)
{
    if (nblocks == 0)
        return hipSuccess;
    switch (fmt)
    {
        case FMT_32:
            if (n >= 1u && n <= 256u)
                return dec_h32w(in, in_bytes, off, nblocks, n, static_cast<uint32_t *>(out), static_cast<const uint32_t *>(starts), err, s);
            return dec_fmt<dev::Fmt::H32>(in, in_bytes, off, nblocks, n, out, starts, err, s);
        case FMT_128V32:
            return dec_fmt<dev::Fmt::V128>(in, in_bytes, off, nblocks, n, out, starts, err, s);
        case FMT_256V32:
            return dec_fmt<dev::Fmt::V256>(in, in_bytes, off, nblocks, n, out, starts, err, s);
        case FMT_64:
            return dec_fmt<dev::Fmt::H64>(in, in_bytes, off, nblocks, n, out, starts, err, s);
        case FMT_128V64: // run-pipelined kernel, p4_dec256v64.hip (n < 128: the generic one)
            if (n < 128u)
                return dec_fmt<dev::Fmt::V128X64>(in, in_bytes, off, nblocks, n, out, starts, err, s);
            return launch_dec128v64(1, in, in_bytes, off, nblocks, static_cast<uint64_t *>(out),
                                    static_cast<const uint64_t *>(starts), err, s);
        case FMT_256V64:
            return launch_dec128v64(2, in, in_bytes, off, nblocks, static_cast<uint64_t *>(out),
                                    static_cast<const uint64_t *>(starts), err, s);
        default:
            return hipErrorInvalidValue;
    }
}

hipError_t launch_enc_generic(int fmt, const void * in, uint64_t nblocks, uint32_t n, bool d1, const void * starts, uint64_t start0,
                              uint8_t * out, uint64_t out_cap, uint64_t * off, void * ws, size_t ws_bytes, hipStream_t s)
{
    if (nblocks == 0)
        return fill_u32(off, 0u, 2, s);
    if (nblocks + 1 > 0x7FFFFFFFull)
        return hipErrorInvalidValue;
    switch (fmt)
    {
        case FMT_32:
            return enc_fmt<dev::Fmt::H32>(in, nblocks, n, d1, starts, start0, out, out_cap, off, ws, ws_bytes, s);
        case FMT_128V32:
            return enc_fmt<dev::Fmt::V128>(in, nblocks, n, d1, starts, start0, out, out_cap, off, ws, ws_bytes, s);
        case FMT_256V32:
            return enc_fmt<dev::Fmt::V256>(in, nblocks, n, d1, starts, start0, out, out_cap, off, ws, ws_bytes, s);
        case FMT_64:
            return enc_fmt<dev::Fmt::H64>(in, nblocks, n, d1, starts, start0, out, out_cap, off, ws, ws_bytes, s);
        case FMT_128V64: // run-pipelined kernels, p4_enc256v64.hip (n < 128: the generic ones)
            if (n < 128u)
                return enc_fmt<dev::Fmt::V128X64>(in, nblocks, n, d1, starts, start0, out, out_cap, off, ws, ws_bytes, s);
            [[fallthrough]];
        case FMT_256V64:
            return launch_enc128v64(fmt == FMT_256V64 ? 2u : 1u, static_cast<const uint64_t *>(in), nblocks, d1,
                                    static_cast<const uint64_t *>(starts), start0, out, out_cap, off, ws, ws_bytes, s);
        default:
            return hipErrorInvalidValue;
    }
}

} // namespace tpf
