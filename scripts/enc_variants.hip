// enc_variants.hip -- measurement tool (NOT part of the library): the 256v32
// encoder designs measured against the two-pass encoder (p4_enc256v32.h) and
// rejected in round 2, kept buildable for re-measurement:
//   modes 4-12   single pass with decoupled look-back over LDS-held tiles
//                (+ the gated two-pass fallback)
//   modes 13-15  the two-pass encoder with nt / sc1 value loads
//   modes 16/17  the two-pass encoder on a persistent grid-stride grid
//   modes >= 18  the single-launch MALL-chunked pipelined encoder
//                (16 + ci + 1024*lag + 65536*minw + 2^20*per_ticket, ci >= 64)
// Every mode writes a valid stream (byte-exact; tests/test_gpu_enc_variants.py).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 -shared -fPIC -munsafe-fp-atomics
//        -I turbopfor-cpp_amd/csrc -I include -o scripts/libencvar.so scripts/enc_variants.hip
//        turbopfor-cpp_amd/lib/libturbopfor_amd.so   (grid_cap, the run scan)
#include "p4_enc256v32.h"

namespace tpf::dev
{

// ---- single-pass encoder: decoupled look-back over workgroup tiles -------
// MEASURED AND REJECTED (round 2): byte-exact in every
// variant, 7.6-9.3 ms per 10M C4 blocks against the two-pass encoder's 5.45.
// Reachable through tpf_probe_enc256v32 modes 4-12 for re-measurement.
// The two-pass encoder reads the values twice (plan, then write: 1.33x the
// round trip's algorithmic bytes).  Here one workgroup = one tile of 4 x K
// consecutive blocks, and the values are read once:
//   1. each wave walks its K blocks (3 in flight), plans each (p4Bits32) and
//      builds it at once into LDS (a fixed slot per block, or packed into a
//      per-wave arena; a block that no longer fits is deferred);
//   2. the tile's byte total is published in status[tile] as an AGGREGATE;
//      wave 0 then looks back over the preceding tiles' status words (256 per
//      poll, 4 per lane): aggregates are summed down to the nearest
//      INCLUSIVE prefix, and the tile publishes its own inclusive prefix;
//   3. every wave writes its blocks' offsets and copies its images out, then
//      loads and builds its deferred blocks one at a time.
// A status word is one 8-byte {flag, value} granule written by one
// write-through (agent-scope) store and polled with agent-scope loads, so
// no fence orders it against anything else (MI355X_MICROARCH.md hand-offs).
// Tiles are taken in blockIdx order: a tile waits only on lower-numbered
// tiles, whose workgroups the dispatcher has placed first (in-order dispatch
// within each XCD), so no residency is assumed beyond that.  Every wait is
// bounded by the real-time clock (kLbWaitTicks): on expiry the launch raises
// the abort word, every waiting workgroup leaves, and the gated two-pass
// encoder enqueued behind it redoes the whole batch -- the result is the
// same bytes either way.
// Why it loses: the images must stay in LDS until the look-back returns, so
// LDS caps the workgroups per CU (16-24 waves against the two passes' 32),
// and the plan + build work alone, with the look-back reduced to one poll
// (mode 4), already takes 5.65 ms -- as long as both passes together.
constexpr uint32_t kLbSlotU32 = 264; // one block image: lead (<= 23 B) + block (<= 1025 B) + read slack, 16-B multiple
constexpr uint32_t kLbK = 8;         // blocks per wave (tile = 4 x kLbK blocks)
constexpr uint32_t kLbArena = 4096;  // bytes of block images per wave
constexpr uint64_t kLbAgg = 1ull << 63, kLbIncl = 1ull << 62, kLbVal = kLbIncl - 1u;
constexpr uint64_t kLbWaitTicks = 2000000; // 20 ms of the 100 MHz real-time clock
static_assert(kPlanHistU32 <= kEncValU32, "plan histogram shares the staging words");

typedef __attribute__((address_space(1))) uint64_t lb_gu64;
typedef __attribute__((address_space(1))) uint32_t lb_gu32;

__device__ __forceinline__ uint64_t lb_ld(const uint64_t * p)
{
    return __hip_atomic_load((lb_gu64 *)(const_cast<uint64_t *>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_st(uint64_t * p, uint64_t v)
{
    __hip_atomic_store((lb_gu64 *)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t x) { return readlane_u64(wave_incl_scan64(x), 63); }

// Wave 0 of tile `tile` (> 0): exclusive byte prefix of the tile, or ~0 on
// abort.  Lane t examines the status words at distances 4t..4t+3 below pos.
__device__ __forceinline__ uint64_t lb_lookback(const uint64_t * status, uint64_t tile, uint32_t * abort, uint32_t t)
{
    uint64_t excl = 0;
    int64_t pos = static_cast<int64_t>(tile) - 1;
    const uint64_t t0 = wall_clock64();
    for (;;)
    {
        uint64_t w[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
        {
            const int64_t idx = pos - static_cast<int64_t>(4u * t + k);
            w[k] = idx >= 0 ? lb_ld(status + idx) : kLbIncl; // before tile 0: inclusive prefix 0
        }
        uint32_t dinc = 0xFFFFu, dinv = 0xFFFFu; // nearest inclusive / unpublished word
#pragma unroll
        for (int k = 3; k >= 0; --k)
        {
            const uint32_t d = 4u * t + static_cast<uint32_t>(k);
            dinc = (w[k] & kLbIncl) ? d : dinc;
            dinv = w[k] == 0u ? d : dinv;
        }
        dinc = uni(wave_min(dinc));
        dinv = uni(wave_min(dinv));
        if (dinv < dinc)
        {
            // a tile before the nearest inclusive prefix has not published yet
            if (__hip_atomic_load((lb_gu32 *)abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)
                return ~0ull;
            if (wall_clock64() - t0 > kLbWaitTicks)
            {
                if (t == 0)
                    __hip_atomic_store((lb_gu32 *)abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return ~0ull;
            }
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        uint64_t s = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            s += (4u * t + k <= dinc) ? (w[k] & kLbVal) : 0u;
        excl += wave_sum64(s);
        if (dinc != 0xFFFFu)
            return excl;
        pos -= 256;
    }
}

// ARENA (bytes per wave, 0 = one fixed 1056-B slot per block): the wave's
// block images are packed one after the other (16-B aligned) into an arena
// sized for typical blocks, so more workgroups fit a CU; a block that no
// longer fits is deferred: after the look-back it is loaded again and built
// in the (then free) arena one block at a time.
template <bool D1, uint32_t K, uint32_t ARENA>
__global__ __launch_bounds__(256) void k_enc256v32_lb(const uint32_t * __restrict in, uint64_t nblocks, const uint32_t * __restrict starts,
                                                       uint32_t start0, uint64_t * __restrict off, uint8_t * __restrict out, uint64_t out_cap,
                                                       uint64_t * status, uint32_t * abort)
{
    constexpr uint32_t kArenaU32 = ARENA ? ARENA / 4u : K * kLbSlotU32;
    static_assert(ARENA == 0 || ARENA >= 4u * kLbSlotU32, "the arena must hold one worst-case block");
    __shared__ __attribute__((aligned(16))) uint32_t arena_all[4][kArenaU32 + 4u]; // + read slack of copy_out_image16
    __shared__ __attribute__((aligned(16))) uint32_t scr_all[4][kEncValU32];      // plan histogram, then the staged values
    __shared__ uint64_t xch[5];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint64_t tile = blockIdx.x;
    uint32_t * const scr = scr_all[wv];
    uint32_t * const arena = arena_all[wv];
    EncRun R;
    R.init_at(in, nblocks, (tile * 4u + wv) * K, K);
    // lane j: size, image start, image slot (u32x4 index) and plan word of block first+j
    uint32_t szv = 0u, sbv = 0u, atv = 0u, pwv = 0u;
    uint32_t built = R.n; // blocks [0, built) are in the arena, the rest deferred
    const uint32_t stv = (D1 && R.n) ? R.start_lane(in, starts, start0, t) : 0u;
    if (R.n)
    {
        uint32_t pos = 0u; // next free u32x4 of the arena
        R.walk(t, [&](u32x4 v, uint32_t jj) {
            if constexpr (D1)
                v = delta_encode(v, rl32(stv, jj), t);
            const Plan32 P = plan_block256(v, scr, t);
            const uint32_t at = ARENA ? pos : jj * (kLbSlotU32 / 4u);
            const bool fits = ARENA == 0u || (built == R.n && 16u * at + kImgLead + 3u + P.size <= ARENA);
            wave_lds_sync();
            uint32_t sb = 0u;
            if (fits)
            {
                uint32_t * img = arena + 4u * at;
                zero_image(img, min((kImgLead + 3u + P.size + 15u) >> 4, kLbSlotU32 / 4u), t);
                wave_lds_sync();
                sb = emit_block256<true>(img, scr, P, v, t);
                wave_lds_sync();
                pos = at + ((sb + P.size + 15u) >> 4);
            }
            else if (built == R.n)
                built = jj;
            szv = t == jj ? P.size : szv;
            sbv = t == jj ? sb : sbv;
            atv = t == jj ? at : atv;
            pwv = t == jj ? plan_word(P) : pwv;
        });
    }
    const uint32_t wt = wave_sum(szv);
    if (t == 0)
        xch[wv] = wt;
    __syncthreads();
    if (wv == 0)
    {
        const uint64_t T = xch[0] + xch[1] + xch[2] + xch[3];
        uint64_t E = 0;
        if (tile == 0)
        {
            if (t == 0)
                lb_st(status, kLbIncl | T);
        }
        else
        {
            if (t == 0)
                lb_st(status + tile, kLbAgg | T);
            E = lb_lookback(status, tile, abort, t);
            if (E != ~0ull && t == 0)
                lb_st(status + tile, kLbIncl | (E + T));
        }
        if (t == 0)
        {
            xch[4] = E;
            if (tile + 1u == gridDim.x && E != ~0ull)
                off[nblocks] = E + T;
        }
    }
    __syncthreads();
    const uint64_t E = xch[4];
    if (E == ~0ull || R.n == 0)
        return;
    uint64_t base = E;
    for (uint32_t w = 0; w < wv; ++w)
        base += xch[w];
    const uint32_t incl = wave_incl_scan(szv);
    const uint64_t ov = base + (incl - szv);
    if (t < R.n)
        off[R.first + t] = ov;
    const uint64_t out_base = reinterpret_cast<uint64_t>(out);
    for (uint32_t j = 0; j < built; ++j)
        copy_out_image16(arena + 4u * rl32(atv, j), rl32(sbv, j), out_base + readlane_u64(ov, j), rl32(szv, j), out_base + out_cap, t);
    for (uint32_t j = built; j < R.n; ++j)
    {
        // deferred block: load it again and build it in the arena
        u32x4 v = R.load(j, t);
        if constexpr (D1)
            v = delta_encode(v, rl32(stv, j), t);
        const uint32_t size = rl32(szv, j);
        const Plan32 P = unplan(rl32(pwv, j), size);
        wave_lds_sync();
        zero_image(arena, (kImgLead + 3u + size + 15u) >> 4, t);
        wave_lds_sync();
        const uint32_t sb = emit_block256<true>(arena, scr, P, v, t);
        wave_lds_sync();
        copy_out_image16(arena, sb, out_base + readlane_u64(ov, j), size, out_base + out_cap, t);
    }
}

// ---- single-launch pipelined encoder: MEASURED AND REJECTED ---
// Reachable only through tpf_probe_enc256v32 (mode >= 16).  Every variant is
// byte-exact, and none is faster than the two-pass encoder above.
// The blocks are cut into chunks of `ci` workgroup items of kPipeItem blocks
// (4 waves x kPipeRun).  ONE persistent launch walks a sequence of items,
// step s = plan items of chunk s interleaved with write items of chunk
// s - lag:
//   plan item  : plans its blocks (p4Bits32 cost model), publishes each
//                block's size and plan word and its run / item byte totals,
//                and arrives on the chunk's counter; the LAST arriving item
//                scans the chunk's item totals (item offsets inside the
//                chunk), chains the chunk's byte offset from the previous
//                chunk's and flags the chunk ready;
//   write item : waits for its chunk's flag, derives every block's byte
//                offset (chunk + item + run offset + in-run scan), writes
//                d_off and builds the blocks as the two-pass write kernel does.
// The aim: a chunk's values are re-read by its write items while the 256 MiB
// Infinity Cache still holds them (no second HBM read: the two-pass encoder
// moves 1.33x the algorithmic bytes), no separate scan launch, planning of one
// chunk beside writing of an earlier one.  Why it loses: a write item cannot
// start before EVERY plan item of its chunk and the chunk chain before it are
// done, while the machine keeps G x kPipeItem blocks (~160 MB of values at
// 1280-2048 workgroups) in flight; a lag that hides that window no longer
// fits the Infinity Cache with the chunks it needs, and any shorter lag makes
// the write items wait (measured 8.3 ms with a static item map, 19-79 ms with
// tickets, vs 5.45 ms two-pass, C4 mix, 10M blocks).
// Hand-offs (MI355X_MICROARCH.md "visibility", cdna_hip_programming.md G16):
// every published word is stored write-through (agent-scope relaxed atomic
// store = sc1) and drained (s_waitcnt vmcnt(0)) by every storing wave before
// the workgroup barrier and the counter add / flag store; consumers poll one
// word relaxed with s_sleep, take ONE agent-scope acquire and read the words
// with sc1 loads.  Items come from a ticket counter in sequence order (no
// residency assumption, see the kernel); every wait is bounded (kSpinLimit
// polls): on expiry the kernel raises an abort word and a finish kernel
// stores UINT64_MAX in d_off[nblocks].
constexpr uint32_t kPipeRun = 32;
constexpr uint32_t kPipeItem = 4u * kPipeRun;
constexpr uint32_t kPipeMaxChunkItems = 512; // the last arriver's scan covers 2 items per thread
// (the measured configurations -- chunk items, lag, launch bound, entries
// per ticket -- are all taken from the probe mode)
constexpr uint32_t kSpinLimit = 1u << 22;    // polls of ~0.2 us

typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint64_t gu64;

__device__ __forceinline__ void st_wt(uint32_t * p, uint32_t v)
{
    __hip_atomic_store((gu32 *)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt64(uint64_t * p, uint64_t v)
{
    __hip_atomic_store((gu64 *)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_wt(const uint32_t * p)
{
    return __hip_atomic_load((gu32 *)(const_cast<uint32_t *>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_wt64(const uint64_t * p)
{
    return __hip_atomic_load((gu64 *)(const_cast<uint64_t *>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Workspace of the pipelined encoder.  The polled words (ticket head,
// counters, flags, abort) sit first, in one 16-byte-padded block zeroed
// before every launch.
struct PipeWs
{
    uint32_t * head;  // [4] ticket counter (word 0)
    uint32_t * abort; // [4] bounded-wait expiry (word 0)
    uint32_t * count; // [nchunks] arrivals of plan items
    uint32_t * ready; // [nchunks] chunk scanned and chained
    uint64_t * cbase; // [nchunks] byte offset of the chunk
    uint64_t * ctot;  // [nchunks] byte total of the chunk
    uint32_t * itot;  // [nitems] byte total of an item
    uint32_t * ibase; // [nitems] byte offset of an item inside its chunk
    uint32_t * rtot;  // [nitems * 4] byte total of a run
    uint32_t * sz;    // [nblocks] block sizes
    uint32_t * plan;  // [nblocks] plan words
};

// Bounded wait (one lane) until *flag != 0; false on expiry or abort.
__device__ __forceinline__ bool wait_set(const uint32_t * flag, uint32_t * abort)
{
    for (uint32_t n = 0;; ++n)
    {
        if (ld_wt(flag) != 0u)
            return true;
        if (ld_wt(abort) != 0u)
            return false;
        if (n >= kSpinLimit)
        {
            st_wt(abort, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(8);
    }
}

struct PipeArgs
{
    const uint32_t * in;
    uint64_t nblocks;
    const uint32_t * starts;
    uint32_t start0;
    uint64_t out_base, cap_end;
    uint64_t * off;
    uint64_t nitems;
    uint32_t nchunks, ci, lag, per_ticket;
};

// Plan item: plan 4 runs of kPipeRun blocks, publish sizes / plan words / run
// and item totals (write-through, drained), arrive on the chunk counter; the
// last arriver scans the chunk's item totals and chains the chunk offset.
template <bool D1>
__device__ __forceinline__ void pipe_plan(const PipeArgs & A, const PipeWs & W, uint32_t c, uint64_t item, uint32_t citems,
                                          uint32_t * hist, uint32_t * xch, uint32_t t, uint32_t wv)
{
    const uint64_t run = item * 4u + wv;
    EncRun R;
    R.init_at(A.in, A.nblocks, run * kPipeRun, kPipeRun);
    uint32_t szv = 0u, pwv = 0u;
    if (R.n)
        plan_run<D1>(R, A.in, A.starts, A.start0, hist, t, szv, pwv);
    if (t < R.n)
    {
        st_wt(W.sz + R.first + t, szv);
        st_wt(W.plan + R.first + t, pwv);
    }
    const uint32_t rt = wave_sum(t < R.n ? szv : 0u);
    if (t == 0)
    {
        st_wt(W.rtot + run, rt);
        xch[wv] = rt;
    }
    drain_stores(); // every storing wave, before the barrier in front of the arrival
    __syncthreads();
    if (threadIdx.x == 0)
    {
        st_wt(W.itot + item, xch[0] + xch[1] + xch[2] + xch[3]);
        drain_stores();
        const uint32_t old = __hip_atomic_fetch_add((gu32 *)(W.count + c), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        xch[4] = (old + 1u == citems) ? 1u : 0u;
        if (xch[4])
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    drain_stores();
    __syncthreads();
    if (xch[4] == 0u)
        return;
    // last arriver of chunk c: exclusive scan of the item totals (<= 2 per thread)
    const uint64_t i0 = static_cast<uint64_t>(c) * A.ci;
    const uint32_t ia = 2u * threadIdx.x, ib = ia + 1u;
    const uint32_t a = ia < citems ? ld_wt(W.itot + i0 + ia) : 0u;
    const uint32_t b = ib < citems ? ld_wt(W.itot + i0 + ib) : 0u;
    const uint32_t incl = wave_incl_scan(a + b);
    if (t == 63)
        xch[8 + wv] = incl;
    __syncthreads();
    uint32_t before = 0u;
    for (uint32_t w = 0; w < wv; ++w)
        before += xch[8 + w];
    const uint32_t ex = before + incl - (a + b);
    if (ia < citems)
        st_wt(W.ibase + i0 + ia, ex);
    if (ib < citems)
        st_wt(W.ibase + i0 + ib, ex + a);
    if (threadIdx.x == 0)
    {
        const uint64_t ctot = static_cast<uint64_t>(xch[8]) + xch[9] + xch[10] + xch[11];
        uint64_t cb = 0u;
        bool ok = true;
        if (c > 0u)
        {
            // chunk c-1's plan items hold earlier tickets: their last arriver is running or done
            ok = wait_set(W.ready + (c - 1u), W.abort);
            cb = ld_wt64(W.cbase + (c - 1u)) + ld_wt64(W.ctot + (c - 1u));
        }
        st_wt64(W.cbase + c, cb);
        st_wt64(W.ctot + c, ctot);
        if (c + 1u == A.nchunks)
            A.off[A.nblocks] = ok ? cb + ctot : ~0ull;
    }
    drain_stores();
    __syncthreads();
    if (threadIdx.x == 0)
        st_wt(W.ready + c, 1u);
}

// Write item: wait for the chunk, derive every block's offset, build the blocks.
template <bool D1>
__device__ __forceinline__ void pipe_write(const PipeArgs & A, const PipeWs & W, uint32_t c, uint64_t item, uint32_t * img,
                                           uint32_t * val, uint32_t * xch, uint32_t t, uint32_t wv)
{
    if (threadIdx.x == 0)
    {
        xch[5] = wait_set(W.ready + c, W.abort) ? 1u : 0u;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    drain_stores();
    __syncthreads();
    if (xch[5] == 0u)
        return;
    const uint64_t run = item * 4u + wv;
    EncRun R;
    if (!R.init_at(A.in, A.nblocks, run * kPipeRun, kPipeRun))
        return;
    uint64_t rb = ld_wt64(W.cbase + c) + ld_wt(W.ibase + item);
    for (uint32_t w = 0; w < wv; ++w)
        rb += ld_wt(W.rtot + item * 4u + w);
    const uint32_t szv = t < R.n ? ld_wt(W.sz + R.first + t) : 0u;
    const uint32_t pwv = t < R.n ? ld_wt(W.plan + R.first + t) : 0u;
    const uint64_t ov = rb + (wave_incl_scan(szv) - szv);
    if (t < R.n)
        A.off[R.first + t] = ov;
    write_run<D1>(R, A.in, A.starts, A.start0, szv, pwv, static_cast<uint32_t>(ov), static_cast<uint32_t>(ov >> 32), img, val,
                  A.out_base, A.cap_end, t);
}

template <bool D1, int MINW>
__global__ __launch_bounds__(256, MINW) void k_enc256v32_pipe(PipeArgs A, PipeWs W)
{
    __shared__ __attribute__((aligned(16))) uint32_t hist[4][kPlanHistU32];
    __shared__ __attribute__((aligned(16))) uint32_t img_all[4][kImgU32];
    __shared__ __attribute__((aligned(16))) uint32_t val_all[4][kEncValU32];
    __shared__ uint32_t xch[16];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t * img = img_all[wv];
    zero_image(img, kImgU32 / 4u, t);
    wave_lds_sync();
    const uint32_t nseq = (A.nchunks + A.lag) * (2u * A.ci);
    // Items come from a ticket counter, A.per_ticket consecutive sequence
    // entries per ticket, and every workgroup runs its entries in order: a
    // write item then waits only on plan items that running workgroups hold,
    // so there is no residency assumption (a static item -> workgroup map
    // would need every workgroup resident).  The next ticket is taken by the
    // last wave after its share of the last entry of the current one, so its
    // latency (one contended word) sits behind that wave's work only.
    if (threadIdx.x == 0)
        xch[12] = __hip_atomic_fetch_add((gu32 *)W.head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * A.per_ticket;
    __syncthreads();
    uint32_t q = xch[12];
    while (q < nseq)
    {
        const bool last_of_ticket = (q + 1u) % A.per_ticket == 0u;
        // sequence: step s = plan items of chunk s interleaved with write items of chunk s - lag
        const uint32_t step = q / (2u * A.ci);
        const uint32_t r = q % (2u * A.ci);
        const bool is_plan = (r & 1u) == 0u;
        if (is_plan || step >= A.lag)
        {
            const uint32_t c = is_plan ? step : step - A.lag;
            const uint64_t item = static_cast<uint64_t>(c) * A.ci + (r >> 1);
            if (c < A.nchunks && item < A.nitems)
            {
                if (is_plan)
                {
                    const uint32_t citems = static_cast<uint32_t>(min_u64(A.ci, A.nitems - static_cast<uint64_t>(c) * A.ci));
                    pipe_plan<D1>(A, W, c, item, citems, hist[wv], xch, t, wv);
                }
                else
                    pipe_write<D1>(A, W, c, item, img, val_all[wv], xch, t, wv);
            }
        }
        if (last_of_ticket)
        {
            if (threadIdx.x == 192)
                xch[12] = __hip_atomic_fetch_add((gu32 *)W.head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * A.per_ticket;
            __syncthreads(); // the new ticket is visible; the item's LDS words are free again
            q = uni(xch[12]);
        }
        else
        {
            __syncthreads(); // the item's LDS words are free again
            ++q;
        }
    }
}

// Abort of the pipelined encoder (a bounded wait expired): mark the stream invalid.
__global__ void k_enc_pipe_finish(const uint32_t * abort, uint64_t * off, uint64_t nblocks)
{
    if (threadIdx.x == 0 && *abort != 0u)
        off[nblocks] = ~0ull;
}
} // namespace tpf::dev

namespace tpf
{

namespace
{

using enc256::al256;
using enc256::twopass_workspace;

struct PipeGeom
{
    uint64_t nitems, nchunks;
    size_t polled; // bytes of the zeroed block (16-B multiple)
    size_t bytes;
};

PipeGeom pipe_geom(uint64_t nblocks, uint32_t ci)
{
    PipeGeom g;
    g.nitems = (nblocks + dev::kPipeItem - 1) / dev::kPipeItem;
    g.nchunks = (g.nitems + ci - 1) / ci;
    g.polled = ((8u + g.nchunks * 2u) * 4u + 15u) & ~size_t(15);
    g.bytes = al256(g.polled) + 2u * al256(g.nchunks * 8u) + 2u * al256(g.nitems * 4u) + al256(g.nitems * 16u)
              + 2u * al256(nblocks * 4u);
    return g;
}

dev::PipeWs pipe_ws(void * ws, uint64_t nblocks, const PipeGeom & g)
{
    uint8_t * p = static_cast<uint8_t *>(ws);
    dev::PipeWs W;
    W.head = reinterpret_cast<uint32_t *>(p);
    W.abort = W.head + 4;
    W.count = W.head + 8;
    W.ready = W.count + g.nchunks;
    p += al256(g.polled);
    W.cbase = reinterpret_cast<uint64_t *>(p);
    p += al256(g.nchunks * 8u);
    W.ctot = reinterpret_cast<uint64_t *>(p);
    p += al256(g.nchunks * 8u);
    W.itot = reinterpret_cast<uint32_t *>(p);
    p += al256(g.nitems * 4u);
    W.ibase = reinterpret_cast<uint32_t *>(p);
    p += al256(g.nitems * 4u);
    W.rtot = reinterpret_cast<uint32_t *>(p);
    p += al256(g.nitems * 16u);
    W.sz = reinterpret_cast<uint32_t *>(p);
    p += al256(nblocks * 4u);
    W.plan = reinterpret_cast<uint32_t *>(p);
    return W;
}

// Workgroups of the persistent grid: as many as the occupancy query admits
// (tickets make residency a speed matter, not a correctness one).
template <bool D1, int MINW>
uint32_t pipe_grid(uint64_t nitems)
{
    static int per_cu[2][3][64] = {};
    int dev_id = 0;
    (void)hipGetDevice(&dev_id);
    dev_id = dev_id < 0 || dev_id >= 64 ? 0 : dev_id;
    int & pc = per_cu[D1][MINW == 8 ? 0 : MINW == 6 ? 1 : 2][dev_id];
    if (pc == 0)
    {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void *>(dev::k_enc256v32_pipe<D1, MINW>), 256, 0)
                != hipSuccess
            || n <= 0)
            n = 1;
        pc = n;
    }
    const uint64_t want = 2u * nitems; // more workgroups than items would only idle
    return static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(want, grid_cap(nullptr, pc))));
}

template <bool D1, int MINW>
hipError_t launch_pipe(const uint32_t * in, uint64_t nblocks, const uint32_t * starts, uint32_t start0, uint8_t * out, uint64_t out_cap,
                       uint64_t * off, void * ws, hipStream_t stream, uint32_t ci, uint32_t lag, uint32_t per_ticket)
{
    const PipeGeom g = pipe_geom(nblocks, ci);
    const dev::PipeWs W = pipe_ws(ws, nblocks, g);
    hipError_t e = hipMemsetAsync(W.head, 0, g.polled, stream);
    if (e != hipSuccess)
        return e;
    dev::PipeArgs A;
    A.in = in;
    A.nblocks = nblocks;
    A.starts = starts;
    A.start0 = start0;
    A.out_base = reinterpret_cast<uint64_t>(out);
    A.cap_end = A.out_base + out_cap;
    A.off = off;
    A.nitems = g.nitems;
    A.nchunks = static_cast<uint32_t>(g.nchunks);
    A.ci = ci;
    A.lag = lag;
    A.per_ticket = per_ticket;
    hipLaunchKernelGGL((dev::k_enc256v32_pipe<D1, MINW>), dim3(pipe_grid<D1, MINW>(g.nitems)), dim3(256), 0, stream, A, W);
    e = hipGetLastError();
    if (e != hipSuccess)
        return e;
    hipLaunchKernelGGL(dev::k_enc_pipe_finish, dim3(1), dim3(64), 0, stream, W.abort, off, nblocks);
    return hipGetLastError();
}

template <bool D1>
hipError_t launch_pipe_w(int minw, const uint32_t * in, uint64_t nblocks, const uint32_t * starts, uint32_t start0, uint8_t * out,
                         uint64_t out_cap, uint64_t * off, void * ws, hipStream_t stream, uint32_t ci, uint32_t lag,
                         uint32_t per_ticket)
{
    switch (minw)
    {
        case 8:
            return launch_pipe<D1, 8>(in, nblocks, starts, start0, out, out_cap, off, ws, stream, ci, lag, per_ticket);
        case 6:
            return launch_pipe<D1, 6>(in, nblocks, starts, start0, out, out_cap, off, ws, stream, ci, lag, per_ticket);
        default:
            return launch_pipe<D1, 1>(in, nblocks, starts, start0, out, out_cap, off, ws, stream, ci, lag, per_ticket);
    }
}

// look-back encoder: one status word per tile + the abort word, then the
// two-pass encoder's workspace for its gated fallback
uint64_t lb_tiles(uint64_t nblocks, uint32_t k) { return (nblocks + 4u * k - 1u) / (4u * k); }
size_t lb_status_bytes(uint64_t nblocks) { return al256(lb_tiles(nblocks, 4) * 8u + 16u); } // the smallest tile measured

// look-back encoder variants: {K, ARENA}
struct LbCfg
{
    uint32_t k, arena;
};

template <bool D1, uint32_t K, uint32_t A>
void launch_lb_one(const uint32_t * in, uint64_t nblocks, const uint32_t * starts, uint32_t start0, uint8_t * out, uint64_t out_cap,
                   uint64_t * off, uint64_t * status, uint32_t * abort, hipStream_t stream)
{
    hipLaunchKernelGGL((dev::k_enc256v32_lb<D1, K, A>), dim3(static_cast<uint32_t>(lb_tiles(nblocks, K))), dim3(256), 0, stream, in, nblocks,
                       starts, start0, off, out, out_cap, status, abort);
}

template <bool D1>
hipError_t launch_lb_k(LbCfg c, const uint32_t * in, uint64_t nblocks, const uint32_t * starts, uint32_t start0, uint8_t * out,
                       uint64_t out_cap, uint64_t * off, uint64_t * status, uint32_t * abort, hipStream_t stream)
{
#define TPF_LB(K, A)                                                                                        \
    if (c.k == K && c.arena == A)                                                                           \
    {                                                                                                       \
        launch_lb_one<D1, K, A>(in, nblocks, starts, start0, out, out_cap, off, status, abort, stream);      \
        return hipGetLastError();                                                                           \
    }
    TPF_LB(4, 0)
    TPF_LB(6, 0)
    TPF_LB(8, 0)
    TPF_LB(8, 5120)
    TPF_LB(8, 4096)
    TPF_LB(6, 3840)
    TPF_LB(12, 7680)
#undef TPF_LB
    return hipErrorInvalidValue;
}

// look-back status + the two-pass workspace, or the pipelined encoder's
// workspace at its smallest chunk (64 items), whichever is larger
size_t encvar_ws(uint64_t nblocks) { return std::max(lb_status_bytes(nblocks) + twopass_workspace(nblocks), pipe_geom(nblocks, 64).bytes); }

hipError_t launch_variant(const uint32_t * in, uint64_t nblocks, const uint32_t * starts, uint32_t start0, bool d1, uint8_t * out,
                          uint64_t out_cap, uint64_t * off, void * ws, size_t ws_bytes, hipStream_t stream, int probe)
{
    if (nblocks == 0)
        return hipMemsetAsync(off, 0, sizeof(uint64_t), stream);
    if (nblocks + 1 > 0x7FFFFFFFull || ws_bytes < encvar_ws(nblocks))
        return hipErrorInvalidValue;
    if (probe == 13)
        return enc256::launch_twopass<256, 256>(in, nblocks, starts, start0, d1, out, out_cap, off, ws, stream);
    if (probe == 14)
        return enc256::launch_twopass<512, 512>(in, nblocks, starts, start0, d1, out, out_cap, off, ws, stream);
    if (probe == 15)
        return enc256::launch_twopass<0, 256>(in, nblocks, starts, start0, d1, out, out_cap, off, ws, stream);
    if (probe == 16 || probe == 17)
    {
        // the two-pass encoder on a persistent grid-stride grid (8 / 4
        // workgroups per CU) instead of one workgroup per 64 blocks; the gate
        // word is set so the gated kernels run
        uint32_t * on = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(ws) + lb_status_bytes(nblocks) - 16u);
        hipError_t e = hipMemsetAsync(on, 1, 4, stream);
        if (e != hipSuccess)
            return e;
        return enc256::launch_twopass<0, 0>(in, nblocks, starts, start0, d1, out, out_cap, off,
                                            static_cast<uint8_t *>(ws) + lb_status_bytes(nblocks), stream, on, probe == 16 ? 8u : 4u);
    }
    if (probe >= 18)
    {
        const uint32_t pv = static_cast<uint32_t>(probe - 16);
        const uint32_t ci = std::min<uint32_t>(dev::kPipeMaxChunkItems, std::max<uint32_t>(64, pv % 1024));
        const uint32_t lag = std::max<uint32_t>(1, (pv / 1024) % 64);
        const int minw = static_cast<int>((pv >> 16) & 15u);
        const uint32_t per_ticket = std::max<uint32_t>(1, pv >> 20);
        return d1 ? launch_pipe_w<true>(minw, in, nblocks, starts, start0, out, out_cap, off, ws, stream, ci, lag, per_ticket)
                  : launch_pipe_w<false>(minw, in, nblocks, starts, start0, out, out_cap, off, ws, stream, ci, lag, per_ticket);
    }
    if (probe < 4 || probe > 12)
        return hipErrorInvalidValue;
    static const LbCfg cfgs[] = {{dev::kLbK, dev::kLbArena}, {4, 0}, {6, 0}, {8, 0}, {8, 5120}, {8, 4096}, {6, 3840}, {12, 7680}};
    const LbCfg c = probe >= 5 && probe <= 11 ? cfgs[probe - 4] : cfgs[0]; // 4, 12: cfgs[0]
    const uint32_t k = c.k;
    uint64_t * status = static_cast<uint64_t *>(ws);
    uint32_t * abort = reinterpret_cast<uint32_t *>(status + lb_tiles(nblocks, k));
    void * tws = static_cast<uint8_t *>(ws) + lb_status_bytes(nblocks);
    hipError_t e = hipMemsetAsync(status, 0, lb_tiles(nblocks, k) * 8u + 16u, stream);
    if (e == hipSuccess && probe == 4)
        e = hipMemsetAsync(abort, 1, 1, stream);
    if (e != hipSuccess)
        return e;
    e = d1 ? launch_lb_k<true>(c, in, nblocks, starts, start0, out, out_cap, off, status, abort, stream)
           : launch_lb_k<false>(c, in, nblocks, starts, start0, out, out_cap, off, status, abort, stream);
    if (e != hipSuccess)
        return e;
    return enc256::launch_twopass<0, 0>(in, nblocks, starts, start0, d1, out, out_cap, off, tws, stream, abort);
}

} // namespace
} // namespace tpf

extern "C" {

size_t encvar_workspace_size(uint64_t nblocks) { return tpf::encvar_ws(nblocks); }

// 0 on success, else the hipError_t
int encvar_launch(int mode, const uint32_t * d_in, uint64_t nblocks, uint8_t * d_out, uint64_t out_cap, uint64_t * d_off, void * d_ws,
                  size_t ws_bytes, void * stream)
{
    return static_cast<int>(tpf::launch_variant(d_in, nblocks, nullptr, 0, false, d_out, out_cap, d_off, d_ws, ws_bytes,
                                                 static_cast<hipStream_t>(stream), mode));
}

} // extern "C"
