// p4_enc256v32.hip -- batch encode of 256v32 P4 blocks (p4Enc256v32 /
// p4D1Enc256v32, reference src/scalar/p4enc256v32_scalar.cpp:216-235 and
// p4d1enc256v32_scalar.cpp:7-15) on gfx950.
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
// probe != 0 (measurement only, reachable only through the separate
// tpf_probe_enc256v32 entry point -- the output is NOT a valid stream): 1 =
// plan kernel with the cost model replaced by a wave OR, 2 = write kernel
// copying the staged values instead of building blocks; same loads and
// stores, so they time each pass's data-movement ceiling
// (scripts/gpu_enc_probe.sh, profiles/r1_v4_enc_probe.txt).
#include "p4_scan.h"

#include "p4_enc32.h"
#include "tpf_kernels.h"

namespace tpf::dev
{

constexpr uint32_t kImgU32 = 592; // bytes per wave image: 4..7 lead + block (<= 2276 B) + slack, 16-B multiple
constexpr uint32_t kEncRun = 16;  // blocks per wave run
constexpr uint32_t kEncNC = 3;    // value chunks in flight per wave (block j+1, j+2 while j is encoded)

// deltaEnc1 (p4_scalar_internal.h:711-719): d[i] = in[i] - in[i-1] - 1, in[-1] = start.
__device__ __forceinline__ u32x4 delta_encode(const u32x4 & v, uint32_t start, uint32_t t)
{
    uint32_t prev = static_cast<uint32_t>(__shfl_up(static_cast<int>(v.w), 1, 64));
    if (t == 0)
        prev = start;
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
struct EncRun
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
        return __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(jj * 1024u + 16u * t), 0, 0);
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
    template <class Body>
    __device__ __forceinline__ void walk(uint32_t t, Body && body) const
    {
        u32x4 C[kEncNC];
#pragma unroll
        for (uint32_t u = 0; u + 1 < kEncNC; ++u)
            C[u] = load(u, t);
        bool more = true;
        for (uint32_t j = 0; more; j += kEncNC)
        {
#pragma unroll
            for (uint32_t u = 0; u < kEncNC; ++u)
            {
                if (more)
                {
                    C[(u + kEncNC - 1) % kEncNC] = load(j + u + kEncNC - 1, t);
                    body(C[u], j + u);
                    more = j + u + 1 < n;
                }
            }
        }
    }
};

__device__ __forceinline__ uint32_t rl32(uint32_t v, uint32_t lane)
{
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(lane)));
}

// Plan a run: lane j of (szv, pwv) = size and plan word of block R.first+j.
template <bool D1, int PROBE = 0>
__device__ __forceinline__ void plan_run(const EncRun & R, const uint32_t * in, const uint32_t * starts, uint32_t start0,
                                         uint32_t * hist, uint32_t t, uint32_t & szv, uint32_t & pwv)
{
    const uint32_t stv = D1 ? R.start_lane(in, starts, start0, t) : 0u;
    szv = 0u;
    pwv = 0u;
    R.walk(t, [&](u32x4 v, uint32_t jj) {
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

// Write a run: lane j of (szv, pwv, olo/ohi) = size, plan word and byte
// offset of block R.first+j.  img: the wave's zeroed LDS image (left zeroed).
template <bool D1, int PROBE = 0>
__device__ __forceinline__ void write_run(const EncRun & R, const uint32_t * in, const uint32_t * starts, uint32_t start0,
                                          uint32_t szv, uint32_t pwv, uint32_t olo, uint32_t ohi, uint32_t * img,
                                          uint32_t * val, uint64_t out_base, uint64_t cap_end, uint32_t t)
{
    const uint32_t stv = D1 ? R.start_lane(in, starts, start0, t) : 0u;
    R.walk(t, [&](u32x4 v, uint32_t jj) {
        if constexpr (D1)
            v = delta_encode(v, rl32(stv, jj), t);
        const uint32_t size = rl32(szv, jj);
        const Plan32 P = unplan(rl32(pwv, jj), size);
        const uint64_t dst = out_base + ((static_cast<uint64_t>(rl32(ohi, jj)) << 32) | rl32(olo, jj));
        if constexpr (PROBE == 2)
        {
            reinterpret_cast<u32x4 *>(img)[4 + t] = v;
            wave_lds_sync();
            copy_out_image16(img, kImgLead, dst, size, cap_end, t);
            wave_lds_sync();
            zero_image(img, kImgU32 / 4u, t);
            wave_lds_sync();
            return;
        }
        const uint32_t sb = emit_block256<true>(img, val, P, v, t);
        wave_lds_sync();
        copy_out_image16(img, sb, dst, size, cap_end, t);
        wave_lds_sync();
        // only [0, sb + size) can be non-zero: clear it for the next block
        zero_image(img, min((sb + size + 15u) >> 4, kImgU32 / 4u), t);
        wave_lds_sync();
    });
}

// ---- two-pass encoder (plan -> run scan -> write): the production path ---
// The plan pass leaves each block's size in off[block] and one total per
// wave run; p4_scan.h scans only the run totals; the write pass rebuilds the
// offsets of its run from the run base and its sizes and writes them back.
template <bool D1, int PROBE = 0>
__global__ __launch_bounds__(256) void k_enc256v32_plan(const uint32_t * __restrict in, uint64_t nblocks,
                                                         const uint32_t * __restrict starts, uint32_t start0,
                                                         uint64_t * __restrict sizes, uint32_t * __restrict plan,
                                                         uint32_t * __restrict run_tot)
{
    __shared__ __attribute__((aligned(16))) uint32_t hist[4][kPlanHistU32];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    EncRun R;
    if (!R.init(in, nblocks, wv))
        return;
    uint32_t szv, pwv; // lane j: block first+j
    plan_run<D1, PROBE>(R, in, starts, start0, hist[wv], t, szv, pwv);
    if (t < R.n)
    {
        sizes[R.first + t] = szv;
        plan[R.first + t] = pwv;
    }
    publish_run_total(run_tot, R.first / kEncRun, t < R.n ? szv : 0u, t);
}

template <bool D1, int PROBE = 0>
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
    EncRun R;
    if (!R.init(in, nblocks, wv))
        return;
    // lane j: destination offset (64-bit), size and plan of block first+j
    uint64_t ov, ev;
    run_offsets(off, R.first, R.n, run_base(run_pre, run_tile, R.first / kEncRun), t, ov, ev);
    const uint32_t szv = static_cast<uint32_t>(ev - ov);
    const uint32_t pwv = t < R.n ? plan[R.first + t] : 0u;
    zero_image(img, kImgU32 / 4u, t);
    wave_lds_sync();
    const uint64_t out_base = reinterpret_cast<uint64_t>(out);
    write_run<D1, PROBE>(R, in, starts, start0, szv, pwv, static_cast<uint32_t>(ov), static_cast<uint32_t>(ov >> 32), img,
                         val_all[wv], out_base, out_base + out_cap, t);
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
constexpr uint32_t kPipeChunkItems = 256;    // default: 32K blocks = 32 MiB of values per chunk
constexpr uint32_t kPipeLag = 2;             // default: chunk c is written in step c + 2
constexpr int kPipeMinWaves = 8;             // default launch bound: 8 waves per SIMD
constexpr uint32_t kPipePerTicket = 8;       // default: sequence entries per ticket
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

size_t al256(size_t x) { return (x + 255u) & ~size_t(255); }

uint64_t enc_runs(uint64_t nblocks) { return (nblocks + dev::kEncRun - 1u) / dev::kEncRun; }

// two-pass encoder workspace: plan words + the run scan (p4_scan.h)
size_t twopass_workspace(uint64_t nblocks) { return al256(nblocks * 4u) + RunScanWs<uint64_t>::bytes(enc_runs(nblocks)); }

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

} // namespace

// the pipelined encoder's workspace is largest at the smallest chunk it may run with (64 items)
size_t enc256v32_workspace(uint64_t nblocks) { return std::max(twopass_workspace(nblocks), pipe_geom(nblocks, 64).bytes); }

hipError_t launch_enc256v32(const uint32_t * in, uint64_t nblocks, const uint32_t * starts, uint32_t start0, bool d1,
                            uint8_t * out, uint64_t out_cap, uint64_t * off, void * ws, size_t ws_bytes, hipStream_t stream,
                            int probe)
{
    if (nblocks == 0)
        return hipMemsetAsync(off, 0, sizeof(uint64_t), stream);
    if (nblocks + 1 > 0x7FFFFFFFull)
        return hipErrorInvalidValue;
    if (probe >= 16)
    {
        // probe >= 16 (measurement): 16 + ci + 1024 * lag + 65536 * minw + 2^20 * per_ticket
        // (minw: launch bound in waves per SIMD, 8 / 6 / other = none)
        const uint32_t pv = static_cast<uint32_t>(probe - 16);
        const uint32_t ci = probe >= 16 ? std::min<uint32_t>(dev::kPipeMaxChunkItems, std::max<uint32_t>(64, pv % 1024))
                                        : dev::kPipeChunkItems;
        const uint32_t lag = probe >= 16 ? std::max<uint32_t>(1, (pv / 1024) % 64) : dev::kPipeLag;
        const int minw = probe >= 16 ? static_cast<int>((pv >> 16) & 15u) : dev::kPipeMinWaves;
        const uint32_t per_ticket = probe >= 16 ? std::max<uint32_t>(1, pv >> 20) : dev::kPipePerTicket;
        return d1 ? launch_pipe_w<true>(minw, in, nblocks, starts, start0, out, out_cap, off, ws, stream, ci, lag, per_ticket)
                  : launch_pipe_w<false>(minw, in, nblocks, starts, start0, out, out_cap, off, ws, stream, ci, lag, per_ticket);
    }
    // the production two-pass encoder (probe 0 / 3), or its passes with the coding removed (probe 1 / 2)
    if (ws_bytes < twopass_workspace(nblocks))
        return hipErrorInvalidValue;
    uint32_t * plan = static_cast<uint32_t *>(ws);
    const uint64_t nruns = enc_runs(nblocks);
    const RunScanWs<uint64_t> rs = RunScanWs<uint64_t>::carve(static_cast<uint8_t *>(ws) + al256(nblocks * 4u), nruns);
    const uint64_t per_wg = 4ull * dev::kEncRun;
    const uint32_t grid = static_cast<uint32_t>((nblocks + per_wg - 1) / per_wg);
    if (d1)
        hipLaunchKernelGGL(dev::k_enc256v32_plan<true>, dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan, rs.tot);
    else if (probe == 1)
        hipLaunchKernelGGL((dev::k_enc256v32_plan<false, 1>), dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan,
                           rs.tot);
    else
        hipLaunchKernelGGL(dev::k_enc256v32_plan<false>, dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan, rs.tot);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return e;
    e = launch_run_scan_u64(rs.tot, nruns, rs.pre, rs.tile, off + nblocks, stream);
    if (e != hipSuccess)
        return e;
    if (d1)
        hipLaunchKernelGGL(dev::k_enc256v32_write<true>, dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan, rs.pre,
                           rs.tile, out, out_cap);
    else if (probe == 2)
        hipLaunchKernelGGL((dev::k_enc256v32_write<false, 2>), dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan,
                           rs.pre, rs.tile, out, out_cap);
    else
        hipLaunchKernelGGL(dev::k_enc256v32_write<false>, dim3(grid), dim3(256), 0, stream, in, nblocks, starts, start0, off, plan,
                           rs.pre, rs.tile, out, out_cap);
    return hipGetLastError();
}

} // namespace tpf
