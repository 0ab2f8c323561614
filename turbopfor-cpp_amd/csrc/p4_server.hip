// p4_server.hip -- resident block server for the per-block drop-in API
// (include/turbopfor.h: one p4Enc* / p4Dec* call = one block).
//
// A launch plus a stream synchronise per call costs ~18-24 us on this stack
// (DESIGN.md 5), 600x slower than the reference's own per-block call
// (src/dispatch.cpp:88-95 on one core).  Here one workgroup stays resident
// while calls keep coming: wave w polls request box w (tpf_server.h: in
// fine-grained device memory the host writes through the BAR, or in pinned
// host memory; 16 workgroups x 4 waves = 64 mailboxes since round 5), decodes
// or encodes the block it finds with the generic wave
// codec (p4_generic.h: every format of turbopfor.h; 256v64 = two 128v64
// blocks, p4enc256v64_scalar.cpp:15-30), writes the result into answer box w
// in pinned host memory and acknowledges.  Host and device exchange only
// plain loads and stores ordered by system-scope fences (no atomics on
// shared memory).  Exit: every wave leaves once all mailboxes have been idle
// for idle_ticks of the 100 MHz real-time counter, after max_ticks in any
// case (a device-wide synchronize elsewhere in the process must not wait for
// it forever), or at once when the host sets `stop`; `alive` drops and the
// host relaunches on the next call.
#include <hip/hip_runtime.h>

#include "p4_generic.h"
#include "tpf_kernels.h"
#include "tpf_server.h"

namespace tpf::dev
{

constexpr uint32_t kSrvImgU32 = (kServerPayload + 64u) / 4u;

struct alignas(16) SrvLds
{
    uint32_t img[kSrvImgU32]; // staged block bytes (decode) / block image (encode)
    uint64_t scr[512];        // vbyte exception scratch of decode_block_g
    uint32_t hist[kPlanGHistU32];
};

// Mailbox words are read with (vector) atomic loads: a uniform plain load
// could be turned into a scalar-cache load, which the fences do not refresh.
__device__ __forceinline__ uint32_t ld_sys(const uint32_t * p)
{
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys64(const uint64_t * p)
{
    return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Round 5: no system-scope fences.  On gfx950 an acquire fence at system
// scope is `buffer_inv sc0 sc1` and a release `buffer_wbl2 sc0 sc1` --
// whole-L2 invalidate / write-back operations of the XCD, which serialised
// concurrent calls (64 mailboxes served ~0.7M calls/s together).  Instead
// every access to the mailboxes' payloads is itself system-coherent (sc0 sc1:
// it bypasses the CU and L2 caches), loads are issued only after the request
// word they depend on has arrived, and the acknowledgement is stored only
// after `s_waitcnt vmcnt(0)` has seen every payload store complete.
constexpr int kSysPol = 1 | 16; // sc0 | sc1
__device__ __forceinline__ void st_sys(uint32_t * p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint64_t * p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ld_sys_v(const uint32_t * p)
{
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys_v(const uint64_t * p)
{
    return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// bytes [0, nbytes) of an LDS buffer (16-byte aligned) to a mailbox answer
// with 16-byte system-coherent stores: the answer crosses PCIe as 16-byte
// writes instead of one write per dword (round 5).  Stores whole chunks (the
// answer payload is larger than any result).
__device__ __forceinline__ void put_answer(uint8_t * dst, const uint32_t * src, uint32_t nbytes, uint32_t t)
{
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(dst, kServerPayload);
    for (uint32_t i = t; i < (nbytes + 15u) >> 4; i += 64u)
        __builtin_amdgcn_raw_buffer_store_b128(reinterpret_cast<const u32x4 *>(src)[i], rs, static_cast<int>(16u * i), 0, kSysPol);
}

// every vector memory operation of the wave complete (stores included: gfx9
// counts them in vmcnt); "memory": the compiler keeps accesses on their side
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint32_t rl32w(uint32_t v, uint32_t lane)
{
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(lane)));
}

// Stage bytes [0, len) of a host buffer into LDS (and zero the 64 after).
__device__ __forceinline__ void srv_stage(uint32_t * img, const uint8_t * src, uint32_t len, uint32_t t)
{
    // system-coherent 16-byte loads (kSysPol); chunks past len read nothing
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(src, kServerPayload);
    u32x4 * d = reinterpret_cast<u32x4 *>(img);
    const uint32_t n16 = (len + 15u) >> 4;
    for (uint32_t i = t; i < n16 + 4u && i < kSrvImgU32 / 4u; i += 64u)
        d[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(i < n16 ? 16u * i : 0x80000000u), 0, kSysPol);
    wave_lds_sync();
    // bytes of the last chunk past len were read from the payload buffer: clear them
    uint8_t * b = reinterpret_cast<uint8_t *>(img);
    if (t < 16u && (len & 15u) && (len & ~15u) + t >= len)
        b[(len & ~15u) + t] = 0;
    wave_lds_sync();
}

// One F block at LDS byte s: values -> out (T), returns bytes consumed;
// *lim = values the reference writes (n for a constant block, else the
// layout's width).  D1: start -> *last (value n-1).  The values go out
// through L.scr (free once the block is decoded) as 16-byte stores.
template <Fmt F>
__device__ __forceinline__ uint32_t srv_dec_one(SrvLds & L, uint32_t s, uint32_t n, bool d1, typename FmtTraits<F>::T start,
                                                uint8_t * out, uint32_t t, uint32_t * lim, typename FmtTraits<F>::T * last)
{
    using T = typename FmtTraits<F>::T;
    const uint32_t NE = FmtTraits<F>::N ? FmtTraits<F>::N : n;
    T v[4];
    uint32_t cm;
    const uint32_t used = decode_block_g<F>(L.img, s, n, L.scr, t, v, &cm);
    if (d1)
        *last = delta1_g<T>(v, n, start, t); // its carry: the value of element n-1
    *lim = cm ? n : NE;
    wave_lds_sync(); // the decoder's scratch reads are done
    T * const st = reinterpret_cast<T *>(L.scr);
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
        st[t + 64u * j] = v[j];
    wave_lds_sync();
    put_answer(out, reinterpret_cast<const uint32_t *>(L.scr), *lim * static_cast<uint32_t>(sizeof(T)), t);
    wave_lds_sync();
    return used;
}

// One F block of n values from in (T, the layout's width) into the LDS
// image at byte s (zeroed), returns its size.
template <Fmt F>
__device__ __forceinline__ uint32_t srv_enc_one(SrvLds & L, uint32_t s, const typename FmtTraits<F>::T * in, uint32_t n, bool d1,
                                                typename FmtTraits<F>::T start, uint32_t t)
{
    using T = typename FmtTraits<F>::T;
    const uint32_t NE = FmtTraits<F>::N ? FmtTraits<F>::N : n;
    T v[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
        v[j] = t + 64u * j < NE ? ld_sys_v(&in[t + 64u * j]) : T(0);
    if (d1)
        delta_enc_g<T>(v, start, n, t);
    const PlanG P = plan_block_g<F>(v, n, L.hist, t);
    emit_block_g<F>(L.img, s, P, v, n, t);
    wave_lds_sync();
    return P.size;
}

template <Fmt F>
__device__ __forceinline__ void srv_serve(SrvLds & L, const ServerReqBox * box, ServerAnsBox * ans, uint32_t op, uint32_t n,
                                          bool d1, uint64_t start, uint32_t in_len, bool pair, uint32_t t)
{
    using T = typename FmtTraits<F>::T;
    const uint32_t n0 = pair ? min(n, 128u) : n;
    if (op == kOpDec)
    {
        srv_stage(L.img, box->in, in_len, t);
        uint8_t * const out = ans->out;
        uint32_t lim = 0;
        T last = T(0);
        uint32_t used = srv_dec_one<F>(L, 0u, n0, d1, static_cast<T>(start), out, t, &lim, &last);
        uint32_t written = lim;
        // a pair whose first block consumes all of in_len disagrees with the
        // host framing of both blocks: corrupt input, not a 128-value success
        // 
        bool ok = true;
        if (pair && n > 128u)
        {
            ok = used < in_len;
            if (ok)
            {
                // second 128v64 block, starting after the first one's value 127
                used += srv_dec_one<F>(L, used, n - 128u, d1, last, out + 128u * sizeof(T), t, &lim, &last);
                written = 128u + lim;
            }
        }
        if (t == 0)
        {
            st_sys(&ans->result, ok && used == in_len ? used : 0xFFFFFFFFu);
            st_sys(&ans->written, written);
        }
        return;
    }
    // encode: values of the layout's width in box->in
    const T * in = reinterpret_cast<const T *>(box->in);
    const uint32_t zero16 = (kSrvImgU32 / 4u);
    for (uint32_t i = t; i < zero16; i += 64u)
        reinterpret_cast<u32x4 *>(L.img)[i] = u32x4{0u, 0u, 0u, 0u};
    wave_lds_sync();
    uint32_t size = srv_enc_one<F>(L, 0u, in, n0, d1, static_cast<T>(start), t);
    if (pair && n > 128u)
    {
        // D1: the second block starts from input value 127 (p4d1enc256v64_scalar.cpp)
        const T s127 = static_cast<T>(uni64(ld_sys64(reinterpret_cast<const uint64_t *>(in + 127))));
        size += srv_enc_one<F>(L, size, in + 128, n - 128u, d1, s127, t);
    }
    // copy the image out (whole 16-byte chunks: the mailbox payload is larger than any block)
    put_answer(ans->out, L.img, size, t);
    if (t == 0)
        st_sys(&ans->result, size);
}

__device__ __forceinline__ uint32_t ld_agent(const uint32_t * p)
{
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void k_block_server(ServerReq * rq, ServerAns * an, ServerCtl * ctl, uint64_t idle_ticks,
                                                      uint64_t max_ticks)
{
    __shared__ SrvLds L[kServerWavesPerWG];
    const uint32_t t = threadIdx.x & 63u;
    const uint32_t w = uni(threadIdx.x >> 6);
    const uint64_t born = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0)
    {
        atomicAdd(&ctl->live, 1u);
        atomicMax(&ctl->last_active, static_cast<unsigned long long>(born));
        __hip_atomic_store(&an->alive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
    const uint32_t bi = blockIdx.x * kServerWavesPerWG + w; // this wave's mailbox
    const ServerReqBox * box = &rq->box[bi];
    ServerAnsBox * ans = &an->box[bi];
    uint32_t last = uni(ld_sys(&ans->ack));
    const uint32_t * line = &box->req;
    // Round 5: the launch's shared words are touched rarely.  Each wave
    // publishes its activity (atomicMax of last_active) at most once per
    // 1 ms of serving, and idle waves read the shared words every 256th
    // poll: one device-scope atomic on one address per request, from every
    // server wave on every XCD, capped all callers together at ~1M
    // calls/s; without it 16 callers reach ~3M (profiles/r5t_*).  The idle
    // exit tolerates the staleness (10 ms idle against 1 ms publication).
    uint64_t pub_a = born;
    for (uint32_t polls = 0;; ++polls)
    {
        // the whole request line in one read: lanes 0..7 hold its first 8
        // words; the launch's quit word is loaded beside it, so both arrive
        // in one memory latency (checked below when no request came)
        const uint32_t word = t < 8u ? ld_sys(line + t) : 0u;
        const uint32_t quit = ld_agent(&ctl->quit);
        const uint32_t r = rl32w(word, 0);
        if (r != last)
        {
            // (no acquire fence: the payload loads are system-coherent and
            // issued after this request word arrived)
            const uint32_t op = rl32w(word, 1), fmt = rl32w(word, 2), n = rl32w(word, 3);
            const uint32_t d1 = rl32w(word, 4), in_len = rl32w(word, 5);
            const uint64_t start = (static_cast<uint64_t>(rl32w(word, 7)) << 32) | rl32w(word, 6);
            const bool ok = n >= 1u && n <= 256u && in_len <= kServerPayload;
            if (!ok)
            {
                if (t == 0)
                    st_sys(&ans->result, 0xFFFFFFFFu);
            }
            else
                switch (fmt)
                {
                    case FMT_32:
                        srv_serve<Fmt::H32>(L[w], box, ans, op, n, d1, start, in_len, false, t);
                        break;
                    case FMT_128V32:
                        srv_serve<Fmt::V128>(L[w], box, ans, op, min(n, 128u), d1, start, in_len, false, t);
                        break;
                    case FMT_256V32:
                        srv_serve<Fmt::V256>(L[w], box, ans, op, n, d1, start, in_len, false, t);
                        break;
                    case FMT_64:
                        srv_serve<Fmt::H64>(L[w], box, ans, op, n, d1, start, in_len, false, t);
                        break;
                    case FMT_128V64:
                        srv_serve<Fmt::V128X64>(L[w], box, ans, op, min(n, 128u), d1, start, in_len, false, t);
                        break;
                    case FMT_256V64:
                        srv_serve<Fmt::V128X64>(L[w], box, ans, op, n, d1, start, in_len, true, t);
                        break;
                    default:
                        if (t == 0)
                            st_sys(&ans->result, 0xFFFFFFFFu);
                }
            wait_vm(); // the results reached memory before the acknowledgement
            if (t == 0)
                __hip_atomic_store(&ans->ack, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            last = r;
            const uint64_t now_a = __builtin_amdgcn_s_memrealtime();
            if (now_a - pub_a > 100000u) // 1 ms of the 100 MHz counter
            {
                if (t == 0)
                    atomicMax(&ctl->last_active, static_cast<unsigned long long>(now_a));
                pub_a = now_a;
            }
            if (__builtin_amdgcn_s_memrealtime() - born > max_ticks) // busy past the lifetime: leave after this answer
            {
                if (t == 0)
                    __hip_atomic_store(&ctl->quit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            continue;
        }
        // leave together: once one wave of the launch quits (idle, past its
        // lifetime, or told to stop) every other follows at its next poll.
        // The quit word (device memory) and the lifetime are checked on every
        // poll (round 6, ADVICE r5: checked every 256th, the launch's waves
        // left over up to 256 poll intervals while the host kept posting to
        // mailboxes whose waves had gone).  The idle test (last_active) and
        // the host's stop word are read every 256th poll (each read of the
        // stop word crosses PCIe in mode 2).
        if (uni(quit) != 0u)
            break;
        bool leave = __builtin_amdgcn_s_memrealtime() - born > max_ticks;
        if ((polls & 255u) == 0u)
        {
            const uint64_t la = uni64(__hip_atomic_load(&ctl->last_active, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            // the clock is read AFTER last_active: another workgroup may have
            // published a later time between an earlier clock read and the
            // load, and `now - la` would wrap to ~2^64 (a spurious
            // idle exit of the whole server)
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            leave = leave || (la < now && now - la > idle_ticks) || uni(ld_sys(&rq->stop)) != 0u;
        }
        if (leave)
        {
            if (t == 0)
                __hip_atomic_store(&ctl->quit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    // every wave of this workgroup has left its poll loop: none serves after
    // this point; the launch's last workgroup out lowers `alive`
    __syncthreads();
    if (threadIdx.x == 0 && atomicSub(&ctl->live, 1u) == 1u)
        __hip_atomic_store(&an->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

} // namespace tpf::dev

namespace tpf
{

hipError_t launch_block_server(ServerReq * d_req, ServerAns * d_ans, ServerCtl * d_ctl, hipStream_t s)
{
    // the control words start at zero for every launch (a kernel, not a
    // memset: DESIGN.md 8)
    hipError_t e = fill_u32(d_ctl, 0u, sizeof(ServerCtl) / 4u, s);
    if (e != hipSuccess)
        return e;
    hipLaunchKernelGGL(dev::k_block_server, dim3(kServerWGs), dim3(256), 0, s, d_req, d_ans, d_ctl, kServerIdleTicks, kServerMaxTicks);
    return hipGetLastError();
}

} // namespace tpf
