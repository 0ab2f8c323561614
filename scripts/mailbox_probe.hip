// mailbox_probe.hip -- measurement tool (not part of the library): round-trip
// latency of a host <-> resident-kernel mailbox, for the per-block block
// server (p4_server.hip).  One workgroup polls a request word; on a new
// request it reads a 1 KB payload, writes 1 KB of answer into host memory and
// acknowledges; the host times request -> acknowledgement.
//   mode 0: request line + payload in coherent pinned host memory (the
//           server's current layout: every device poll is a PCIe read)
//   mode 1: request line + payload in fine-grained DEVICE memory written by
//           the host CPU over the BAR (device polls its own memory)
//   mode 2: request word only in device memory, payload in host memory
// Answers and acknowledgements always go to host memory (the host polls its
// own cache).  Device loads of mailbox words are vector atomic loads; all
// device stores are vector stores.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/mailbox_probe scripts/mailbox_probe.hip
// usage: mailbox_probe MODE [calls]
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct alignas(128) Req
{
    uint32_t req;
    uint32_t stop;
    uint32_t pad[30];
    u32x4 payload[64];
};

struct alignas(128) Ans
{
    uint32_t ack;
    uint32_t pad[31];
    u32x4 out[64];
};

__device__ __forceinline__ uint32_t ld_sys(const uint32_t * p)
{
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void k_server(Req * rq, const u32x4 * payload, Ans * an, uint32_t calls)
{
    const uint32_t t = threadIdx.x;
    uint32_t last = 0;
    uint64_t active = __builtin_amdgcn_s_memrealtime();
    for (uint64_t polls = 0;; ++polls)
    {
        const uint32_t r = __builtin_amdgcn_readfirstlane(ld_sys(&rq->req));
        if (r != last)
        {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            const u32x4 v = payload[t];
            an->out[t] = v ^ u32x4{r, r, r, r};
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            if (t == 0)
                __hip_atomic_store(&an->ack, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            last = r;
            if (r >= calls)
                return;
            active = __builtin_amdgcn_s_memrealtime();
            continue;
        }
        // leave after 2 s without a request (100 MHz counter) or when told to stop
        if (__builtin_amdgcn_s_memrealtime() - active > 200000000ull)
            return;
        if ((polls & 1023u) == 0u && __builtin_amdgcn_readfirstlane(ld_sys(&rq->stop)) != 0u)
            return;
        __builtin_amdgcn_s_sleep(1);
    }
}

#define CK(x)                                                                                                   \
    do                                                                                                          \
    {                                                                                                           \
        hipError_t e_ = (x);                                                                                    \
        if (e_ != hipSuccess)                                                                                   \
        {                                                                                                       \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));                                          \
            return 1;                                                                                           \
        }                                                                                                       \
    } while (0)

int main(int argc, char ** argv)
{
    const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
    const uint32_t calls = argc > 2 ? static_cast<uint32_t>(std::atoi(argv[2])) : 2000;
    Req * rq = nullptr; // request word (+ payload in modes 0/1)
    Req * hp = nullptr; // host payload (mode 2)
    Ans * an = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void **>(&an), sizeof(Ans), hipHostMallocCoherent | hipHostMallocPortable));
    if (mode == 0)
        CK(hipHostMalloc(reinterpret_cast<void **>(&rq), sizeof(Req), hipHostMallocCoherent | hipHostMallocPortable));
    else
    {
        CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&rq), sizeof(Req), hipDeviceMallocFinegrained));
        CK(hipMemset(rq, 0, sizeof(Req)));
        if (mode == 2)
            CK(hipHostMalloc(reinterpret_cast<void **>(&hp), sizeof(Req), hipHostMallocCoherent | hipHostMallocPortable));
    }
    CK(hipDeviceSynchronize());
    hipPointerAttribute_t at{};
    CK(hipPointerGetAttributes(&at, rq));
    std::printf("mode %d: request at %p (type %d, host ptr %p, device ptr %p)\n", mode, static_cast<void *>(rq), static_cast<int>(at.type),
                at.hostPointer, at.devicePointer);
    std::fflush(stdout);
    // host view of the request block: the same pointer (fine-grained device memory is mapped for the host when
    // the BAR covers it); a fault here ends the process before any kernel runs
    volatile uint32_t * hreq = &rq->req;
    if (mode != 0)
    {
        std::printf("host write to device memory...\n");
        std::fflush(stdout);
        hreq[1] = 0; // stop word
        std::printf("host write ok, read back %u\n", hreq[1]);
        std::fflush(stdout);
    }
    else
        std::memset(rq, 0, sizeof(Req));
    std::memset(an, 0, sizeof(Ans));
    const u32x4 * payload = mode == 2 ? hp->payload : rq->payload;
    u32x4 * hpay = mode == 2 ? hp->payload : rq->payload;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(k_server, dim3(1), dim3(64), 0, s, rq, payload, an, calls);
    CK(hipGetLastError());
    std::vector<double> us;
    us.reserve(calls);
    volatile uint32_t * hack = &an->ack;
    bool bad = false;
    for (uint32_t i = 1; i <= calls; ++i)
    {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t k = 0; k < 64; ++k)
            hpay[k] = u32x4{i, k, i ^ k, 7u};
        _mm_sfence();
        std::atomic_thread_fence(std::memory_order_release);
        *hreq = i;
        _mm_sfence();
        while (*hack != i)
        {
            _mm_pause();
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1))
            {
                std::printf("timeout at call %u\n", i);
                bad = true;
                break;
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        const auto t1 = std::chrono::steady_clock::now();
        if (bad)
            break;
        const u32x4 o = an->out[5];
        if (o.x != (i ^ i) || o.y != (5u ^ i))
        {
            std::printf("wrong answer at call %u\n", i);
            bad = true;
            break;
        }
        us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    if (bad)
        hreq[1] = 1;
    CK(hipStreamSynchronize(s));
    if (us.size() > 100)
    {
        std::vector<double> w(us.begin() + 50, us.end());
        std::sort(w.begin(), w.end());
        std::printf("mode %d: %zu calls, median %.2f us, p10 %.2f, p90 %.2f, p99 %.2f\n", mode, w.size(), w[w.size() / 2],
                    w[w.size() / 10], w[w.size() * 9 / 10], w[w.size() * 99 / 100]);
    }
    return bad ? 2 : 0;
}
