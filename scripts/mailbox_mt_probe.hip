// mailbox_mt_probe.hip -- measurement tool (not part of the library):
// aggregate rate of T host threads each doing request -> acknowledgement
// round trips with its own resident wave (the block server's mechanism
// without the codec), to tell the round trip's own ceiling from the
// server's.  Request words live in fine-grained device memory written by the
// host through the BAR (the server's mode 0); acknowledgements (and, with
// PAYLOAD=1, a 1 KB answer of 16-byte system-coherent stores) go to coherent
// pinned host memory.  No system-scope fences: sc0 sc1 accesses and
// s_waitcnt vmcnt(0) before the acknowledgement, as p4_server.hip.
// Build: hipcc --offload-arch=gfx950 -O3 -o mailbox_mt_probe scripts/mailbox_mt_probe.hip -lpthread
// usage: mailbox_mt_probe CALLS PAYLOAD T1 [T2 ...]   (T <= 64)
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kBoxes = 64;

struct alignas(128) Req
{
    uint32_t req;
    uint32_t pad[31];
};
struct alignas(128) Ans
{
    uint32_t ack;
    uint32_t pad[31];
    u32x4 out[64];
};
struct alignas(128) Ctl
{
    uint32_t stop;
    uint32_t pad[31];
};

__device__ __forceinline__ uint32_t ld_sys(const uint32_t * p)
{
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void k_echo(Req * rq, Ans * an, Ctl * ctl, int payload)
{
    const uint32_t t = threadIdx.x;
    Req * q = rq + blockIdx.x;
    Ans * a = an + blockIdx.x;
    uint32_t last = 0;
    uint64_t active = __builtin_amdgcn_s_memrealtime();
    for (uint64_t polls = 0;; ++polls)
    {
        const uint32_t r = __builtin_amdgcn_readfirstlane(ld_sys(&q->req));
        if (r != last)
        {
            if (payload)
            {
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a->out, static_cast<short>(0), 1024, 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{r, t, r ^ t, 7u}, rs, static_cast<int>(16u * t), 0, 1 | 16);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (t == 0)
                __hip_atomic_store(&a->ack, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            last = r;
            active = __builtin_amdgcn_s_memrealtime();
            continue;
        }
        if (__builtin_amdgcn_s_memrealtime() - active > 2000000000ull) // 20 s idle
            return;
        if ((polls & 255u) == 0u && __builtin_amdgcn_readfirstlane(ld_sys(&ctl->stop)) != 0u)
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
    if (argc < 4)
    {
        std::fprintf(stderr, "usage: %s CALLS PAYLOAD T1 [T2 ...]\n", argv[0]);
        return 2;
    }
    const uint32_t calls = static_cast<uint32_t>(std::atoi(argv[1]));
    const int payload = std::atoi(argv[2]);
    Req * rq = nullptr;
    Ans * an = nullptr;
    Ctl * ctl = nullptr;
    CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&rq), sizeof(Req) * kBoxes, hipDeviceMallocFinegrained));
    CK(hipMemset(rq, 0, sizeof(Req) * kBoxes));
    CK(hipHostMalloc(reinterpret_cast<void **>(&an), sizeof(Ans) * kBoxes, hipHostMallocCoherent | hipHostMallocPortable));
    CK(hipHostMalloc(reinterpret_cast<void **>(&ctl), sizeof(Ctl), hipHostMallocCoherent | hipHostMallocPortable));
    std::memset(an, 0, sizeof(Ans) * kBoxes);
    ctl->stop = 0;
    CK(hipDeviceSynchronize());
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(k_echo, dim3(kBoxes), dim3(64), 0, s, rq, an, ctl, payload);
    CK(hipGetLastError());
    uint32_t next[kBoxes] = {};
    int rc = 0;
    for (int a = 3; a < argc && rc == 0; ++a)
    {
        const int T = std::min(std::atoi(argv[a]), kBoxes);
        std::atomic<int> ready{0}, bad{0};
        std::atomic<bool> go{false};
        std::vector<std::thread> th;
        for (int i = 0; i < T; ++i)
            th.emplace_back([&, i] {
                volatile uint32_t * hreq = &rq[i].req;
                volatile uint32_t * hack = &an[i].ack;
                ready++;
                while (!go.load())
                    std::this_thread::yield();
                for (uint32_t k = 0; k < calls; ++k)
                {
                    const uint32_t r = ++next[i];
                    _mm_sfence();
                    *hreq = r;
                    _mm_sfence();
                    const auto t0 = std::chrono::steady_clock::now();
                    while (*hack != r)
                    {
                        _mm_pause();
                        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1))
                        {
                            bad++;
                            return;
                        }
                    }
                }
            });
        while (ready.load() < T)
            std::this_thread::yield();
        const auto t0 = std::chrono::steady_clock::now();
        go = true;
        for (auto & t : th)
            t.join();
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("{\"threads\": %d, \"payload\": %d, \"calls_per_thread\": %u, \"calls_per_s\": %.0f, \"us_per_call\": %.2f, \"bad\": %d}\n",
                    T, payload, calls, T * calls / sec, sec * 1e6 / calls, bad.load());
        std::fflush(stdout);
        if (bad.load())
            rc = 1;
    }
    ctl->stop = 1;
    _mm_sfence();
    CK(hipStreamSynchronize(s));
    return rc;
}
