// perblock_threads.cpp -- aggregate throughput of the per-block drop-in calls
// (include/turbopfor.h: one 256-value block per call, any number of calling
// threads, src/dispatch.cpp:88-104) at T concurrent callers: each thread
// encodes / decodes ITS OWN block K times with turbopfor::p4Enc256v32 /
// p4Dec256v32, checking every returned end pointer and the decoded values.
// One JSON line per T.  PBT_MODE=2: request mailboxes in pinned host memory
// (tpf_perblock_mode(2)) instead of device memory written through the BAR.
// PBT_N=n (< 256): p4Enc32 / p4Dec32 blocks of n values instead (a small
// payload: separates the per-call round trip from moving the block).
// usage: perblock_threads K T1 [T2 ...]
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <latch>
#include <thread>
#include <vector>

#include "turbopfor.h"
#include "turbopfor_capi.h"

// weak: the tool also runs against older library builds without the counter
#pragma weak tpf_perblock_launches
static uint64_t launches_now() { return tpf_perblock_launches ? tpf_perblock_launches() : 0; }

static void fill_block(uint32_t * v, uint32_t seed)
{
    // bw 8 base with 10% exceptions in [2^8, 2^32): the ab_test-style mix (ab_test.cpp:1611-1626)
    uint64_t x = 0x9E3779B97F4A7C15ull * (seed + 1);
    for (int i = 0; i < 256; ++i)
    {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        v[i] = (x % 10 == 0) ? static_cast<uint32_t>(256u + (x >> 32) % 0xFFFFFEFFu) : static_cast<uint32_t>((x >> 20) & 255u);
    }
}

int main(int argc, char ** argv)
{
    if (argc < 3)
    {
        std::fprintf(stderr, "usage: %s K T1 [T2 ...]\n", argv[0]);
        return 2;
    }
    const int K = std::atoi(argv[1]);
    const int mode = std::getenv("PBT_MODE") ? std::atoi(std::getenv("PBT_MODE")) : 0;
    const unsigned nv = std::getenv("PBT_N") ? static_cast<unsigned>(std::atoi(std::getenv("PBT_N"))) : 256u;
    auto enc = [nv](uint32_t * v, unsigned char * o) {
        return nv >= 256u ? turbopfor::p4Enc256v32(v, 256, o) : turbopfor::p4Enc32(v, nv, o);
    };
    auto dec = [nv](const unsigned char * i, uint32_t * o) {
        return nv >= 256u ? turbopfor::p4Dec256v32(i, 256, o) : turbopfor::p4Dec32(i, nv, o);
    };
    if (mode != 0 && tpf_perblock_mode(mode) < 0)
    {
        std::fprintf(stderr, "tpf_perblock_mode(%d) failed\n", mode);
        return 2;
    }
    for (int a = 2; a < argc; ++a)
    {
        const int T = std::atoi(argv[a]);
        std::atomic<int> bad{0};
        double dec_s = 0, enc_s = 0;
        uint64_t launches[2] = {0, 0}; // block-server launches during each timed phase
        for (int phase = 0; phase < 2; ++phase) // 0 = encode, 1 = decode
        {
            // blocking latches, not yield loops: on a machine whose CPU time is
            // capped by a cgroup quota, T threads yield-spinning between their
            // warm-up call and the start burn the quota, and the timed phase
            // then runs throttled (round 6: the spread of the 48-128 thread
            // numbers before this)
            std::latch ready(T), go(1);
            std::vector<std::thread> th;
            std::vector<double> secs(T);
            for (int i = 0; i < T; ++i)
                th.emplace_back([&, i] {
                    uint32_t v[256], out[256];
                    unsigned char buf[4096];
                    fill_block(v, static_cast<uint32_t>(i));
                    unsigned char * end = enc(v, buf); // warm: also relaunches the server
                    if (!end)
                        bad++;
                    ready.count_down();
                    go.wait();
                    if (!end)
                        return;
                    const auto t0 = std::chrono::steady_clock::now();
                    for (int k = 0; k < K; ++k)
                    {
                        if (phase == 0)
                        {
                            if (enc(v, buf) != end)
                                bad++;
                        }
                        else if (dec(buf, out) != end)
                            bad++;
                    }
                    secs[i] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                    if (phase == 1 && std::memcmp(out, v, 4u * (nv >= 256u ? 256u : nv)) != 0)
                        bad++;
                });
            ready.wait();
            // let a cgroup quota period pass: the warm-up's CPU time (thread
            // creation, T first calls) is not charged to the timed phase
            std::this_thread::sleep_for(std::chrono::milliseconds(200));
            const uint64_t l0 = launches_now();
            const auto t0 = std::chrono::steady_clock::now();
            go.count_down();
            for (auto & t : th)
                t.join();
            const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            launches[phase] = launches_now() - l0;
            (phase == 0 ? enc_s : dec_s) = wall;
        }
        const double calls = static_cast<double>(T) * K;
        std::printf("{\"mode\": %d, \"n\": %u, \"threads\": %d, \"calls_per_thread\": %d, \"dec_calls_per_s\": %.0f, \"dec_G_int32_per_s\": %.4f, "
                    "\"dec_us_per_call\": %.2f, \"enc_calls_per_s\": %.0f, \"enc_G_int32_per_s\": %.4f, \"enc_us_per_call\": %.2f, "
                    "\"enc_launches\": %llu, \"dec_launches\": %llu, \"bad\": %d}\n",
                    mode, nv, T, K, calls / dec_s, calls * (nv >= 256u ? 256u : nv) / dec_s / 1e9, dec_s * T / calls * 1e6, calls / enc_s, calls * (nv >= 256u ? 256u : nv) / enc_s / 1e9,
                    enc_s * T / calls * 1e6, static_cast<unsigned long long>(launches[0]), static_cast<unsigned long long>(launches[1]), bad.load());
        std::fflush(stdout);
        if (bad.load())
            return 1;
    }
    return 0;
}
