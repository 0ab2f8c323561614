// shard_exec_mock.cpp -- CPU test of the multi-GPU host streams' device
// discipline (turbopfor-cpp_amd/csrc/shard_exec.h, used by
// tpf_host_dec_multi / tpf_host_enc_multi) through a mock device map: a
// thread-local "current device" stands for hipSetDevice / hipGetDevice, and a
// mock pipeline checks that it is made, used and destroyed only while its own
// device is selected (the multi-device code had never met a
// second physical GPU).  Prints "shard exec ok" on success.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "shard_exec.h"

static thread_local int t_dev = 0;       // the mock current device of this thread
static std::set<int> g_bad_devs;         // devices whose selection fails
static std::atomic<int> g_violations{0}; // operations seen on the wrong device
static std::atomic<int> g_made{0}, g_destroyed{0};

#define CHECK(c)                                                                                                                   \
    do                                                                                                                             \
    {                                                                                                                              \
        if (!(c))                                                                                                                  \
        {                                                                                                                          \
            std::fprintf(stderr, "CHECK failed line %d: %s\n", __LINE__, #c);                                                    \
            std::exit(1);                                                                                                          \
        }                                                                                                                          \
    } while (0)

struct MockPipe
{
    int dev;
    explicit MockPipe(int d) : dev(d)
    {
        if (t_dev != d)
            g_violations++;
        g_made++;
    }
    void use() const // a stream / event / allocation call on this pipeline
    {
        if (t_dev != dev)
            g_violations++;
    }
    ~MockPipe()
    {
        if (t_dev != dev)
            g_violations++;
        g_destroyed++;
    }
};

struct MockOps
{
    int get_dev() { return t_dev; }
    bool set_dev(int d)
    {
        if (g_bad_devs.count(d))
            return false;
        t_dev = d;
        return true;
    }
    MockPipe * make(int d) { return new MockPipe(d); }
};

static tpf::DevicePool<MockPipe> g_pool;

// one shard's body: lease a pipeline of the thread's device, use it, give it back
static int shard_body(int expect_dev, bool fail, bool throw_it, std::string & msg)
{
    if (t_dev != expect_dev)
        g_violations++;
    MockOps ops;
    MockPipe * p = g_pool.acquire(ops);
    CHECK(p->dev == expect_dev);
    for (int i = 0; i < 100; ++i)
        p->use();
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    g_pool.give_back(p);
    if (throw_it)
        throw std::runtime_error("shard exploded");
    if (fail)
    {
        msg = "shard failed on purpose";
        return -4;
    }
    return 0;
}

int main()
{
    auto set_dev = [](int d) {
        MockOps o;
        return o.set_dev(d);
    };
    // 1. eight devices, then repeated / permuted device lists, several rounds:
    //    every shard runs bound to its device and gets a pipeline of that device
    const std::vector<std::vector<int>> lists = {{0, 1, 2, 3, 4, 5, 6, 7}, {7, 6, 5, 4, 3, 2, 1, 0}, {0, 0, 1, 1}, {3}, {2, 5, 2, 5, 2, 5}};
    for (int round = 0; round < 3; ++round)
        for (const auto & devs : lists)
        {
            const auto res = tpf::run_shards(
                devs.data(), static_cast<int>(devs.size()), set_dev,
                [&](int d, std::string & msg) { return shard_body(devs[d], false, false, msg); }, -2, -3);
            for (const auto & r : res)
                CHECK(r.rc == 0);
        }
    CHECK(g_violations.load() == 0);
    // pipelines are reused per device: no more than the peak number of
    // concurrent shards on one device were ever made for it
    CHECK(g_made.load() <= 14); // per device the most shards a list puts on it at once: 2,2,3,1,1,3,1,1
    // 2. one shard fails, one throws, one cannot select its device: each is
    //    recorded for its own shard, every other shard completes, all joined
    g_bad_devs = {6};
    {
        const std::vector<int> devs = {0, 1, 2, 3, 4, 5, 6, 7};
        std::atomic<int> done{0};
        const auto res = tpf::run_shards(
            devs.data(), 8, set_dev,
            [&](int d, std::string & msg) {
                const int rc = shard_body(devs[d], d == 2, d == 4, msg);
                done++;
                return rc;
            },
            -2, -3);
        CHECK(res[2].rc == -4 && res[2].msg == "shard failed on purpose");
        CHECK(res[4].rc == -3 && res[4].msg == "shard exploded");
        CHECK(res[6].rc == -2 && res[6].msg.find("device 6") != std::string::npos);
        for (int d : {0, 1, 3, 5, 7})
            CHECK(res[d].rc == 0);
        CHECK(done.load() == 6); // device 6's body never ran, shard 4 threw
    }
    g_bad_devs.clear();
    CHECK(g_violations.load() == 0);
    // 3. release from a thread on another device: each pipeline is destroyed
    //    with its own device selected and the caller's device is restored
    t_dev = 3;
    {
        MockOps ops;
        g_pool.drain(ops);
    }
    CHECK(t_dev == 3);
    CHECK(g_violations.load() == 0);
    CHECK(g_made.load() == g_destroyed.load());
    CHECK(g_pool.idle.empty());
    std::printf("shard exec ok: %d pipelines made and destroyed on their own devices\n", g_made.load());
    return 0;
}
