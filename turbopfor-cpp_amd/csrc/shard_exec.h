// shard_exec.h -- the device-affinity skeleton of the multi-GPU host streams
// (tpf_host_dec_multi / tpf_host_enc_multi, host_stream.cpp): one thread per
// shard bound to its device before it touches anything, and a pool of
// per-device pipelines.  Free of HIP so that a CPU test can drive it with a
// mock device map (tests/cpp/shard_exec_mock.cpp): the multi-device code had
// only ever met one physical GPU, so its device discipline is
// checked here by construction and by that test.
//
// Rules it enforces:
//   * a shard thread selects its device (set_dev) before its body runs, and
//     the body runs only if that succeeded;
//   * every shard thread is joined, whatever the others did: an error or an
//     exception in one shard is recorded for that shard and never leaves
//     another shard's thread blocked or unjoined (a failed thread creation
//     joins the threads already started before it reports);
//   * a pooled object is created, handed out, returned and destroyed with
//     its own device selected (DevicePool: acquire on device d only ever
//     returns an object made on d; destroy selects the object's device and
//     restores the caller's).
#pragma once

#include <exception>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace tpf
{

struct ShardResult
{
    int rc = 0; // 0 = ok, else the shard's error code
    std::string msg;
};

// Run body(d) for d in [0, ndev) on ndev threads, thread d bound to devs[d]
// by set_dev(dev) -> bool.  Returns one result per shard; err_dev / err_exc =
// the codes recorded for a failed set_dev / an exception out of body.
template <class SetDev, class Body>
std::vector<ShardResult> run_shards(const int * devs, int ndev, SetDev && set_dev, Body && body, int err_dev, int err_exc)
{
    std::vector<ShardResult> res(static_cast<size_t>(ndev));
    std::vector<std::thread> th;
    th.reserve(static_cast<size_t>(ndev));
    std::exception_ptr spawn_failed;
    for (int d = 0; d < ndev; ++d)
    {
        try
        {
            th.emplace_back([&, d] {
                ShardResult & r = res[static_cast<size_t>(d)];
                if (!set_dev(devs[d]))
                {
                    r.rc = err_dev;
                    r.msg = "selecting device " + std::to_string(devs[d]) + " failed";
                    return;
                }
                try
                {
                    r.rc = body(d, r.msg);
                }
                catch (const std::exception & e)
                {
                    r.rc = err_exc;
                    r.msg = e.what();
                }
                catch (...)
                {
                    r.rc = err_exc;
                    r.msg = "unknown exception";
                }
            });
        }
        catch (...)
        {
            spawn_failed = std::current_exception(); // join what runs, then report
            break;
        }
    }
    for (std::thread & t : th)
        t.join();
    if (spawn_failed)
        std::rethrow_exception(spawn_failed);
    return res;
}

// Idle objects of type T (each made on one device, T::dev), shared by all
// threads.  Ops: get_dev() -> int (the calling thread's device), set_dev(int)
// -> bool, make(dev) -> T* (called with dev selected).
template <class T>
struct DevicePool
{
    std::mutex mu;
    std::vector<T *> idle;

    // an object of the calling thread's current device
    template <class Ops>
    T * acquire(Ops & ops)
    {
        const int dev = ops.get_dev();
        {
            std::lock_guard<std::mutex> g(mu);
            for (size_t i = 0; i < idle.size(); ++i)
                if (idle[i]->dev == dev)
                {
                    T * p = idle[i];
                    idle.erase(idle.begin() + static_cast<std::ptrdiff_t>(i));
                    return p;
                }
        }
        return ops.make(dev);
    }
    void give_back(T * p)
    {
        std::lock_guard<std::mutex> g(mu);
        idle.push_back(p);
    }
    // destroy p with its own device selected, then restore the caller's
    template <class Ops>
    static void destroy(Ops & ops, T * p)
    {
        const int cur = ops.get_dev();
        const bool sw = cur != p->dev && ops.set_dev(p->dev);
        delete p;
        if (sw)
            (void)ops.set_dev(cur);
    }
    // every idle object, each destroyed on its own device
    template <class Ops>
    void drain(Ops & ops)
    {
        std::vector<T *> all;
        {
            std::lock_guard<std::mutex> g(mu);
            all.swap(idle);
        }
        for (T * p : all)
            destroy(ops, p);
    }
};

} // namespace tpf
