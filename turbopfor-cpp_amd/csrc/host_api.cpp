// host_api.cpp -- the drop-in boundary: include/turbopfor.h (C++ linkage,
// signature-identical to the reference's include/turbopfor.h:9-80), its
// extern "C" mirror include/turbopfor_capi.h, and the host-memory stream
// entry points.  Every call runs the gfx950 kernels; nothing here encodes or
// decodes a value on the CPU.
//
// Per-block calls (one block per call, as reference callers chain them) go
// to the resident block server (p4_server.hip, tpf_server.h): the call
// writes the block into a request mailbox in fine-grained device memory
// (through the BAR), bumps the request word and spins on the acknowledgement
// in pinned host memory -- no launch, no stream synchronise per call.
// tpf_perblock_mode(2) keeps the request mailboxes in pinned host memory
// (the first server layout: the kernel polls across PCIe);
// tpf_perblock_mode(1) selects the first design (a thread-local stream and
// pinned staging, one batched launch with nblocks = 1 on the staging's
// device addresses, synchronise: 18-25 us per call, the launch + synchronise
// floor).  All give identical bytes; throughput callers use
// tpf_host_dec/tpf_host_enc (pipelined host streams) or turbopfor_gpu.h
// (device-resident batches).
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <sched.h>
#include <sys/prctl.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/turbopfor.h"
#include "../../include/turbopfor_capi.h"
#include "../../include/turbopfor_gpu.h"
#include "tpf_kernels.h"
#include "tpf_server.h"

namespace
{

void hip_check(hipError_t e, const char * what)
{
    if (e != hipSuccess)
        throw std::runtime_error(std::string("turbopfor_amd: ") + what + ": " + hipGetErrorString(e));
}

void tpf_check(int rc, const char * what)
{
    if (rc != TPF_OK)
        throw std::runtime_error(std::string("turbopfor_amd: ") + what + ": " + tpf_last_error());
}

bool wide_fmt(int fmt) { return fmt == TPF_FMT_64 || fmt == TPF_FMT_128V64 || fmt == TPF_FMT_256V64; }

unsigned unit_values(int fmt, unsigned n)
{
    switch (fmt)
    {
        case TPF_FMT_128V32:
        case TPF_FMT_128V64:
            return 128;
        case TPF_FMT_256V32:
        case TPF_FMT_256V64:
            return 256;
        default:
            return n;
    }
}

struct DevBuf
{
    void * p = nullptr;
    size_t n = 0;
    void release()
    {
        if (p)
            (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void * get(size_t want)
    {
        if (want > n)
        {
            if (p)
                (void)hipFree(p);
            p = nullptr;
            hip_check(hipMalloc(&p, want), "hipMalloc");
            n = want;
        }
        return p;
    }
    ~DevBuf()
    {
        if (p)
            (void)hipFree(p);
    }
};

// Pinned staging; `d` is its device address (hipHostMalloc memory is mapped
// into the device's address space), looked up once per allocation.
struct HostBuf
{
    void * p = nullptr;
    void * d = nullptr;
    size_t n = 0;
    void release()
    {
        if (p)
            (void)hipHostFree(p);
        p = d = nullptr;
        n = 0;
    }
    void * get(size_t want)
    {
        if (want > n)
        {
            release();
            hip_check(hipHostMalloc(&p, want, hipHostMallocDefault), "hipHostMalloc");
            hip_check(hipHostGetDevicePointer(&d, p, 0), "hipHostGetDevicePointer");
            n = want;
        }
        return p;
    }
    ~HostBuf() { release(); }
};

// Thread-local per-block context.
struct Ctx
{
    int device = -1;
    hipStream_t stream = nullptr;

    DevBuf d_ws;
    HostBuf h_in, h_vals, h_off;

    static Ctx & get()
    {
        thread_local Ctx c;
        thread_local int count = -1;
        if (count <= 0 && (hipGetDeviceCount(&count) != hipSuccess || count <= 0))
            throw std::runtime_error("turbopfor_amd: no HIP device visible (this library has no CPU fallback)");
        int dev = 0;
        hip_check(hipGetDevice(&dev), "hipGetDevice");
        if (c.device != dev)
        {
            c.reset();
            c.device = dev;
            hip_check(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking), "hipStreamCreate");
        }
        return c;
    }
    void reset()
    {
        d_ws.release();
        for (HostBuf * b : {&h_in, &h_vals, &h_off})
            b->release();
        if (stream)
            (void)hipStreamDestroy(stream);
        stream = nullptr;
    }
    ~Ctx() { reset(); }
};

// ---- waiting for an answer: spin, or sleep when callers outnumber CPUs ------
// Round 6.  A waiting caller spun on its answer word.  With
// more calling threads than CPUs the spinners took the CPUs from the threads
// that would post requests and read answers; on a machine whose CPU time is
// capped by a cgroup quota (the GPU boxes: 256 visible CPUs, 16 CPUs of
// quota) every spinner sits on a CPU of its own and burns quota, the cgroup is
// throttled for the rest of each period, and the aggregate collapsed (64
// callers: 1.17M calls/s at 55 us per call, against 3.8M at 24).  Yielding
// does not help there (a thread alone on its CPU gets it straight back).  So
// when the threads that call the library outnumber the CPUs the process may
// use, a waiter sleeps between polls instead (1 us of timer slack on the
// calling thread, set once); otherwise it spins as before.

// CPUs this process may use: its affinity mask, capped by a cgroup CPU quota
// (v2 cpu.max, v1 cfs_quota_us / cfs_period_us).
unsigned effective_cpus()
{
    cpu_set_t set;
    unsigned n = 0;
    if (sched_getaffinity(0, sizeof(set), &set) == 0)
        n = static_cast<unsigned>(CPU_COUNT(&set));
    if (n == 0)
        n = std::max(1u, std::thread::hardware_concurrency());
    double quota = -1, period = -1;
    {
        std::ifstream f("/sys/fs/cgroup/cpu.max");
        std::string q;
        if (f >> q >> period && q != "max")
            quota = std::atof(q.c_str());
    }
    if (quota <= 0)
    {
        std::ifstream fq("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"), fp("/sys/fs/cgroup/cpu/cpu.cfs_period_us");
        if (!(fq >> quota && fp >> period))
            quota = -1;
    }
    if (quota > 0 && period > 0)
        n = std::min(n, std::max(1u, static_cast<unsigned>(quota / period + 0.999)));
    return n;
}

// Threads that have made a per-block call and still exist (each registers on
// its first call, deregisters at exit): the one word a call reads for the
// policy is written only when threads come and go.
std::atomic<unsigned> g_callers{0};
struct CallerReg
{
    bool on = false;
    void enter()
    {
        if (!on)
        {
            on = true;
            g_callers.fetch_add(1u, std::memory_order_relaxed);
        }
    }
    ~CallerReg()
    {
        if (on)
            g_callers.fetch_sub(1u, std::memory_order_relaxed);
    }
};

// TPF_PERBLOCK_WAIT=spin / sleep forces one policy (A/B runs); default: auto.
int wait_policy()
{
    const char * e = std::getenv("TPF_PERBLOCK_WAIT");
    if (e && std::strcmp(e, "spin") == 0)
        return 1;
    if (e && std::strcmp(e, "sleep") == 0)
        return 2;
    return 0;
}

// calling threads (registers the calling thread)
unsigned callers()
{
    thread_local CallerReg reg;
    reg.enter();
    return g_callers.load(std::memory_order_relaxed);
}

// Sleeping costs a wake-up per nap, spinning a CPU per waiter: spinning
// still wins up to about twice as many callers as CPUs (r6j, 16 CPUs: 24-32
// spinning callers 3.6-4.9M calls/s, sleeping 2.3-3.7M; 48 and more sleeping
// 4.6-4.9M at 48-64 and 2.1-2.6M at 96-128, spinning 1.0-3.9M).
bool crowded()
{
    static const unsigned cpus = effective_cpus();
    static const int policy = wait_policy();
    return policy == 2 || (policy == 0 && callers() > 2u * cpus);
}

void nap_ns(long ns)
{
    thread_local bool slack = [] {
        (void)prctl(PR_SET_TIMERSLACK, 1000ul, 0ul, 0ul, 0ul); // 1 us (the default 50 us would set every nap's length)
        return true;
    }();
    (void)slack;
    timespec ts{0, ns};
    (void)nanosleep(&ts, nullptr);
}

// ---- resident block server (per device) ------------------------------------
// 0 = block server with request mailboxes in device memory, 1 = launch +
// synchronise per call, 2 = block server with request mailboxes in host memory
std::atomic<int> g_mode{0};
// launches of the block server on every device (tpf_perblock_launches)
std::atomic<uint64_t> g_launches{0};

struct Server
{
    int dev = -1;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr; // recorded after the current launch
    bool launched = false;
    // request halves: fine-grained device memory written through the BAR
    // (mode 0; its host and device addresses coincide) and pinned host memory
    // (mode 2)
    tpf::ServerReq * rq_dev = nullptr; // stays null without a CPU-mapped (large) BAR
    tpf::ServerReq * rq_host = nullptr;
    tpf::ServerReq * rq_host_d = nullptr;
    tpf::ServerAns * an = nullptr;   // answers: coherent pinned host memory (host view)
    tpf::ServerAns * an_d = nullptr; // the same memory, device view
    tpf::ServerCtl * ctl = nullptr; // device memory shared by the launch's workgroups
    std::atomic<tpf::ServerReq *> launched_rq{nullptr};
    std::mutex mu; // launches, event queries
    // Mailbox leases (round 5): one lock word per mailbox, each on its own
    // cache line, tried from a per-thread starting mailbox, so concurrent
    // callers touch no shared line per call.  A pause (tpf::PerblockPause)
    // takes every mailbox: the mailboxes are also the per-block calls' side
    // of the pause.  (A shared free mask, a std::shared_mutex for the pause
    // and packed request counters -- six contended read-modify-writes per
    // call -- capped 8-64 callers at ~630k calls/s together.)
    struct alignas(64) Box
    {
        std::atomic<uint32_t> busy{0};
        std::atomic<uint32_t> reqno{0};   // last request number posted to this mailbox
        std::atomic<uint32_t> waiters{0}; // callers blocked on `busy` (lease, crowded)
    };
    Box box[tpf::kServerBoxes];
    bool held = false; // every mailbox taken by the pause (pause thread only)


    static void * pinned(size_t bytes, void ** dev_view)
    {
        void * p = nullptr;
        hip_check(hipHostMalloc(&p, bytes, hipHostMallocCoherent | hipHostMallocPortable), "server mailboxes");
        std::memset(p, 0, bytes);
        hip_check(hipHostGetDevicePointer(dev_view, p, 0), "server mailbox device address");
        return p;
    }

    explicit Server(int device) : dev(device)
    {
        hip_check(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "server stream");
        hip_check(hipEventCreateWithFlags(&done, hipEventDisableTiming), "server event");
        void * dv = nullptr;
        an = static_cast<tpf::ServerAns *>(pinned(sizeof(tpf::ServerAns), &dv));
        an_d = static_cast<tpf::ServerAns *>(dv);
        rq_host = static_cast<tpf::ServerReq *>(pinned(sizeof(tpf::ServerReq), &dv));
        rq_host_d = static_cast<tpf::ServerReq *>(dv);
        void * c = nullptr;
        hip_check(hipMalloc(&c, sizeof(tpf::ServerCtl)), "server control words");
        ctl = static_cast<tpf::ServerCtl *>(c);
        // Mode 0 writes the request mailboxes in device memory from the CPU,
        // which needs the whole of VRAM mapped into the CPU's address space
        // (a large BAR).  Without one the device-memory half is never created
        // and every call uses the host-memory mailboxes (mode 2's layout).
        int large_bar = 0;
        if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, dev) != hipSuccess)
        {
            large_bar = 0;
            (void)hipGetLastError();
        }
        if (large_bar)
        {
            void * q = nullptr;
            hip_check(hipExtMallocWithFlags(&q, sizeof(tpf::ServerReq), hipDeviceMallocFinegrained), "request mailboxes");
            hip_check(hipMemsetAsync(q, 0, sizeof(tpf::ServerReq), stream), "request mailboxes");
            hip_check(hipStreamSynchronize(stream), "request mailboxes");
            rq_dev = static_cast<tpf::ServerReq *>(q);
        }
    }

    // the request half the current mode uses (host view)
    tpf::ServerReq * current() const
    {
        return g_mode.load(std::memory_order_relaxed) == 2 || rq_dev == nullptr ? rq_host : rq_dev;
    }

    // caller holds mu, no launch running
    void launch(tpf::ServerReq * rq)
    {
        hip_check(tpf::launch_block_server(rq == rq_host ? rq_host_d : rq, an_d, ctl, stream), "block server launch");
        hip_check(hipEventRecord(done, stream), "block server event");
        launched = true;
        g_launches.fetch_add(1u, std::memory_order_relaxed);
        launched_rq.store(rq, std::memory_order_release);
    }
    // caller holds mu: has the current launch ended (idle exit or stop)?
    bool ended()
    {
        if (!launched)
            return true;
        const hipError_t e = hipEventQuery(done);
        if (e == hipErrorNotReady)
            return false;
        hip_check(e, "block server");
        return true;
    }
    // caller holds mu
    void stop_locked()
    {
        tpf::ServerReq * rq = launched_rq.load(std::memory_order_acquire);
        if (!launched || rq == nullptr)
            return;
        __atomic_store_n(&rq->stop, 1u, __ATOMIC_RELEASE);
        _mm_sfence();
        (void)hipEventSynchronize(done);
        __atomic_store_n(&rq->stop, 0u, __ATOMIC_RELEASE);
        _mm_sfence();
    }
    // Mode switch (no call in flight): retire the launch and bring both
    // request halves' numbers up to date -- a half unused for a while holds
    // stale request words, which a new launch would take for new requests.
    void switch_halves()
    {
        std::lock_guard<std::mutex> g(mu);
        stop_locked();
        for (uint32_t i = 0; i < tpf::kServerBoxes; ++i)
        {
            const uint32_t r = box[i].reqno.load();
            if (rq_dev)
                __atomic_store_n(&rq_dev->box[i].req, r, __ATOMIC_RELAXED);
            __atomic_store_n(&rq_host->box[i].req, r, __ATOMIC_RELAXED);
        }
        _mm_sfence();
        std::atomic_thread_fence(std::memory_order_seq_cst);
    }

    bool try_lease(uint32_t i)
    {
        uint32_t z = 0u;
        return box[i].busy.load(std::memory_order_relaxed) == 0u &&
               box[i].busy.compare_exchange_strong(z, 1u, std::memory_order_seq_cst);
    }
    // A free mailbox, searched from a per-thread starting mailbox (up to 64
    // threads get distinct ones).  With more calling threads than CPUs a
    // caller tries its own mailbox and three others a quarter of the ring
    // apart, then blocks on its own mailbox's lock word until that mailbox is
    // released (a futex wait: no CPU, no polling).  Round 6: a full pass over
    // 64 lock words owned by other cores costs microseconds of CPU, and with
    // 128 callers every waiting thread made such passes between naps (0.9M
    // calls/s, r6b); a semaphore admitting 64 callers at a time paid a futex
    // wake per call (0.75M, r6f); napping waiters paid a wake-up per nap (r6g).
    int lease()
    {
        thread_local const uint32_t hint = [] {
            static std::atomic<uint32_t> next{0};
            return next.fetch_add(1u) % tpf::kServerBoxes;
        }();
        for (;;)
        {
            const bool crowd = crowded();
            const uint32_t tries = crowd ? 4u : tpf::kServerBoxes;
            const uint32_t step = crowd ? tpf::kServerBoxes / 4u : 1u;
            for (uint32_t k = 0; k < tries; ++k)
            {
                const uint32_t i = (hint + k * step) % tpf::kServerBoxes;
                if (try_lease(i))
                    return static_cast<int>(i);
            }
            if (crowd)
            {
                // seq_cst on both sides (the count, then the lock word here;
                // the lock word, then the count in release): one of the two
                // sees the other's store, so a release never skips a waiter
                box[hint].waiters.fetch_add(1u, std::memory_order_seq_cst);
                box[hint].busy.wait(1u, std::memory_order_seq_cst); // returns at once if it is free by now
                box[hint].waiters.fetch_sub(1u, std::memory_order_relaxed);
            }
            else
                std::this_thread::yield();
        }
    }
    void release(int i)
    {
        box[i].busy.store(0u, std::memory_order_seq_cst);
        if (box[i].waiters.load(std::memory_order_seq_cst) != 0u) // only with more callers than mailboxes
            box[i].busy.notify_one();
    }
    // the pause side: every mailbox, as the calls holding them return
    void hold_all()
    {
        for (uint32_t i = 0; i < tpf::kServerBoxes; ++i)
            while (!try_lease(i))
                std::this_thread::yield();
        held = true;
    }
    void release_all()
    {
        if (!held)
            return; // created during the pause: its calls wait on the pending word
        held = false;
        for (uint32_t i = 0; i < tpf::kServerBoxes; ++i)
            release(static_cast<int>(i));
    }

    // Make sure a launch serves `rq`.  Fast path: the running launch raised
    // `alive` and polls this request half -- no event query, no lock.
    void ensure(tpf::ServerReq * rq)
    {
        if (__atomic_load_n(&an->alive, __ATOMIC_ACQUIRE) != 0u && launched_rq.load(std::memory_order_acquire) == rq)
            return;
        std::lock_guard<std::mutex> g(mu);
        if (ended())
            launch(rq);
    }

    // Post the request prepared in box i of `rq` and wait for its acknowledgement.
    void call(tpf::ServerReq * rq, int i)
    {
        tpf::ServerReqBox * b = &rq->box[i];
        tpf::ServerAnsBox * a = &an->box[i];
        const uint32_t r = box[i].reqno.fetch_add(1u, std::memory_order_relaxed) + 1u;
        ensure(rq);
        _mm_sfence(); // the payload and fields (write-combined device memory) before the request word
        std::atomic_thread_fence(std::memory_order_release);
        __atomic_store_n(&b->req, r, __ATOMIC_RELEASE);
        _mm_sfence();
        // Spin (a call takes ~5 us), or with more calling threads than CPUs
        // sleep between polls (see crowded()); a spinner that has waited
        // kSpinNs -- over twice a call's latency -- yields between polls.
        constexpr auto kSpinNs = std::chrono::nanoseconds(12000);
        const bool crowd = crowded();
        const auto t0 = std::chrono::steady_clock::now();
        bool patient = false;
        // crowded: a first nap of about one call's latency (most answers are
        // in by then; every wake-up costs CPU time the callers share), later
        // naps 2 us.  (A first nap tracking the thread's own latency fed back
        // on itself -- the latency includes the nap -- and doubled it, r6h.)
        if (crowd)
            nap_ns(4000);
        for (uint64_t spin = 1;; ++spin)
        {
            if (__atomic_load_n(&a->ack, __ATOMIC_ACQUIRE) == r)
                break;
            if (crowd)
                nap_ns(2000);
            else if (patient)
                std::this_thread::yield();
            else
            {
                _mm_pause();
                if ((spin & 31u) == 0u && std::chrono::steady_clock::now() - t0 > kSpinNs)
                    patient = true;
            }
            if ((spin & (crowd || patient ? 15u : 1023u)) == 0u)
            {
                // the launch may have idled out just before this request:
                // relaunch.  Only when it shows signs of having ended (alive
                // lowered, or another half launched): the mutex and the event
                // query it guards, taken by every waiting caller, serialised
                // many concurrent callers (round 5)
                if (__atomic_load_n(&an->alive, __ATOMIC_ACQUIRE) == 0u || launched_rq.load(std::memory_order_acquire) != rq)
                {
                    std::lock_guard<std::mutex> g(mu);
                    if (ended() && __atomic_load_n(&a->ack, __ATOMIC_ACQUIRE) != r)
                        launch(rq);
                }
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(20))
                    throw std::runtime_error("turbopfor_amd: block server did not answer within 20 s");
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    }

    void stop()
    {
        std::lock_guard<std::mutex> g(mu);
        stop_locked();
    }
};

std::mutex g_srv_mu;
Server * g_srv[64] = {};

// A resident server kernel keeps its stream busy, and HIP waits for every
// stream of the device in hipFree / hipHostFree / hipDeviceSynchronize.  So
// the library's own frees (host_stream.cpp) run inside a tpf::PerblockPause:
// it raises g_pause_pending, takes every mailbox of every server (waiting for
// the calls that hold them), stops the servers, and keeps the mailboxes until
// it ends, so no server runs during the free and no call can relaunch one.
// A call leases its mailbox and THEN reads g_pause_pending (both sequentially
// consistent): either the pause sees the mailbox taken and waits for it, or
// the call sees the pause and gives the mailbox back.  Pauses of different
// threads take turns on g_pause_mu; a thread's nested pauses count depth.
std::mutex g_pause_mu;
std::atomic<int> g_pause_pending{0};

// pauses this thread holds (tpf::PerblockPause nests; only depth 0 -> 1 locks)
thread_local int t_pause_depth = 0;

void pause_lock();
void pause_unlock();

void stop_servers()
{
    std::lock_guard<std::mutex> g(g_srv_mu);
    for (Server * s : g_srv)
        if (s)
            s->stop();
}

// The calling thread's server: a thread-local cache in front of the table,
// so a call takes no lock (round 5: the table's mutex, taken on every call,
// capped 16-64 concurrent callers at ~560k calls/s together).
Server & server()
{
    int dev = 0;
    hip_check(hipGetDevice(&dev), "hipGetDevice");
    thread_local int t_dev = -1;
    thread_local Server * t_srv = nullptr;
    if (dev == t_dev && t_srv != nullptr)
        return *t_srv;
    if (dev < 0 || dev >= 64)
        throw std::runtime_error("turbopfor_amd: device index out of range");
    std::lock_guard<std::mutex> g(g_srv_mu);
    t_dev = dev;
    if (!g_srv[dev])
    {
        static bool registered = false;
        if (!registered)
        {
            std::atexit(stop_servers); // before HIP's own teardown (registered earlier, runs later)
            registered = true;
        }
        g_srv[dev] = new Server(dev);
    }
    t_srv = g_srv[dev];
    return *t_srv;
}

void pause_lock()
{
    g_pause_mu.lock();
    g_pause_pending.fetch_add(1, std::memory_order_seq_cst);
    std::lock_guard<std::mutex> g(g_srv_mu);
    for (Server * s : g_srv)
        if (s)
            s->hold_all();
}

void pause_unlock()
{
    {
        std::lock_guard<std::mutex> g(g_srv_mu);
        for (Server * s : g_srv)
            if (s)
                s->release_all();
    }
    g_pause_pending.fetch_sub(1, std::memory_order_seq_cst);
    g_pause_mu.unlock();
}

// A call's mailbox.  Inside a pause (the pausing thread holds every
// mailbox) a call uses mailbox 0 without leasing it.
struct BoxLease
{
    Server & s;
    tpf::ServerReq * rq;
    int i = 0;
    bool own = false;
    explicit BoxLease(Server & srv) : s(srv), rq(nullptr)
    {
        if (t_pause_depth == 0)
            for (;;)
            {
                while (g_pause_pending.load(std::memory_order_acquire) != 0)
                    std::this_thread::yield();
                i = s.lease();
                if (g_pause_pending.load(std::memory_order_seq_cst) == 0)
                    break;
                s.release(i);
            }
        own = t_pause_depth == 0;
        rq = s.current();
    }
    ~BoxLease()
    {
        if (own)
            s.release(i);
    }
    tpf::ServerReqBox * req() const { return &rq->box[i]; }
    tpf::ServerAnsBox * ans() const { return &s.an->box[i]; }
    void call() { s.call(rq, i); }
};

unsigned char * enc_srv(int fmt, const void * in, unsigned n, unsigned char * out, bool d1, uint64_t start)
{
    Server & S = server();
    BoxLease L(S);
    tpf::ServerReqBox * b = L.req();
    const size_t es = wide_fmt(fmt) ? 8 : 4;
    const size_t vbytes = es * unit_values(fmt, n); // the reference also reads the full block width
    std::memcpy(b->in, in, vbytes);
    b->op = tpf::kOpEnc;
    b->fmt = static_cast<uint32_t>(fmt);
    b->n = n;
    b->d1 = d1 ? 1u : 0u;
    b->start_lo = static_cast<uint32_t>(start);
    b->start_hi = static_cast<uint32_t>(start >> 32);
    b->in_len = static_cast<uint32_t>(vbytes);
    L.call();
    const tpf::ServerAnsBox * a = L.ans();
    const uint32_t size = a->result;
    if (size == 0xFFFFFFFFu || size > tpf::kServerPayload)
        throw std::runtime_error("turbopfor_amd: block server rejected the encode request");
    std::memcpy(out, a->out, size);
    return out + size;
}

const unsigned char * dec_srv(int fmt, const unsigned char * in, unsigned n, void * out, bool d1, uint64_t start)
{
    int written = 0;
    const uint64_t size = tpf_block_size(fmt, in, uint64_t(1) << 20, n, &written);
    if (size == 0 || size > tpf::kServerPayload)
        throw std::runtime_error("turbopfor_amd: malformed P4 block header");
    Server & S = server();
    BoxLease L(S);
    tpf::ServerReqBox * b = L.req();
    std::memcpy(b->in, in, size);
    b->op = tpf::kOpDec;
    b->fmt = static_cast<uint32_t>(fmt);
    b->n = n;
    b->d1 = d1 ? 1u : 0u;
    b->start_lo = static_cast<uint32_t>(start);
    b->start_hi = static_cast<uint32_t>(start >> 32);
    b->in_len = static_cast<uint32_t>(size);
    L.call();
    const tpf::ServerAnsBox * a = L.ans();
    if (a->result != size)
        throw std::runtime_error("turbopfor_amd: malformed P4 block (length check failed on the device)");
    const size_t es = wide_fmt(fmt) ? 8 : 4;
    std::memcpy(out, a->out, es * a->written);
    return in + size;
}

// One-block encode through tpf_enc_batch.  Zero-copy: the kernels read the
// values from, and write the bytes and offsets to, pinned host staging, so a
// call is one launch sequence and one synchronise (the first version staged
// through HBM with three copies: 26.5 us per call).
unsigned char * enc_one(int fmt, const void * in, unsigned n, unsigned char * out, bool d1, uint64_t start)
{
    if (n == 0)
        return out;
    if (g_mode.load(std::memory_order_relaxed) != 1)
        return enc_srv(fmt, in, n, out, d1, start);
    Ctx & c = Ctx::get();
    const size_t es = wide_fmt(fmt) ? 8 : 4;
    const size_t vbytes = es * unit_values(fmt, n);
    const uint64_t cap = tpf_enc_bound(fmt, 1, n);
    void * hv = c.h_vals.get(vbytes);
    std::memcpy(hv, in, vbytes); // the reference also reads the full block width
    auto * hoff = static_cast<uint64_t *>(c.h_off.get(4 * sizeof(uint64_t)));
    auto * hin = static_cast<uint8_t *>(c.h_in.get(cap));
    const size_t wsb = std::max<size_t>(tpf_enc_workspace_size(fmt, 1, n), 256);
    void * ws = c.d_ws.get(wsb);
    tpf_check(tpf_enc_batch(fmt, c.h_vals.d, 1, n, d1 ? 1 : 0, nullptr, start, static_cast<uint8_t *>(c.h_in.d), cap,
                            static_cast<uint64_t *>(c.h_off.d), ws, wsb, c.stream),
              "tpf_enc_batch");
    hip_check(hipStreamSynchronize(c.stream), "sync");
    const uint64_t size = hoff[1];
    std::memcpy(out, hin, size);
    return out + size;
}

// One-block decode through tpf_dec_batch, zero-copy as enc_one (the first
// version: two H2D copies, the launch, one D2H copy: 21.8 us per call).
const unsigned char * dec_one(int fmt, const unsigned char * in, unsigned n, void * out, bool d1, uint64_t start)
{
    if (n == 0)
        return in;
    if (g_mode.load(std::memory_order_relaxed) != 1)
        return dec_srv(fmt, in, n, out, d1, start);
    Ctx & c = Ctx::get();
    int written = 0;
    // the block's length comes from its own header (framing.cpp); 1 MiB is far
    // above any block's size and only bounds the header walk
    const uint64_t size = tpf_block_size(fmt, in, uint64_t(1) << 20, n, &written);
    if (size == 0)
        throw std::runtime_error("turbopfor_amd: malformed P4 block header");
    const size_t es = wide_fmt(fmt) ? 8 : 4;
    const size_t vbytes = es * unit_values(fmt, n);
    auto * hin = static_cast<uint8_t *>(c.h_in.get(size));
    std::memcpy(hin, in, size);
    auto * hoff = static_cast<uint64_t *>(c.h_off.get(4 * sizeof(uint64_t)));
    hoff[0] = 0;
    hoff[1] = size;
    hoff[2] = start;
    void * hv = c.h_vals.get(vbytes);
    auto * doff = static_cast<uint64_t *>(c.h_off.d);
    tpf_check(tpf_dec_batch(fmt, static_cast<const uint8_t *>(c.h_in.d), size, doff, 1, n, c.h_vals.d, d1 ? doff + 2 : nullptr,
                            nullptr, c.stream),
              "tpf_dec_batch");
    hip_check(hipStreamSynchronize(c.stream), "sync");
    std::memcpy(out, hv, es * written);
    return in + size;
}

} // namespace

namespace tpf
{
void set_last_error(const std::string & msg);

PerblockPause::PerblockPause()
{
    if (t_pause_depth++ == 0)
    {
        try
        {
            pause_lock();
        }
        catch (...)
        {
            --t_pause_depth;
            throw;
        }
    }
    stop_servers();
}
PerblockPause::~PerblockPause()
{
    if (--t_pause_depth == 0)
        pause_unlock();
}
} // namespace tpf

namespace
{

template <class F>
auto guarded(F && f) -> decltype(f())
{
    try
    {
        return f();
    }
    catch (const std::exception & e)
    {
        tpf::set_last_error(e.what());
        std::fprintf(stderr, "%s\n", e.what());
        return nullptr;
    }
}

} // namespace

// ---------------------------------------------------------------- turbopfor::
namespace turbopfor
{
unsigned char * p4Enc32(uint32_t * in, unsigned n, unsigned char * out) { return enc_one(TPF_FMT_32, in, n, out, false, 0); }
unsigned char * p4D1Enc32(uint32_t * in, unsigned n, unsigned char * out, uint32_t start)
{
    return enc_one(TPF_FMT_32, in, n, out, true, start);
}
const unsigned char * p4Dec32(const unsigned char * in, unsigned n, uint32_t * out) { return dec_one(TPF_FMT_32, in, n, out, false, 0); }
const unsigned char * p4D1Dec32(const unsigned char * in, unsigned n, uint32_t * out, uint32_t start)
{
    return dec_one(TPF_FMT_32, in, n, out, true, start);
}

unsigned char * p4Enc128v32(uint32_t * in, unsigned n, unsigned char * out) { return enc_one(TPF_FMT_128V32, in, n, out, false, 0); }
unsigned char * p4D1Enc128v32(uint32_t * in, unsigned n, unsigned char * out, uint32_t start)
{
    return enc_one(TPF_FMT_128V32, in, n, out, true, start);
}
const unsigned char * p4Dec128v32(const unsigned char * in, unsigned n, uint32_t * out)
{
    return dec_one(TPF_FMT_128V32, in, n, out, false, 0);
}
const unsigned char * p4D1Dec128v32(const unsigned char * in, unsigned n, uint32_t * out, uint32_t start)
{
    return dec_one(TPF_FMT_128V32, in, n, out, true, start);
}

unsigned char * p4Enc256v32(uint32_t * in, unsigned n, unsigned char * out) { return enc_one(TPF_FMT_256V32, in, n, out, false, 0); }
unsigned char * p4D1Enc256v32(uint32_t * in, unsigned n, unsigned char * out, uint32_t start)
{
    return enc_one(TPF_FMT_256V32, in, n, out, true, start);
}
const unsigned char * p4Dec256v32(const unsigned char * in, unsigned n, uint32_t * out)
{
    return dec_one(TPF_FMT_256V32, in, n, out, false, 0);
}
const unsigned char * p4D1Dec256v32(const unsigned char * in, unsigned n, uint32_t * out, uint32_t start)
{
    return dec_one(TPF_FMT_256V32, in, n, out, true, start);
}

unsigned char * p4Enc64(uint64_t * in, unsigned n, unsigned char * out) { return enc_one(TPF_FMT_64, in, n, out, false, 0); }
unsigned char * p4D1Enc64(uint64_t * in, unsigned n, unsigned char * out, uint64_t start)
{
    return enc_one(TPF_FMT_64, in, n, out, true, start);
}
const unsigned char * p4Dec64(const unsigned char * in, unsigned n, uint64_t * out) { return dec_one(TPF_FMT_64, in, n, out, false, 0); }
const unsigned char * p4D1Dec64(const unsigned char * in, unsigned n, uint64_t * out, uint64_t start)
{
    return dec_one(TPF_FMT_64, in, n, out, true, start);
}

unsigned char * p4Enc128v64(uint64_t * in, unsigned n, unsigned char * out) { return enc_one(TPF_FMT_128V64, in, n, out, false, 0); }
unsigned char * p4D1Enc128v64(uint64_t * in, unsigned n, unsigned char * out, uint64_t start)
{
    return enc_one(TPF_FMT_128V64, in, n, out, true, start);
}
const unsigned char * p4Dec128v64(const unsigned char * in, unsigned n, uint64_t * out)
{
    return dec_one(TPF_FMT_128V64, in, n, out, false, 0);
}
const unsigned char * p4D1Dec128v64(const unsigned char * in, unsigned n, uint64_t * out, uint64_t start)
{
    return dec_one(TPF_FMT_128V64, in, n, out, true, start);
}

// 256v64 = consecutive 128v64 blocks of min(remaining, 128) values
// (p4enc256v64_scalar.cpp:15-30, p4d1dec256v64_scalar.cpp:15-49): a full
// 256-value unit goes to the paired kernels in one launch, a shorter one as
// its 128v64 blocks (the second starting from value 127 for D1).
unsigned char * p4Enc256v64(uint64_t * in, unsigned n, unsigned char * out)
{
    if (n == 256u || n == 0u)
        return enc_one(TPF_FMT_256V64, in, n, out, false, 0);
    out = enc_one(TPF_FMT_128V64, in, std::min(n, 128u), out, false, 0);
    return n > 128u ? enc_one(TPF_FMT_128V64, in + 128, n - 128u, out, false, 0) : out;
}
unsigned char * p4D1Enc256v64(uint64_t * in, unsigned n, unsigned char * out, uint64_t start)
{
    if (n == 256u || n == 0u)
        return enc_one(TPF_FMT_256V64, in, n, out, true, start);
    out = enc_one(TPF_FMT_128V64, in, std::min(n, 128u), out, true, start);
    return n > 128u ? enc_one(TPF_FMT_128V64, in + 128, n - 128u, out, true, in[127]) : out;
}
const unsigned char * p4Dec256v64(const unsigned char * in, unsigned n, uint64_t * out)
{
    if (n == 256u || n == 0u)
        return dec_one(TPF_FMT_256V64, in, n, out, false, 0);
    in = dec_one(TPF_FMT_128V64, in, std::min(n, 128u), out, false, 0);
    return n > 128u ? dec_one(TPF_FMT_128V64, in, n - 128u, out + 128, false, 0) : in;
}
const unsigned char * p4D1Dec256v64(const unsigned char * in, unsigned n, uint64_t * out, uint64_t start)
{
    if (n == 256u || n == 0u)
        return dec_one(TPF_FMT_256V64, in, n, out, true, start);
    in = dec_one(TPF_FMT_128V64, in, std::min(n, 128u), out, true, start);
    return n > 128u ? dec_one(TPF_FMT_128V64, in, n - 128u, out + 128, true, out[127]) : in;
}
} // namespace turbopfor

// ----------------------------------------------------------- extern "C" mirror
extern "C" {

void tpf_perblock_quiesce(void)
{
    const tpf::PerblockPause p; // nests inside a pause this thread already holds
}

uint64_t tpf_perblock_launches(void) { return g_launches.load(std::memory_order_relaxed); }

int tpf_perblock_mode(int mode)
{
    if (mode < 0)
        return g_mode.load();
    const int m = mode == 1 || mode == 2 ? mode : 0;
    const tpf::PerblockPause p; // no call in flight while the halves switch
    const int old = g_mode.exchange(m);
    if (old != m)
    {
        std::lock_guard<std::mutex> g(g_srv_mu);
        for (Server * s : g_srv)
            if (s)
                s->switch_halves();
    }
    return old;
}

#define TPF_MIRROR_ENC(NAME, T)                                                                                  \
    unsigned char * tpf_##NAME(T * in, unsigned n, unsigned char * out)                                          \
    {                                                                                                            \
        return guarded([&]() -> unsigned char * { return turbopfor::NAME(in, n, out); });                      \
    }
#define TPF_MIRROR_D1ENC(NAME, T)                                                                                \
    unsigned char * tpf_##NAME(T * in, unsigned n, unsigned char * out, T start)                                 \
    {                                                                                                            \
        return guarded([&]() -> unsigned char * { return turbopfor::NAME(in, n, out, start); });               \
    }
#define TPF_MIRROR_DEC(NAME, T)                                                                                  \
    const unsigned char * tpf_##NAME(const unsigned char * in, unsigned n, T * out)                              \
    {                                                                                                            \
        return guarded([&]() -> const unsigned char * { return turbopfor::NAME(in, n, out); });                \
    }
#define TPF_MIRROR_D1DEC(NAME, T)                                                                                \
    const unsigned char * tpf_##NAME(const unsigned char * in, unsigned n, T * out, T start)                     \
    {                                                                                                            \
        return guarded([&]() -> const unsigned char * { return turbopfor::NAME(in, n, out, start); });         \
    }

TPF_MIRROR_ENC(p4Enc32, uint32_t)
TPF_MIRROR_D1ENC(p4D1Enc32, uint32_t)
TPF_MIRROR_DEC(p4Dec32, uint32_t)
TPF_MIRROR_D1DEC(p4D1Dec32, uint32_t)
TPF_MIRROR_ENC(p4Enc128v32, uint32_t)
TPF_MIRROR_D1ENC(p4D1Enc128v32, uint32_t)
TPF_MIRROR_DEC(p4Dec128v32, uint32_t)
TPF_MIRROR_D1DEC(p4D1Dec128v32, uint32_t)
TPF_MIRROR_ENC(p4Enc256v32, uint32_t)
TPF_MIRROR_D1ENC(p4D1Enc256v32, uint32_t)
TPF_MIRROR_DEC(p4Dec256v32, uint32_t)
TPF_MIRROR_D1DEC(p4D1Dec256v32, uint32_t)
TPF_MIRROR_ENC(p4Enc64, uint64_t)
TPF_MIRROR_D1ENC(p4D1Enc64, uint64_t)
TPF_MIRROR_DEC(p4Dec64, uint64_t)
TPF_MIRROR_D1DEC(p4D1Dec64, uint64_t)
TPF_MIRROR_ENC(p4Enc128v64, uint64_t)
TPF_MIRROR_D1ENC(p4D1Enc128v64, uint64_t)
TPF_MIRROR_DEC(p4Dec128v64, uint64_t)
TPF_MIRROR_D1DEC(p4D1Dec128v64, uint64_t)
TPF_MIRROR_ENC(p4Enc256v64, uint64_t)
TPF_MIRROR_D1ENC(p4D1Enc256v64, uint64_t)
TPF_MIRROR_DEC(p4Dec256v64, uint64_t)
TPF_MIRROR_D1DEC(p4D1Dec256v64, uint64_t)

} // extern "C"
