// ref_shim.cpp -- extern "C" wrappers around the REFERENCE library compiled
// from its own sources under /root/reference (oracle/Makefile, target
// `ref`).  TEST INFRASTRUCTURE ONLY: used to generate the golden fixtures
// (oracle/gen_golden.cpp) and as bench.py's cpu_baseline (kind "reference").
// The output library lives in oracle/_ref/ (git-ignored).
//
// Two entry families:
//   tpref_s_*  -> turbopfor::scalar::*   (src/scalar, the bit-exact oracle)
//   tpref_d_*  -> turbopfor::*           (src/dispatch.cpp; AVX2/SSE4.2 paths
//                                         when built with ENABLE_AVX2/SSE42)
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>
#include <chrono>

#include "turbopfor.h"           // /root/reference/include
#include "scalar/p4_scalar.h"    // /root/reference/src

namespace
{
template <class T, class Enc, class D1Enc>
static uint64_t enc_batch(const T * in, uint64_t nb, const T * starts, uint8_t * out, uint64_t * off, Enc enc, D1Enc d1enc)
{
    T tmp[256 + 64];
    uint8_t * p = out;
    for (uint64_t i = 0; i < nb; ++i)
    {
        off[i] = static_cast<uint64_t>(p - out);
        std::memcpy(tmp, in + i * 256u, 256u * sizeof(T));
        p = starts ? d1enc(tmp, 256u, p, starts[i]) : enc(tmp, 256u, p);
    }
    off[nb] = static_cast<uint64_t>(p - out);
    return off[nb];
}

template <class T, class Dec, class D1Dec>
static int64_t dec_batch(const uint8_t * in, const uint64_t * off, uint64_t nb, const T * starts, T * out, Dec dec, D1Dec d1dec)
{
    for (uint64_t i = 0; i < nb; ++i)
    {
        const uint8_t * e = starts ? d1dec(in + off[i], 256u, out + i * 256u, starts[i]) : dec(in + off[i], 256u, out + i * 256u);
        if (e != in + off[i + 1])
            return static_cast<int64_t>(i);
    }
    return -1;
}

} // namespace

extern "C" {

#define W32ENC(name, ns, fn) \
    uint8_t * name(uint32_t * in, unsigned n, uint8_t * out) { return ns::fn(in, n, out); }
#define W32D1ENC(name, ns, fn) \
    uint8_t * name(uint32_t * in, unsigned n, uint8_t * out, uint32_t s) { return ns::fn(in, n, out, s); }
#define W32DEC(name, ns, fn) \
    const uint8_t * name(const uint8_t * in, unsigned n, uint32_t * out) { return ns::fn(in, n, out); }
#define W32D1DEC(name, ns, fn) \
    const uint8_t * name(const uint8_t * in, unsigned n, uint32_t * out, uint32_t s) { return ns::fn(in, n, out, s); }
#define W64ENC(name, ns, fn) \
    uint8_t * name(uint64_t * in, unsigned n, uint8_t * out) { return ns::fn(in, n, out); }
#define W64D1ENC(name, ns, fn) \
    uint8_t * name(uint64_t * in, unsigned n, uint8_t * out, uint64_t s) { return ns::fn(in, n, out, s); }
#define W64DEC(name, ns, fn) \
    const uint8_t * name(const uint8_t * in, unsigned n, uint64_t * out) { return ns::fn(in, n, out); }
#define W64D1DEC(name, ns, fn) \
    const uint8_t * name(const uint8_t * in, unsigned n, uint64_t * out, uint64_t s) { return ns::fn(in, n, out, s); }

#define FAMILY(prefix, ns)                                   \
    W32ENC(prefix##p4enc32, ns, p4Enc32)                     \
    W32D1ENC(prefix##p4d1enc32, ns, p4D1Enc32)               \
    W32DEC(prefix##p4dec32, ns, p4Dec32)                     \
    W32D1DEC(prefix##p4d1dec32, ns, p4D1Dec32)               \
    W32ENC(prefix##p4enc128v32, ns, p4Enc128v32)             \
    W32D1ENC(prefix##p4d1enc128v32, ns, p4D1Enc128v32)       \
    W32DEC(prefix##p4dec128v32, ns, p4Dec128v32)             \
    W32D1DEC(prefix##p4d1dec128v32, ns, p4D1Dec128v32)       \
    W32ENC(prefix##p4enc256v32, ns, p4Enc256v32)             \
    W32D1ENC(prefix##p4d1enc256v32, ns, p4D1Enc256v32)       \
    W32DEC(prefix##p4dec256v32, ns, p4Dec256v32)             \
    W32D1DEC(prefix##p4d1dec256v32, ns, p4D1Dec256v32)       \
    W64ENC(prefix##p4enc128v64, ns, p4Enc128v64)             \
    W64D1ENC(prefix##p4d1enc128v64, ns, p4D1Enc128v64)       \
    W64DEC(prefix##p4dec128v64, ns, p4Dec128v64)             \
    W64D1DEC(prefix##p4d1dec128v64, ns, p4D1Dec128v64)       \
    W64ENC(prefix##p4enc256v64, ns, p4Enc256v64)             \
    W64D1ENC(prefix##p4d1enc256v64, ns, p4D1Enc256v64)       \
    W64DEC(prefix##p4dec256v64, ns, p4Dec256v64)             \
    W64D1DEC(prefix##p4d1dec256v64, ns, p4D1Dec256v64)

FAMILY(tpref_s_, turbopfor::scalar)
FAMILY(tpref_d_, turbopfor)

// Batch round trips through the reference SCALAR path (the parity oracle),
// for tests that pin the C restatement on the bench distributions: block i
// is in[256i..] (D1 when starts != nullptr, starts[i] = the value before the
// block); encodings end to end with off[i] the byte offset of block i.
// Decode returns -1 when every block ends exactly at off[i+1], else the
// first block that does not.
uint64_t tpref_s_enc256v32_batch(const uint32_t * in, uint64_t nb, const uint32_t * starts, uint8_t * out, uint64_t * off)
{
    return enc_batch<uint32_t>(in, nb, starts, out, off, turbopfor::scalar::p4Enc256v32, turbopfor::scalar::p4D1Enc256v32);
}

int64_t tpref_s_dec256v32_batch(const uint8_t * in, const uint64_t * off, uint64_t nb, const uint32_t * starts, uint32_t * out)
{
    return dec_batch<uint32_t>(in, off, nb, starts, out, turbopfor::scalar::p4Dec256v32, turbopfor::scalar::p4D1Dec256v32);
}

uint64_t tpref_s_enc256v64_batch(const uint64_t * in, uint64_t nb, const uint64_t * starts, uint8_t * out, uint64_t * off)
{
    return enc_batch<uint64_t>(in, nb, starts, out, off, turbopfor::scalar::p4Enc256v64, turbopfor::scalar::p4D1Enc256v64);
}

int64_t tpref_s_dec256v64_batch(const uint8_t * in, const uint64_t * off, uint64_t nb, const uint64_t * starts, uint64_t * out)
{
    return dec_batch<uint64_t>(in, off, nb, starts, out, turbopfor::scalar::p4Dec256v64, turbopfor::scalar::p4D1Dec256v64);
}

// Streaming decode of nblocks consecutive 256v32 blocks (block i at
// in+off[i]) on nthreads std::threads, each a contiguous block range.
// use_dispatch=1 -> turbopfor::p4Dec256v32 (AVX2 path), 0 -> scalar.
// Returns wall seconds of the parallel region.
double tpref_dec256v32_stream_mt(const uint8_t * in, const uint64_t * off, uint64_t nblocks, uint32_t * out,
                                 int nthreads, int use_dispatch, int d1)
{
    if (nthreads < 1)
        nthreads = 1;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
    {
        uint64_t lo = nblocks * (uint64_t)t / (uint64_t)nthreads;
        uint64_t hi = nblocks * (uint64_t)(t + 1) / (uint64_t)nthreads;
        th.emplace_back([=] {
            for (uint64_t i = lo; i < hi; ++i)
            {
                uint32_t * o = out + i * 256u;
                if (d1)
                {
                    uint32_t st = i ? 0u : 0u;
                    if (use_dispatch)
                        turbopfor::p4D1Dec256v32(in + off[i], 256u, o, st);
                    else
                        turbopfor::scalar::p4D1Dec256v32(in + off[i], 256u, o, st);
                }
                else if (use_dispatch)
                    turbopfor::p4Dec256v32(in + off[i], 256u, o);
                else
                    turbopfor::scalar::p4Dec256v32(in + off[i], 256u, o);
            }
        });
    }
    for (auto & x : th)
        x.join();
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// Streaming p4D1Dec256v32 of nblocks blocks with their starts, the way a
// posting-list reader calls the reference (README.md:108-123): chained != 0
// takes starts[] only for each thread's first block and carries the previous
// block's last value after that; chained == 0 passes starts[i] per block.
// Returns wall seconds of the parallel region.
double tpref_d1dec256v32_stream_mt(const uint8_t * in, const uint64_t * off, const uint32_t * starts,
                                   uint64_t nblocks, uint32_t * out, int nthreads, int use_dispatch, int chained)
{
    if (nthreads < 1)
        nthreads = 1;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
    {
        uint64_t lo = nblocks * (uint64_t)t / (uint64_t)nthreads;
        uint64_t hi = nblocks * (uint64_t)(t + 1) / (uint64_t)nthreads;
        th.emplace_back([=] {
            for (uint64_t i = lo; i < hi; ++i)
            {
                uint32_t * o = out + i * 256u;
                const uint32_t st = (chained && i > lo) ? o[-1] : starts[i];
                if (use_dispatch)
                    turbopfor::p4D1Dec256v32(in + off[i], 256u, o, st);
                else
                    turbopfor::scalar::p4D1Dec256v32(in + off[i], 256u, o, st);
            }
        });
    }
    for (auto & x : th)
        x.join();
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// The 64-bit posting-list reader: p4D1Dec256v64 over nunits consecutive
// 256v64 units, each thread a contiguous range; chained != 0 takes starts[]
// only for a thread's first unit and carries the previous unit's last value
// (README.md:116-123).  Returns wall seconds of the parallel region.
double tpref_d1dec256v64_stream_mt(const uint8_t * in, const uint64_t * off, const uint64_t * starts, uint64_t nunits, uint64_t * out,
                                   int nthreads, int use_dispatch, int chained)
{
    if (nthreads < 1)
        nthreads = 1;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
    {
        uint64_t lo = nunits * (uint64_t)t / (uint64_t)nthreads;
        uint64_t hi = nunits * (uint64_t)(t + 1) / (uint64_t)nthreads;
        th.emplace_back([=] {
            for (uint64_t i = lo; i < hi; ++i)
            {
                uint64_t * o = out + i * 256u;
                const uint64_t st = (chained && i > lo) ? o[-1] : starts[i];
                if (use_dispatch)
                    turbopfor::p4D1Dec256v64(in + off[i], 256u, o, st);
                else
                    turbopfor::scalar::p4D1Dec256v64(in + off[i], 256u, o, st);
            }
        });
    }
    for (auto & x : th)
        x.join();
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// The posting-list writer: p4D1Enc256v32 over nblocks blocks of one list,
// each thread a contiguous range chained through the returned end pointers
// into its own slice of `scratch` (range x `slot` bytes), block i started
// from starts[i] for a thread's first block and from the previous block's
// last input value after that (README.md:108-123).  off[i] = block i's
// offset in scratch.  Returns wall seconds, or -1 on a bad slot.
double tpref_d1enc256v32_stream_mt(const uint32_t * vals, const uint32_t * starts, uint64_t nblocks, uint8_t * scratch, uint64_t slot,
                                   uint64_t * off, int nthreads, int use_dispatch)
{
    if (nthreads < 1)
        nthreads = 1;
    if (slot < 1040)
        return -1.0;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
    {
        uint64_t lo = nblocks * (uint64_t)t / (uint64_t)nthreads;
        uint64_t hi = nblocks * (uint64_t)(t + 1) / (uint64_t)nthreads;
        th.emplace_back([=] {
            uint8_t * e = scratch + lo * slot;
            for (uint64_t i = lo; i < hi; ++i)
            {
                off[i] = static_cast<uint64_t>(e - scratch);
                uint32_t * in = const_cast<uint32_t *>(vals + i * 256u);
                const uint32_t st = i > lo ? vals[i * 256u - 1u] : starts[i];
                e = use_dispatch ? turbopfor::p4D1Enc256v32(in, 256u, e, st) : turbopfor::scalar::p4D1Enc256v32(in, 256u, e, st);
            }
        });
    }
    for (auto & x : th)
        x.join();
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// Round trip of nblocks blocks of 256 u32 (block i at vals + 256 i): each
// thread encodes its contiguous range with p4Enc256v32, chaining through the
// returned end pointers into its own slice of `scratch` (slice = range x
// `slot` bytes) and noting each block's start in off[i], then decodes the
// blocks back with p4Dec256v32 from off[i] (not through the decoder's end
// pointer: the dispatch path's is wrong for bitmap blocks with >= 32
// exceptions).  `slot` must be >= 1040 (a 256v32 block is
// at most 1 + 32*32 bytes, plus the encoder's 4-byte over-write).  Returns
// wall seconds of the parallel region, or -1 on a bad slot.
double tpref_rt256v32_stream_mt(const uint32_t * vals, uint64_t nblocks, uint8_t * scratch, uint64_t slot,
                                uint64_t * off, uint32_t * out, int nthreads, int use_dispatch)
{
    if (nthreads < 1)
        nthreads = 1;
    if (slot < 1040)
        return -1.0;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
    {
        uint64_t lo = nblocks * (uint64_t)t / (uint64_t)nthreads;
        uint64_t hi = nblocks * (uint64_t)(t + 1) / (uint64_t)nthreads;
        th.emplace_back([=] {
            uint8_t * e = scratch + lo * slot;
            for (uint64_t i = lo; i < hi; ++i)
            {
                off[i] = static_cast<uint64_t>(e - scratch);
                uint32_t * in = const_cast<uint32_t *>(vals + i * 256u);
                e = use_dispatch ? turbopfor::p4Enc256v32(in, 256u, e) : turbopfor::scalar::p4Enc256v32(in, 256u, e);
            }
            for (uint64_t i = lo; i < hi; ++i)
                use_dispatch ? (void)turbopfor::p4Dec256v32(scratch + off[i], 256u, out + i * 256u)
                             : (void)turbopfor::scalar::p4Dec256v32(scratch + off[i], 256u, out + i * 256u);
        });
    }
    for (auto & x : th)
        x.join();
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// ab_test methodology (benchmarks/ab_test.cpp:553-701): one block decoded in
// an L1-hot loop, `iters` iterations per chunk, best of `runs` runs.  Returns
// best seconds per decode call.
double tpref_abtest_dec256v32(const uint8_t * blk, unsigned iters, unsigned runs, int use_dispatch)
{
    alignas(64) uint32_t out[256 + 64];
    volatile uint32_t sink = 0;
    for (unsigned w = 0; w < 1000; ++w)
        use_dispatch ? (void)turbopfor::p4Dec256v32(blk, 256u, out) : (void)turbopfor::scalar::p4Dec256v32(blk, 256u, out);
    double best = 1e30;
    for (unsigned r = 0; r < runs; ++r)
    {
        auto t0 = std::chrono::steady_clock::now();
        for (unsigned i = 0; i < iters; ++i)
        {
            if (use_dispatch)
                turbopfor::p4Dec256v32(blk, 256u, out);
            else
                turbopfor::scalar::p4Dec256v32(blk, 256u, out);
            sink = sink + out[i & 255u];
        }
        auto t1 = std::chrono::steady_clock::now();
        double s = std::chrono::duration<double>(t1 - t0).count() / iters;
        if (s < best)
            best = s;
    }
    return best;
}

// The same methodology for configs[0] of BASELINE.json (C1): p4Enc32 /
// p4Dec32 of one n-value block (ab_test.cpp:1610-1631 uses n = 127, bw 8).
// enc != 0 times the encoder on `vals`, else the decoder on `blk`.  Returns
// best seconds per call.
double tpref_abtest_p4_32(const uint32_t * vals, const uint8_t * blk, unsigned n, unsigned iters, unsigned runs,
                          int use_dispatch, int enc)
{
    alignas(64) uint32_t in[256 + 64];
    alignas(64) uint32_t out[256 + 64];
    alignas(64) uint8_t buf[256 * 5 + 512];
    std::memcpy(in, vals, n * sizeof(uint32_t));
    volatile uint32_t sink = 0;
    auto call = [&](unsigned i) {
        if (enc)
        {
            uint8_t * e = use_dispatch ? turbopfor::p4Enc32(in, n, buf) : turbopfor::scalar::p4Enc32(in, n, buf);
            sink = sink + static_cast<uint32_t>(e - buf) + buf[i & 63u];
        }
        else
        {
            use_dispatch ? (void)turbopfor::p4Dec32(blk, n, out) : (void)turbopfor::scalar::p4Dec32(blk, n, out);
            sink = sink + out[i % n];
        }
    };
    for (unsigned w = 0; w < 1000; ++w)
        call(w);
    double best = 1e30;
    for (unsigned r = 0; r < runs; ++r)
    {
        auto t0 = std::chrono::steady_clock::now();
        for (unsigned i = 0; i < iters; ++i)
            call(i);
        auto t1 = std::chrono::steady_clock::now();
        const double sec = std::chrono::duration<double>(t1 - t0).count() / iters;
        if (sec < best)
            best = sec;
    }
    return best;
}

} // extern "C"
