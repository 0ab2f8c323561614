// gen_golden.cpp -- generates tests/golden/*.bin from the REFERENCE scalar
// codec (turbopfor::scalar::*, compiled from /root/reference/src by
// oracle/Makefile target `ref`).  Test infrastructure only.
//
// Inputs are produced by our own splitmix64 generator and STORED in the
// fixtures (std::uniform_int_distribution is implementation-defined, so the
// reference tests' seeds would not reproduce).  Patterns follow the
// reference tests: tests/test_helpers.h:90-155 (sequential, random, constant,
// fillWithExceptions), tests/test_p4dec_32.cpp:248-264, tests/test_d1enc.cpp:154
// (sorted, maxDelta 1/15/255/65535), tests/test_p4_64.cpp:587-611 (64-bit bit
// widths, 32/64-bit exceptions, 63->64 quirk) and benchmarks/ab_test.cpp:1610-1631
// (exception distribution).
//
// File format (little endian):
//   "TPFG" u32 version(1) u32 count
//   record: u32 flags  (bit0 = delta-1, bit1 = decode-only vector)
//           u32 n      (values per call)
//           u64 start  (delta-1 start)
//           u32 esize  (4 or 8)
//           u32 enc_len
//           u8  values[n*esize]   (encoder input == expected decoder output)
//           u8  enc[enc_len]      (expected encoder output / decoder input)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>
#include <cmath>

#include "turbopfor.h"
#include "scalar/p4_scalar.h"

namespace sc = turbopfor::scalar;

struct Rng
{
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) { }
    uint64_t next()
    {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint64_t range(uint64_t lo, uint64_t hi) // inclusive
    {
        uint64_t span = hi - lo + 1u;
        if (span == 0u)
            return next();
        return lo + next() % span;
    }
    double unit() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

struct Writer
{
    std::vector<uint8_t> buf;
    uint32_t count = 0;
    void put(const void * p, size_t n)
    {
        const uint8_t * b = static_cast<const uint8_t *>(p);
        buf.insert(buf.end(), b, b + n);
    }
    template <class T>
    void put(T v) { put(&v, sizeof(T)); }
    void record(uint32_t flags, uint32_t n, uint64_t start, uint32_t esize, const void * vals, const uint8_t * enc, uint32_t enc_len)
    {
        put(flags);
        put(n);
        put(start);
        put(esize);
        put(enc_len);
        put(vals, size_t(n) * esize);
        put(enc, enc_len);
        ++count;
    }
    void save(const std::string & path)
    {
        FILE * f = std::fopen(path.c_str(), "wb");
        if (!f)
        {
            std::perror(path.c_str());
            std::exit(1);
        }
        std::fwrite("TPFG", 1, 4, f);
        uint32_t ver = 1;
        std::fwrite(&ver, 4, 1, f);
        std::fwrite(&count, 4, 1, f);
        std::fwrite(buf.data(), 1, buf.size(), f);
        std::fclose(f);
        std::printf("%s: %u records, %zu bytes\n", path.c_str(), count, buf.size() + 12);
    }
};

static void die(const char * what, unsigned idx)
{
    std::fprintf(stderr, "reference self-check failed: %s (case %u)\n", what, idx);
    std::exit(2);
}

// ---------------------------------------------------------------- 32-bit
enum Fmt32
{
    F256V32,
    F128V32,
    FH32
};

static unsigned blockN(Fmt32 f, unsigned n) { return f == F256V32 ? 256u : f == F128V32 ? 128u : n; }

static void add32(Writer & w, Fmt32 f, std::vector<uint32_t> v, bool d1, uint32_t start)
{
    unsigned n = static_cast<unsigned>(v.size());
    std::vector<uint8_t> enc(n * 5 + 4096, 0);
    std::vector<uint32_t> in(std::max<size_t>(v.size(), 256) + 64, 0);
    std::copy(v.begin(), v.end(), in.begin());
    uint8_t * e = nullptr;
    if (f == F256V32)
        e = d1 ? sc::p4D1Enc256v32(in.data(), n, enc.data(), start) : sc::p4Enc256v32(in.data(), n, enc.data());
    else if (f == F128V32)
        e = d1 ? sc::p4D1Enc128v32(in.data(), n, enc.data(), start) : sc::p4Enc128v32(in.data(), n, enc.data());
    else
        e = d1 ? sc::p4D1Enc32(in.data(), n, enc.data(), start) : sc::p4Enc32(in.data(), n, enc.data());
    uint32_t len = static_cast<uint32_t>(e - enc.data());
    std::vector<uint32_t> dec(512 + 64, 0xDEADBEEFu);
    const uint8_t * r = nullptr;
    if (f == F256V32)
        r = d1 ? sc::p4D1Dec256v32(enc.data(), n, dec.data(), start) : sc::p4Dec256v32(enc.data(), n, dec.data());
    else if (f == F128V32)
        r = d1 ? sc::p4D1Dec128v32(enc.data(), n, dec.data(), start) : sc::p4Dec128v32(enc.data(), n, dec.data());
    else
        r = d1 ? sc::p4D1Dec32(enc.data(), n, dec.data(), start) : sc::p4Dec32(enc.data(), n, dec.data());
    if (r != e)
        die("decode end pointer", w.count);
    if (std::memcmp(dec.data(), v.data(), n * 4u) != 0)
        die("round trip", w.count);
    w.record(d1 ? 1u : 0u, n, start, 4u, v.data(), enc.data(), len);
}

static std::vector<uint32_t> sortedSeq(Rng & r, unsigned n, uint32_t max_delta, uint32_t & start_out)
{
    std::vector<uint32_t> v(n);
    uint32_t cur = static_cast<uint32_t>(r.range(0, 1000));
    start_out = cur;
    for (unsigned i = 0; i < n; ++i)
    {
        cur += static_cast<uint32_t>(r.range(1, max_delta));
        v[i] = cur;
    }
    return v;
}

// Zipf-ish posting-list gaps: 95% gaps from a bounded
// continuous Zipf(s=1.1) on [1,64], 5% gaps 64+U[0,2^16).
static uint32_t zipfGap(Rng & r)
{
    if (r.unit() < 0.05)
        return 64u + static_cast<uint32_t>(r.range(0, 65535));
    const double s = 1.1, a = 1.0, b = 65.0;
    double u = r.unit();
    double x = std::pow(std::pow(a, 1 - s) + u * (std::pow(b, 1 - s) - std::pow(a, 1 - s)), 1.0 / (1 - s));
    uint32_t g = static_cast<uint32_t>(std::floor(x));
    return g < 1u ? 1u : (g > 64u ? 64u : g);
}

static void gen32(Writer & w, Fmt32 f, uint64_t seed)
{
    Rng r(seed);
    std::vector<unsigned> ns;
    if (f == FH32)
        ns = {1, 2, 3, 5, 7, 8, 31, 32, 33, 63, 64, 65, 100, 127, 128, 129, 200, 255, 256};
    else
        ns = {blockN(f, 0)};
    for (unsigned n : ns)
    {
        std::vector<uint32_t> v(n);
        // sequential / zeros / constant 42 (test_p4dec_32.cpp:248-264)
        for (unsigned i = 0; i < n; ++i)
            v[i] = 1000u + i * 3u;
        add32(w, f, v, false, 0);
        std::fill(v.begin(), v.end(), 0u);
        add32(w, f, v, false, 0);
        std::fill(v.begin(), v.end(), 42u);
        add32(w, f, v, false, 0);
        // constant blocks of every bit width (constant payload = ceil(b/8) bytes)
        for (unsigned b = 1; b <= 32; b += (f == FH32 && n != 127 ? 7 : 1))
        {
            uint32_t c = (b == 32) ? 0xF0000001u : ((1u << (b - 1)) | static_cast<uint32_t>(r.range(0, (1u << (b - 1)) - 1)));
            std::fill(v.begin(), v.end(), c);
            add32(w, f, v, false, 0);
        }
        // random, every bit width
        unsigned reps = (f == FH32 && n != 127) ? 1u : 2u;
        for (unsigned b = 1; b <= 32; ++b)
            for (unsigned rep = 0; rep < reps; ++rep)
            {
                uint32_t mx = b == 32 ? 0xFFFFFFFFu : ((1u << b) - 1u);
                for (auto & x : v)
                    x = static_cast<uint32_t>(r.range(0, mx));
                add32(w, f, v, false, 0);
            }
        // fillWithExceptions(255, 100000, pct) (test_helpers.h:109-121)
        for (unsigned pct : {1u, 5u, 10u, 25u, 50u})
        {
            for (auto & x : v)
                x = (r.range(0, 99) < pct) ? 100000u : static_cast<uint32_t>(r.range(0, 255));
            add32(w, f, v, false, 0);
        }
        // ab_test distribution (ab_test.cpp:1610-1631): base U[0,2^bw), exc U[2^bw, 2^32)
        for (unsigned bw = 1; bw <= 28; bw += (f == FH32 && n != 127 ? 5 : 1))
            for (double pct : {0.0, 5.0, 10.0, 25.0})
            {
                for (auto & x : v)
                    x = (r.unit() * 100.0 < pct) ? static_cast<uint32_t>(r.range(1ull << bw, 0xFFFFFFFFull))
                                                 : static_cast<uint32_t>(r.range(0, (1ull << bw) - 1));
                add32(w, f, v, false, 0);
            }
        // mostly zero with a few large values (b = 0 with patches / vbyte at b = 0)
        for (unsigned k : {1u, 2u, 3u, 8u, 40u})
        {
            std::fill(v.begin(), v.end(), 0u);
            for (unsigned j = 0; j < k && j < n; ++j)
                v[r.range(0, n - 1)] = static_cast<uint32_t>(r.range(1, 0xFFFFFFFFull));
            add32(w, f, v, false, 0);
        }
        // small values + moderately sized exceptions: vbyte compressed vs raw escape
        for (unsigned k : {4u, 12u, 20u, 30u, 60u, 100u})
            for (uint32_t emax : {300u, 20000u, 3000000u, 0x7FFFFFFu})
            {
                for (auto & x : v)
                    x = static_cast<uint32_t>(r.range(0, 15));
                for (unsigned j = 0; j < k && j < n; ++j)
                    v[r.range(0, n - 1)] = static_cast<uint32_t>(r.range(16, emax));
                add32(w, f, v, false, 0);
            }
        // delta-1: sorted inputs (test_d1enc.cpp:154)
        for (uint32_t md : {1u, 15u, 255u, 65535u})
        {
            uint32_t st;
            auto s = sortedSeq(r, n, md, st);
            add32(w, f, s, true, st);
        }
        {
            // wrap-around start
            uint32_t st = 0xFFFFFF00u, cur = st;
            for (auto & x : v)
                x = (cur += static_cast<uint32_t>(r.range(1, 9)));
            add32(w, f, v, true, st);
        }
        for (unsigned rep = 0; rep < 6; ++rep)
        {
            uint32_t cur = static_cast<uint32_t>(r.range(0, 1u << 20)), st = cur;
            for (auto & x : v)
                x = (cur += zipfGap(r));
            add32(w, f, v, true, st);
        }
    }
}

// ---------------------------------------------------------------- 64-bit
static void add64(Writer & w, std::vector<uint64_t> v, bool d1, uint64_t start, bool v128)
{
    unsigned n = static_cast<unsigned>(v.size());
    std::vector<uint8_t> enc(n * 10 + 4096, 0);
    std::vector<uint64_t> in(256 + 64, 0);
    std::copy(v.begin(), v.end(), in.begin());
    uint8_t * e = v128 ? (d1 ? sc::p4D1Enc128v64(in.data(), n, enc.data(), start) : sc::p4Enc128v64(in.data(), n, enc.data()))
                       : (d1 ? sc::p4D1Enc256v64(in.data(), n, enc.data(), start) : sc::p4Enc256v64(in.data(), n, enc.data()));
    uint32_t len = static_cast<uint32_t>(e - enc.data());
    std::vector<uint64_t> dec(256 + 64, 0);
    const uint8_t * rp = v128 ? (d1 ? sc::p4D1Dec128v64(enc.data(), n, dec.data(), start) : sc::p4Dec128v64(enc.data(), n, dec.data()))
                              : (d1 ? sc::p4D1Dec256v64(enc.data(), n, dec.data(), start) : sc::p4Dec256v64(enc.data(), n, dec.data()));
    if (rp != e)
        die("64 decode end pointer", w.count);
    if (std::memcmp(dec.data(), v.data(), n * 8u) != 0)
        die("64 round trip", w.count);
    w.record(d1 ? 1u : 0u, n, start, 8u, v.data(), enc.data(), len);
}

static void gen64(Writer & w, uint64_t seed, bool v128)
{
    Rng r(seed);
    const unsigned n = v128 ? 128u : 256u;
    std::vector<uint64_t> v(n);
    for (unsigned i = 0; i < n; ++i)
        v[i] = 1000000ull + i * 7ull;
    add64(w, v, false, 0, v128);
    std::fill(v.begin(), v.end(), 0ull);
    add64(w, v, false, 0, v128);
    for (unsigned b : {1u, 8u, 31u, 32u, 33u, 40u, 56u, 63u, 64u})
    {
        uint64_t c = (b == 64) ? 0xF000000000000001ull : ((1ull << (b - 1)) | 1ull);
        std::fill(v.begin(), v.end(), c);
        add64(w, v, false, 0, v128);
    }
    // bit widths of test_p4_64.cpp:587-611
    for (unsigned b : {1u, 2u, 4u, 8u, 16u, 24u, 31u, 32u, 33u, 40u, 48u, 56u, 62u, 63u, 64u})
        for (unsigned rep = 0; rep < 3; ++rep)
        {
            uint64_t mx = b == 64 ? ~0ull : ((1ull << b) - 1ull);
            for (auto & x : v)
                x = r.range(0, mx);
            add64(w, v, false, 0, v128);
        }
    // exceptions above bit 32 and at bit 63/64
    for (unsigned bw : {4u, 8u, 16u, 20u, 31u, 32u, 40u})
        for (unsigned pct : {1u, 5u, 10u, 25u})
            for (unsigned hi : {33u, 48u, 63u, 64u})
            {
                for (auto & x : v)
                    x = (r.range(0, 99) < pct) ? r.range(1ull << (hi - 1), hi == 64 ? ~0ull : ((1ull << hi) - 1ull))
                                               : r.range(0, (1ull << bw) - 1ull);
                add64(w, v, false, 0, v128);
            }
    // vbyte-friendly: small base + a few moderately sized exceptions
    for (unsigned k : {3u, 10u, 20u, 40u})
        for (uint64_t emax : {300ull, 20000ull, 3000000ull, (1ull << 40), ~0ull})
        {
            for (auto & x : v)
                x = r.range(0, 15);
            for (unsigned j = 0; j < k; ++j)
                v[r.range(0, n - 1)] = r.range(16, emax);
            add64(w, v, false, 0, v128);
        }
    // 63->64 quirk: values whose width is exactly 63
    for (unsigned rep = 0; rep < 4; ++rep)
    {
        for (auto & x : v)
            x = r.range(1ull << 62, (1ull << 63) - 1ull);
        add64(w, v, false, 0, v128);
        for (auto & x : v)
            x = r.range(0, (1ull << 62) - 1ull);
        v[r.range(0, n - 1)] = (1ull << 62) | 5ull; // max width 63 with few at top
        add64(w, v, false, 0, v128);
    }
    // delta-1 (test_d1enc.cpp:300-339)
    for (uint64_t md : {1ull, 15ull, 255ull, 65535ull, (1ull << 40)})
        for (unsigned rep = 0; rep < 2; ++rep)
        {
            uint64_t cur = r.range(0, 100000), st = cur;
            for (auto & x : v)
                x = (cur += r.range(1, md));
            add64(w, v, true, st, v128);
        }
    {
        // 32-bit prefix overflow inside a 128 chunk (the simd::p4D1Dec256v64 bug of SURVEY a10)
        uint64_t cur = 0xFFFFF000ull, st = cur;
        for (auto & x : v)
            x = (cur += r.range(1 << 17, 1 << 22));
        add64(w, v, true, st, v128);
    }
}

// n below the layout width (128v64 n < 128, 256v64 n < 256).  The reference
// leaves the base slots past n of an exception block, and the delta slots
// past n of a D1 block, uninitialised (p4enc128v64_scalar.cpp:59,
// p4d1enc256v64_scalar.cpp:12): those payload bits are whatever its stack
// held.  Each vector is encoded after zero-filling the stack (the convention
// the oracle and the GPU path implement: padding slots are 0) and again after
// filling it with 0xA5; where the two differ the record carries flag 4
// ("padding bits follow the zero convention, not pinned by the reference").
__attribute__((noinline)) static void fill_stack(uint8_t v)
{
    volatile uint8_t junk[1 << 16];
    for (size_t i = 0; i < sizeof(junk); ++i)
        junk[i] = v;
    asm volatile("" ::"r"(junk) : "memory");
}

// p4Enc256v64 is a loop of p4Enc128v64 over 128-value chunks
// (p4enc256v64_scalar.cpp:15-30), so with `chunked` the 256v64 encoding is
// made chunk by chunk with the stack refilled before each call (the direct
// call's second chunk would see the first chunk's stale stack instead).
static uint32_t enc64_ref(const std::vector<uint64_t> & in, unsigned n, bool d1, uint64_t start, bool v128, uint8_t fill,
                          std::vector<uint8_t> & enc, bool chunked)
{
    std::vector<uint64_t> buf(in);
    std::fill(enc.begin(), enc.end(), 0);
    if (v128 || !chunked)
    {
        fill_stack(fill);
        uint8_t * e = v128 ? (d1 ? sc::p4D1Enc128v64(buf.data(), n, enc.data(), start) : sc::p4Enc128v64(buf.data(), n, enc.data()))
                           : (d1 ? sc::p4D1Enc256v64(buf.data(), n, enc.data(), start) : sc::p4Enc256v64(buf.data(), n, enc.data()));
        return static_cast<uint32_t>(e - enc.data());
    }
    uint8_t * e = enc.data();
    for (unsigned c0 = 0; c0 < n; c0 += 128u)
    {
        const unsigned c = std::min(n - c0, 128u);
        fill_stack(fill);
        e = d1 ? sc::p4D1Enc128v64(buf.data() + c0, c, e, c0 ? buf[c0 - 1] : start) : sc::p4Enc128v64(buf.data() + c0, c, e);
    }
    return static_cast<uint32_t>(e - enc.data());
}

static void add64_short(Writer & w, std::vector<uint64_t> v, bool d1, uint64_t start, bool v128)
{
    const unsigned n = static_cast<unsigned>(v.size());
    std::vector<uint64_t> in(256 + 64, 0);
    std::copy(v.begin(), v.end(), in.begin());
    std::vector<uint8_t> e0(n * 10 + 4096), e1(n * 10 + 4096), ed(n * 10 + 4096);
    const uint32_t len0 = enc64_ref(in, n, d1, start, v128, 0x00, e0, true);
    const uint32_t len1 = enc64_ref(in, n, d1, start, v128, 0xA5, e1, true);
    const uint32_t lend = enc64_ref(in, n, d1, start, v128, 0x00, ed, false);
    if (len0 != len1 || len0 != lend)
        die("64 short: length depends on stack contents", w.count);
    const bool unpinned = std::memcmp(e0.data(), e1.data(), len0) != 0 || std::memcmp(e0.data(), ed.data(), len0) != 0;
    std::vector<uint64_t> dec(256 + 64, 0);
    const uint8_t * rp = v128 ? (d1 ? sc::p4D1Dec128v64(e0.data(), n, dec.data(), start) : sc::p4Dec128v64(e0.data(), n, dec.data()))
                              : (d1 ? sc::p4D1Dec256v64(e0.data(), n, dec.data(), start) : sc::p4Dec256v64(e0.data(), n, dec.data()));
    if (rp != e0.data() + len0)
        die("64 short decode end pointer", w.count);
    if (std::memcmp(dec.data(), v.data(), n * 8u) != 0)
        die("64 short round trip", w.count);
    w.record((d1 ? 1u : 0u) | (unpinned ? 4u : 0u), n, start, 8u, v.data(), e0.data(), len0);
}

static void gen64_short(Writer & w, uint64_t seed, bool v128)
{
    Rng r(seed);
    const std::vector<unsigned> ns = v128 ? std::vector<unsigned>{1u, 7u, 64u, 100u, 127u}
                                          : std::vector<unsigned>{1u, 100u, 128u, 129u, 200u, 255u};
    for (unsigned n : ns)
    {
        std::vector<uint64_t> v(n);
        std::fill(v.begin(), v.end(), 0ull);
        add64_short(w, v, false, 0, v128);
        std::fill(v.begin(), v.end(), 0x123456789ull);
        add64_short(w, v, false, 0, v128); // constant
        for (unsigned b : {8u, 40u})
        {
            for (auto & x : v)
                x = r.range(0, (1ull << b) - 1ull);
            add64_short(w, v, false, 0, v128); // plain (or patched by chance)
        }
        for (unsigned pct : {10u, 30u})
            for (unsigned hi : {33u, 64u})
            {
                for (auto & x : v)
                    x = (r.range(0, 99) < pct) ? r.range(1ull << (hi - 1), hi == 64 ? ~0ull : ((1ull << hi) - 1ull)) : r.range(0, 255);
                add64_short(w, v, false, 0, v128); // bitmap or vbyte exceptions
            }
        for (auto & x : v)
            x = r.range(0, 15);
        v[r.range(0, n - 1)] = r.range(1u << 20, 1u << 30);
        add64_short(w, v, false, 0, v128); // one exception: vbyte
        for (uint64_t md : {1ull, 255ull, (1ull << 40)})
        {
            uint64_t cur = r.range(0, 100000), st = cur;
            for (auto & x : v)
                x = (cur += r.range(1, md));
            add64_short(w, v, true, st, v128);
        }
    }
}

// Hand-made decode-only vectors: valid streams the encoder never emits.
static void genDecodeOnly(Writer & w)
{
    // header 0x88, bx = 0: "bitmap says no exceptions" (p4dec256v32_scalar.cpp:80-83)
    Rng r(7);
    std::vector<uint8_t> enc(2 + 256 + 64, 0);
    enc[0] = 0x80 | 8;
    enc[1] = 0;
    for (unsigned i = 0; i < 256; ++i)
        enc[2 + i] = static_cast<uint8_t>(r.next());
    std::vector<uint32_t> dec(256 + 64);
    const uint8_t * e = sc::p4Dec256v32(enc.data(), 256, dec.data());
    w.record(2u, 256, 0, 4u, dec.data(), enc.data(), static_cast<uint32_t>(e - enc.data()));
    const uint8_t * e1 = sc::p4D1Dec256v32(enc.data(), 256, dec.data(), 12345u);
    w.record(3u, 256, 12345u, 4u, dec.data(), enc.data(), static_cast<uint32_t>(e1 - enc.data()));
}

int main(int argc, char ** argv)
{
    std::string dir = argc > 1 ? argv[1] : "../tests/golden";
    {
        Writer w;
        gen32(w, F256V32, 0x256032);
        genDecodeOnly(w);
        w.save(dir + "/g256v32.bin");
    }
    {
        Writer w;
        gen32(w, F128V32, 0x128032);
        w.save(dir + "/g128v32.bin");
    }
    {
        Writer w;
        gen32(w, FH32, 0x32);
        w.save(dir + "/g32.bin");
    }
    {
        Writer w;
        gen64(w, 0x256064, false);
        gen64_short(w, 0x256065, false);
        w.save(dir + "/g256v64.bin");
    }
    {
        Writer w;
        gen64(w, 0x128064, true);
        gen64_short(w, 0x128065, true);
        w.save(dir + "/g128v64.bin");
    }
    return 0;
}
