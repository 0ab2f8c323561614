// Host-side sanitizer driver (built with -fsanitize=address,undefined by
// tests/test_sanitize_cpu.py): the CPU code of the library that parses
// untrusted bytes -- stream framing (turbopfor-cpp_amd/csrc/framing.cpp:
// tpf_block_size, tpf_scan_offsets) and the caller-offset check the host
// streams run before any copy (tpf_check_offsets) -- plus the oracle's
// decoders (oracle/tpf_oracle.c, the test-side restatement of the reference),
// fed valid, corrupted and random streams of every format.  Every stream sits
// in a heap buffer of exactly its size, so any read past it is an ASan error.
// The oracle decodes only blocks the framing accepts, from a copy with the
// reference's documented read slack (SURVEY.md §8 b: at most 8 bytes for the
// scalar decoders), and must end exactly where the framing says.
// Reference analogue: src/simd/p4_simd_internal.h:10-19 (MSan unpoison).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/turbopfor_capi.h"
#include "../../include/turbopfor_gpu.h"
#include "../../oracle/tpf_oracle.h"

namespace
{

struct Fmt
{
    int id;
    const char * name;
    unsigned unit; // values per block
    bool wide;
};

// (the oracle restates the five families the GPU tests pin; horizontal 64-bit
// streams are framed by the same code path as 128v64's b > 32 blocks)
const Fmt kFmts[] = {{TPF_FMT_32, "32", 127, false},     {TPF_FMT_128V32, "128v32", 128, false}, {TPF_FMT_256V32, "256v32", 256, false},
                     {TPF_FMT_128V64, "128v64", 128, true}, {TPF_FMT_256V64, "256v64", 256, true}};

uint8_t * enc_one(const Fmt & f, const void * v, uint8_t * out)
{
    switch (f.id)
    {
        case TPF_FMT_32: return orc_p4enc32(static_cast<const uint32_t *>(v), f.unit, out);
        case TPF_FMT_128V32: return orc_p4enc128v32(static_cast<const uint32_t *>(v), f.unit, out);
        case TPF_FMT_256V32: return orc_p4enc256v32(static_cast<const uint32_t *>(v), f.unit, out);
        case TPF_FMT_128V64: return orc_p4enc128v64(static_cast<const uint64_t *>(v), f.unit, out);
        default: return orc_p4enc256v64(static_cast<const uint64_t *>(v), f.unit, out);
    }
}

const uint8_t * dec_one(const Fmt & f, const uint8_t * in, void * out)
{
    switch (f.id)
    {
        case TPF_FMT_32: return orc_p4dec32(in, f.unit, static_cast<uint32_t *>(out));
        case TPF_FMT_128V32: return orc_p4dec128v32(in, f.unit, static_cast<uint32_t *>(out));
        case TPF_FMT_256V32: return orc_p4dec256v32(in, f.unit, static_cast<uint32_t *>(out));
        case TPF_FMT_128V64: return orc_p4dec128v64(in, f.unit, static_cast<uint64_t *>(out));
        default: return orc_p4dec256v64(in, f.unit, static_cast<uint64_t *>(out));
    }
}

int fails = 0;
#define CHECK(c)                                                                                                                 \
    do                                                                                                                           \
    {                                                                                                                            \
        if (!(c))                                                                                                                \
        {                                                                                                                        \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);                                          \
            ++fails;                                                                                                             \
        }                                                                                                                        \
    } while (0)

// Frame a stream of exactly `len` heap bytes; decode every accepted block.
void frame_and_decode(const Fmt & f, const uint8_t * bytes, uint64_t len, uint64_t nblocks, bool valid)
{
    uint8_t * buf = static_cast<uint8_t *>(std::malloc(len ? len : 1));
    std::memcpy(buf, bytes, len);
    std::vector<uint64_t> off(nblocks + 1);
    const int64_t r = tpf_scan_offsets(f.id, buf, len, f.unit, nblocks, off.data());
    if (valid)
        CHECK(r == static_cast<int64_t>(len));
    const uint64_t ok_blocks = r >= 0 ? nblocks : static_cast<uint64_t>(-r - 1);
    CHECK(tpf_check_offsets(off.data(), ok_blocks, len) == 0);
    std::vector<uint64_t> out(512 + 64);
    for (uint64_t i = 0; i < ok_blocks; ++i)
    {
        const uint64_t sz = off[i + 1] - off[i];
        int written = 0;
        CHECK(tpf_block_size(f.id, buf + off[i], len - off[i], f.unit, &written) == sz);
        uint8_t * blk = static_cast<uint8_t *>(std::malloc(sz + 8)); // + the scalar decoders' read slack
        std::memcpy(blk, buf + off[i], sz);
        std::memset(blk + sz, 0, 8);
        const uint8_t * end = dec_one(f, blk, out.data());
        CHECK(end == blk + sz);
        std::free(blk);
    }
    // the framing must also stop cleanly on every truncation of the stream
    for (uint64_t cut = 0; cut < len && cut < 64; ++cut)
    {
        uint8_t * tb = static_cast<uint8_t *>(std::malloc(cut ? cut : 1));
        std::memcpy(tb, buf, cut);
        (void)tpf_scan_offsets(f.id, tb, cut, f.unit, nblocks, off.data());
        std::free(tb);
    }
    std::free(buf);
}

} // namespace

int main(int argc, char ** argv)
{
    const unsigned rounds = argc > 1 ? static_cast<unsigned>(std::atoi(argv[1])) : 40;
    std::mt19937_64 rng(12345);
    uint64_t blocks = 0;
    for (unsigned rd = 0; rd < rounds; ++rd)
    {
        for (const Fmt & f : kFmts)
        {
            const uint64_t nb = 1 + rng() % 40;
            std::vector<uint8_t> stream(nb * (f.unit * 9 + 64) + 64);
            uint8_t * p = stream.data();
            for (uint64_t i = 0; i < nb; ++i)
            {
                const unsigned bw = 1 + rng() % (f.wide ? 64 : 32);
                const unsigned pct = (rng() % 4) * 8;
                std::vector<uint64_t> v(f.unit);
                for (auto & x : v)
                {
                    x = bw >= 64 ? rng() : rng() & ((1ull << bw) - 1);
                    if (rng() % 100 < pct)
                        x = f.wide ? rng() : (rng() & 0xFFFFFFFFull);
                }
                if (rng() % 9 == 0)
                    std::fill(v.begin(), v.end(), v[0]); // constant blocks
                if (f.wide)
                    p = enc_one(f, v.data(), p);
                else
                {
                    std::vector<uint32_t> w(v.begin(), v.end());
                    p = enc_one(f, w.data(), p);
                }
            }
            const uint64_t len = static_cast<uint64_t>(p - stream.data());
            frame_and_decode(f, stream.data(), len, nb, true);
            // corrupted: flip bytes (headers included)
            std::vector<uint8_t> bad(stream.begin(), stream.begin() + len);
            for (int k = 0; k < 1 + static_cast<int>(rng() % 6); ++k)
                bad[rng() % len] ^= static_cast<uint8_t>(1 + rng() % 255);
            frame_and_decode(f, bad.data(), len, nb, false);
            // random bytes
            std::vector<uint8_t> junk(1 + rng() % 3000);
            for (auto & x : junk)
                x = static_cast<uint8_t>(rng());
            frame_and_decode(f, junk.data(), junk.size(), 1 + rng() % 20, false);
            blocks += nb;
        }
        // offset checks on random arrays
        std::vector<uint64_t> off(33);
        for (auto & x : off)
            x = rng() % 5000;
        (void)tpf_check_offsets(off.data(), 32, 4000);
    }
    std::printf("sanitize_framing: %llu blocks, %d failures\n", static_cast<unsigned long long>(blocks), fails);
    return fails ? 1 : 0;
}
