// dropin_example.cpp -- a reference-style caller of include/turbopfor.h,
// written the way the reference's README (README.md:92-127) and tests chain
// blocks: encode a sorted posting list block by block with p4D1Enc256v32,
// passing the previous block's last value as `start`, then decode it back
// through the returned end pointers.  Built against libturbopfor_amd.so with
// nothing but the header; exits non-zero on any mismatch.
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

#include "turbopfor.h"

int main()
{
    const size_t nblocks = 64, n = 256;
    std::vector<uint32_t> docs(nblocks * n);
    uint32_t cur = 17;
    uint64_t x = 88172645463325252ull;
    for (auto & d : docs)
    {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        cur += 1 + static_cast<uint32_t>(x % ((x >> 32) % 8 == 0 ? 70000 : 40));
        d = cur;
    }
    std::vector<unsigned char> buf(nblocks * (n * 4 + 1024));
    unsigned char * op = buf.data();
    uint32_t start = 0;
    for (size_t b = 0; b < nblocks; ++b)
    {
        op = turbopfor::p4D1Enc256v32(&docs[b * n], n, op, start);
        start = docs[b * n + n - 1];
    }
    const size_t total = op - buf.data();
    std::vector<uint32_t> back(nblocks * n);
    const unsigned char * ip = buf.data();
    start = 0;
    for (size_t b = 0; b < nblocks; ++b)
    {
        ip = turbopfor::p4D1Dec256v32(ip, n, &back[b * n], start);
        start = back[b * n + n - 1];
    }
    if (static_cast<size_t>(ip - buf.data()) != total || std::memcmp(back.data(), docs.data(), docs.size() * 4) != 0)
    {
        std::printf("MISMATCH\n");
        return 1;
    }
    // 64-bit and horizontal families round trip too
    std::vector<uint64_t> v64(256), r64(256);
    for (size_t i = 0; i < 256; ++i)
        v64[i] = (uint64_t(i) * 0x9E3779B97F4A7C15ull) >> (i % 40);
    std::vector<unsigned char> b64(256 * 10 + 1024);
    unsigned char * e64 = turbopfor::p4Enc256v64(v64.data(), 256, b64.data());
    const unsigned char * d64 = turbopfor::p4Dec256v64(b64.data(), 256, r64.data());
    std::vector<uint32_t> v32(127), r32(127);
    for (size_t i = 0; i < 127; ++i)
        v32[i] = static_cast<uint32_t>((i * 37) & 255);
    std::vector<unsigned char> b32(127 * 5 + 64);
    unsigned char * e32 = turbopfor::p4Enc32(v32.data(), 127, b32.data());
    const unsigned char * d32 = turbopfor::p4Dec32(b32.data(), 127, r32.data());
    if (d64 != e64 || r64 != v64 || d32 != e32 || r32 != v32)
    {
        std::printf("MISMATCH 64/32\n");
        return 1;
    }
    std::printf("ok: %zu blocks, %zu bytes (%.2f B/int); 256v64 %td B; p4Enc32(n=127) %td B\n", nblocks, total,
                double(total) / double(docs.size()), e64 - b64.data(), e32 - b32.data());
    return 0;
}
