// framing.cpp -- host-side P4 stream framing: the encoded byte length of one
// block from its header, without decoding any value.  The reference has no
// offsets (callers chain blocks through the returned end pointer,
// README.md:108-123), so this is what turns a legacy stream into the
// (bytes, offsets) pair the batched GPU decoders take, and
// what the per-block drop-in decoders use to copy exactly one block to HBM.
//
// Length rules (reference decoders):
//   constant  (h&0xC0)==0xC0: 1 + ceil(b/8)                 p4dec256v32_scalar.cpp:100-112
//   plain     (h&0xC0)==0   : 1 + base(b)                   p4dec256v32_scalar.cpp:114-121
//   bitmap    h&0x80, bx    : 2 + pad8(n) + pad8(xn*bx) + base(b)   :10-66
//   vbyte     (h&0xC0)==0x40: 2 + base(b) + |V| + xn        :123-136, vbDec32 p4_scalar_internal.cpp:215-237
//   64-bit: header b == 63 means 64 (p4d1dec128v64_scalar.cpp:190-200)
#include <cstdint>
#include <cstring>

#include "../../include/turbopfor_capi.h"
#include "../../include/turbopfor_gpu.h"

namespace
{

inline uint32_t pad8(uint32_t bits) { return (bits + 7u) / 8u; }

uint32_t base_bytes(int fmt, uint32_t n, uint32_t b)
{
    switch (fmt)
    {
        case TPF_FMT_256V32:
            return 32u * b;
        case TPF_FMT_128V32:
        case TPF_FMT_128V64:
            return 16u * b;
        default:
            return pad8(n * b);
    }
}

bool is_wide(int fmt) { return fmt == TPF_FMT_64 || fmt == TPF_FMT_128V64 || fmt == TPF_FMT_256V64; }

// One block (for 256v64: one 128v64 half).  Returns 0 on malformed / truncated input.
uint64_t one_block(int fmt, const uint8_t * in, uint64_t avail, uint32_t n, int * constant)
{
    if (avail < 1)
        return 0;
    const bool wide = is_wide(fmt);
    const uint32_t W = wide ? 64u : 32u;
    const uint32_t h = in[0];
    *constant = 0;
    if ((h & 0xC0u) == 0xC0u)
    {
        uint32_t b = h & 0x3Fu;
        if (wide && b == 63u)
            b = 64u;
        if (fmt == TPF_FMT_32 && b > 32u) // more than 4 value bytes: undefined in the reference (p4dec32.cpp:100-116)
            return 0;
        *constant = 1;
        const uint64_t sz = 1u + (b + 7u) / 8u;
        return sz <= avail ? sz : 0;
    }
    if ((h & 0x40u) == 0u)
    {
        uint32_t bx = 0, hdr = 1, b = h & 0x7Fu;
        if (h & 0x80u)
        {
            if (avail < 2)
                return 0;
            bx = in[1];
            hdr = 2;
        }
        if (wide && b == 63u)
            b = 64u;
        if (b > W || bx > W)
            return 0;
        if (bx == 0u)
        {
            const uint64_t sz = hdr + base_bytes(fmt, n, b);
            return sz <= avail ? sz : 0;
        }
        const uint32_t bm_bytes = pad8(n);
        if (avail < 2u + bm_bytes)
            return 0;
        uint32_t xn = 0;
        for (uint32_t i = 0; i < n; ++i)
            xn += (in[2 + (i >> 3)] >> (i & 7u)) & 1u;
        const uint64_t sz = 2u + bm_bytes + pad8(xn * bx) + base_bytes(fmt, n, b);
        return sz <= avail ? sz : 0;
    }
    uint32_t b = h & 0x3Fu;
    if (wide && b == 63u)
        b = 64u;
    if (b > W || avail < 2) // a 32-bit vbyte block wider than 32 bits: the reference's unpack is undefined there
        return 0;
    const uint32_t xn = in[1];
    uint64_t p = 2u + base_bytes(fmt, n, b);
    if (p >= avail)
        return 0; // V always has at least one byte (0xFF escape when xn == 0)
    if (in[p] == 0xFFu)
        p += 1u + (wide ? 8u : 4u) * xn;
    else
    {
        for (uint32_t k = 0; k < xn; ++k)
        {
            if (p >= avail)
                return 0;
            const uint32_t m = in[p];
            uint32_t len;
            if (!wide)
                len = m < 0x9Cu ? 1u : m < 0xDCu ? 2u : m < 0xFCu ? 3u : m == 0xFCu ? 4u : 5u;
            else
                len = m < 0x98u ? 1u : m < 0xD8u ? 2u : m < 0xF8u ? 3u : (m - 0xF8u + 4u);
            p += len;
        }
    }
    p += xn;
    return p <= avail ? p : 0;
}

} // namespace

extern "C" {

uint64_t tpf_block_size(int fmt, const uint8_t * in, uint64_t avail, unsigned n, int * values_written)
{
    int cst = 0;
    if (!in || n == 0)
        return 0;
    if (fmt == TPF_FMT_256V64)
    {
        // consecutive 128v64 blocks of min(remaining, 128) values (p4dec256v64_scalar.cpp:37-51);
        // a non-constant block writes all 128 slots, a constant one its n values
        const unsigned n0 = n < 128u ? n : 128u;
        int c1 = 0;
        const uint64_t a = one_block(TPF_FMT_128V64, in, avail, n0, &cst);
        if (!a)
            return 0;
        uint64_t b = 0;
        if (n > 128u && !(b = one_block(TPF_FMT_128V64, in + a, avail - a, n - 128u, &c1)))
            return 0;
        if (values_written)
            *values_written = n > 128u ? static_cast<int>(128u + (c1 ? n - 128u : 128u)) : static_cast<int>(cst ? n : 128u);
        return a + b;
    }
    const uint64_t sz = one_block(fmt, in, avail, n, &cst);
    if (values_written)
    {
        uint32_t full = n;
        if (fmt == TPF_FMT_256V32)
            full = 256;
        else if (fmt == TPF_FMT_128V32 || fmt == TPF_FMT_128V64)
            full = 128;
        *values_written = static_cast<int>(cst ? n : full);
    }
    return sz;
}

int64_t tpf_check_offsets(const uint64_t * off, uint64_t nblocks, uint64_t in_bytes)
{
    if (!off)
        return -1;
    for (uint64_t i = 0; i < nblocks; ++i)
        if (off[i] > off[i + 1])
            return -static_cast<int64_t>(i) - 1;
    if (off[nblocks] > in_bytes)
        return -static_cast<int64_t>(nblocks) - 1;
    return 0;
}

int64_t tpf_scan_offsets(int fmt, const uint8_t * in, uint64_t in_bytes, unsigned n, uint64_t nblocks, uint64_t * off)
{
    uint64_t pos = 0;
    for (uint64_t i = 0; i < nblocks; ++i)
    {
        off[i] = pos;
        const uint64_t sz = tpf_block_size(fmt, in + pos, in_bytes - pos, n, nullptr);
        if (sz == 0)
            return -static_cast<int64_t>(i) - 1;
        pos += sz;
    }
    off[nblocks] = pos;
    return static_cast<int64_t>(pos);
}

} // extern "C"
