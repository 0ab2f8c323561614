/*
 * tpf_oracle.c -- CPU restatement of the reference's src/scalar P4 codec.
 *
 * TEST INFRASTRUCTURE ONLY (see tpf_oracle.h).  Written for clarity, not
 * speed: bit streams are handled with a generic little-endian bit reader /
 * writer instead of the reference's unrolled templates.  Each function cites
 * the reference function it restates (src/scalar/...).
 */
#include "tpf_oracle.h"

#include <pthread.h>
#include <string.h>

enum { LAY_H = 0, LAY_V128 = 1, LAY_V256 = 2 };

/* ---------------------------------------------------------------- helpers */

/* pad8 -- p4_scalar_internal.h:123-126 */
static unsigned pad8(unsigned bits) { return (bits + 7u) / 8u; }

/* bitWidth32 / bitWidth64 -- p4_scalar_internal.h:159-169, :196-206 */
static unsigned bw32(uint32_t x) { return x ? 32u - (unsigned)__builtin_clz(x) : 0u; }
static unsigned bw64(uint64_t x) { return x ? 64u - (unsigned)__builtin_clzll(x) : 0u; }

static uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint64_t ld64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static void st32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static void st64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }

static uint64_t mask64(unsigned b) { return b >= 64u ? ~0ull : ((1ull << b) - 1ull); }
/* Exception patch shifts: the reference writes `exc << b`, undefined in C for
 * b >= the type's width (only reachable from malformed headers); here such a
 * shift yields 0, as the GPU decoders' shl32 does. */
static uint32_t shl32u(uint32_t v, unsigned b) { return b >= 32u ? 0u : v << b; }
static uint64_t shl64u(uint64_t v, unsigned b) { return b >= 64u ? 0u : v << b; }

/* Write the b low bits of v at bit position pos of an LSB-first stream
 * (the buffer must be zero-initialised where bits are written). */
static void put_bits(uint8_t *buf, uint64_t pos, uint64_t v, unsigned b)
{
    v &= mask64(b);
    while (b) {
        unsigned sh = (unsigned)(pos & 7u);
        unsigned take = 8u - sh;
        if (take > b) take = b;
        buf[pos >> 3] |= (uint8_t)((v & ((1u << take) - 1u)) << sh);
        v >>= take;
        pos += take;
        b -= take;
    }
}

static uint64_t get_bits(const uint8_t *buf, uint64_t pos, unsigned b)
{
    uint64_t v = 0;
    unsigned got = 0;
    while (got < b) {
        unsigned sh = (unsigned)(pos & 7u);
        unsigned take = 8u - sh;
        if (take > b - got) take = b - got;
        v |= (uint64_t)((buf[pos >> 3] >> sh) & ((1u << take) - 1u)) << got;
        got += take;
        pos += take;
    }
    return v;
}

/* Horizontal bitpack of n values, b bits each: one continuous LSB-first
 * stream of pad8(n*b) bytes.  Restates bitpack32Scalar / bitpack64Scalar
 * (p4_scalar_bitpack_impl.h:194-236, p4_scalar_bitpack64_impl.h): full
 * 32-value chunks are 4*b bytes, and choose_block_size
 * (p4_scalar_internal.h:428-451) only cuts the tail at byte-aligned
 * boundaries, so the concatenation is a single continuous stream. */
static uint8_t *hpack(const uint64_t *in, unsigned n, uint8_t *out, unsigned b)
{
    unsigned bytes = pad8(n * b);
    memset(out, 0, bytes);
    for (unsigned i = 0; i < n; ++i) put_bits(out, (uint64_t)i * b, in[i], b);
    return out + bytes;
}

/* bitunpack32Scalar / bitunpack64Scalar (p4_scalar_bitunpack_impl.h:308-368) */
static const uint8_t *hunpack(const uint8_t *in, unsigned n, uint64_t *out, unsigned b)
{
    for (unsigned i = 0; i < n; ++i) out[i] = b ? get_bits(in, (uint64_t)i * b, b) : 0u;
    return in + pad8(n * b);
}

/* Vertical (lane-interleaved) layouts: L lanes of 32 bits; element i sits in
 * lane i % L at lane-bit offset (i / L) * b; lane word k of lane l is at byte
 * 4*(L*k + l).  bitpack256v32Scalar / bitunpack256v32Scalar
 * (bitpack256v32_scalar.cpp:57-231) for L=8, bitpack128v32Scalar /
 * bitunpack128v32Scalar (bitpack128v32_scalar.cpp:57-231) for L=4.  The
 * block always holds 32*L values, output size 4*L*b bytes. */
static uint8_t *vpack(const uint32_t *in, unsigned L, uint8_t *out, unsigned b)
{
    unsigned N = 32u * L;
    unsigned bytes = 4u * L * b;
    if (b == 0u) return out;
    memset(out, 0, bytes);
    for (unsigned i = 0; i < N; ++i) {
        unsigned l = i % L, g = i / L;
        uint32_t v = (uint32_t)(in[i] & mask64(b));
        for (unsigned j = 0; j < b; ++j) {
            unsigned o = g * b + j; /* bit inside the lane stream */
            unsigned k = o >> 5, bit = o & 31u;
            unsigned byte = 4u * (L * k + l) + (bit >> 3);
            out[byte] |= (uint8_t)(((v >> j) & 1u) << (bit & 7u));
        }
    }
    return out + bytes;
}

static const uint8_t *vunpack(const uint8_t *in, unsigned L, uint32_t *out, unsigned b)
{
    unsigned N = 32u * L;
    for (unsigned i = 0; i < N; ++i) {
        unsigned l = i % L, g = i / L;
        uint32_t v = 0;
        for (unsigned j = 0; j < b; ++j) {
            unsigned o = g * b + j;
            unsigned k = o >> 5, bit = o & 31u;
            unsigned byte = 4u * (L * k + l) + (bit >> 3);
            v |= (uint32_t)((in[byte] >> (bit & 7u)) & 1u) << j;
        }
        out[i] = v;
    }
    return in + 4u * L * b;
}

/* ---------------------------------------------------------------- vbyte */

/* vbPut32 -- p4_scalar_internal.cpp:47-89 */
static uint8_t *vbput32(uint8_t *op, uint32_t x)
{
    if (x < 156u) {
        *op++ = (uint8_t)x;
    } else if (x < 16540u) {
        unsigned d = x - 156u;
        *op++ = (uint8_t)(0x9Cu + (d >> 8));
        *op++ = (uint8_t)d;
    } else if (x < 2113692u) {
        unsigned d = x - 16540u;
        *op++ = (uint8_t)(0xDCu + (d >> 16));
        *op++ = (uint8_t)d;
        *op++ = (uint8_t)(d >> 8);
    } else if (x <= 0xFFFFFFu) {
        *op++ = 0xFC;
        *op++ = (uint8_t)x;
        *op++ = (uint8_t)(x >> 8);
        *op++ = (uint8_t)(x >> 16);
    } else {
        *op++ = 0xFD;
        st32(op, x);
        op += 4;
    }
    return op;
}

/* vbEnc32 -- p4_scalar_internal.cpp:163-197 (0xFF raw escape when the
 * compressed form saves fewer than 32 bytes) */
static uint8_t *vbenc32(const uint32_t *in, unsigned n, uint8_t *out)
{
    uint8_t *op = out;
    for (unsigned i = 0; i < n; ++i) op = vbput32(op, in[i]);
    if (op + 32 > out + (size_t)n * 4u) {
        *out = 0xFF;
        memcpy(out + 1, in, (size_t)n * 4u);
        return out + 1 + (size_t)n * 4u;
    }
    return op;
}

/* vbDec32 / vbGet32Inline -- p4_scalar_internal.cpp:215-237, p4_scalar_internal.h:589-625 */
static const uint8_t *vbdec32(const uint8_t *in, unsigned n, uint32_t *out)
{
    if (*in == 0xFF) {
        memcpy(out, in + 1, (size_t)n * 4u);
        return in + 1 + (size_t)n * 4u;
    }
    const uint8_t *ip = in;
    for (unsigned i = 0; i < n; ++i) {
        unsigned m = *ip++;
        if (m < 0x9Cu) {
            out[i] = m;
        } else if (m < 0xDCu) {
            out[i] = ((m - 0x9Cu) << 8) + *ip++ + 156u;
        } else if (m < 0xFCu) {
            out[i] = (unsigned)(ip[0] | (ip[1] << 8)) + ((m - 0xDCu) << 16) + 16540u;
            ip += 2;
        } else if (m == 0xFCu) {
            out[i] = (uint32_t)ip[0] | ((uint32_t)ip[1] << 8) | ((uint32_t)ip[2] << 16);
            ip += 3;
        } else {
            out[i] = ld32(ip);
            ip += 4;
        }
    }
    return ip;
}

/* vbPut64 -- p4_scalar_internal.cpp:447-476 (raw markers 0xF8..0xFD write
 * 8 bytes and advance by the byte count; we write only the counted bytes) */
static uint8_t *vbput64(uint8_t *op, uint64_t x)
{
    if (x < 152u) {
        *op++ = (uint8_t)x;
    } else if (x < 16536u) {
        unsigned d = (unsigned)x - 152u;
        *op++ = (uint8_t)(0x98u + (d >> 8));
        *op++ = (uint8_t)d;
    } else if (x < 2113688u) {
        unsigned d = (unsigned)x - 16536u;
        *op++ = (uint8_t)(0xD8u + (d >> 16));
        *op++ = (uint8_t)d;
        *op++ = (uint8_t)(d >> 8);
    } else {
        unsigned nb = (bw64(x) + 7u) / 8u;
        *op++ = (uint8_t)(0xF8u + (nb - 3u));
        for (unsigned i = 0; i < nb; ++i) *op++ = (uint8_t)(x >> (8u * i));
    }
    return op;
}

/* vbEnc64 -- p4_scalar_internal.cpp:480-495 */
static uint8_t *vbenc64(const uint64_t *in, unsigned n, uint8_t *out)
{
    uint8_t *op = out;
    for (unsigned i = 0; i < n; ++i) op = vbput64(op, in[i]);
    if (op + 32 > out + (size_t)n * 8u) {
        *out = 0xFF;
        memcpy(out + 1, in, (size_t)n * 8u);
        return out + 1 + (size_t)n * 8u;
    }
    return op;
}

/* vbDec64 / vbGet64Inline -- p4_scalar_internal.cpp:497-526, p4_scalar_internal.h:638-670 */
static const uint8_t *vbdec64(const uint8_t *in, unsigned n, uint64_t *out)
{
    if (*in == 0xFF) {
        memcpy(out, in + 1, (size_t)n * 8u);
        return in + 1 + (size_t)n * 8u;
    }
    const uint8_t *ip = in;
    for (unsigned i = 0; i < n; ++i) {
        unsigned m = *ip++;
        if (m < 0x98u) {
            out[i] = m;
        } else if (m < 0xD8u) {
            out[i] = ((m - 0x98u) << 8) + *ip++ + 152u;
        } else if (m < 0xF8u) {
            out[i] = (uint64_t)((unsigned)(ip[0] | (ip[1] << 8)) + ((m - 0xD8u) << 16) + 16536u);
            ip += 2;
        } else {
            unsigned nb = (m - 0xF8u) + 3u;
            uint64_t v = 0;
            for (unsigned j = 0; j < nb && j < 8u; ++j) v |= (uint64_t)ip[j] << (8u * j);
            out[i] = v;
            ip += nb;
        }
    }
    return ip;
}

/* ------------------------------------------------------------ cost model */

/* p4Bits32 / p4Bits64 -- p4_scalar_internal.cpp:270-387 and :538-652.
 * W = 32 or 64.  Returns b; *bx = 0 (plain), 1..W (bitmap patch bits),
 * W+1 (vbyte exceptions), W+2 (constant block). */
static unsigned p4bits_generic(const uint64_t *in, unsigned n, unsigned W, unsigned *out_bx)
{
    uint64_t orv = 0;
    const uint64_t first = in[0];
    unsigned eq = 0;
    for (unsigned i = 0; i < n; ++i) {
        orv |= in[i];
        eq += (in[i] == first);
    }
    if (orv == 0) {
        *out_bx = 0;
        return 0;
    }
    unsigned max_bits = bw64(orv);
    if (eq == n) {
        *out_bx = W + 2u;
        return max_bits;
    }
    unsigned cnt[64 + 8];
    memset(cnt, 0, sizeof(cnt));
    for (unsigned i = 0; i < n; ++i) ++cnt[bw64(in[i])];

    /* vb[] is indexed from -25 .. W; stored with an offset of 32 */
    int vbstore[64 + 64];
    memset(vbstore, 0, sizeof(vbstore));
    int *vb = vbstore + 32;

    unsigned best_b = max_bits;
    unsigned xc = cnt[max_bits];
    unsigned min_size = pad8(n * max_bits) + 1u;
    unsigned vbsum = xc;
#define VB_UPDATE(count, bits)                    \
    do {                                          \
        vb[(int)(bits) - 7] += (int)(count);      \
        vb[(int)(bits) - 15] += (int)(count) * 2; \
        vb[(int)(bits) - 19] += (int)(count) * 3; \
        vb[(int)(bits) - 25] += (int)(count) * 4; \
    } while (0)
    VB_UPDATE(xc, max_bits);
    unsigned use_vb = 0;
    const unsigned bmp = pad8(n);
    unsigned b = max_bits - 1u;
    for (;;) {
        unsigned pb = max_bits - b;
        unsigned vsz = pad8(n * b) + 2u + xc + vbsum;
        unsigned psz = pad8(n * b) + 2u + bmp + pad8(xc * pb);
        if (psz < min_size && psz <= vsz) {
            min_size = psz;
            best_b = b;
            use_vb = 0;
        } else if (vsz < min_size) {
            min_size = vsz;
            best_b = b;
            use_vb = 1;
        }
        if (b == 0) break;
        xc += cnt[b];
        vbsum += cnt[b] + (unsigned)vb[b];
        VB_UPDATE(cnt[b], b);
        --b;
    }
#undef VB_UPDATE
    *out_bx = use_vb ? (W + 1u) : (max_bits - best_b);
    if (W == 64u && best_b == 63u) { /* 63->64 quirk, p4_scalar_internal.cpp:645-649 */
        best_b = 64u;
        *out_bx = 0;
    }
    return best_b;
}

unsigned orc_p4bits32(const uint32_t *in, unsigned n, unsigned *bx)
{
    uint64_t t[256];
    for (unsigned i = 0; i < n; ++i) t[i] = in[i];
    return p4bits_generic(t, n, 32u, bx);
}

unsigned orc_p4bits64(const uint64_t *in, unsigned n, unsigned *bx)
{
    return p4bits_generic(in, n, 64u, bx);
}

/* writeHeader -- p4_scalar_internal.cpp:409-429; writeHeader64 -- :675-695 */
static uint8_t *write_header(uint8_t *out, unsigned b, unsigned bx, unsigned W)
{
    unsigned bh = (W == 64u && b >= 64u) ? 63u : b;
    if (bx == 0u) {
        *out++ = (uint8_t)bh;
    } else if (bx <= W) {
        *out++ = (uint8_t)(0x80u | bh);
        *out++ = (uint8_t)bx;
    } else {
        *out++ = (uint8_t)(((bx == W + 1u) ? 0x40u : 0xC0u) | bh);
    }
    return out;
}

/* ---------------------------------------------------------- 32-bit codec */

static unsigned lay_count(int lay, unsigned n)
{
    return lay == LAY_V256 ? 256u : lay == LAY_V128 ? 128u : n;
}

static uint8_t *pack_base32(const uint32_t *in, unsigned n, uint8_t *out, unsigned b, int lay)
{
    if (lay == LAY_V256) return vpack(in, 8u, out, b);
    if (lay == LAY_V128) return vpack(in, 4u, out, b);
    uint64_t t[256];
    for (unsigned i = 0; i < n; ++i) t[i] = in[i];
    return hpack(t, n, out, b);
}

static const uint8_t *unpack_base32(const uint8_t *in, unsigned n, uint32_t *out, unsigned b, int lay)
{
    if (lay == LAY_V256) return vunpack(in, 8u, out, b);
    if (lay == LAY_V128) return vunpack(in, 4u, out, b);
    uint64_t t[256];
    const uint8_t *r = hunpack(in, n, t, b);
    for (unsigned i = 0; i < n; ++i) out[i] = (uint32_t)t[i];
    return r;
}

/* p4Enc256v32 / p4Enc128v32 / p4Enc32 with their payload helpers:
 *   p4enc256v32_scalar.cpp:49-151 (exceptions), :170-194 (payload), :216-235
 *   p4enc128v32_scalar.cpp (same structure, 128v32 base layout)
 *   p4enc32.cpp:30-119, :139-180, :201-217 (horizontal base layout; the
 *   constant block writes exactly ceil(b/8) bytes instead of 4) */
static uint8_t *p4enc32_generic(const uint32_t *in_raw, unsigned n, uint8_t *out, int lay)
{
    if (n == 0u) return out;
    const unsigned N = lay_count(lay, n);
    uint32_t in[256];
    memset(in, 0, sizeof(in));
    memcpy(in, in_raw, (size_t)((lay == LAY_H) ? n : N) * 4u);

    unsigned bx;
    unsigned b = orc_p4bits32(in, n, &bx);
    out = write_header(out, b, bx, 32u);

    if (bx == 0u) return pack_base32(in, n, out, b, lay);
    if (bx == 34u) {
        if (lay == LAY_H) {
            uint32_t v = (uint32_t)(in[0] & mask64(b));
            for (unsigned i = 0; i < (b + 7u) / 8u; ++i) out[i] = (uint8_t)(v >> (8u * i));
        } else {
            st32(out, in[0]); /* over-writes up to 4 bytes, like storeU32 */
        }
        return out + (b + 7u) / 8u;
    }

    const uint32_t bmask = (uint32_t)mask64(b);
    uint32_t base[256];
    uint64_t exc[256];
    uint32_t exc32[256];
    unsigned pos[256];
    unsigned xn = 0;
    memset(base, 0, sizeof(base));
    for (unsigned i = 0; i < n; ++i) {
        base[i] = in[i] & bmask;
        if (in[i] > bmask) {
            pos[xn] = i;
            exc32[xn] = in[i] >> b;
            exc[xn] = exc32[xn];
            ++xn;
        }
    }
    (void)N;
    if (bx <= 32u) {
        uint8_t bm[32];
        memset(bm, 0, sizeof(bm));
        for (unsigned k = 0; k < xn; ++k) bm[pos[k] >> 3] |= (uint8_t)(1u << (pos[k] & 7u));
        memcpy(out, bm, pad8(n));
        out += pad8(n);
        out = hpack(exc, xn, out, bx);
        return pack_base32(base, n, out, b, lay);
    }
    *out++ = (uint8_t)xn;
    out = pack_base32(base, n, out, b, lay);
    out = vbenc32(exc32, xn, out);
    for (unsigned k = 0; k < xn; ++k) *out++ = (uint8_t)pos[k];
    return out;
}

/* p4Dec256v32 (p4dec256v32_scalar.cpp:10-137), p4Dec128v32
 * (p4dec128v32_scalar.cpp), p4Dec32 (p4dec32.cpp:12-142). */
static const uint8_t *p4dec32_generic(const uint8_t *in, unsigned n, uint32_t *out, int lay)
{
    if (n == 0u) return in;
    const uint8_t *ip = in;
    unsigned b = *ip++;

    if ((b & 0xC0u) == 0xC0u) { /* constant */
        b &= 0x3Fu;
        uint32_t v;
        unsigned nbytes = (b + 7u) / 8u;
        if (lay == LAY_H) { /* reads exactly ceil(b/8) bytes, p4dec32.cpp:100-124 */
            uint64_t v64 = 0; /* b > 32 is undefined in the reference (p4dec32.cpp:100-116): low 32 bits here */
            for (unsigned i = 0; i < nbytes; ++i) v64 |= (uint64_t)ip[i] << (8u * i);
            v = (uint32_t)v64;
        } else {
            v = ld32(ip);
        }
        if (b < 32u) v &= (uint32_t)mask64(b);
        for (unsigned i = 0; i < n; ++i) out[i] = v;
        return ip + nbytes;
    }
    if ((b & 0x40u) == 0u) { /* plain or bitmap */
        unsigned bx = 0;
        if (b & 0x80u) bx = *ip++;
        b &= 0x7Fu;
        if (bx == 0u) return unpack_base32(ip, n, out, b, lay);

        uint64_t bm[4] = {0, 0, 0, 0};
        unsigned words = (n + 63u) / 64u, xn = 0;
        for (unsigned w = 0; w < words; ++w) {
            uint64_t word = ld64(ip + 8u * w);
            if (w == words - 1u && (n & 63u)) word &= (1ull << (n & 63u)) - 1ull;
            bm[w] = word;
            xn += (unsigned)__builtin_popcountll(word);
        }
        ip += pad8(n);
        uint64_t exc[256 + 64];
        ip = hunpack(ip, xn, exc, bx);
        ip = unpack_base32(ip, n, out, b, lay);
        unsigned k = 0;
        for (unsigned w = 0; w < words; ++w) {
            uint64_t word = bm[w];
            while (word) {
                unsigned bit = (unsigned)__builtin_ctzll(word);
                out[w * 64u + bit] |= shl32u((uint32_t)exc[k++], b);
                word &= word - 1ull;
            }
        }
        return ip;
    }
    /* vbyte exceptions */
    unsigned xn = *ip++;
    b &= 0x3Fu;
    if (b > 32u) b = 32u; /* malformed (the reference's unpack is undefined there): clamped as the GPU decoders do */
    ip = unpack_base32(ip, n, out, b, lay);
    uint32_t exc[256 + 64];
    ip = vbdec32(ip, xn, exc);
    for (unsigned k = 0; k < xn; ++k) out[ip[k]] |= shl32u(exc[k], b);
    return ip + xn;
}

/* applyDelta1_256 -- p4d1dec256v32_scalar.cpp:39-50 (also p4d1dec32.cpp:68) */
static void delta1_32(uint32_t *out, unsigned n, uint32_t start)
{
    uint32_t acc = start;
    for (unsigned i = 0; i < n; ++i) {
        acc += out[i] + 1u;
        out[i] = acc;
    }
}

/* deltaEnc1 -- p4_scalar_internal.h:711-719 */
static void deltaenc1_32(const uint32_t *in, unsigned n, uint32_t *out, uint32_t start)
{
    for (unsigned i = 0; i < n; ++i) {
        out[i] = in[i] - start - 1u;
        start = in[i];
    }
}

uint8_t *orc_p4enc256v32(const uint32_t *in, unsigned n, uint8_t *out) { return p4enc32_generic(in, n, out, LAY_V256); }
uint8_t *orc_p4enc128v32(const uint32_t *in, unsigned n, uint8_t *out) { return p4enc32_generic(in, n, out, LAY_V128); }
uint8_t *orc_p4enc32(const uint32_t *in, unsigned n, uint8_t *out) { return p4enc32_generic(in, n, out, LAY_H); }

/* p4D1Enc256v32 (p4d1enc256v32_scalar.cpp:7-15), p4D1Enc128v32, p4D1Enc32:
 * deltaEnc1 into a temporary, then the plain encoder.  For the vertical
 * layouts the temporary holds only n deltas; the tail up to the block size is
 * taken from the caller's input like the reference's stack buffer would not
 * be -- callers use n equal to the block size. */
static uint8_t *p4d1enc32_generic(const uint32_t *in, unsigned n, uint8_t *out, uint32_t start, int lay)
{
    if (n == 0u) return out;
    uint32_t t[256 + 8];
    memset(t, 0, sizeof(t));
    deltaenc1_32(in, n, t, start);
    return p4enc32_generic(t, n, out, lay);
}
uint8_t *orc_p4d1enc256v32(const uint32_t *in, unsigned n, uint8_t *out, uint32_t s) { return p4d1enc32_generic(in, n, out, s, LAY_V256); }
uint8_t *orc_p4d1enc128v32(const uint32_t *in, unsigned n, uint8_t *out, uint32_t s) { return p4d1enc32_generic(in, n, out, s, LAY_V128); }
uint8_t *orc_p4d1enc32(const uint32_t *in, unsigned n, uint8_t *out, uint32_t s) { return p4d1enc32_generic(in, n, out, s, LAY_H); }

const uint8_t *orc_p4dec256v32(const uint8_t *in, unsigned n, uint32_t *out) { return p4dec32_generic(in, n, out, LAY_V256); }
const uint8_t *orc_p4dec128v32(const uint8_t *in, unsigned n, uint32_t *out) { return p4dec32_generic(in, n, out, LAY_V128); }
const uint8_t *orc_p4dec32(const uint8_t *in, unsigned n, uint32_t *out) { return p4dec32_generic(in, n, out, LAY_H); }

/* p4D1Dec256v32 (p4d1dec256v32_scalar.cpp:198-268), p4D1Dec128v32,
 * p4D1Dec32 (p4d1dec32.cpp): decode, then the delta-1 prefix scan. */
static const uint8_t *p4d1dec32_generic(const uint8_t *in, unsigned n, uint32_t *out, uint32_t start, int lay)
{
    if (n == 0u) return in;
    const uint8_t *r = p4dec32_generic(in, n, out, lay);
    delta1_32(out, n, start);
    return r;
}
const uint8_t *orc_p4d1dec256v32(const uint8_t *in, unsigned n, uint32_t *out, uint32_t s) { return p4d1dec32_generic(in, n, out, s, LAY_V256); }
const uint8_t *orc_p4d1dec128v32(const uint8_t *in, unsigned n, uint32_t *out, uint32_t s) { return p4d1dec32_generic(in, n, out, s, LAY_V128); }
const uint8_t *orc_p4d1dec32(const uint8_t *in, unsigned n, uint32_t *out, uint32_t s) { return p4d1dec32_generic(in, n, out, s, LAY_H); }

/* ---------------------------------------------------------- 64-bit codec */

/* bitpack128v64Scalar / bitunpack128v64Scalar -- bitpack128v64_scalar.cpp:38-104:
 * b<=32: 128v32 layout of the low halves with each group of 4 pair-swapped
 * ([v2,v3,v0,v1], the IP32 shuffle); b>32: horizontal 64-bit stream. */
static uint8_t *pack128v64(const uint64_t *in, uint8_t *out, unsigned b)
{
    if (b <= 32u) {
        uint32_t t[128];
        for (unsigned i = 0; i < 128u; i += 4) {
            t[i + 0] = (uint32_t)in[i + 2];
            t[i + 1] = (uint32_t)in[i + 3];
            t[i + 2] = (uint32_t)in[i + 0];
            t[i + 3] = (uint32_t)in[i + 1];
        }
        return vpack(t, 4u, out, b);
    }
    return hpack(in, 128u, out, b);
}

static const uint8_t *unpack128v64(const uint8_t *in, uint64_t *out, unsigned b)
{
    if (b <= 32u) {
        uint32_t t[128];
        const uint8_t *r = vunpack(in, 4u, t, b);
        for (unsigned i = 0; i < 128u; i += 4) {
            out[i + 0] = t[i + 2];
            out[i + 1] = t[i + 3];
            out[i + 2] = t[i + 0];
            out[i + 3] = t[i + 1];
        }
        return r;
    }
    return hunpack(in, 128u, out, b);
}

/* p4Enc128v64 -- p4enc128v64_scalar.cpp:51-224 */
uint8_t *orc_p4enc128v64(const uint64_t *in_raw, unsigned n, uint8_t *out)
{
    if (n == 0u) return out;
    uint64_t in[128];
    memset(in, 0, sizeof(in));
    memcpy(in, in_raw, 128u * 8u);
    unsigned bx;
    unsigned b = orc_p4bits64(in, n, &bx);
    out = write_header(out, b, bx, 64u);
    if (bx == 0u) return pack128v64(in, out, b);
    if (bx == 66u) {
        st64(out, in[0]); /* storeU64Fast over-write, :173-175 */
        return out + (b + 7u) / 8u;
    }
    const uint64_t bmask = mask64(b);
    uint64_t base[128], exc[128];
    unsigned pos[128], xn = 0;
    memset(base, 0, sizeof(base));
    for (unsigned i = 0; i < n; ++i) {
        base[i] = in[i] & bmask;
        if (in[i] > bmask) {
            pos[xn] = i;
            exc[xn] = in[i] >> b;
            ++xn;
        }
    }
    if (bx <= 64u) {
        uint8_t bm[16];
        memset(bm, 0, sizeof(bm));
        for (unsigned k = 0; k < xn; ++k) bm[pos[k] >> 3] |= (uint8_t)(1u << (pos[k] & 7u));
        memcpy(out, bm, pad8(n));
        out += pad8(n);
        out = hpack(exc, xn, out, bx);
        return pack128v64(base, out, b);
    }
    *out++ = (uint8_t)xn;
    out = pack128v64(base, out, b);
    out = vbenc64(exc, xn, out);
    for (unsigned k = 0; k < xn; ++k) *out++ = (uint8_t)pos[k];
    return out;
}

/* p4Dec128v64 -- p4d1dec128v64_scalar.cpp:257-375 */
const uint8_t *orc_p4dec128v64(const uint8_t *in, unsigned n, uint64_t *out)
{
    if (n == 0u) return in;
    const uint8_t *ip = in;
    unsigned b = *ip++;
    if ((b & 0xC0u) == 0xC0u) {
        b &= 0x3Fu;
        if (b == 63u) b = 64u;
        uint64_t v = ld64(ip);
        if (b < 64u) v &= mask64(b);
        for (unsigned i = 0; i < n; ++i) out[i] = v;
        return ip + (b + 7u) / 8u;
    }
    if ((b & 0x40u) == 0u) {
        unsigned bx = 0;
        if (b & 0x80u) {
            bx = *ip++;
            b &= 0x7Fu;
        }
        if (b == 63u) b = 64u;
        if (bx == 0u) return unpack128v64(ip, out, b);
        uint64_t bm[4] = {0, 0, 0, 0};
        unsigned words = (n + 63u) / 64u, xn = 0;
        for (unsigned w = 0; w < words; ++w) {
            uint64_t word = ld64(ip + 8u * w);
            if (w == words - 1u && (n & 63u)) word &= (1ull << (n & 63u)) - 1ull;
            bm[w] = word;
            xn += (unsigned)__builtin_popcountll(word);
        }
        ip += pad8(n);
        uint64_t exc[256 + 64];
        ip = hunpack(ip, xn, exc, bx);
        ip = unpack128v64(ip, out, b);
        unsigned k = 0;
        for (unsigned w = 0; w < words; ++w) {
            uint64_t word = bm[w];
            while (word) {
                unsigned bit = (unsigned)__builtin_ctzll(word);
                out[w * 64u + bit] |= shl64u(exc[k++], b);
                word &= word - 1ull;
            }
        }
        return ip;
    }
    b &= 0x3Fu;
    if (b == 63u) b = 64u;
    unsigned xn = *ip++;
    ip = unpack128v64(ip, out, b);
    uint64_t exc[256 + 64];
    ip = vbdec64(ip, xn, exc);
    for (unsigned k = 0; k < xn; ++k) out[ip[k]] |= shl64u(exc[k], b);
    return ip + xn;
}

/* applyDelta1_64 -- p4d1dec128v64_scalar.cpp (top of file) */
static void delta1_64(uint64_t *out, unsigned n, uint64_t start)
{
    for (unsigned i = 0; i < n; ++i) out[i] = (start += out[i]) + (i + 1u);
}

/* p4D1Dec128v64 -- p4d1dec128v64_scalar.cpp:157-251 */
const uint8_t *orc_p4d1dec128v64(const uint8_t *in, unsigned n, uint64_t *out, uint64_t start)
{
    if (n == 0u) return in;
    const uint8_t *r = orc_p4dec128v64(in, n, out);
    delta1_64(out, n, start);
    return r;
}

/* p4D1Enc128v64 -- p4d1enc128v64_scalar.cpp */
uint8_t *orc_p4d1enc128v64(const uint64_t *in, unsigned n, uint8_t *out, uint64_t start)
{
    if (n == 0u) return out;
    uint64_t t[128 + 8];
    memset(t, 0, sizeof(t));
    for (unsigned i = 0; i < n; ++i) {
        t[i] = in[i] - start - 1u;
        start = in[i];
    }
    return orc_p4enc128v64(t, n, out);
}

/* p4Enc256v64 / p4Dec256v64 / p4D1Dec256v64 / p4D1Enc256v64:
 * two consecutive 128v64 blocks (p4enc256v64_scalar.cpp:15-30,
 * p4d1dec256v64_scalar.cpp:15-49, p4d1enc256v64_scalar.cpp). */
uint8_t *orc_p4enc256v64(const uint64_t *in, unsigned n, uint8_t *out)
{
    while (n > 0u) {
        unsigned c = n < 128u ? n : 128u;
        out = orc_p4enc128v64(in, c, out);
        in += c;
        n -= c;
    }
    return out;
}

uint8_t *orc_p4d1enc256v64(const uint64_t *in, unsigned n, uint8_t *out, uint64_t start)
{
    if (n == 0u) return out;
    uint64_t t[256 + 8];
    memset(t, 0, sizeof(t));
    for (unsigned i = 0; i < n; ++i) {
        t[i] = in[i] - start - 1u;
        start = in[i];
    }
    return orc_p4enc256v64(t, n, out);
}

const uint8_t *orc_p4dec256v64(const uint8_t *in, unsigned n, uint64_t *out)
{
    while (n > 0u) {
        unsigned c = n < 128u ? n : 128u;
        in = orc_p4dec128v64(in, c, out);
        out += c;
        n -= c;
    }
    return in;
}

const uint8_t *orc_p4d1dec256v64(const uint8_t *in, unsigned n, uint64_t *out, uint64_t start)
{
    while (n > 0u) {
        unsigned c = n < 128u ? n : 128u;
        in = orc_p4d1dec128v64(in, c, out, start);
        start = out[c - 1];
        out += c;
        n -= c;
    }
    return in;
}

/* ---------------------------------------------------------- batch helpers */

uint64_t orc_enc256v32_batch(const uint32_t *in, uint64_t nb, uint8_t *out, uint64_t *off)
{
    uint8_t *op = out;
    for (uint64_t i = 0; i < nb; ++i) {
        off[i] = (uint64_t)(op - out);
        op = orc_p4enc256v32(in + i * 256u, 256u, op);
    }
    off[nb] = (uint64_t)(op - out);
    return off[nb];
}

uint64_t orc_d1enc256v32_batch(const uint32_t *in, uint64_t nb, uint8_t *out, uint64_t *off, const uint32_t *st)
{
    uint8_t *op = out;
    for (uint64_t i = 0; i < nb; ++i) {
        off[i] = (uint64_t)(op - out);
        op = orc_p4d1enc256v32(in + i * 256u, 256u, op, st[i]);
    }
    off[nb] = (uint64_t)(op - out);
    return off[nb];
}

int orc_dec256v32_batch(const uint8_t *in, const uint64_t *off, uint64_t nb, uint32_t *out)
{
    for (uint64_t i = 0; i < nb; ++i) {
        const uint8_t *e = orc_p4dec256v32(in + off[i], 256u, out + i * 256u);
        if ((uint64_t)(e - in) != off[i + 1]) return -1 - (int)(i & 0x3fffffff);
    }
    return 0;
}

int orc_d1dec256v32_batch(const uint8_t *in, const uint64_t *off, uint64_t nb, uint32_t *out, const uint32_t *st)
{
    for (uint64_t i = 0; i < nb; ++i) {
        const uint8_t *e = orc_p4d1dec256v32(in + off[i], 256u, out + i * 256u, st[i]);
        if ((uint64_t)(e - in) != off[i + 1]) return -1 - (int)(i & 0x3fffffff);
    }
    return 0;
}

uint64_t orc_enc256v64_batch(const uint64_t *in, uint64_t nb, uint8_t *out, uint64_t *off)
{
    uint8_t *op = out;
    for (uint64_t i = 0; i < nb; ++i) {
        off[i] = (uint64_t)(op - out);
        op = orc_p4enc256v64(in + i * 256u, 256u, op);
    }
    off[nb] = (uint64_t)(op - out);
    return off[nb];
}

uint64_t orc_d1enc256v64_batch(const uint64_t *in, uint64_t nb, uint8_t *out, uint64_t *off, const uint64_t *st)
{
    uint8_t *op = out;
    for (uint64_t i = 0; i < nb; ++i) {
        off[i] = (uint64_t)(op - out);
        op = orc_p4d1enc256v64(in + i * 256u, 256u, op, st[i]);
    }
    off[nb] = (uint64_t)(op - out);
    return off[nb];
}

int orc_dec256v64_batch(const uint8_t *in, const uint64_t *off, uint64_t nb, uint64_t *out)
{
    for (uint64_t i = 0; i < nb; ++i) {
        const uint8_t *e = orc_p4dec256v64(in + off[i], 256u, out + i * 256u);
        if ((uint64_t)(e - in) != off[i + 1]) return -1 - (int)(i & 0x3fffffff);
    }
    return 0;
}

int orc_d1dec256v64_batch(const uint8_t *in, const uint64_t *off, uint64_t nb, uint64_t *out, const uint64_t *st)
{
    for (uint64_t i = 0; i < nb; ++i) {
        const uint8_t *e = orc_p4d1dec256v64(in + off[i], 256u, out + i * 256u, st[i]);
        if ((uint64_t)(e - in) != off[i + 1]) return -1 - (int)(i & 0x3fffffff);
    }
    return 0;
}

uint64_t orc_enc32_batch(const uint32_t *in, uint64_t nb, unsigned bn, uint8_t *out, uint64_t *off)
{
    uint8_t *op = out;
    for (uint64_t i = 0; i < nb; ++i) {
        off[i] = (uint64_t)(op - out);
        op = orc_p4enc32(in + i * bn, bn, op);
    }
    off[nb] = (uint64_t)(op - out);
    return off[nb];
}

uint64_t orc_d1enc32_batch(const uint32_t *in, uint64_t nb, unsigned bn, uint8_t *out, uint64_t *off, const uint32_t *st)
{
    uint8_t *op = out;
    for (uint64_t i = 0; i < nb; ++i) {
        off[i] = (uint64_t)(op - out);
        op = orc_p4d1enc32(in + i * bn, bn, op, st[i]);
    }
    off[nb] = (uint64_t)(op - out);
    return off[nb];
}

int orc_dec32_batch(const uint8_t *in, const uint64_t *off, uint64_t nb, unsigned bn, uint32_t *out)
{
    for (uint64_t i = 0; i < nb; ++i) {
        const uint8_t *e = orc_p4dec32(in + off[i], bn, out + i * bn);
        if ((uint64_t)(e - in) != off[i + 1]) return -1 - (int)(i & 0x3fffffff);
    }
    return 0;
}

int orc_d1dec32_batch(const uint8_t *in, const uint64_t *off, uint64_t nb, unsigned bn, uint32_t *out, const uint32_t *st)
{
    for (uint64_t i = 0; i < nb; ++i) {
        const uint8_t *e = orc_p4d1dec32(in + off[i], bn, out + i * bn, st[i]);
        if ((uint64_t)(e - in) != off[i + 1]) return -1 - (int)(i & 0x3fffffff);
    }
    return 0;
}

struct mt_job {
    const uint8_t *in;
    const uint64_t *off;
    uint64_t lo, hi;
    uint32_t *out;
    int rc;
};

static void *mt_worker(void *arg)
{
    struct mt_job *j = (struct mt_job *)arg;
    j->rc = 0;
    for (uint64_t i = j->lo; i < j->hi; ++i) orc_p4dec256v32(j->in + j->off[i], 256u, j->out + i * 256u);
    return 0;
}

int orc_dec256v32_batch_mt(const uint8_t *in, const uint64_t *off, uint64_t nb, uint32_t *out, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    struct mt_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].in = in;
        jobs[t].off = off;
        jobs[t].lo = nb * (uint64_t)t / (uint64_t)nthreads;
        jobs[t].hi = nb * (uint64_t)(t + 1) / (uint64_t)nthreads;
        jobs[t].out = out;
        pthread_create(&th[t], 0, mt_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], 0);
    return 0;
}
