/*
 * tpf_oracle.h -- CPU restatement of the reference's scalar P4 codec.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it, and only as the checker.  The product path (turbopfor-cpp_amd/)
 * never links or calls it.
 *
 * Parity: pinned against golden vectors generated from the reference's own
 * src/scalar sources (oracle/gen_golden.cpp -> tests/golden/), see
 * tests/test_oracle_golden.py.
 *
 * Every function restates the reference function named beside it
 * (paths relative to the reference checkout: src/scalar/...).
 * Formats:
 *   256v32 : 8-lane interleaved base layout   (bitpack256v32_scalar.cpp:57-231)
 *   128v32 : 4-lane interleaved base layout   (bitpack128v32_scalar.cpp:57-231)
 *   32     : horizontal LSB-first bitstream   (p4_scalar_bitpack_impl.h:194-236)
 *   128v64 : hybrid (128v32 of pair-swapped low halves if b<=32, horizontal
 *            64-bit stream if b>32)          (bitpack128v64_scalar.cpp:38-104)
 *   256v64 : two consecutive 128v64 blocks    (p4enc256v64_scalar.cpp:15-30)
 */
#ifndef TPF_ORACLE_H
#define TPF_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* --- per-block functions, same argument meaning as turbopfor.h --- */
uint8_t *orc_p4enc256v32(const uint32_t *in, unsigned n, uint8_t *out);
uint8_t *orc_p4d1enc256v32(const uint32_t *in, unsigned n, uint8_t *out, uint32_t start);
const uint8_t *orc_p4dec256v32(const uint8_t *in, unsigned n, uint32_t *out);
const uint8_t *orc_p4d1dec256v32(const uint8_t *in, unsigned n, uint32_t *out, uint32_t start);

uint8_t *orc_p4enc128v32(const uint32_t *in, unsigned n, uint8_t *out);
uint8_t *orc_p4d1enc128v32(const uint32_t *in, unsigned n, uint8_t *out, uint32_t start);
const uint8_t *orc_p4dec128v32(const uint8_t *in, unsigned n, uint32_t *out);
const uint8_t *orc_p4d1dec128v32(const uint8_t *in, unsigned n, uint32_t *out, uint32_t start);

uint8_t *orc_p4enc32(const uint32_t *in, unsigned n, uint8_t *out);
uint8_t *orc_p4d1enc32(const uint32_t *in, unsigned n, uint8_t *out, uint32_t start);
const uint8_t *orc_p4dec32(const uint8_t *in, unsigned n, uint32_t *out);
const uint8_t *orc_p4d1dec32(const uint8_t *in, unsigned n, uint32_t *out, uint32_t start);

uint8_t *orc_p4enc128v64(const uint64_t *in, unsigned n, uint8_t *out);
uint8_t *orc_p4d1enc128v64(const uint64_t *in, unsigned n, uint8_t *out, uint64_t start);
const uint8_t *orc_p4dec128v64(const uint8_t *in, unsigned n, uint64_t *out);
const uint8_t *orc_p4d1dec128v64(const uint8_t *in, unsigned n, uint64_t *out, uint64_t start);

uint8_t *orc_p4enc256v64(const uint64_t *in, unsigned n, uint8_t *out);
uint8_t *orc_p4d1enc256v64(const uint64_t *in, unsigned n, uint8_t *out, uint64_t start);
const uint8_t *orc_p4dec256v64(const uint8_t *in, unsigned n, uint64_t *out);
const uint8_t *orc_p4d1dec256v64(const uint8_t *in, unsigned n, uint64_t *out, uint64_t start);

/* p4Bits32 / p4Bits64 cost model (p4_scalar_internal.cpp:270-387, :538-652) */
unsigned orc_p4bits32(const uint32_t *in, unsigned n, unsigned *bx);
unsigned orc_p4bits64(const uint64_t *in, unsigned n, unsigned *bx);

/* --- batch helpers for the tests: block i occupies [off[i], off[i+1]) --- */
/* kind: 0 = 256v32, 1 = 128v32(n=128 blocks), 2 = 32 (n per block = blk_n) */
uint64_t orc_enc256v32_batch(const uint32_t *in, uint64_t nblocks, uint8_t *out, uint64_t *off);
uint64_t orc_d1enc256v32_batch(const uint32_t *in, uint64_t nblocks, uint8_t *out, uint64_t *off,
                               const uint32_t *starts);
int orc_dec256v32_batch(const uint8_t *in, const uint64_t *off, uint64_t nblocks, uint32_t *out);
int orc_d1dec256v32_batch(const uint8_t *in, const uint64_t *off, uint64_t nblocks, uint32_t *out,
                          const uint32_t *starts);
uint64_t orc_enc256v64_batch(const uint64_t *in, uint64_t nblocks, uint8_t *out, uint64_t *off);
uint64_t orc_d1enc256v64_batch(const uint64_t *in, uint64_t nblocks, uint8_t *out, uint64_t *off,
                               const uint64_t *starts);
int orc_dec256v64_batch(const uint8_t *in, const uint64_t *off, uint64_t nblocks, uint64_t *out);
int orc_d1dec256v64_batch(const uint8_t *in, const uint64_t *off, uint64_t nblocks, uint64_t *out,
                          const uint64_t *starts);
uint64_t orc_enc32_batch(const uint32_t *in, uint64_t nblocks, unsigned blk_n, uint8_t *out, uint64_t *off);
int orc_dec32_batch(const uint8_t *in, const uint64_t *off, uint64_t nblocks, unsigned blk_n, uint32_t *out);
uint64_t orc_d1enc32_batch(const uint32_t *in, uint64_t nblocks, unsigned blk_n, uint8_t *out, uint64_t *off,
                           const uint32_t *starts);
int orc_d1dec32_batch(const uint8_t *in, const uint64_t *off, uint64_t nblocks, unsigned blk_n, uint32_t *out,
                      const uint32_t *starts);

/* Multi-threaded streaming decode used by bench.py's cpu_baseline leg
 * (kind "port"): nthreads workers each decode a contiguous block range. */
int orc_dec256v32_batch_mt(const uint8_t *in, const uint64_t *off, uint64_t nblocks, uint32_t *out, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
