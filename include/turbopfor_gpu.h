/*
 * turbopfor_gpu.h -- C-ABI of the MI355X (gfx950) P4 codec: batched device
 * entry points.  Plain C types only (no HIP/torch types): `stream` is a
 * hipStream_t passed as void* (NULL = the default stream).  All pointers named
 * d_* are device pointers; inputs are expected to be resident in HBM.
 *
 * Layout contract for the batched 256v32 / 256v64 formats:
 *   - the packed stream is the reference's per-block encodings laid end to
 *     end, exactly as the reference's callers chain them with the returned end
 *     pointer (README.md:108-123);
 *   - d_off[0..nblocks] are byte offsets of each block (d_off[nblocks] = end);
 *     the reference has no offsets (block sizes are implicit), so the batch
 *     encoders produce them and tpf_scan_offsets recovers them from a legacy
 *     stream;
 *   - OFFSETS CONTRACT (every entry below that takes d_off / h_off): the
 *     array has nblocks + 1 readable entries.  The kernels read d_off[i] and
 *     d_off[i+1] of every block they decode; the array's length is not passed
 *     and cannot be checked on the device, so a shorter array is an
 *     out-of-bounds device read (round 5 saw one fault from a test that broke
 *     this).  The VALUES are checked: an offset outside [0, in_bytes] or a
 *     block whose parse disagrees with its offsets is reported through d_err,
 *     never followed;
 *   - decoded values are nblocks * 256 contiguous integers.
 * No device-side slack is required: all device reads are bounds-checked
 * against in_bytes.
 *
 * Return value: TPF_OK (0) or a negative TPF_E* code; tpf_last_error()
 * returns a thread-local message for the last failure.
 */
#ifndef TURBOPFOR_GPU_H
#define TURBOPFOR_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TPF_OK 0
#define TPF_EINVAL (-1)  /* bad argument */
#define TPF_EHIP (-2)    /* HIP runtime error (see tpf_last_error) */
#define TPF_ENODEV (-3)  /* no HIP device: the library has no CPU fallback */
#define TPF_ECORRUPT (-4) /* a block's parsed length disagrees with its offsets */

const char *tpf_last_error(void);
int tpf_device_count(void);

/* ---- 256v32 decode (hot path) ------------------------------------------
 * Replaces per-block turbopfor::p4Dec256v32 (reference include/turbopfor.h:39,
 * src/dispatch.cpp:88-95).  d_err (optional, may be NULL): receives the index
 * of the first block whose parsed byte length differs from
 * d_off[i+1]-d_off[i], or UINT64_MAX when every block is consistent. */
int tpf_p4dec256v32_batch(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nblocks,
                          uint32_t *d_out, uint64_t *d_err, void *stream);


/* Replaces turbopfor::p4D1Dec256v32 (include/turbopfor.h:42, dispatch.cpp:97-104):
 * block i is decoded with start d_starts[i] (the value preceding the block). */
int tpf_p4d1dec256v32_batch(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nblocks,
                            uint32_t *d_out, const uint32_t *d_starts, uint64_t *d_err, void *stream);

/* ---- 256v32 chained delta-1 decode -------------------
 * One posting list split into nblocks consecutive 256v32 D1 blocks, encoded
 * the way reference callers chain them (start of block i = last value of
 * block i-1, README.md:116-123): decode the whole list on the device with
 * only the list's initial start0.  Phase A (chain_sums) decodes every block's
 * delta sum and prefix-sums them into the workspace; phase B (chain_decode)
 * decodes with start(i) = base + prefix(i-1).  tpf_p4d1dec256v32_chained = A+B
 * with base = start0.  For a list sharded over GPUs, each rank runs A, the
 * ranks exchange their totals (d_total, one u32 each) and each runs B with
 * base = start0 + the totals of all earlier shards (mod 2^32). */
size_t tpf_p4d1dec256v32_chain_workspace_size(uint64_t nblocks);
int tpf_p4d1dec256v32_chained(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nblocks,
                              uint32_t *d_out, uint32_t start0, void *d_ws, size_t ws_bytes, uint64_t *d_err,
                              void *stream);
int tpf_p4d1dec256v32_chain_sums(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nblocks,
                                 void *d_ws, size_t ws_bytes, uint32_t *d_total, uint64_t *d_err, void *stream);
int tpf_p4d1dec256v32_chain_decode(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nblocks,
                                   uint32_t *d_out, uint32_t base, const void *d_ws, uint64_t *d_err, void *stream);

/* ---- 64-bit chained delta-1 decode (128v64 / 256v64) --------------------
 * The 64-bit counterpart of the chained 256v32 decode: nunits consecutive
 * p4D1Enc256v64 (fmt TPF_FMT_256V64, 256 values per unit) or p4D1Enc128v64
 * (TPF_FMT_128V64, 128) units chained the way reference callers chain them
 * (start of unit i = last value of unit i-1, README.md:116-123; reference
 * decoder p4d1dec256v64_scalar.cpp:15-32, which carries the start across its
 * two 128-value blocks the same way).  Phase A (chain_sums) decodes every
 * unit's delta total sum(v + 1) mod 2^64 and prefix-sums them into the
 * workspace; phase B (chain_decode) decodes with start(i) = base + the totals
 * before i.  tpf_d1dec64_chained = A + B with base = start0; for a sharded list
 * exchange the d_total of each shard (one u64) as for 256v32.  d_out: nunits *
 * 128 * (1 or 2) u64. */
size_t tpf_d1dec64_chain_workspace_size(uint64_t nunits);
int tpf_d1dec64_chained(int fmt, const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nunits,
                        uint64_t *d_out, uint64_t start0, void *d_ws, size_t ws_bytes, uint64_t *d_err, void *stream);
int tpf_d1dec64_chain_sums(int fmt, const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nunits,
                           void *d_ws, size_t ws_bytes, uint64_t *d_total, uint64_t *d_err, void *stream);
int tpf_d1dec64_chain_decode(int fmt, const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nunits,
                             uint64_t *d_out, uint64_t base, const void *d_ws, uint64_t *d_err, void *stream);
/* Named forms: replace a caller's loop of turbopfor::p4D1Dec256v64 /
 * p4D1Dec128v64 calls (include/turbopfor.h:80,67) over one chained list. */
int tpf_p4d1dec256v64_chained(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nunits,
                              uint64_t *d_out, uint64_t start0, void *d_ws, size_t ws_bytes, uint64_t *d_err, void *stream);
int tpf_p4d1dec128v64_chained(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nunits,
                              uint64_t *d_out, uint64_t start0, void *d_ws, size_t ws_bytes, uint64_t *d_err, void *stream);

/* ---- 256v32 encode ---------------------------------------------------
 * Replaces turbopfor::p4Enc256v32 (include/turbopfor.h:33, dispatch.cpp:70-77)
 * and p4D1Enc256v32 (:36, dispatch.cpp:79-86) for nblocks blocks of 256
 * values (d_in: nblocks*256 u32).  Writes the blocks end to end into d_out
 * (capacity out_cap bytes, at least tpf_p4enc256v32_bound(nblocks): the
 * sizes are only known on the device, so a smaller out_cap is rejected with
 * TPF_EINVAL instead of risking a silently cut-off block)
 * and their byte offsets into d_off[0..nblocks] (d_off[nblocks] = total).
 * d_ws: device workspace of tpf_p4enc256v32_workspace_size(nblocks) bytes.
 * D1: d_starts[i] is the value preceding block i; with d_starts == NULL the
 * blocks are one chained posting list: block 0 starts from start0 and block
 * i>0 from the last input value of block i-1. */
uint64_t tpf_p4enc256v32_bound(uint64_t nblocks);
size_t tpf_p4enc256v32_workspace_size(uint64_t nblocks);
int tpf_p4enc256v32_batch(const uint32_t *d_in, uint64_t nblocks, uint8_t *d_out, uint64_t out_cap, uint64_t *d_off,
                          void *d_ws, size_t ws_bytes, void *stream);
int tpf_p4d1enc256v32_batch(const uint32_t *d_in, uint64_t nblocks, const uint32_t *d_starts, uint32_t start0,
                            uint8_t *d_out, uint64_t out_cap, uint64_t *d_off, void *d_ws, size_t ws_bytes, void *stream);

/* ---- every format of include/turbopfor.h, batched ----------------------
 * fmt selects the reference function family:
 *   TPF_FMT_32     p4{,D1}{Enc,Dec}32      (turbopfor.h:9-18)   n = 1..256 values per block
 *   TPF_FMT_128V32 p4{,D1}{Enc,Dec}128v32  (turbopfor.h:21-30)  n <= 128
 *   TPF_FMT_256V32 p4{,D1}{Enc,Dec}256v32  (turbopfor.h:33-42)  n <= 256 (n == 256 -> hot path)
 *   TPF_FMT_64     p4{,D1}{Enc,Dec}64      (turbopfor.h:45-54)  n = 1..256 (uint64)
 *   TPF_FMT_128V64 p4{,D1}{Enc,Dec}128v64  (turbopfor.h:57-67)  n <= 128 (uint64)
 *   TPF_FMT_256V64 p4{,D1}{Enc,Dec}256v64  (turbopfor.h:69-80)  n == 256 (uint64; one unit = two 128v64 blocks;
 *                  the per-block turbopfor::p4*256v64 calls take any n and split it into 128v64 blocks
 *                  of min(remaining, 128) values like the reference, p4enc256v64_scalar.cpp:15-30)
 * A batch holds nblocks units; unit i's values are at d_vals + i*stride with
 * stride = n for the horizontal formats and the layout's full width (128 or
 * 256) for the interleaved ones (the reference packs the full width).
 * Values are uint32 or uint64 as the family requires.  D1 (delta-1): starts
 * per unit, or NULL = one chained list (encode: start0 then the previous
 * unit's last input; decode requires starts). */
#define TPF_FMT_32 0
#define TPF_FMT_128V32 1
#define TPF_FMT_256V32 2
#define TPF_FMT_64 3
#define TPF_FMT_128V64 4
#define TPF_FMT_256V64 5

/* tpf_enc_batch requires out_cap >= tpf_enc_bound(fmt, nblocks, n) (TPF_EINVAL otherwise).
 * tpf_dec_batch reports through d_err (first such block index) any block whose
 * parse disagrees with its offsets; for TPF_FMT_32 (the windowed decoder) also
 * any block whose offsets span more than 2,544 bytes or run past in_bytes --
 * a p4Enc32 block of n <= 256 values is at most about 1 KB. */
uint64_t tpf_enc_bound(int fmt, uint64_t nblocks, unsigned n);
size_t tpf_enc_workspace_size(int fmt, uint64_t nblocks, unsigned n);
int tpf_dec_batch(int fmt, const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nblocks, unsigned n,
                  void *d_vals, const void *d_starts, uint64_t *d_err, void *stream);
int tpf_enc_batch(int fmt, const void *d_vals, uint64_t nblocks, unsigned n, int d1, const void *d_starts, uint64_t start0,
                  uint8_t *d_out, uint64_t out_cap, uint64_t *d_off, void *d_ws, size_t ws_bytes, void *stream);

/* ---- n-variant streams --------------------------------
 * n values of any count as floor(n/256) p4Enc256v32 blocks followed, when
 * n % 256 != 0, by one p4Enc32 block of the remaining values: the stream a
 * caller produces by chaining turbopfor::p4Enc256v32 over the full blocks
 * and turbopfor::p4Enc32 over the tail (reference include/turbopfor.h:9,
 * :33; D1: p4D1Enc256v32 / p4D1Enc32 with each block's start = the value
 * before it, the first = start0).  d_off receives nunits + 1 byte offsets
 * (nunits = n/256 + (n%256 != 0)); d_off[nunits] is the stream's length.
 * Decode takes the same offsets (tpf_scan_offsets of the parts, or the
 * encoder's) and writes exactly n values. */
uint64_t tpf_p4nenc256v32_bound(uint64_t n);
size_t tpf_p4nenc256v32_workspace_size(uint64_t n);
int tpf_p4nenc256v32(const uint32_t *d_in, uint64_t n, int d1, uint32_t start0, uint8_t *d_out, uint64_t out_cap,
                     uint64_t *d_off, void *d_ws, size_t ws_bytes, void *stream);
size_t tpf_p4ndec256v32_workspace_size(uint64_t n);
int tpf_p4ndec256v32(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t n, int d1, uint32_t start0,
                     uint32_t *d_out, void *d_ws, size_t ws_bytes, uint64_t *d_err, void *stream);

/* ---- host pipeline utility ----------------------------------------------
 * Copies `bytes` bytes with a kernel (16-byte non-temporal stores) instead of
 * an SDMA engine; either side may be pinned/registered host memory, at any
 * byte alignment.  The tpf_host_* pipelines use it for downloads under
 * TPF_HOST_DOWN=kernel (SDMA is their default: faster on MI355X). */
int tpf_copy_async(void *dst, const void *src, uint64_t bytes, void *stream);

#ifdef __cplusplus
}
#endif
#endif
