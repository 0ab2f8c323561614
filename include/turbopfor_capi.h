/*
 * turbopfor_capi.h -- extern "C" mirror of the reference's per-block API plus
 * host-memory stream entry points.  This is the surface a foreign-language
 * binding (cgo, JNI, N-API, ctypes) binds: plain C types, C linkage, one symbol
 * per reference function.  See INTEGRATION.md.
 *
 * tpf_<name>(...) has exactly the argument meaning and return value of
 * turbopfor::<name>(...) in the reference's include/turbopfor.h (line cited
 * per family).  On failure (no HIP device, HIP error) these return NULL and
 * tpf_last_error() describes why; they never fall back to a CPU codec.
 */
#ifndef TURBOPFOR_CAPI_H
#define TURBOPFOR_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char *tpf_last_error(void);

/* reference include/turbopfor.h:9-18 */
unsigned char *tpf_p4Enc32(uint32_t *in, unsigned n, unsigned char *out);
unsigned char *tpf_p4D1Enc32(uint32_t *in, unsigned n, unsigned char *out, uint32_t start);
const unsigned char *tpf_p4Dec32(const unsigned char *in, unsigned n, uint32_t *out);
const unsigned char *tpf_p4D1Dec32(const unsigned char *in, unsigned n, uint32_t *out, uint32_t start);
/* :21-30 */
unsigned char *tpf_p4Enc128v32(uint32_t *in, unsigned n, unsigned char *out);
unsigned char *tpf_p4D1Enc128v32(uint32_t *in, unsigned n, unsigned char *out, uint32_t start);
const unsigned char *tpf_p4Dec128v32(const unsigned char *in, unsigned n, uint32_t *out);
const unsigned char *tpf_p4D1Dec128v32(const unsigned char *in, unsigned n, uint32_t *out, uint32_t start);
/* :33-42 (hot path) */
unsigned char *tpf_p4Enc256v32(uint32_t *in, unsigned n, unsigned char *out);
unsigned char *tpf_p4D1Enc256v32(uint32_t *in, unsigned n, unsigned char *out, uint32_t start);
const unsigned char *tpf_p4Dec256v32(const unsigned char *in, unsigned n, uint32_t *out);
const unsigned char *tpf_p4D1Dec256v32(const unsigned char *in, unsigned n, uint32_t *out, uint32_t start);
/* :45-54 */
unsigned char *tpf_p4Enc64(uint64_t *in, unsigned n, unsigned char *out);
unsigned char *tpf_p4D1Enc64(uint64_t *in, unsigned n, unsigned char *out, uint64_t start);
const unsigned char *tpf_p4Dec64(const unsigned char *in, unsigned n, uint64_t *out);
const unsigned char *tpf_p4D1Dec64(const unsigned char *in, unsigned n, uint64_t *out, uint64_t start);
/* :57-67 */
unsigned char *tpf_p4Enc128v64(uint64_t *in, unsigned n, unsigned char *out);
unsigned char *tpf_p4D1Enc128v64(uint64_t *in, unsigned n, unsigned char *out, uint64_t start);
const unsigned char *tpf_p4Dec128v64(const unsigned char *in, unsigned n, uint64_t *out);
const unsigned char *tpf_p4D1Dec128v64(const unsigned char *in, unsigned n, uint64_t *out, uint64_t start);
/* :69-80 */
unsigned char *tpf_p4Enc256v64(uint64_t *in, unsigned n, unsigned char *out);
unsigned char *tpf_p4D1Enc256v64(uint64_t *in, unsigned n, unsigned char *out, uint64_t start);
const unsigned char *tpf_p4Dec256v64(const unsigned char *in, unsigned n, uint64_t *out);
const unsigned char *tpf_p4D1Dec256v64(const unsigned char *in, unsigned n, uint64_t *out, uint64_t start);

/* How the per-block calls above reach the GPU (identical bytes either way):
 * 0 (default) = a resident block server kernel (no launch per call; it exits
 * after 10 ms without calls and is relaunched on the next one) whose request
 * mailboxes sit in fine-grained device memory the host writes through the
 * BAR, answers in pinned host memory; 2 = the same server with the request
 * mailboxes in pinned host memory (the kernel polls across PCIe); 1 = one
 * batched launch plus a stream synchronise per call.  mode < 0 only queries.
 * Switch between calls, not while a per-block call is in flight.  Returns
 * the previous mode. */
int tpf_perblock_mode(int mode);

/* Stops the resident block server on every device (the next per-block call
 * relaunches it).  The server kernel occupies a stream of its own until it
 * idles out (10 ms without calls), and HIP's hipDeviceSynchronize, hipFree
 * and hipHostFree wait for every stream of the device: a caller about to do
 * one of those right after per-block calls calls this first to avoid that
 * wait.  The host streams do so themselves around their own allocations and
 * frees (only there: host streams of different threads run concurrently).  Mode 0 needs a large BAR
 * (VRAM mapped into the CPU's address space); without one the server uses the
 * host-memory mailboxes of mode 2. */
void tpf_perblock_quiesce(void);

/* Diagnostics: launches of the block server since the process started (every
 * device).  A launch serves until it has been idle for 10 ms, or for 5 ms of
 * service at most; calls/launch shows whether it leaves early. */
uint64_t tpf_perblock_launches(void);

/* ---- stream framing (host, no decoding) -------------------
 * Encoded length of the block at `in` (fmt = TPF_FMT_*, n = values per call),
 * reading at most `avail` bytes; 0 if malformed/truncated.  values_written
 * (optional) receives how many values the reference decoder stores (n for a
 * constant block, else the layout's full width). */
uint64_t tpf_block_size(int fmt, const uint8_t *in, uint64_t avail, unsigned n, int *values_written);
/* Offsets of nblocks consecutive blocks (off[nblocks] = total).  Returns the
 * total byte length, or -(i+1) if block i is malformed/truncated. */
int64_t tpf_scan_offsets(int fmt, const uint8_t *in, uint64_t in_bytes, unsigned n, uint64_t nblocks, uint64_t *off);
/* Caller-supplied offsets (off[0..nblocks]): 0 when they never decrease and
 * off[nblocks] <= in_bytes; -(i+1) when off[i] > off[i+1]; -(nblocks+1) when
 * the last offset is past in_bytes (-1 for a NULL array).  The host streams
 * run this before any copy. */
int64_t tpf_check_offsets(const uint64_t *off, uint64_t nblocks, uint64_t in_bytes);

/* ---- host-memory streams (end-to-end path) ----------------
 * Decode / encode nblocks blocks whose bytes and values live in HOST memory:
 * the work is split into chunks that are copied to HBM, processed and copied
 * back, the upload of chunk k+1 overlapping the kernel and the download of
 * chunk k (a copy stream and a kernel stream).  Host buffers allocated with
 * hipHostMalloc (or registered by the caller) are used as they are (full PCIe
 * rate); pageable buffers are staged through the pipeline's pinned buffers by
 * host copies -- the library never page-locks caller memory.  Staging buffers and
 * streams are pooled per device across calls; tpf_host_release() frees them.
 * h_off may be NULL for decode (offsets are scanned with tpf_scan_offsets);
 * given offsets have nblocks + 1 readable entries (the length cannot be
 * checked: a shorter array is an out-of-bounds host read), must not decrease
 * and must end at or below in_bytes (TPF_EINVAL otherwise, checked on the host
 * before any device is touched), and a block whose parsed length disagrees
 * with its offsets fails the call with TPF_ECORRUPT (tpf_last_error names the
 * block).  Encode writes nblocks + 1 entries to h_off.
 * Encode fails with TPF_EINVAL when the blocks do not fit in out_cap.
 * Value arrays use the unit strides documented in turbopfor_gpu.h. */
int tpf_host_dec(int fmt, const uint8_t *h_in, uint64_t in_bytes, const uint64_t *h_off, uint64_t nblocks, unsigned n,
                 void *h_vals, const void *h_starts);
int tpf_host_enc(int fmt, const void *h_vals, uint64_t nblocks, unsigned n, int d1, const void *h_starts, uint64_t start0,
                 uint8_t *h_out, uint64_t out_cap, uint64_t *h_off);
void tpf_host_release(void);
/* Decode one host stream on several GPUs at once: the blocks are cut into ndev
 * contiguous shards of about equal bytes and shard d runs tpf_host_dec's
 * pipeline on device devs[d] from its own thread (each GPU brings its own
 * PCIe link).  Arguments and checks as tpf_host_dec; a failing shard's
 * message names the shard (its block numbers are shard-relative).  devs may
 * repeat a device (two pipelines on one GPU). */
int tpf_host_dec_multi(const int *devs, int ndev, int fmt, const uint8_t *h_in, uint64_t in_bytes, const uint64_t *h_off,
                       uint64_t nblocks, unsigned n, void *h_vals, const void *h_starts);
/* Encode one host array on several GPUs at once: the blocks are cut into ndev
 * contiguous shards of equal block counts and shard d runs tpf_host_enc's
 * pipeline on device devs[d] from its own thread.  Shard 0 writes straight
 * into h_out; the others into pooled host staging, moved into place (and
 * their offsets rebased) once the sizes before them are known.  The bytes
 * and offsets are identical to tpf_host_enc's (a chained D1 list continues
 * across shard cuts: each shard starts from the value before its first
 * block).  Arguments and checks as tpf_host_enc. */
int tpf_host_enc_multi(const int *devs, int ndev, int fmt, const void *h_vals, uint64_t nblocks, unsigned n, int d1,
                       const void *h_starts, uint64_t start0, uint8_t *h_out, uint64_t out_cap, uint64_t *h_off);

#ifdef __cplusplus
}
#endif
#endif
