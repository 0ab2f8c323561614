/* tpf_measure.h -- the measurement and test library (lib/libtpf_measure.so).
 *
 * NOT part of the codec's interface (include/ holds that): bench.py, the GPU
 * tests and scripts/ load this library beside libturbopfor_amd.so for the
 * data-movement probes of the kernels, the device's own streaming ceilings,
 * forced encoder paths for A/B runs and the run-scan test hook.  It is built
 * from the same kernel headers as the codec (csrc/ headers), so a probe runs the
 * very load / store code of the kernel it is compared against, and links the
 * codec library for the shared launch helpers.  All functions return 0 on
 * success, -1 on a bad argument, or the hipError_t of a failed launch; all
 * pointers are device pointers, stream a hipStream_t (NULL = default). */
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The 256v32 decode kernel's exact load and store pattern with the decoding
 * removed (k_dec256v32w<Probe>): block i's staged bytes are written to
 * d_out[256*i..] unchanged.  The data-movement ceiling bench.py compares the
 * decoder with. */
// the plain 256v32 decode through a forced load path: grouped = 0 single-block
// pipeline, 1 grouped 1 KB loads (the library picks one per launch)
int tpfm_dec256v32_path(int grouped, const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nblocks, uint32_t *d_out,
                        void *stream);
int tpfm_probe256v32(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nblocks, uint32_t *d_out,
                     void *stream);

/* The same for the 256v64 decoder (nunits units at d_off; each unit's first
 * staged bytes written to both 1 KB halves of its 2 KB output). */
int tpfm_probe256v64(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_off, uint64_t nunits, uint64_t *d_out,
                     void *stream);

/* Streaming ceilings of the device: kind 0 = read `bytes` of d_src (d_dst
 * gets at most one 16-byte sink word), 1 = write `bytes` to d_dst, 2 = copy;
 * 16-byte lanes, non-temporal, grid-stride.  bytes is rounded down to 16. */
int tpfm_probe_hbm(int kind, void *d_dst, const void *d_src, uint64_t bytes, void *stream);

/* 256v32 encoder paths, arguments as tpf_p4d1enc256v32_batch (d1 = 0: plain;
 * d1 = 1 with d_starts NULL: one chained list from start0):
 *   mode 1 = the two-pass encoder's plan pass reduced to a wave OR, 2 = its
 *            write pass copying the staged values (plain only; the output is
 *            NOT a valid stream): each pass's data-movement ceiling;
 *   mode 3 = the two-pass encoder (plan, run scan, write);
 *   mode 4 = the slot encoder (plan + build into per-run slots, run scan,
 *            compaction: measured and not adopted, enc_slot.h);
 *   mode 5 = the slot encoder without the fused plan/build scans.
 * d_ws: tpfm_enc256v32_workspace_size(mode, nblocks) bytes. */
size_t tpfm_enc256v32_workspace_size(int mode, uint64_t nblocks);
int tpfm_enc256v32(int mode, const uint32_t *d_in, uint64_t nblocks, int d1, const uint32_t *d_starts, uint32_t start0,
                   uint8_t *d_out, uint64_t out_cap, uint64_t *d_off, void *d_ws, size_t ws_bytes, void *stream);

/* The run scan every two-pass kernel pair uses between its passes
 * (p4_scan.h): d_tot holds nruns u32 totals; writes d_base[r] = sum of
 * d_tot[0..r) (u64, exclusive) and *d_total = the sum of all. */
size_t tpfm_run_scan_workspace_size(uint64_t nruns);
int tpfm_run_scan(const uint32_t *d_tot, uint64_t nruns, uint64_t *d_base, uint64_t *d_total, void *d_ws, size_t ws_bytes,
                  void *stream);

#ifdef __cplusplus
}
#endif
