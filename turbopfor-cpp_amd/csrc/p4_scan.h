// p4_scan.h -- offsets of variable-size units without a device-wide scan of
// every unit (internal).
//
// Every two-pass kernel pair here works in wave runs of a fixed number of
// units.  The first pass leaves each unit's size in place (the encoders: in
// d_off[unit]; the chained decode: in its block-sum array) and ONE total per
// run in run_tot[run].  Two small kernels then scan only the run totals
// (p4_scan.hip): 16 x fewer entries than units, 4096 per workgroup tile,
// then the tile totals in one workgroup.  The second pass rebuilds each
// unit's offset from its run's base and a wave scan of its own run's sizes,
// and (encoders) writes the final offset back over the size.  This replaces
// a library device scan over every unit (two launches reading and writing
// 8 B per unit) between the passes.
#pragma once

#include "tpf_device.h"

namespace tpf::dev
{

constexpr uint32_t kScanTile = 4096; // run totals per workgroup of k_run_scan_tiles (256 threads x 16)

// First pass: this wave's run total (lanes >= the run's length pass 0).
__device__ __forceinline__ void publish_run_total(uint32_t * __restrict run_tot, uint64_t run, uint32_t size_or_zero, uint32_t t)
{
    const uint32_t s = wave_sum(size_or_zero);
    if (t == 0)
        run_tot[run] = s;
}

// Second pass: base of `run` = exclusive prefix of the run totals.
template <class T>
__device__ __forceinline__ T run_base(const T * __restrict pre, const T * __restrict tile, uint64_t run)
{
    return tile[run / kScanTile] + pre[run];
}

// Second pass of an encoder: lane t < n gets the byte offset of unit
// first+t (and its size) from the size the first pass left in off[first+t],
// and stores the offset there (each run owns its own entries).
__device__ __forceinline__ void run_offsets(uint64_t * __restrict off, uint64_t first, uint32_t n, uint64_t base, uint32_t t,
                                            uint64_t & ov, uint64_t & ev)
{
    const uint32_t sz = t < n ? static_cast<uint32_t>(off[first + t]) : 0u;
    const uint32_t incl = wave_incl_scan(sz); // a run's bytes fit 32 bits
    ov = base + (incl - sz);
    ev = ov + sz;
    if (t < n)
        off[first + t] = ov;
}

} // namespace tpf::dev

namespace tpf
{

// Workspace of the run scan: run totals (u32), in-tile prefixes and tile
// totals (T), each 256-byte aligned.
template <class T>
struct RunScanWs
{
    uint32_t * tot = nullptr;
    T * pre = nullptr;
    T * tile = nullptr;

    static size_t al(size_t x) { return (x + 255u) & ~size_t(255); }
    static uint64_t tiles(uint64_t nruns) { return (nruns + dev::kScanTile - 1u) / dev::kScanTile; }
    static size_t bytes(uint64_t nruns) { return al(4u * nruns) + al(sizeof(T) * nruns) + al(sizeof(T) * tiles(nruns)) + 256u; }
    static RunScanWs carve(void * ws, uint64_t nruns)
    {
        RunScanWs w;
        auto * p = static_cast<uint8_t *>(ws);
        w.tot = reinterpret_cast<uint32_t *>(p);
        p += al(4u * nruns);
        w.pre = reinterpret_cast<T *>(p);
        p += al(sizeof(T) * nruns);
        w.tile = reinterpret_cast<T *>(p);
        return w;
    }
};

// pre[r] = sum of tot[0..r) within r's tile, tile[k] = sum of the tiles
// before k (so run_base = tile[r / kScanTile] + pre[r]); *total (optional) =
// sum of all run totals.  T = uint64_t: byte offsets; uint32_t: sums mod 2^32.
hipError_t launch_run_scan_u64(const uint32_t * tot, uint64_t nruns, uint64_t * pre, uint64_t * tile, uint64_t * total, hipStream_t s);
hipError_t launch_run_scan_u32(const uint32_t * tot, uint64_t nruns, uint32_t * pre, uint32_t * tile, uint32_t * total, hipStream_t s);
// u64 run totals (the 64-bit chained decode's unit sums, mod 2^64)
hipError_t launch_run_scan_u64t(const uint64_t * tot, uint64_t nruns, uint64_t * pre, uint64_t * tile, uint64_t * total, hipStream_t s);

} // namespace tpf
