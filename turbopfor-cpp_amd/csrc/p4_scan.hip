// p4_scan.hip -- the run-total scan of p4_scan.h: two small kernels over one
// entry per wave run (10M units in runs of 16: 625K entries, 153 tiles).
#include "p4_scan.h"
#include "tpf_kernels.h"

namespace tpf::dev
{

template <class T>
__device__ __forceinline__ T wave_incl_scan_t(T x)
{
    if constexpr (sizeof(T) == 8)
        return wave_incl_scan64(x);
    else
        return wave_incl_scan(x);
}

template <class T>
__device__ __forceinline__ T readlane_t(T x, uint32_t l)
{
    if constexpr (sizeof(T) == 8)
        return readlane_u64(x, l);
    else
        return static_cast<T>(__builtin_amdgcn_readlane(static_cast<int>(x), static_cast<int>(l)));
}

// Tile k = run totals [k*4096, (k+1)*4096): thread i sums its 16 consecutive
// entries serially, the 256 thread sums are scanned (wave scans + 4 wave
// totals in LDS); pre[] = exclusive prefix inside the tile, tile[k] = total.
template <class T, class TT>
__global__ __launch_bounds__(256) void k_run_scan_tiles(const TT * __restrict tot, uint64_t nruns, T * __restrict pre,
                                                         T * __restrict tile)
{
    __shared__ T wsum[4];
    const uint32_t t = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kScanTile + 16u * threadIdx.x;
    T v[16];
    T s = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k)
    {
        const T x = b + k < nruns ? static_cast<T>(tot[b + k]) : T(0);
        v[k] = s;
        s += x;
    }
    const T incl = wave_incl_scan_t<T>(s);
    if (t == 63u)
        wsum[w] = incl;
    __syncthreads();
    T wb = 0;
    for (uint32_t k = 0; k < w; ++k)
        wb += wsum[k];
    const T ex = wb + incl - s;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k)
        if (b + k < nruns)
            pre[b + k] = ex + v[k];
    if (threadIdx.x == 255u)
        tile[blockIdx.x] = wb + incl;
}

// One workgroup: exclusive scan of the tile totals in place, 1024 per step
// with a running carry; *total = the sum of everything.
template <class T>
__global__ __launch_bounds__(1024) void k_run_scan_tops(T * __restrict tile, uint64_t ntiles, T * __restrict total)
{
    __shared__ T wsum[16];
    const uint32_t t = threadIdx.x & 63u, w = threadIdx.x >> 6;
    T carry = 0;
    for (uint64_t c = 0; c < ntiles; c += 1024u)
    {
        const uint64_t i = c + threadIdx.x;
        const T x = i < ntiles ? tile[i] : T(0);
        const T incl = wave_incl_scan_t<T>(x);
        if (t == 63u)
            wsum[w] = incl;
        __syncthreads();
        T wb = 0, all = 0;
        for (uint32_t k = 0; k < 16; ++k)
        {
            wb += k < w ? wsum[k] : T(0);
            all += wsum[k];
        }
        if (i < ntiles)
            tile[i] = carry + wb + incl - x;
        carry += all;
        __syncthreads(); // wsum is rewritten by the next step
    }
    if (threadIdx.x == 0 && total != nullptr)
        *total = carry;
}

} // namespace tpf::dev

namespace tpf
{

namespace
{
template <class T, class TT = uint32_t>
hipError_t run_scan(const TT * tot, uint64_t nruns, T * pre, T * tile, T * total, hipStream_t s)
{
    if (nruns == 0)
        return total ? fill_u32(total, 0u, sizeof(T) / 4u, s) : hipSuccess;
    const uint64_t ntiles = RunScanWs<T>::tiles(nruns);
    hipLaunchKernelGGL((dev::k_run_scan_tiles<T, TT>), dim3(static_cast<uint32_t>(ntiles)), dim3(256), 0, s, tot, nruns, pre, tile);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return e;
    hipLaunchKernelGGL(dev::k_run_scan_tops<T>, dim3(1), dim3(1024), 0, s, tile, ntiles, total);
    return hipGetLastError();
}
} // namespace

hipError_t launch_run_scan_u64(const uint32_t * tot, uint64_t nruns, uint64_t * pre, uint64_t * tile, uint64_t * total, hipStream_t s)
{
    return run_scan<uint64_t>(tot, nruns, pre, tile, total, s);
}

hipError_t launch_run_scan_u64t(const uint64_t * tot, uint64_t nruns, uint64_t * pre, uint64_t * tile, uint64_t * total, hipStream_t s)
{
    return run_scan<uint64_t, uint64_t>(tot, nruns, pre, tile, total, s);
}

hipError_t launch_run_scan_u32(const uint32_t * tot, uint64_t nruns, uint32_t * pre, uint32_t * tile, uint32_t * total, hipStream_t s)
{
    return run_scan<uint32_t>(tot, nruns, pre, tile, total, s);
}

} // namespace tpf
