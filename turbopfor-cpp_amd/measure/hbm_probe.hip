// hbm_probe.hip -- measurement-library streaming kernels (no reference
// counterpart; not in the codec library): the box's own HBM ceilings, timed inside bench.py in the same
// process as the codec so the line's "ceiling" numbers are measured in-run.
//
//   kind 0  read : every lane XOR-folds 16-byte non-temporal loads (a sink
//                  word in dst keeps the loads alive)
//   kind 1  write: 16-byte non-temporal stores of a constant
//   kind 2  copy : 16-byte loads, 16-byte non-temporal stores
//
// Grid-stride over 16-byte vectors, 256-thread workgroups, 128 workgroups per
// CU (the best of 32/128 per CU in scripts/hbm_probe.hip,
// profiles/archive/r1/r1_v3_hbm_probes.txt).
#include <hip/hip_runtime.h>

#include "../csrc/tpf_device.h"
#include "../csrc/tpf_kernels.h"
#include "tpf_measure.h"

namespace tpf::dev
{

__global__ __launch_bounds__(256) void k_probe_read(const u32x4 * __restrict__ a, uint64_t n, u32x4 * __restrict__ sink)
{
    u32x4 acc{0u, 0u, 0u, 0u};
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
        acc ^= __builtin_nontemporal_load(a + i);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) // data-dependent, practically never taken
        sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_probe_write(u32x4 * __restrict__ b, uint64_t n)
{
    const u32x4 v{1u, 2u, 3u, 4u};
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(v, b + i);
}

__global__ __launch_bounds__(256) void k_probe_copy(const u32x4 * __restrict__ a, u32x4 * __restrict__ b, uint64_t n)
{
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(a[i], b + i);
}

} // namespace tpf::dev

namespace tpfm
{

hipError_t launch_probe_hbm(int kind, void * dst, const void * src, uint64_t bytes, hipStream_t s)
{
    using tpf::grid_cap;
    namespace dev = tpf::dev;
    const uint64_t n = bytes / 16u;
    if (n == 0)
        return hipSuccess;
    const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(grid_cap(s, 128), (n + 255u) / 256u));
    switch (kind)
    {
        case 0:
            hipLaunchKernelGGL(dev::k_probe_read, dim3(grid), dim3(256), 0, s, static_cast<const dev::u32x4 *>(src), n,
                               static_cast<dev::u32x4 *>(dst));
            break;
        case 1:
            hipLaunchKernelGGL(dev::k_probe_write, dim3(grid), dim3(256), 0, s, static_cast<dev::u32x4 *>(dst), n);
            break;
        case 2:
            hipLaunchKernelGGL(dev::k_probe_copy, dim3(grid), dim3(256), 0, s, static_cast<const dev::u32x4 *>(src),
                               static_cast<dev::u32x4 *>(dst), n);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

} // namespace tpfm
