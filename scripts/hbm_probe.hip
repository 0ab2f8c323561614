// hbm_probe.hip -- standalone data-movement ceilings on this box (measurement
// tool, not part of the library): grid-stride read-only, write-only and copy
// streams of 16-byte lanes, and a write-heavy mix with the decode's 0.6:1
// read:write ratio.  Build: hipcc --offload-arch=gfx950 -O3 -o hbm_probe hbm_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_read(const u32x4 * __restrict__ a, size_t n, u32x4 * sink)
{
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= __builtin_nontemporal_load(a + i);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u)
        sink[0] = acc;
}

__global__ void k_write(u32x4 * __restrict__ b, size_t n, int nt)
{
    const u32x4 v = {1, 2, 3, 4};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (nt)
            __builtin_nontemporal_store(v, b + i);
        else
            b[i] = v;
}

template <int AUX>
__global__ void k_write_aux(u32x4 * __restrict__ b, size_t n)
{
    const u32x4 v = {1, 2, 3, 4};
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(b, 0, 0x7FFFFFFF, 0x00020000);
    const size_t per = 0x7FFFFFF0 / 16;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n && i < per; i += (size_t)gridDim.x * blockDim.x)
        __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(i * 16), 0, AUX);
}

__global__ void k_copy(const u32x4 * __restrict__ a, u32x4 * __restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(a[i], b + i);
}

// read 0.6 KB, write 1 KB per "block", per-wave contiguous runs like the decoder
__global__ void k_mix(const u32x4 * __restrict__ a, u32x4 * __restrict__ b, size_t nblk)
{
    const uint32_t t = threadIdx.x & 63u;
    const size_t w = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t W = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t blk = w; blk < nblk; blk += W)
    {
        u32x4 v = {0, 0, 0, 0};
        if (t < 38)
            v = a[blk * 38 + t];
        __builtin_nontemporal_store(v, b + blk * 64 + t);
    }
}

int main()
{
    const size_t bytes = 4ull << 30;
    const size_t n = bytes / 16;
    u32x4 *a, *b, *sink;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMalloc(&sink, 64);
    hipMemset(a, 1, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int grid : {8192, 32768})
    {
        float ms;
        auto run = [&](const char * name, double moved, auto launch) {
            for (int i = 0; i < 3; ++i)
                launch();
            hipEventRecord(e0);
            for (int i = 0; i < 10; ++i)
                launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            printf("grid %6d %-10s %8.1f GB/s\n", grid, name, moved * 10 / (ms * 1e-3) / 1e9);
        };
        run("read", (double)bytes, [&] { k_read<<<grid, 256>>>(a, n, sink); });
        run("write", (double)bytes, [&] { k_write<<<grid, 256>>>(b, n, 0); });
        run("write_nt", (double)bytes, [&] { k_write<<<grid, 256>>>(b, n, 1); });
        run("copy", 1.0 * bytes, [&] { k_copy<<<grid, 256>>>(a, b, n / 2); });
        const double wb = (double)(0x7FFFFFF0 / 16) * 16;
        run("w_aux0", wb, [&] { k_write_aux<0><<<grid, 256>>>(b, n); });
        run("w_aux1", wb, [&] { k_write_aux<1><<<grid, 256>>>(b, n); });
        run("w_aux2", wb, [&] { k_write_aux<2><<<grid, 256>>>(b, n); });
        run("w_aux3", wb, [&] { k_write_aux<3><<<grid, 256>>>(b, n); });
        run("w_aux16", wb, [&] { k_write_aux<16><<<grid, 256>>>(b, n); });
        run("w_aux17", wb, [&] { k_write_aux<17><<<grid, 256>>>(b, n); });
        run("w_aux18", wb, [&] { k_write_aux<18><<<grid, 256>>>(b, n); });
        run("w_aux19", wb, [&] { k_write_aux<19><<<grid, 256>>>(b, n); });
        const size_t nblk = bytes / 1024;
        run("mix0.6", (double)nblk * (608 + 1024), [&] { k_mix<<<grid, 256>>>(a, b, nblk); });
    }
    return 0;
}
