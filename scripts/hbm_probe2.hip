// hbm_probe2.hip -- data-movement ceilings shaped like the 256v32 decode
// (measurement tool, not part of the library).  Per "block": read R packed
// bytes (contiguous stream, blocks back to back), write 1 KB of output.  Each
// wave owns a run of 16 consecutive blocks, as k_dec256v32w does.
//   blk   : per block, lanes t < ceil(R/16) issue one 16 B load (the decode's shape)
//   run   : the run's 16*R bytes read with full-wave 16 B loads, then 16 x 1 KB stores
//   wonly : stores only (write ceiling of the same grid)
// Build: hipcc --offload-arch=gfx950 -O3 -o hbm_probe2 hbm_probe2.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE, int NT>
__global__ __launch_bounds__(256) void k_probe(const u32x4 * __restrict__ a, u32x4 * __restrict__ b, size_t nblk, uint32_t R16)
{
    const uint32_t t = threadIdx.x & 63u;
    const size_t run = (blockIdx.x * 4ull + (threadIdx.x >> 6));
    const size_t first = run * 16u;
    if (first >= nblk)
        return;
    u32x4 acc = {t, 0, 0, 0};
    if (MODE == 0)
    {
        u32x4 v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j)
            v[j] = t < R16 ? a[(first + j) * R16 + t] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 16; ++j)
        {
            if (NT)
                __builtin_nontemporal_store(v[j] ^ acc, b + (first + j) * 64 + t);
            else
                b[(first + j) * 64 + t] = v[j] ^ acc;
        }
    }
    else if (MODE == 1)
    {
        const uint32_t n16 = 16u * R16; // 16-byte words in the run
        u32x4 x = acc;
        for (uint32_t i = t; i < n16; i += 64u)
            x ^= a[first * R16 + i];
#pragma unroll
        for (int j = 0; j < 16; ++j)
        {
            if (NT)
                __builtin_nontemporal_store(x, b + (first + j) * 64 + t);
            else
                b[(first + j) * 64 + t] = x;
        }
    }
    else
    {
#pragma unroll
        for (int j = 0; j < 16; ++j)
        {
            if (NT)
                __builtin_nontemporal_store(acc, b + (first + j) * 64 + t);
            else
                b[(first + j) * 64 + t] = acc;
        }
    }
}

int main()
{
    const size_t nblk = 10000000;
    u32x4 *a, *b;
    hipMalloc(&a, nblk * 1040);
    hipMalloc(&b, nblk * 1024);
    hipMemset(a, 1, nblk * 1040);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const uint32_t grid = (uint32_t)((nblk + 63) / 64);
    for (uint32_t R : {176u, 368u, 608u, 944u, 1024u})
    {
        const uint32_t R16 = R / 16;
        auto run = [&](const char * name, double moved, auto launch) {
            float ms;
            for (int i = 0; i < 3; ++i)
                launch();
            hipEventRecord(e0);
            for (int i = 0; i < 10; ++i)
                launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            const double s = ms * 1e-3 / 10;
            printf("R=%4u %-10s %8.1f GB/s  %8.1f G int/s  %.3f ms\n", R, name, moved / s / 1e9, nblk * 256.0 / s / 1e9, s * 1e3);
        };
        const double mv = (double)nblk * (R + 1024);
        run("blk_nt", mv, [&] { k_probe<0, 1><<<grid, 256>>>(a, b, nblk, R16); });
        run("blk", mv, [&] { k_probe<0, 0><<<grid, 256>>>(a, b, nblk, R16); });
        run("run_nt", mv, [&] { k_probe<1, 1><<<grid, 256>>>(a, b, nblk, R16); });
        run("run", mv, [&] { k_probe<1, 0><<<grid, 256>>>(a, b, nblk, R16); });
        if (R == 176u)
        {
            run("wonly_nt", nblk * 1024.0, [&] { k_probe<2, 1><<<grid, 256>>>(a, b, nblk, R16); });
            run("wonly", nblk * 1024.0, [&] { k_probe<2, 0><<<grid, 256>>>(a, b, nblk, R16); });
        }
    }
    return 0;
}
