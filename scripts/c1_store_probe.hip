// c1_store_probe.hip -- data-movement ceilings of the C1 (p4Dec32 n=127)
// output shape (measurement tool, not part of the library): per block read
// 128 B of a contiguous stream, write 127 u32 = 508 B at byte 508*k (4-byte
// aligned only).  A wave owns 64 consecutive blocks (k_dec_h32w's grid).
//   dw   : lane t stores elements t and t+64 (two dword store instructions per block, k_dec_h32w)
//   x4   : lane t stores elements 4t..4t+3 with one 16-byte store (4-byte aligned), the ragged
//          last lane with dword stores
//   a16  : (round 6) the wave's whole output range (64 blocks x 508 B = 32,512 B, 16-byte aligned:
//          the run starts at a multiple of 64 blocks) in 16-byte aligned chunks, one chunk per lane per
//          store instruction -- the store pattern an LDS-staged output would issue, with the staging's
//          own cost left out
//   Each with default and nt store policy (a16 also sc1 nt).
// Build: hipcc --offload-arch=gfx950 -O3 -o c1_store_probe c1_store_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk(const void * p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, bytes, 0x00020000);
}

template <int MODE, int AUX>
__global__ __launch_bounds__(256) void k_probe(const uint8_t * __restrict in, uint32_t * __restrict out, uint64_t nblk)
{
    const uint32_t t = threadIdx.x & 63u;
    const uint64_t first = (blockIdx.x * 4ull + (threadIdx.x >> 6)) * 64u;
    if (first >= nblk)
        return;
    const uint32_t nr = static_cast<uint32_t>(nblk - first < 64u ? nblk - first : 64u);
    const __amdgpu_buffer_rsrc_t rs = mk(in + first * 128u, nr * 128u);
    const __amdgpu_buffer_rsrc_t os = mk(out + first * 127u, nr * 508u);
    // the run's bytes: 8 KB, 8 loads per lane, XOR-folded into the stored values
    u32x4 acc{t, 0u, 0u, 0u};
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i)
        acc ^= __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(1024u * i + 16u * t), 0, 0);
    const uint32_t v = acc.x ^ acc.y ^ acc.z ^ acc.w;
    for (uint32_t jj = 0; jj < nr; ++jj)
    {
        const uint32_t v2 = v + jj;
        if (MODE == 2)
            break;
        if (MODE == 0)
        {
            __builtin_amdgcn_raw_buffer_store_b32(v2, os, static_cast<int>((jj * 127u + t) * 4u), 0, AUX);
            __builtin_amdgcn_raw_buffer_store_b32(v2, os, static_cast<int>(t + 64u < 127u ? (jj * 127u + t + 64u) * 4u : 0x80000000u), 0, AUX);
        }
        else
        {
            const uint32_t e = 4u * t;
            if (e + 4u <= 127u)
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{v2, v2, v2, v2}, os, static_cast<int>((jj * 127u + e) * 4u), 0, AUX);
            else if (e < 127u)
                for (uint32_t i = 0; e + i < 127u; ++i)
                    __builtin_amdgcn_raw_buffer_store_b32(v2, os, static_cast<int>((jj * 127u + e + i) * 4u), 0, AUX);
        }
    }
    if (MODE == 2)
    {
        const uint32_t chunks = nr * 508u / 16u; // nr = 64: 2,032 whole chunks
        for (uint32_t c = t; c < chunks; c += 64u)
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{v, v + c, v, v}, os, static_cast<int>(16u * c), 0, AUX);
    }
}

int main()
{
    const uint64_t nblk = 10000000;
    uint8_t * in;
    uint32_t * out;
    hipMalloc(&in, nblk * 128);
    hipMalloc(&out, nblk * 508 + 64);
    hipMemset(in, 1, nblk * 128);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const uint32_t grid = static_cast<uint32_t>((nblk + 255) / 256);
    auto run = [&](const char * name, auto launch) {
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
        printf("%-12s %8.1f GB/s  %7.1f G int32/s  %.3f ms\n", name, nblk * 636.0 / s / 1e9, nblk * 127.0 / s / 1e9, s * 1e3);
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep)
    {
        run("dw", [&] { k_probe<0, 0><<<grid, 256>>>(in, out, nblk); });
        run("dw nt", [&] { k_probe<0, 2><<<grid, 256>>>(in, out, nblk); });
        run("x4", [&] { k_probe<1, 0><<<grid, 256>>>(in, out, nblk); });
        run("x4 nt", [&] { k_probe<1, 2><<<grid, 256>>>(in, out, nblk); });
        run("a16", [&] { k_probe<2, 0><<<grid, 256>>>(in, out, nblk); });
        run("a16 nt", [&] { k_probe<2, 2><<<grid, 256>>>(in, out, nblk); });
        run("a16 sc1nt", [&] { k_probe<2, 18><<<grid, 256>>>(in, out, nblk); });
    }
    return 0;
}
