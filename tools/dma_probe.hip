// LDS-DMA ingest rate per CU by piece shape (tuning aid, not shipped): every wave streams 1-KiB pieces
// (64 lanes x 16 B) from an L2-resident buffer into LDS with global_load_lds_dwordx4; a piece covers either
// 16 rows x 64 B (the planes GEMM's BK = 32 image rows) or 8 rows x 128 B (full lines), rows `stride` apart.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/dma_probe.hip -o tools/bin/dma_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                        \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);              \
            exit(1);                                                                                 \
        }                                                                                            \
    } while (0)

template <int ROWB, int INFLIGHT>
__global__ __launch_bounds__(512) void dma_kernel(const char* __restrict__ src, long long rows, int stride, int iters,
                                                   int* sink) {
    __shared__ __attribute__((aligned(16))) char lds[8 * 64 * 16 * INFLIGHT];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int LPR = ROWB / 16;  // lanes per row
    constexpr int RPP = 64 / LPR;   // rows per piece
    long long row = ((long long)blockIdx.x * 8 + wave) * RPP * 7 % rows;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int q = 0; q < INFLIGHT; ++q) {
            const long long r = (row + lane / LPR) % rows;
            const char* g = src + r * stride + (lane % LPR) * 16;
            __builtin_amdgcn_global_load_lds((const void*)g,
                                             (__attribute__((address_space(3))) void*)(lds + (wave * INFLIGHT + q) * 1024),
                                             16, 0, 0);
            row += RPP * 2048 + 64;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (threadIdx.x == 0 && sink) sink[blockIdx.x] = lds[7];
}

int main() {
    const long long bytes = 3LL << 20;  // 3 MiB: stays in one XCD's L2
    char* src;
    int* sink;
    CK(hipMalloc(&src, bytes));
    CK(hipMemset(src, 1, bytes));
    CK(hipMalloc(&sink, 4096 * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grid = 256, iters = 2000;
    auto run = [&](auto kern, int rowb, int stride, const char* name) {
        const long long rows = bytes / stride;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, 0, src, rows, stride, 10, sink);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, 0, src, rows, stride, iters, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double moved = (double)grid * 8 * iters * 4 * 1024.0;
        printf("%-36s %8.3f ms  %7.1f GB/s per CU  %6.2f TB/s total\n", name, ms, moved / grid / (ms * 1e-3) / 1e9,
               moved / (ms * 1e-3) / 1e12);
        (void)rowb;
    };
    run(dma_kernel<64, 4>, 64, 256, "16 rows x 64 B (stride 256 B)");
    run(dma_kernel<128, 4>, 128, 256, "8 rows x 128 B (stride 256 B)");
    run(dma_kernel<64, 4>, 64, 1024, "16 rows x 64 B (stride 1 KiB)");
    run(dma_kernel<128, 4>, 128, 1024, "8 rows x 128 B (stride 1 KiB)");
    run(dma_kernel<256, 4>, 256, 1024, "4 rows x 256 B (stride 1 KiB)");
    run(dma_kernel<64, 8>, 64, 256, "16 x 64 B, 8 in flight");
    run(dma_kernel<128, 8>, 128, 256, "8 x 128 B, 8 in flight");
    return 0;
}
