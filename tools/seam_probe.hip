// What a phase seam costs on this GPU (tuning aid, not shipped; VERDICT r4 #5 "measure the persistent transformer"):
//   (a) kernel boundary: N back-to-back launches of a tiny kernel captured in a hipGraph (the engine's batch-1 form)
//   (b) grid barrier: ONE persistent launch doing the same N phases with a grid-wide barrier between them (vector
//       atomics on a per-launch counter; bounded spins, so every wave exits even if a peer never arrives)
// Each phase is the same trivial work per workgroup (one read-modify-write of 1 KB), so the difference is the seam.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/seam_probe.hip -o ab/seam_probe && ab/seam_probe
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

__global__ __launch_bounds__(256) void phase_kernel(float* buf, int phase) {
    float* p = buf + (size_t)blockIdx.x * 256 + threadIdx.x;
    *p = *p * 0.5f + (float)phase;
}

// bar: [0] arrivals (monotonic within a launch; zeroed by a memset node before it), [1] give-up count
__global__ __launch_bounds__(256) void persistent_kernel(float* buf, unsigned* bar, int phases) {
    float* p = buf + (size_t)blockIdx.x * 256 + threadIdx.x;
    const unsigned n = gridDim.x;
    __shared__ int bail;
    if (threadIdx.x == 0) bail = 0;
    __syncthreads();
    for (int ph = 0; ph < phases; ++ph) {
        *p = *p * 0.5f + (float)ph;
        if (ph + 1 == phases) break;
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned want = n * (unsigned)(ph + 1);
            int spins = 0;
            while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < want) {
                if (++spins > (1 << 18)) {  // a peer never arrived: give up (counted), every wave still exits
                    __hip_atomic_fetch_add(bar + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    bail = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        if (bail) break;
    }
}

// two-level barrier: a workgroup arrives on its XCD's counter (workgroups are dealt to the 8 XCDs round-robin), the
// XCD's last arrival bumps the global counter, the last of those publishes the generation everyone waits on.
// bar (uints): [16 (x + 1)] XCD counters x = 0..7 (64 B apart), [192] global count, [224] generation, [1] give-ups
// RELAXED: the same barrier with relaxed atomics and no fences -- no cache write-back / invalidate per arrival, so
// not a correct barrier for data; the synchronisation's own floor
template <bool RELAXED>
__global__ __launch_bounds__(256) void persistent2_kernel(float* buf, unsigned* bar, int phases) {
    constexpr int ORD_RMW = RELAXED ? __ATOMIC_RELAXED : __ATOMIC_ACQ_REL;
    constexpr int ORD_ST = RELAXED ? __ATOMIC_RELAXED : __ATOMIC_RELEASE;
    constexpr int ORD_LD = RELAXED ? __ATOMIC_RELAXED : __ATOMIC_ACQUIRE;
    float* p = buf + (size_t)blockIdx.x * 256 + threadIdx.x;
    const unsigned per_xcd = gridDim.x / 8, x = blockIdx.x & 7;
    __shared__ int bail;
    if (threadIdx.x == 0) bail = 0;
    __syncthreads();
    for (int ph = 0; ph < phases; ++ph) {
        *p = *p * 0.5f + (float)ph;
        if (ph + 1 == phases) break;
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned gen = (unsigned)ph + 1;
            const unsigned old = __hip_atomic_fetch_add(bar + 16 * (x + 1), 1u, ORD_RMW, __HIP_MEMORY_SCOPE_AGENT);
            if (old == per_xcd * gen - 1) {
                const unsigned g = __hip_atomic_fetch_add(bar + 192, 1u, ORD_RMW, __HIP_MEMORY_SCOPE_AGENT);
                if (g == 8 * gen - 1) __hip_atomic_store(bar + 224, gen, ORD_ST, __HIP_MEMORY_SCOPE_AGENT);
            }
            int spins = 0;
            while (__hip_atomic_load(bar + 224, ORD_LD, __HIP_MEMORY_SCOPE_AGENT) < gen) {
                if (++spins > (1 << 18)) {
                    __hip_atomic_fetch_add(bar + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    bail = 1;
                    break;
                }
            }
        }
        __syncthreads();
        if (bail) break;
    }
}

int main(int argc, char** argv) {
    const int phases = argc > 1 ? atoi(argv[1]) : 56;  // 7 kernels per layer x 8 layers
    int dev = 0, ncu = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    float* buf;
    unsigned* bar;
    CK(hipMalloc(&buf, (size_t)4 * ncu * 256 * 4));
    CK(hipMalloc(&bar, 1024));
    CK(hipMemset(buf, 0, (size_t)4 * ncu * 256 * 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int mult = 1; mult <= 4; mult *= 2) {
        const int grid = ncu * mult;
        // (a) graph of `phases` launches
        hipGraph_t g;
        hipGraphExec_t gx;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        for (int ph = 0; ph < phases; ++ph) hipLaunchKernelGGL(phase_kernel, dim3(grid), dim3(256), 0, s, buf, ph);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&gx, g, nullptr, nullptr, 0));
        for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(gx, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(gx, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms_a;
        CK(hipEventElapsedTime(&ms_a, e0, e1));
        // (b) one persistent launch per pass (a memset node zeroes the counter first), also as a graph
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        CK(hipMemsetAsync(bar, 0, 8, s));
        hipLaunchKernelGGL(persistent_kernel, dim3(grid), dim3(256), 0, s, buf, bar, phases);
        hipGraph_t g2;
        hipGraphExec_t gx2;
        CK(hipStreamEndCapture(s, &g2));
        CK(hipGraphInstantiate(&gx2, g2, nullptr, nullptr, 0));
        for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(gx2, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(gx2, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms_b;
        CK(hipEventElapsedTime(&ms_b, e0, e1));
        unsigned hb[2];
        CK(hipMemcpy(hb, bar, 8, hipMemcpyDeviceToHost));
        // (b2) the two-level barrier; (b3) the same, relaxed
        float ms_b3 = 0.0f, ms_b2 = 0.0f;
        unsigned hb2[2] = {0, 0};
        for (int relaxed = 1; relaxed >= 0; --relaxed) {
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        CK(hipMemsetAsync(bar, 0, 1024, s));
        if (relaxed)
            hipLaunchKernelGGL(persistent2_kernel<true>, dim3(grid), dim3(256), 0, s, buf, bar, phases);
        else
            hipLaunchKernelGGL(persistent2_kernel<false>, dim3(grid), dim3(256), 0, s, buf, bar, phases);
        hipGraph_t g3;
        hipGraphExec_t gx3;
        CK(hipStreamEndCapture(s, &g3));
        CK(hipGraphInstantiate(&gx3, g3, nullptr, nullptr, 0));
        for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(gx3, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(gx3, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms_b2, e0, e1));
        CK(hipMemcpy(hb2, bar, 8, hipMemcpyDeviceToHost));
        CK(hipGraphExecDestroy(gx3));
        CK(hipGraphDestroy(g3));
        if (relaxed) ms_b3 = ms_b2;
        }
        // (c) one launch of one phase: the floor both forms pay once
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(phase_kernel, dim3(grid), dim3(256), 0, s, buf, i);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms_c;
        CK(hipEventElapsedTime(&ms_c, e0, e1));
        printf("grid %4d: relaxed two-level barrier (synchronisation floor) %7.2f us (%.2f us per seam)\n", grid,
               ms_b3 * 1000 / 20, ms_b3 * 1000 / 20 / (phases - 1));
        printf("grid %4d (%d per CU), %d phases: graph of launches %7.2f us (%.2f us per seam); persistent + grid "
               "barriers %7.2f us (%.2f us per seam; gave up: %u); two-level barrier %7.2f us (%.2f us per seam; "
               "gave up: %u); single launch %.2f us\n",
               grid, mult, phases, ms_a * 1000 / 20, ms_a * 1000 / 20 / phases, ms_b * 1000 / 20,
               ms_b * 1000 / 20 / (phases - 1), hb[1], ms_b2 * 1000 / 20, ms_b2 * 1000 / 20 / (phases - 1), hb2[1],
               ms_c * 1000 / 20);
        CK(hipGraphExecDestroy(gx));
        CK(hipGraphDestroy(g));
        CK(hipGraphExecDestroy(gx2));
        CK(hipGraphDestroy(g2));
    }
    CK(hipFree(buf));
    CK(hipFree(bar));
    return 0;
}
