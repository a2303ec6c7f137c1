// Packed f32 under concurrent load: which operand form of v_pk_*_f32 gives different results while other kernels
// run on the GPU?  (DESIGN.md "Packed f32"; round 5 caught ds_edge_fix_kernel's
// `v_pk_fma_f32 v[2:3], v[60:61], v[56:57], v[2:3] op_sel_hi:[1,0,1]` changing its low lanes under load.)
//
// A victim kernel walks ds_edge_fix_kernel's access pattern (16 float4 weight rows and 4 float4 inputs per round,
// every FMA right behind the load wait it depends on) and forms each round's 4 accumulators twice: once with the
// packed form under test (inline asm, so the compiler cannot change the form) and once with scalar v_fma_f32 (or
// v_mul_f32 + v_add_f32).  Every round compares the two bitwise per half and counts low / high lane mismatches.
//   form 0  scalar vs scalar (control)
//   form 1  v_pk_fma_f32 vD, vW, vX, vD op_sel_hi:[1,0,1]    (VGPR pair, hi half broadcast from lo: the caught form)
//   form 2  v_pk_fma_f32 vD, vW, vXX, vD                      (VGPR pair holding x twice, no op_sel)
//   form 3  v_pk_fma_f32 vD, vW, sX, vD op_sel_hi:[1,0,1]     (SGPR pair, wave-uniform x)
//   form 4  v_pk_mul_f32 + v_pk_add_f32, VGPR pairs, broadcast op_sel_hi
// Each form runs IDLE (alone) and LOADED (an MFMA-bound and an HBM-bound kernel on two other streams).
// Build: hipcc -O3 --offload-arch=gfx950 tools/pk_probe.hip -o tools/bin/pk_probe
// Run:   tools/bin/pk_probe [launches per form and condition, default 40]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                                         \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) {                                                                          \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
            std::exit(1);                                                                                \
        }                                                                                                \
    } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int kTable = 1 << 14;  // float4 rows in the weight / input tables (256 KB each)

__device__ __forceinline__ float sfma(float a, float b, float c) {
    asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
    return c;
}
__device__ __forceinline__ float smuladd(float a, float b, float c) {
    float t;
    asm volatile("v_mul_f32 %0, %1, %2" : "=v"(t) : "v"(a), "v"(b));
    asm volatile("v_add_f32 %0, %1, %0" : "+v"(c) : "v"(t));
    return c;
}

template <int FORM>
__device__ __forceinline__ f2 pk(f2 acc, f2 w, float x, float xs) {
    if constexpr (FORM == 0) {
        acc.x = sfma(w.x, x, acc.x);
        acc.y = sfma(w.y, x, acc.y);
    } else if constexpr (FORM == 1) {
        f2 xp = {x, 0.0f};
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(acc) : "v"(w), "v"(xp));
    } else if constexpr (FORM == 2) {
        f2 xp = {x, x};
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(w), "v"(xp));
    } else if constexpr (FORM == 3) {
        f2 xp = {xs, 0.0f};
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(acc) : "v"(w), "s"(xp));
    } else {
        f2 xp = {x, 0.0f}, t;
        asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t) : "v"(w), "v"(xp));
        asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(acc) : "v"(t));
    }
    return acc;
}

template <int FORM>
__device__ __forceinline__ float ref(float acc, float w, float x, float xs) {
    if constexpr (FORM == 3) return sfma(w, xs, acc);
    if constexpr (FORM == 4) return smuladd(w, x, acc);
    return sfma(w, x, acc);
}

template <int FORM>
__global__ __launch_bounds__(256) void victim_kernel(const f4* __restrict__ wt, const f4* __restrict__ xt,
                                                     unsigned long long* __restrict__ bad, int rounds) {
    const int tid = blockIdx.x * 256 + threadIdx.x;
    unsigned lo = 0, hi = 0;
    f2 a01 = {0.f, 0.f}, a23 = {0.f, 0.f};
    float r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f;
    for (int r = 0; r < rounds; ++r) {
        const int base = (tid * 7 + r * 613) & (kTable - 1);
        f4 w[16], xv[4];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = wt[(base + i * 97) & (kTable - 1)];
#pragma unroll
        for (int i = 0; i < 4; ++i) xv[i] = xt[(base + i * 31) & (kTable - 1)];
        // wave-uniform copy of the inputs for the SGPR form
        const int ub = __builtin_amdgcn_readfirstlane(base);
        f4 xu[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) xu[i] = xt[(ub + i * 31) & (kTable - 1)];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float x1 = xv[i >> 2][i & 3];
            const float xs = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(xu[i >> 2][i & 3])));
            a01 = pk<FORM>(a01, f2{w[i].x, w[i].y}, x1, xs);
            a23 = pk<FORM>(a23, f2{w[i].z, w[i].w}, x1, xs);
            r0 = ref<FORM>(r0, w[i].x, x1, xs);
            r1 = ref<FORM>(r1, w[i].y, x1, xs);
            r2 = ref<FORM>(r2, w[i].z, x1, xs);
            r3 = ref<FORM>(r3, w[i].w, x1, xs);
        }
        lo += (__float_as_uint(a01.x) != __float_as_uint(r0)) + (__float_as_uint(a23.x) != __float_as_uint(r2));
        hi += (__float_as_uint(a01.y) != __float_as_uint(r1)) + (__float_as_uint(a23.y) != __float_as_uint(r3));
        a01 = f2{r0, r1};  // resynchronise, so one flip counts once
        a23 = f2{r2, r3};
        if ((r & 15) == 15) {  // keep the values bounded
            r0 = r1 = r2 = r3 = 0.f;
            a01 = a23 = f2{0.f, 0.f};
        }
    }
    if (lo) atomicAdd(&bad[0], (unsigned long long)lo);
    if (hi) atomicAdd(&bad[1], (unsigned long long)hi);
    atomicAdd(&bad[2], 2ULL * (unsigned long long)rounds);  // compared results per half (2 per round)
}

// load 1: MFMA-bound (dependent 32x32x16 f16 chains), writes one value per lane so nothing is removed
__global__ __launch_bounds__(256) void mfma_load_kernel(float* __restrict__ out, int iters) {
    h8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = (_Float16)(0.001f * (threadIdx.x + i));
        b[i] = (_Float16)(0.002f * (blockIdx.x + i));
    }
    f16v c0 = {}, c1 = {};
    for (int it = 0; it < iters; ++it) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, c1, 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

// load 2: HBM-bound stream (float4 copy with a scale)
__global__ __launch_bounds__(256) void mem_load_kernel(const f4* __restrict__ src, f4* __restrict__ dst, long long n,
                                                       int reps) {
    for (int r = 0; r < reps; ++r)
        for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
            dst[i] = src[i] * 1.0001f;
}

template <int FORM>
static void launch_victim(const f4* wt, const f4* xt, unsigned long long* bad, hipStream_t s) {
    hipLaunchKernelGGL(victim_kernel<FORM>, dim3(512), dim3(256), 0, s, wt, xt, bad, 64);
}

int main(int argc, char** argv) {
    const int launches = argc > 1 ? std::atoi(argv[1]) : 40;
    if (launches < 1 || launches > 2000) return 2;
    std::vector<float> h(kTable * 4);
    unsigned seed = 12345u;
    for (auto& v : h) {
        seed = seed * 1664525u + 1013904223u;
        v = (float)((int)(seed >> 8) - (1 << 23)) / (float)(1 << 23);
    }
    f4 *wt, *xt, *msrc, *mdst;
    float* mout;
    unsigned long long* bad;
    const long long mn = 64LL << 20;  // 64 M float4 = 1 GiB per buffer
    CHECK(hipMalloc(&wt, kTable * sizeof(f4)));
    CHECK(hipMalloc(&xt, kTable * sizeof(f4)));
    CHECK(hipMemcpy(wt, h.data(), kTable * sizeof(f4), hipMemcpyHostToDevice));
    for (auto& v : h) {
        seed = seed * 1664525u + 1013904223u;
        v = (float)((int)(seed >> 8) - (1 << 23)) / (float)(1 << 23);
    }
    CHECK(hipMemcpy(xt, h.data(), kTable * sizeof(f4), hipMemcpyHostToDevice));
    CHECK(hipMalloc(&msrc, mn * sizeof(f4)));
    CHECK(hipMalloc(&mdst, mn * sizeof(f4)));
    CHECK(hipMemset(msrc, 0, mn * sizeof(f4)));
    CHECK(hipMalloc(&mout, 4096 * 256 * sizeof(float)));
    CHECK(hipMalloc(&bad, 3 * sizeof(unsigned long long)));
    hipStream_t sv, sm, sh;
    CHECK(hipStreamCreateWithFlags(&sv, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&sm, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&sh, hipStreamNonBlocking));

    typedef void (*Launch)(const f4*, const f4*, unsigned long long*, hipStream_t);
    const Launch forms[5] = {launch_victim<0>, launch_victim<1>, launch_victim<2>, launch_victim<3>, launch_victim<4>};
    const char* names[5] = {"scalar control", "pk_fma VGPR-pair broadcast", "pk_fma VGPR pair (x,x)",
                            "pk_fma SGPR-pair broadcast", "pk_mul+pk_add VGPR broadcast"};
    for (int round = 0; round < 2; ++round) {
        for (int f = 0; f < 5; ++f) {
            for (int loaded = 0; loaded < 2; ++loaded) {
                CHECK(hipMemset(bad, 0, 3 * sizeof(unsigned long long)));
                CHECK(hipDeviceSynchronize());
                const auto t0 = std::chrono::steady_clock::now();
                for (int l = 0; l < launches; ++l) {
                    if (loaded && l % 8 == 0) {
                        hipLaunchKernelGGL(mfma_load_kernel, dim3(2048), dim3(256), 0, sm, mout, 20000);
                        hipLaunchKernelGGL(mem_load_kernel, dim3(2048), dim3(256), 0, sh, msrc, mdst, mn, 8);
                    }
                    forms[f](wt, xt, bad, sv);
                }
                CHECK(hipGetLastError());
                CHECK(hipDeviceSynchronize());
                const double ms =
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                unsigned long long hb[3];
                CHECK(hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost));
                std::printf("round %d form %d %-30s %-6s low %llu high %llu of %llu per half  (%.0f ms)\n", round, f,
                            names[f], loaded ? "loaded" : "idle", hb[0], hb[1], hb[2], ms);
                std::fflush(stdout);
            }
        }
    }
    return 0;
}
