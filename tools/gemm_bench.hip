// Microbenchmark of planes-GEMM variants on the encode's real GEMM shapes (tuning aid, not shipped).
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I tokenize-audio_amd/csrc -I tools \
//     tools/gemm_bench.hip -o tools/bin/gemm_bench
//   tools/bin/gemm_bench REPS down_s0,down_s1,...   (shape names, comma-separated)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gemm_planes.h"
#include "gemm_stream_proto.h"

using namespace mimi;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

struct Shape {
    const char* name;
    int cin, k, s;
    long long tin, tout;
    int batch, N;
};

typedef void (*LaunchFn)(const GemmArgs&, hipStream_t);

template <int BM, int BN, int WM, int WN, int BK, int NBUF, bool NFAST>
void launch(const GemmArgs& a, hipStream_t s) {
    dim3 grid((a.M + BM - 1) / BM, (a.N + BN - 1) / BN, a.batch);
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, BK, NBUF, NFAST, false, PAD_ZERO, EPI_BIAS, 0>), grid,
                       dim3(WM * WN * 64), 0, s, a);
}

template <int BM, int BN, int WM, int WN, int NS>
void launch_bf(const GemmArgs& a, hipStream_t s) {
    dim3 grid((a.M + BM - 1) / BM, (a.N + BN - 1) / BN, a.batch);
    hipLaunchKernelGGL((gemm_bf16x_kernel<BM, BN, WM, WN, NS, false, PAD_ZERO, EPI_BIAS, 0>), grid,
                       dim3(WM * WN * 64), 0, s, a);
}

template <int BM, int BN, int WM, int WN, int ST, int LW, int FL>
void launch_st(const GemmArgs& a, hipStream_t s) {
    int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN) * a.batch;
    int occ = 1;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &occ, gemm_stream_kernel<BM, BN, WM, WN, ST, EPI_BIAS, 0, 0, LW, FL>, (WM * WN + LW) * 64, 0);
    nwg = std::min(nwg, 256 * std::max(1, occ));
    hipLaunchKernelGGL((gemm_stream_kernel<BM, BN, WM, WN, ST, EPI_BIAS, 0, 0, LW, FL>), dim3(nwg),
                       dim3((WM * WN + LW) * 64), 0, s, a);
}

template <int BM, int BN, int WM, int WN, int NS, int ST, int LW = 0, int BK = 32, int MF = 32, int FL = 0,
          bool F16 = false>
void launch_pl(const GemmArgs& a, hipStream_t s) {
    int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN) * a.batch;
    if (FL & FL_PERSIST) {
        int occ = 1;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &occ, gemm_planes_kernel<BM, BN, WM, WN, NS, ST, EPI_BIAS, 0, 0, LW, BK, MF, FL, F16>, (WM * WN + LW) * 64, 0);
        nwg = std::min(nwg, 256 * std::max(1, occ));
    }
    hipLaunchKernelGGL((gemm_planes_kernel<BM, BN, WM, WN, NS, ST, EPI_BIAS, 0, 0, LW, BK, MF, FL, F16>), dim3(nwg),
                       dim3((WM * WN + LW) * 64), 0, s, a);
}

__global__ void split_planes(const float* x, __bf16* out, long long n) {
    const long long i = blockIdx.x * 256LL + threadIdx.x;
    if (i >= n) return;
    float r = x[i];
    for (int p = 0; p < 3; ++p) {
        const __bf16 h = (__bf16)r;
        out[p * n + i] = h;
        r -= (float)h;
    }
}

__global__ void split_planes_f16(const float* x, _Float16* out, long long n, float sc) {
    const long long i = blockIdx.x * 256LL + threadIdx.x;
    if (i >= n) return;
    const float r = x[i] * sc;
    const _Float16 h = (_Float16)r;
    out[i] = h;
    out[n + i] = (_Float16)(r - (float)h);
}

struct Variant {
    const char* name;
    LaunchFn fn;
    int bk;
    int ns;  // 0 = fp32 weights, else bf16 planes (2, 3) or fp16 planes (12)
    bool pair = false;  // FL_PAIR: k = 2s convs only
};

static uint16_t f2bf(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    u += 0x7FFF + ((u >> 16) & 1);
    return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    Shape shapes[] = {
        {"down_s0", 64, 8, 4, 240000, 60000, 32, 128},  {"down_s1", 128, 10, 5, 60000, 12000, 32, 256},
        {"down_s2", 256, 12, 6, 12000, 2000, 32, 512},  {"down_s3", 512, 16, 8, 2000, 250, 32, 1024},
        {"final", 1024, 3, 1, 250, 250, 32, 512},        {"fc1", 512, 1, 1, 8000, 8000, 1, 2048},
        {"fc2", 2048, 1, 1, 8000, 8000, 1, 512},         {"qkv", 512, 1, 1, 250, 250, 32, 1536},
        {"o_proj", 512, 1, 1, 8000, 8000, 1, 512},
        {"res3_s2", 256, 3, 1, 12000, 12000, 32, 128},   {"res1_s2", 128, 1, 1, 12000, 12000, 32, 256},
        {"res3_s3", 512, 3, 1, 2000, 2000, 32, 256},     {"res1_s3", 256, 1, 1, 2000, 2000, 32, 512},
        // batch 1 (launch / latency bound)
        {"b1_fc2", 2048, 1, 1, 250, 250, 1, 512},        {"b1_fc1", 512, 1, 1, 250, 250, 1, 2048},
        {"b1_qkv", 512, 1, 1, 250, 250, 1, 1536},        {"b1_oproj", 512, 1, 1, 250, 250, 1, 512},
        {"b1_down_s3", 512, 16, 8, 2000, 250, 1, 1024},  {"b1_final", 1024, 3, 1, 250, 250, 1, 512},
        {"b1_down_s1", 128, 10, 5, 60000, 12000, 1, 256},
        {"b8_dn_s1", 128, 10, 5, 60000, 12000, 8, 256}, {"b1_down_s0", 64, 8, 4, 240000, 60000, 1, 128},
    };
    Variant vars[] = {
        // references: loader-free kernels (the LW > 0 loop under test must give the same bits)
        {"ref 256x128 8w s3", launch_pl<256, 128, 4, 2, 2, 3, 0, 32, 16, 0, true>, 32, 12},
        {"pair ref 256x128 8w s2 0ld", launch_pl<256, 128, 4, 2, 2, 2, 0, 32, 16, FL_PAIR | FL_PERSIST, true>, 64, 12, true},
        {"pair PERSIST 8w+4ld s2", launch_pl<256, 128, 4, 2, 2, 2, 4, 32, 16, FL_PAIR | FL_PERSIST, true>, 64, 12, true},
        {"pair 64x64 4w+4ld s2", launch_pl<64, 64, 2, 2, 2, 2, 4, 32, 16, FL_PAIR, true>, 64, 12, true},
        {"pair 64x64 4w+4ld s4 KG2", launch_pl<64, 64, 2, 2, 2, 4, 4, 32, 16, FL_PAIR | FL_KG2, true>, 64, 12, true},
        {"64x64 4w+4ld s4", launch_pl<64, 64, 2, 2, 2, 4, 4, 32, 16, 0, true>, 32, 12},
        {"128x128 4w+4ld s3", launch_pl<128, 128, 2, 2, 2, 3, 4, 32, 16, 0, true>, 32, 12},
        {"128x128 8w+4ld s2", launch_pl<128, 128, 4, 2, 2, 2, 4, 32, 16, 0, true>, 32, 12},
        {"256x128 8w+4ld s3", launch_pl<256, 128, 4, 2, 2, 3, 4, 32, 16, 0, true>, 32, 12},
        {"128x128 8w s2 (fc1/qkv/res3)", launch_pl<128, 128, 4, 2, 2, 2, 0, 32, 16, 0, true>, 32, 12},
        {"128x64 4w s2 (res1)", launch_pl<128, 64, 2, 2, 2, 2, 0, 32, 16, 0, true>, 32, 12},
        {"128x64 4w+4ld s2", launch_pl<128, 64, 2, 2, 2, 2, 4, 32, 16, 0, true>, 32, 12},
        {"128x64 4w+4ld s3", launch_pl<128, 64, 2, 2, 2, 3, 4, 32, 16, 0, true>, 32, 12},
        {"128x128 4w+4ld s4", launch_pl<128, 128, 2, 2, 2, 4, 4, 32, 16, 0, true>, 32, 12},
        {"128x128 8w+4ld s3", launch_pl<128, 128, 4, 2, 2, 3, 4, 32, 16, 0, true>, 32, 12},
        {"64x128 2w+4ld s4", launch_pl<64, 128, 1, 2, 2, 4, 4, 32, 16, 0, true>, 32, 12},
        {"pair PERSIST bk16 mf32 s4", launch_pl<256, 128, 4, 2, 2, 4, 4, 16, 32, FL_PAIR | FL_PERSIST, true>, 64, 12, true},
        {"pair PERSIST bk16 mf32 s3", launch_pl<256, 128, 4, 2, 2, 3, 4, 16, 32, FL_PAIR | FL_PERSIST, true>, 64, 12, true},
        {"pair PERSIST bk16 mf32 s4 KG2", launch_pl<256, 128, 4, 2, 2, 4, 4, 16, 32, FL_PAIR | FL_PERSIST | FL_KG2, true>, 64, 12, true},
        {"pair PERSIST mf32 s2", launch_pl<256, 128, 4, 2, 2, 2, 4, 32, 32, FL_PAIR | FL_PERSIST, true>, 64, 12, true},
        {"pair PERSIST 4w(2x2)+4ld s2", launch_pl<256, 128, 2, 2, 2, 2, 4, 32, 16, FL_PAIR | FL_PERSIST, true>, 64, 12, true},
        {"pair PERSIST 4w(4x1)+4ld s2", launch_pl<256, 128, 4, 1, 2, 2, 4, 32, 16, FL_PAIR | FL_PERSIST, true>, 64, 12, true},
        {"pair PERSIST 4w(2x2) mf32+4ld s2", launch_pl<256, 128, 2, 2, 2, 2, 4, 32, 32, FL_PAIR | FL_PERSIST, true>, 64, 12, true},
        {"128x128 8w+4ld s2 P", launch_pl<128, 128, 4, 2, 2, 2, 4, 32, 16, FL_PERSIST | FL_PF, true>, 32, 12},
        {"128x128 8w+4ld s3 P", launch_pl<128, 128, 4, 2, 2, 3, 4, 32, 16, FL_PERSIST | FL_PF, true>, 32, 12},
        {"128x128 4w+4ld s3 P", launch_pl<128, 128, 2, 2, 2, 3, 4, 32, 16, FL_PERSIST | FL_PF, true>, 32, 12},
        {"256x128 8w+4ld s3 P", launch_pl<256, 128, 4, 2, 2, 3, 4, 32, 16, FL_PERSIST | FL_PF, true>, 32, 12},
        {"pair 256x256 bk16 mf32 8w(2x4) s3 0ld", launch_pl<256, 256, 2, 4, 2, 3, 0, 16, 32, FL_PAIR | FL_PERSIST, true>, 64, 12, true},
        {"pair 256x256 bk16 mf32 8w(2x4)+4ld s3", launch_pl<256, 256, 2, 4, 2, 3, 4, 16, 32, FL_PAIR | FL_PERSIST, true>, 64, 12, true},
        {"pair 256x256 bk16 mf32 8w(4x2)+4ld s3", launch_pl<256, 256, 4, 2, 2, 3, 4, 16, 32, FL_PAIR | FL_PERSIST, true>, 64, 12, true},
        {"pair PERSIST DIAG nodma", launch_pl<256, 128, 4, 2, 2, 2, 4, 32, 16, FL_PAIR | FL_PERSIST | FL_DIAG_NODMA, true>, 64, 12, true},
        {"pair PERSIST DIAG nomma", launch_pl<256, 128, 4, 2, 2, 2, 4, 32, 16, FL_PAIR | FL_PERSIST | FL_DIAG_NOMMA, true>, 64, 12, true},
        {"pair PERSIST DIAG both", launch_pl<256, 128, 4, 2, 2, 2, 4, 32, 16, FL_PAIR | FL_PERSIST | FL_DIAG_NODMA | FL_DIAG_NOMMA, true>, 64, 12, true},
        // transformer tiles (qkv: 8w+4ld s2; fc1: 8w s2; o_proj / fc2: 8w+4ld s3) with the DMA refills or the MFMAs removed
        {"T 128x128 8w+4ld s2 DIAG nodma", launch_pl<128, 128, 4, 2, 2, 2, 4, 32, 16, FL_DIAG_NODMA, true>, 32, 12},
        {"T 128x128 8w+4ld s2 DIAG nomma", launch_pl<128, 128, 4, 2, 2, 2, 4, 32, 16, FL_DIAG_NOMMA, true>, 32, 12},
        {"T 128x128 8w+4ld s2 DIAG both", launch_pl<128, 128, 4, 2, 2, 2, 4, 32, 16, FL_DIAG_NODMA | FL_DIAG_NOMMA, true>, 32, 12},
        {"T 128x128 8w s2 DIAG nodma", launch_pl<128, 128, 4, 2, 2, 2, 0, 32, 16, FL_DIAG_NODMA, true>, 32, 12},
        {"T 128x128 8w s2 DIAG nomma", launch_pl<128, 128, 4, 2, 2, 2, 0, 32, 16, FL_DIAG_NOMMA, true>, 32, 12},
        {"T 128x128 8w+4ld s3 DIAG nodma", launch_pl<128, 128, 4, 2, 2, 3, 4, 32, 16, FL_DIAG_NODMA, true>, 32, 12},
        {"T 128x128 8w+4ld s3 DIAG nomma", launch_pl<128, 128, 4, 2, 2, 3, 4, 32, 16, FL_DIAG_NOMMA, true>, 32, 12},
        {"T 128x128 8w+4ld s4", launch_pl<128, 128, 4, 2, 2, 4, 4, 32, 16, 0, true>, 32, 12},
        {"T 256x128 8w+4ld s2", launch_pl<256, 128, 4, 2, 2, 2, 4, 32, 16, 0, true>, 32, 12},
        {"T 128x256 8w+4ld s2", launch_pl<128, 256, 2, 4, 2, 2, 4, 32, 16, 0, true>, 32, 12},
        {"T 256x256 8w+4ld s2", launch_pl<256, 256, 4, 2, 2, 2, 4, 32, 16, 0, true>, 32, 12},
        // batch-1 tiles (round 4): ring depth / grouping on the latency-bound small grids (16 K steps at K = 512)
        {"B1 16x64 1w+4ld s4", launch_pl<16, 64, 1, 1, 2, 4, 4, 32, 16, 0, true>, 32, 12},
        {"B1 16x64 1w+4ld s6", launch_pl<16, 64, 1, 1, 2, 6, 4, 32, 16, 0, true>, 32, 12},
        {"B1 16x64 1w+4ld s8", launch_pl<16, 64, 1, 1, 2, 8, 4, 32, 16, 0, true>, 32, 12},
        {"B1 16x64 1w+4ld s8 KG2", launch_pl<16, 64, 1, 1, 2, 8, 4, 32, 16, FL_KG2, true>, 32, 12},
        {"B1 16x64 1w+4ld s8 KG4", launch_pl<16, 64, 1, 1, 2, 8, 4, 32, 16, FL_KG4, true>, 32, 12},
        {"B1 16x64 2w+4ld s8", launch_pl<16, 64, 1, 2, 2, 8, 4, 32, 16, 0, true>, 32, 12},
        {"B1 32x32 2w+4ld s4", launch_pl<32, 32, 2, 1, 2, 4, 4, 32, 16, 0, true>, 32, 12},
        {"B1 32x32 2w+4ld s8", launch_pl<32, 32, 2, 1, 2, 8, 4, 32, 16, 0, true>, 32, 12},
        {"B1 32x64 4w+4ld s4", launch_pl<32, 64, 2, 2, 2, 4, 4, 32, 16, 0, true>, 32, 12},
        {"B1 32x64 4w+4ld s8", launch_pl<32, 64, 2, 2, 2, 8, 4, 32, 16, 0, true>, 32, 12},
        {"B1 32x64 4w+4ld s8 KG2", launch_pl<32, 64, 2, 2, 2, 8, 4, 32, 16, FL_KG2, true>, 32, 12},
        {"B1 16x32 1w+4ld s4", launch_pl<16, 32, 1, 1, 2, 4, 4, 32, 16, 0, true>, 32, 12},
        {"B1 16x32 1w+4ld s8", launch_pl<16, 32, 1, 1, 2, 8, 4, 32, 16, 0, true>, 32, 12},
        {"B1 16x32 1w+2ld s8", launch_pl<16, 32, 1, 1, 2, 8, 2, 32, 16, 0, true>, 32, 12},
        {"B1 16x32 1w+4ld s6 KG2", launch_pl<16, 32, 1, 1, 2, 6, 4, 32, 16, FL_KG2, true>, 32, 12},
        {"B1 64x64 4w+4ld s8", launch_pl<64, 64, 2, 2, 2, 8, 4, 32, 16, 0, true>, 32, 12},
        // deeper rings (round 4, late): more bytes in flight per CU for the latency-bound small grids
        {"B1 16x32 1w+4ld s12 KG2", launch_pl<16, 32, 1, 1, 2, 12, 4, 32, 16, FL_KG2, true>, 32, 12},
        {"B1 16x32 1w+4ld s16 KG4", launch_pl<16, 32, 1, 1, 2, 16, 4, 32, 16, FL_KG4, true>, 32, 12},
        {"B1 16x32 1w+4ld s16 KG2", launch_pl<16, 32, 1, 1, 2, 16, 4, 32, 16, FL_KG2, true>, 32, 12},
        {"B1 16x64 1w+4ld s12 KG2", launch_pl<16, 64, 1, 1, 2, 12, 4, 32, 16, FL_KG2, true>, 32, 12},
        {"B1 16x64 1w+4ld s16 KG4", launch_pl<16, 64, 1, 1, 2, 16, 4, 32, 16, FL_KG4, true>, 32, 12},
        {"B1 32x32 2w+4ld s12 KG2", launch_pl<32, 32, 2, 1, 2, 12, 4, 32, 16, FL_KG2, true>, 32, 12},
        {"B1 16x32 1w+4ld s6 KG2 (fc2)", launch_pl<16, 32, 1, 1, 2, 6, 4, 32, 16, FL_KG2, true>, 32, 12},
        // interleaved-plane timing probe (FL_DIAG_ILV: 8 rows x 128 B pieces; results garbage)
        {"pair PERSIST 8w+4ld s2 ILV", launch_pl<256, 128, 4, 2, 2, 2, 4, 32, 16, FL_PAIR | FL_PERSIST | FL_DIAG_ILV, true>, 64, 12, true},
        {"pair PERSIST DIAG nomma ILV", launch_pl<256, 128, 4, 2, 2, 2, 4, 32, 16, FL_PAIR | FL_PERSIST | FL_DIAG_NOMMA | FL_DIAG_ILV, true>, 64, 12, true},
        {"T 128x128 8w+4ld s2 ILV", launch_pl<128, 128, 4, 2, 2, 2, 4, 32, 16, FL_DIAG_ILV, true>, 32, 12},
        {"T 128x128 8w+4ld s3 ILV", launch_pl<128, 128, 4, 2, 2, 3, 4, 32, 16, FL_DIAG_ILV, true>, 32, 12},
        {"T 128x128 8w+4ld s2 DIAG nomma ILV", launch_pl<128, 128, 4, 2, 2, 2, 4, 32, 16, FL_DIAG_NOMMA | FL_DIAG_ILV, true>, 32, 12},
        {"256x128 8w+4ld s3 ILV", launch_pl<256, 128, 4, 2, 2, 3, 4, 32, 16, FL_DIAG_ILV, true>, 32, 12},
    };
    const int nv = sizeof(vars) / sizeof(vars[0]);
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* only = argc > 2 ? argv[2] : nullptr;
    for (const Shape& sh : shapes) {
        if (only && !strstr(only, sh.name)) continue;
        const long long K = (long long)sh.k * sh.cin;
        const size_t nA = (size_t)sh.batch * sh.tin * sh.cin, nW = (size_t)sh.N * K,
                     nC = (size_t)sh.batch * sh.tout * sh.N;
        std::vector<float> hA(nA), hW(nW), hb(sh.N);
        unsigned long long x = 0x9E3779B97F4A7C15ull;
        auto rnd = [&]() {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            return (float)((x >> 40) * (1.0 / (1ull << 24)) - 0.5);
        };
        for (auto& v : hA) v = rnd();
        for (auto& v : hW) v = rnd() * 0.1f;
        for (auto& v : hb) v = rnd();
        float *A, *W, *bias, *C, *Cref, *Cref2;
        uint16_t* Wp;
        CK(hipMalloc(&Wp, 3 * nW * 2));
        {
            std::vector<uint16_t> hp(3 * nW);
            for (size_t i = 0; i < nW; ++i) {
                float r = hW[i];
                for (int pl = 0; pl < 3; ++pl) {
                    const uint16_t h = f2bf(r);
                    hp[pl * nW + i] = h;
                    r -= bf2f(h);
                }
            }
            // planes for NS = 2 are the first two planes of the NS = 3 split (same leading terms)
            CK(hipMemcpy(Wp, hp.data(), 3 * nW * 2, hipMemcpyHostToDevice));
        }
        CK(hipMalloc(&A, nA * 4));
        CK(hipMalloc(&W, nW * 4));
        CK(hipMalloc(&bias, sh.N * 4));
        CK(hipMalloc(&C, nC * 4));
        CK(hipMalloc(&Cref, nC * 4));
        CK(hipMalloc(&Cref2, nC * 4));
        CK(hipMemcpy(A, hA.data(), nA * 4, hipMemcpyHostToDevice));
        __bf16* Apl;
        CK(hipMalloc(&Apl, 3 * nA * 2));
        hipLaunchKernelGGL(split_planes, dim3((unsigned)((nA + 255) / 256)), dim3(256), 0, 0, A, Apl, (long long)nA);
        CK(hipDeviceSynchronize());
        // fp16 planes (2) of A * sa and W * sw, sa / sw powers of two putting max|A| at 2^7, max|W| at 2^14
        float amax = 0, wmax = 0;
        for (float v : hA) amax = fmaxf(amax, fabsf(v));
        for (float v : hW) wmax = fmaxf(wmax, fabsf(v));
        const float sa = ldexpf(1.0f, 7 - (int)ceilf(log2f(amax))), sw = ldexpf(1.0f, 14 - (int)ceilf(log2f(wmax)));
        _Float16 *Ah, *Wh;
        float* unsc;
        CK(hipMalloc(&Ah, 2 * nA * 2));
        CK(hipMalloc(&Wh, 2 * nW * 2));
        CK(hipMalloc(&unsc, sh.batch * 4));
        CK(hipMemcpy(W, hW.data(), nW * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(split_planes_f16, dim3((unsigned)((nA + 255) / 256)), dim3(256), 0, 0, A, Ah, (long long)nA, sa);
        hipLaunchKernelGGL(split_planes_f16, dim3((unsigned)((nW + 255) / 256)), dim3(256), 0, 0, W, Wh, (long long)nW, sw);
        {
            std::vector<float> hu(sh.batch, 1.0f / (sa * sw));
            CK(hipMemcpy(unsc, hu.data(), sh.batch * 4, hipMemcpyHostToDevice));
        }
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(bias, hb.data(), sh.N * 4, hipMemcpyHostToDevice));
        GemmArgs a{};
        a.A = A;
        a.a_bstride = sh.tin * sh.cin;
        a.a_off = -(long long)(sh.k - sh.s) * sh.cin;
        a.a_rs = sh.s * sh.cin;
        a.a_cin = sh.cin;
        a.a_len = sh.tin * sh.cin;
        a.Ap = Apl;
        a.a_pstride = (long long)nA;
        a.W = W;
        a.M = (int)sh.tout;
        a.N = sh.N;
        a.K = (int)K;
        a.batch = sh.batch;
        a.bias = bias;
        a.c_bstride = sh.tout * sh.N;
        a.ldc = sh.N;
        const double flops = 2.0 * sh.batch * sh.tout * sh.N * K;
        std::vector<float> ref(nC), out(nC);
        const char* vonly = argc > 3 ? argv[3] : nullptr;  // variant-name substrings, '|'-separated
        for (int v = 0; v < nv; ++v) {
            if (vonly) {
                bool hit = false;
                for (const char* q = vonly; *q;) {
                    const char* e = strchr(q, '|');
                    const size_t n = e ? (size_t)(e - q) : strlen(q);
                    if (n && std::string(vars[v].name).find(std::string(q, n)) != std::string::npos) hit = true;
                    q += n + (e ? 1 : 0);
                }
                if (!hit) continue;
            }
            if (K % vars[v].bk) continue;
            if (vars[v].pair && sh.k != 2 * sh.s) continue;
            a.C = v == 0 ? Cref : (v == 1 ? Cref2 : C);
            a.W = W;
            a.Wsplit = Wp;
            a.Ap = Apl;
            a.unscale = 0.0f;
            if (vars[v].ns == 12) {
                a.Wsplit = Wh;
                a.Ap = Ah;
                a.unscale = 1.0f / (sa * sw);
            }
            if (vars[v].ns == 2) {
                // NS = 2 reads planes [2][N][K]: the first two planes of the 3-plane buffer are exactly that
            }
            vars[v].fn(a, st);
            CK(hipGetLastError());
            CK(hipStreamSynchronize(st));
            float best = 1e30f, tot = 0;
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(e0, st));
                vars[v].fn(a, st);
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = fminf(best, ms);
                tot += ms;
            }
            double maxrel = 0;
            if (v > 1) {
                CK(hipMemcpy(out.data(), C, nC * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(ref.data(), vars[v].pair ? Cref2 : Cref, nC * 4, hipMemcpyDeviceToHost));
                double mx = 0, md = 0;
                for (size_t i = 0; i < nC; ++i) {
                    mx = fmax(mx, fabs((double)ref[i]));
                    md = fmax(md, fabs((double)out[i] - (double)ref[i]));
                }
                maxrel = md / (mx + 1e-30);
            }
            printf("%-8s %-22s best %8.3f ms  mean %8.3f ms  %7.1f TF/s(f32-equiv)  max|d|/max|ref| %.2e\n", sh.name,
                   vars[v].name, best, tot / reps, flops / (best * 1e-3) / 1e12, maxrel);
            fflush(stdout);
        }
        CK(hipFree(A)); CK(hipFree(Apl)); CK(hipFree(W)); CK(hipFree(Wp)); CK(hipFree(bias)); CK(hipFree(C)); CK(hipFree(Cref)); CK(hipFree(Cref2));
        CK(hipFree(Ah)); CK(hipFree(Wh)); CK(hipFree(unsc));
    }
    return 0;
}
