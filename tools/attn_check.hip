// Determinism / accuracy probe of the attention kernels (tuning aid, not shipped):
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I tokenize-audio_amd/csrc \
//     tools/attn_check.hip tokenize-audio_amd/csrc/ops.hip -o tools/bin/attn_check
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kernels.h"

using namespace mimi;
#define CK(x)                                                                                        \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);              \
            exit(1);                                                                                 \
        }                                                                                            \
    } while (0)

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 32, T = argc > 2 ? atoi(argv[2]) : 500, H = 8, D = 64, W = 250;
    const size_t nq = (size_t)B * T * 3 * H * D, no = (size_t)B * T * H * D;
    std::vector<float> hq(nq);
    unsigned long long x = 88172645463325252ull;
    for (auto& v : hq) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        v = (float)((x >> 40) * (1.0 / (1ull << 24)) - 0.5) * 4.0f;
    }
    float *q, *ref;
    _Float16* pl;
    unsigned* amax;
    CK(hipMalloc(&q, nq * 4));
    CK(hipMalloc(&ref, no * 4));
    CK(hipMalloc(&pl, 2 * no * 2));
    CK(hipMalloc(&amax, 64 * 16 * 4));
    if (argc > 3) {  // raw fp32 qkv [B][T][3 H D] (e.g. the engine's qkv0 tap)
        FILE* f = fopen(argv[3], "rb");
        if (!f || fread(hq.data(), 4, nq, f) != nq) {
            fprintf(stderr, "read %s failed\n", argv[3]);
            return 1;
        }
        fclose(f);
    }
    CK(hipMemcpy(q, hq.data(), nq * 4, hipMemcpyHostToDevice));
    CK(launch_attention(q, ref, B, T, H, D, W, 0.125f, 0, nullptr, 0, 0, 0.0f, nullptr, false));
    CK(hipDeviceSynchronize());
    std::vector<float> r(no);
    CK(hipMemcpy(r.data(), ref, no * 4, hipMemcpyDeviceToHost));
    std::vector<_Float16> first(2 * no), cur(2 * no);
    const float os = 4096.0f;
    for (int rep = 0; rep < 6; ++rep) {
        CK(launch_attention(q, nullptr, B, T, H, D, W, 0.125f, 0, pl, (long long)no, 2, os, amax, true));
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(cur.data(), pl, 2 * no * 2, hipMemcpyDeviceToHost));
        size_t ndiff = 0, first_i = 0;
        double md = 0, mx = 0;
        for (size_t i = 0; i < no; ++i) {
            const double v = ((double)(float)cur[i] + (double)(float)cur[no + i]) / os;
            md = fmax(md, fabs(v - r[i]));
            mx = fmax(mx, fabs(r[i]));
        }
        if (rep == 0) first = cur;
        for (size_t i = 0; i < 2 * no; ++i)
            if (*(uint16_t*)&cur[i] != *(uint16_t*)&first[i]) {
                if (!ndiff) first_i = i;
                ++ndiff;
            }
        size_t fi = first_i % no;
        printf("rep %d: max|h16 - f32| / max|f32| = %.3e, differs from rep 0 in %zu halves (first: b %zu t %zu h %zu d %zu)\n",
               rep, md / mx, ndiff, fi / ((size_t)T * H * D), (fi / (H * D)) % T, (fi / D) % H, fi % D);
    }
    // timing: the two fp16-plane kernels on this shape (T <= 256 only for the whole-head one)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto&& launch, const char* name) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 20; ++i) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s B %d T %d: %8.2f us per launch\n", name, B, T, ms * 1000.0f / 20);
    };
    timeit([&] { (void)launch_attention(q, nullptr, B, T, H, D, W, 0.125f, 0, pl, (long long)no, 2, os, amax, true); },
           T <= 256 ? "attention_t256_h16" : "attention_band_h16");
    if (T <= 256) {
        timeit([&] { (void)launch_attention_band(q, B, T, H, W, 0.125f, 0, pl, (long long)no, os, amax); },
               "attention_band_h16");
    }
    timeit([&] { (void)launch_attention(q, ref, B, T, H, D, W, 0.125f, 0, nullptr, 0, 0, 0.0f, nullptr, false); },
           "fp32");
    return 0;
}
