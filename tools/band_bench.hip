// Timing + bit check of the banded attention kernel's two forms (tuning aid, not shipped):
//   hipcc -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -I tokenize-audio_amd/csrc \
//     tools/band_bench.hip tokenize-audio_amd/csrc/ops.hip -o tools/bin/band_bench
//   tools/bin/band_bench [B T]...     (default: the YODAS2-like long items 17 x 378, 32 x 500, 1 x 500)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
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

static void run(int B, int T) {
    const int H = 8, D = 64, W = 250;
    const size_t nq = (size_t)B * T * 3 * H * D, no = (size_t)B * T * H * D;
    std::vector<float> hq(nq);
    unsigned long long x = 88172645463325252ull;
    for (auto& v : hq) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        v = (float)((x >> 40) * (1.0 / (1ull << 24)) - 0.5) * 4.0f;
    }
    float* q;
    _Float16 *pa, *pb;
    unsigned* amax;
    CK(hipMalloc(&q, nq * 4));
    CK(hipMalloc(&pa, 2 * no * 2));
    CK(hipMalloc(&pb, 2 * no * 2));
    CK(hipMalloc(&amax, 64 * 16 * 4));
    CK(hipMemcpy(q, hq.data(), nq * 4, hipMemcpyHostToDevice));
    const float os = 4096.0f;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float us[3] = {0, 0, 0};
    for (int split = 0; split <= 2; split += 2) {
        _Float16* p = split ? pb : pa;
        auto launch = [&] { CK(launch_attention_band(q, B, T, H, W, 0.125f, 0, p, (long long)no, os, amax, split)); };
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 20; ++i) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        us[split] = ms * 1000.0f / 20;
    }
    std::vector<uint16_t> a(2 * no), b(2 * no);
    CK(hipMemcpy(a.data(), pa, 2 * no * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), pb, 2 * no * 2, hipMemcpyDeviceToHost));
    size_t nd = 0;
    for (size_t i = 0; i < 2 * no; ++i) nd += a[i] != b[i];
    printf("B %3d T %4d: wide %8.2f us, split %8.2f us per launch; wide vs split: %zu halves differ\n", B, T, us[0],
           us[2], nd);
    CK(hipFree(q));
    CK(hipFree(pa));
    CK(hipFree(pb));
    CK(hipFree(amax));
}

int main(int argc, char** argv) {
    if (argc > 2) {
        for (int i = 1; i + 1 < argc; i += 2) run(atoi(argv[i]), atoi(argv[i + 1]));
    } else {
        run(17, 378);
        run(32, 500);
        run(8, 500);
        run(1, 500);
    }
    return 0;
}
