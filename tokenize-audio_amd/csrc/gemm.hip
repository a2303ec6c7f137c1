// Implicit-GEMM Conv1d / Linear on fp32 MFMA (v_mfma_f32_32x32x2_f32) for gfx950.
//
// Every conv of the Mimi encoder (TF/modeling_mimi.py:210-347, causal MimiConv1d) and every dense
// projection of its transformer (:657-726, :602-615) is one GEMM over a channels-last activation:
//   out[t][co] = sum_{kk, ci} x[t*s - pad + kk][ci] * W'[co][kk*Cin + ci]
// With channels-last storage, row t of the im2col matrix is the CONTIGUOUS span
//   x_flat[(t*s - pad)*Cin, (t*s - pad + k)*Cin)
// so A is an ordinary row-major operand with row stride s*Cin (rows overlap in memory when k > s); no
// im2col buffer, no gather.  Causal left padding / right "extra" padding are bounds checks on that span.
//
// Tile: BM x BN x 32, WM x WN waves, each wave a (BM/WM) x (BN/WN) block of 32x32 MFMA tiles.
// Operands are staged global -> registers -> LDS ([row][32+4] fp32, +4 pad makes the ds_read_b128
// fragment reads conflict-free); the next K-slice's global loads are issued before the current slice's
// MFMAs so their latency hides under 64 * (BM/WM/32) * (BN/WN/32) MFMA cycles per wave.
// Fused prologue: ELU on A as it is written to LDS.  Fused epilogues: bias, ELU, residual add, GELU(erf),
// layer scale + residual, RoPE (rotate-half pairs (d, d+32) live in the same lane of tiles tn, tn+1).
#include "kernels.h"

#include <cstdio>

namespace mimi {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float elu1(float x) { return x > 0.0f ? x : expm1f(x); }

// torch CPU GELU(approximate='none'): (x * 0.5) * (1 + erf(x * M_SQRT1_2))
__device__ __forceinline__ float gelu_erf(float x) {
    return (x * 0.5f) * (1.0f + erff(x * 0.70710678118654752440f));
}

template <int BM, int BN, int WM, int WN, bool ELU_IN, int PAD, int EPI, int TAG>
__global__ __launch_bounds__(WM* WN * 64) void gemm_f32_kernel(GemmArgs p) {
    constexpr int NT = WM * WN * 64;
    constexpr int BK = 32;
    constexpr int LDK = BK + 4;
    constexpr int TM = BM / WM / 32;
    constexpr int TN = BN / WN / 32;
    constexpr int A_F4 = BM * (BK / 4) / NT;
    constexpr int B_F4 = BN * (BK / 4) / NT;
    static_assert(TM >= 1 && TN >= 1, "tile");
    static_assert(A_F4 * NT == BM * (BK / 4) && B_F4 * NT == BN * (BK / 4), "loader");
    static_assert(EPI != EPI_ROPE || (TN % 2 == 0), "rope pairs need even TN");

    __shared__ __attribute__((aligned(16))) float lds[(BM + BN) * LDK];
    float* As = lds;
    float* Bs = lds + BM * LDK;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN;
    const int wn = wave % WN;
    const int b = blockIdx.z;
    const int m0 = blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const int M = p.M, N = p.N, K = p.K;

    const float* __restrict__ Ab = p.A + (long long)b * p.a_bstride;
    const float* __restrict__ W = p.W;

    f32x4 ra[A_F4];
    f32x4 rb[B_F4];

    auto gload = [&](int k0) {
#pragma unroll
        for (int i = 0; i < A_F4; ++i) {
            const int idx = tid + i * NT;
            const int r = idx >> 3;
            const int c = (idx & 7) * 4;
            const int m = m0 + r;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (m < M) {
                long long e = p.a_off + (long long)m * p.a_rs + k0 + c;
                if (PAD == PAD_ZERO) {
                    if (e >= 0 && e < p.a_len) v = *reinterpret_cast<const f32x4*>(Ab + e);
                } else {
                    const long long cin = p.a_cin;
                    long long t = e >= 0 ? e / cin : -((-e + cin - 1) / cin);
                    const long long ch = e - t * cin;
                    const long long tmax = p.a_len / cin - 1;
                    t = t < 0 ? 0 : (t > tmax ? tmax : t);
                    v = *reinterpret_cast<const f32x4*>(Ab + t * cin + ch);
                }
            }
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < B_F4; ++i) {
            const int idx = tid + i * NT;
            const int r = idx >> 3;
            const int c = (idx & 7) * 4;
            const int n = n0 + r;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (n < N) v = *reinterpret_cast<const f32x4*>(W + (long long)n * K + k0 + c);
            rb[i] = v;
        }
    };
    auto sstore = [&]() {
#pragma unroll
        for (int i = 0; i < A_F4; ++i) {
            const int idx = tid + i * NT;
            const int r = idx >> 3;
            const int c = (idx & 7) * 4;
            f32x4 v = ra[i];
            if (ELU_IN) {
                v.x = elu1(v.x); v.y = elu1(v.y); v.z = elu1(v.z); v.w = elu1(v.w);
            }
            *reinterpret_cast<f32x4*>(As + r * LDK + c) = v;
        }
#pragma unroll
        for (int i = 0; i < B_F4; ++i) {
            const int idx = tid + i * NT;
            const int r = idx >> 3;
            const int c = (idx & 7) * 4;
            *reinterpret_cast<f32x4*>(Bs + r * LDK + c) = rb[i];
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    const int KT = K / BK;
    const int arow = wm * TM * 32 + (lane & 31);
    const int brow = wn * TN * 32 + (lane & 31);
    const int kh = (lane >> 5) * 4;

    gload(0);
    sstore();
    __syncthreads();
    for (int kt = 0; kt < KT; ++kt) {
        if (kt + 1 < KT) gload((kt + 1) * BK);
#pragma unroll
        for (int kq = 0; kq < BK / 8; ++kq) {
            f32x4 af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                af[i] = *reinterpret_cast<const f32x4*>(As + (arow + i * 32) * LDK + kq * 8 + kh);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bf[j] = *reinterpret_cast<const f32x4*>(Bs + (brow + j * 32) * LDK + kq * 8 + kh);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < KT) {
            __syncthreads();
            sstore();
            __syncthreads();
        }
    }

    // ---- epilogue: lane holds col (lane&31), rows (r&3) + 8*(r>>2) + 4*(lane>>5) of each 32x32 tile
    float* __restrict__ Cb = p.C + (long long)b * p.c_bstride;
    const float* __restrict__ Rb = p.R ? p.R + (long long)b * p.c_bstride : nullptr;
    const int rbase = m0 + wm * TM * 32 + 4 * (lane >> 5);
    const int cbase = n0 + wn * TN * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = cbase + j * 32;
            float bias = 0.0f, scale = 0.0f;
            if (col < N) {
                if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU || EPI == EPI_BIAS_RES_ELU || EPI == EPI_BIAS_OUT)
                    bias = p.bias[col];
                if (EPI == EPI_SCALE_RES) scale = p.scale[col];
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = rbase + i * 32 + (r & 3) + 8 * (r >> 2);
                if (row >= M || col >= N) continue;
                float v = acc[i][j][r];
                const long long off = (long long)row * p.ldc + col;
                if (EPI == EPI_BIAS || EPI == EPI_BIAS_OUT) {
                    v = v + bias;
                } else if (EPI == EPI_BIAS_ELU) {
                    v = elu1(v + bias);
                } else if (EPI == EPI_BIAS_RES_ELU) {
                    v = elu1(Rb[off] + (v + bias));
                } else if (EPI == EPI_GELU) {
                    v = gelu_erf(v);
                } else if (EPI == EPI_SCALE_RES) {
                    v = Rb[off] + scale * v;
                } else if (EPI == EPI_ROPE) {
                    // pair (j even -> first half d, j+1 -> second half d+32) of one head
                    const int hd2 = 32;
                    if (col < p.rope_cols) {
                        const int d = (col % 64);  // head_dim = 64
                        const float c = p.rope_cos[(long long)row * hd2 + (d & 31)];
                        const float sn = p.rope_sin[(long long)row * hd2 + (d & 31)];
                        if ((j & 1) == 0) {
                            const float x2 = acc[i][j + 1][r];
                            v = v * c + (-x2) * sn;
                        } else {
                            const float x1 = acc[i][j - 1][r];
                            v = v * c + x1 * sn;
                        }
                    }
                }
                Cb[off] = v;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// role -> instantiation
// ------------------------------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, bool ELU_IN, int PAD, int EPI, int TAG>
static const char* kernel_symbol() {
    static char name[128];
    if (!name[0])
        snprintf(name, sizeof(name), "mimi::gemm_f32_kernel<%d, %d, %d, %d, %s, %d, %d, %d>", BM, BN, WM, WN,
                 ELU_IN ? "true" : "false", PAD, EPI, TAG);
    return name;
}

static thread_local const char* g_last_kernel = nullptr;

template <int BM, int BN, int WM, int WN, bool ELU_IN, int PAD, int EPI, int TAG>
static hipError_t run(const GemmArgs& a, hipStream_t s) {
    g_last_kernel = kernel_symbol<BM, BN, WM, WN, ELU_IN, PAD, EPI, TAG>();
    dim3 grid((a.M + BM - 1) / BM, (a.N + BN - 1) / BN, a.batch);
    dim3 block(WM * WN * 64);
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, ELU_IN, PAD, EPI, TAG>), grid, block, 0, s, a);
    return hipGetLastError();
}

// Tile choice by output width: N = 32 (res0 conv k3) gets 256x32, N = 64 gets 256x64, wider gets 128x128;
// the transformer-sized problems (M <= 1024 per item) use 64-row tiles to keep >1 workgroup per CU.
template <bool ELU_IN, int PAD, int EPI, int TAG>
static hipError_t run_auto(const GemmArgs& a, hipStream_t s) {
    if (a.N <= 32) return run<256, 32, 4, 1, ELU_IN, PAD, EPI, TAG>(a, s);
    if (a.N <= 64) return run<256, 64, 4, 1, ELU_IN, PAD, EPI, TAG>(a, s);
    if (a.M <= 1024) return run<64, 128, 1, 2, ELU_IN, PAD, EPI, TAG>(a, s);
    return run<128, 128, 2, 2, ELU_IN, PAD, EPI, TAG>(a, s);
}

static hipError_t dispatch(int role, const GemmArgs& a, hipStream_t s);

hipError_t launch_gemm(int role, const GemmArgs& a, hipStream_t s, const char** kname) {
    if (a.K % 32 != 0 || a.a_cin % 4 != 0 || a.a_rs % 4 != 0 || a.M <= 0 || a.N <= 0 || a.batch <= 0)
        return hipErrorInvalidValue;
    g_last_kernel = nullptr;
    hipError_t e = dispatch(role, a, s);
    if (kname) *kname = g_last_kernel ? g_last_kernel : "?";
    return e;
}

static hipError_t dispatch(int role, const GemmArgs& a, hipStream_t s) {
    switch (role) {
        case ROLE_RES3: return run_auto<true, PAD_ZERO, EPI_BIAS_ELU, 0>(a, s);
        case ROLE_RES1: return run_auto<false, PAD_ZERO, EPI_BIAS_RES_ELU, 1>(a, s);
        case ROLE_DOWN: return run_auto<false, PAD_ZERO, EPI_BIAS, 2>(a, s);
        case ROLE_DOWN_ELU: return run_auto<false, PAD_ZERO, EPI_BIAS_ELU, 3>(a, s);
        case ROLE_FINAL: return run_auto<false, PAD_ZERO, EPI_BIAS_OUT, 4>(a, s);
        case ROLE_QKV: return run<64, 128, 1, 2, false, PAD_ZERO, EPI_ROPE, 5>(a, s);
        case ROLE_OPROJ: return run_auto<false, PAD_ZERO, EPI_SCALE_RES, 6>(a, s);
        case ROLE_FC1: return run_auto<false, PAD_ZERO, EPI_GELU, 7>(a, s);
        case ROLE_FC2: return run_auto<false, PAD_ZERO, EPI_SCALE_RES, 8>(a, s);
        case ROLE_DOWNSAMPLE: return run_auto<false, PAD_REPLICATE, EPI_NONE, 9>(a, s);
        case ROLE_INPROJ: return run_auto<false, PAD_ZERO, EPI_NONE, 10>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mimi
