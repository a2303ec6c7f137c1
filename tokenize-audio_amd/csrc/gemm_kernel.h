// The implicit-GEMM Conv1d / Linear kernel template (included by gemm.hip and by tools/gemm_bench.hip).
#pragma once
#include "kernels.h"

namespace mimi {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float elu1(float x) { return elu_fast(x); }

// GELU(x) = x Phi(x) = x erfc(-x / sqrt 2) / 2 with one branch-free erfc (Numerical Recipes' erfcc Chebyshev fit,
// fractional error < 1.2e-7 for every argument): erfc(a) = t exp(-a^2 + P(t)), t = 1 / (1 + a / 2), a = |x| / sqrt 2;
// Phi(-|x|) = erfc(a) / 2 carries full relative precision where GELU's (1 + erf) cancels.  ~19 VALU (one rcp, one
// exp2) against ~40 for both of OCML erff's branches under divergence.  P's coefficients carry the log2(e) of exp2.
__device__ __forceinline__ float gelu_fast(float x) {
    constexpr float L2E = 1.4426950408889634f;
    const float a = fabsf(x) * 0.70710678118654752440f;
    const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.5f, a, 1.0f));
    float p = 0.17087277f * L2E;
    p = __builtin_fmaf(p, t, -0.82215223f * L2E);
    p = __builtin_fmaf(p, t, 1.48851587f * L2E);
    p = __builtin_fmaf(p, t, -1.13520398f * L2E);
    p = __builtin_fmaf(p, t, 0.27886807f * L2E);
    p = __builtin_fmaf(p, t, -0.18628806f * L2E);
    p = __builtin_fmaf(p, t, 0.09678418f * L2E);
    p = __builtin_fmaf(p, t, 0.37409196f * L2E);
    p = __builtin_fmaf(p, t, 1.00002368f * L2E);
    const float y = __builtin_fmaf(t, p, __builtin_fmaf(-a * L2E, a, -1.26551223f * L2E));
    const float h = 0.5f * (t * __builtin_amdgcn_exp2f(y));  // Phi(-|x|)
    return x * (x > 0.0f ? 1.0f - h : h);
}

// torch CPU GELU(approximate='none'): (x * 0.5) * (1 + erf(x * M_SQRT1_2))
__device__ __forceinline__ float gelu_erf(float x) {
#ifdef MIMI_GELU_DIAG  // timing diagnostic builds only (results wrong): the epilogue without erf
    return (x * 0.5f) * (1.0f + x * 0.70710678118654752440f);
#else
    return (x * 0.5f) * (1.0f + erff(x * 0.70710678118654752440f));
#endif
}

// RoPE rotate-half of the pair (x1 = dim d, x2 = dim d + 32), d < 32 (TF/modeling_mimi.py:384-404): the q/k/v
// GEMM epilogue (gemm_planes.h EPI_ROPE) and the fused q/k/v + attention kernel (qkv_attn.hip) form it with
// these two expressions, so both give the same bits
__device__ __forceinline__ float rope_lo(float x1, float x2, float c, float sn) { return x1 * c + (-x2) * sn; }
__device__ __forceinline__ float rope_hi(float x2, float x1, float c, float sn) { return x2 * c + x1 * sn; }

template <int BM, int BN, int WM, int WN, int BK, int NBUF, bool NFAST, bool ELU_IN, int PAD, int EPI, int TAG>
__global__ __launch_bounds__(WM* WN * 64) void gemm_f32_kernel(GemmArgs p) {
    constexpr int NT = WM * WN * 64;
    constexpr int LDK = BK + 4;
    constexpr int TM = BM / WM / 32;
    constexpr int TN = BN / WN / 32;
    constexpr int KQ = BK / 4;  // float4 per LDS row
    constexpr int A_F4 = BM * KQ / NT;
    constexpr int B_F4 = BN * KQ / NT;
    static_assert(NBUF == 1 || NBUF == 2, "buffers");
    static_assert(TM >= 1 && TN >= 1, "tile");
    static_assert(A_F4 * NT == BM * (BK / 4) && B_F4 * NT == BN * (BK / 4), "loader");
    static_assert(EPI != EPI_ROPE || (TN % 2 == 0), "rope pairs need even TN");

    __shared__ __attribute__((aligned(16))) float lds[NBUF * (BM + BN) * LDK];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN;
    const int wn = wave % WN;
    const int b = blockIdx.z;
    // NFAST: consecutive workgroups walk the N tiles of one M tile, so an activation tile is re-read by the
    // other N tiles while it is still in L2 / the Infinity Cache instead of one full pass over M later.
    int mt, nt;
    if (NFAST) {
        const int ntn = gridDim.y;
        const int lin = blockIdx.x * ntn + blockIdx.y;
        mt = lin / ntn;
        nt = lin % ntn;
        (void)ntn;
    } else {
        mt = blockIdx.x;
        nt = blockIdx.y;
    }
    const int m0 = mt * BM;
    const int n0 = nt * BN;
    const int M = p.M, N = p.N, K = p.K;

    const float* __restrict__ Ab = p.A + (long long)b * p.a_bstride;
    const float* __restrict__ W = p.W;

    f32x4 ra[A_F4];
    f32x4 rb[B_F4];

    auto gload = [&](int k0) {
#pragma unroll
        for (int i = 0; i < A_F4; ++i) {
            const int idx = tid + i * NT;
            const int r = idx / KQ;
            const int c = (idx % KQ) * 4;
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
            const int r = idx / KQ;
            const int c = (idx % KQ) * 4;
            const int n = n0 + r;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (n < N) v = *reinterpret_cast<const f32x4*>(W + (long long)n * K + k0 + c);
            rb[i] = v;
        }
    };
    auto sstore = [&](int buf) {
        float* As = lds + buf * (BM + BN) * LDK;
        float* Bs = As + BM * LDK;
#pragma unroll
        for (int i = 0; i < A_F4; ++i) {
            const int idx = tid + i * NT;
            const int r = idx / KQ;
            const int c = (idx % KQ) * 4;
            f32x4 v = ra[i];
            if (ELU_IN) {
                v.x = elu1(v.x); v.y = elu1(v.y); v.z = elu1(v.z); v.w = elu1(v.w);
            }
            *reinterpret_cast<f32x4*>(As + r * LDK + c) = v;
        }
#pragma unroll
        for (int i = 0; i < B_F4; ++i) {
            const int idx = tid + i * NT;
            const int r = idx / KQ;
            const int c = (idx % KQ) * 4;
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
    sstore(0);
    __syncthreads();
    for (int kt = 0; kt < KT; ++kt) {
        const int cur = NBUF == 2 ? (kt & 1) : 0;
        const float* As = lds + cur * (BM + BN) * LDK;
        const float* Bs = As + BM * LDK;
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
            if (NBUF == 1) __syncthreads();  // single buffer: every wave is done reading before the overwrite
            sstore(NBUF == 2 ? (cur ^ 1) : 0);
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


// ================================================================================================
// Split-bf16 variant: fp32 accuracy from the bf16 matrix cores.
//
// gfx950 has no xf32/tf32; its bf16 MFMA (v_mfma_f32_32x32x16_bf16) runs 16x the f32-MFMA rate.  Each fp32
// operand is split exactly into NS bf16 planes (x = x0 + x1 [+ x2], x_p = bf16(x - x0 - ... - x_{p-1})) and
// the product is the sum of the plane products whose plane indices add to < NS:
//   NS = 3: a0b0 + a0b1 + a1b0 + a0b2 + a1b1 + a2b0  (6 MFMAs, ~24-bit operands: fp32-level error, 2.7x f32 rate)
//   NS = 2: a0b0 + a0b1 + a1b0                       (3 MFMAs, ~16-bit operands: ~1e-5 rel error, 5.3x)
// bf16 x bf16 products are exact in fp32 and accumulate in fp32, so what is dropped is only the plane
// truncation (2^-24 resp. 2^-16 relative).  Activations are split as they are staged into LDS (after the
// optional ELU); weights are split once at load time and read from global as NS bf16 planes [NS][N][K].
// ================================================================================================
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// K-step order of the implicit-GEMM convs.  A K step reads a 64-B half line (32 channels) of one tap of
// every tile row.  Tap kk + s of output row m reads the input row that tap kk of row m + 1 reads, so each
// 128-B input line is touched 4 times per tile: 2 channel halves x 2 taps (k = 2s; 3 x 2 for k = 3, s = 1).
// Order (outer -> inner): chain start j < s, 128-B channel block hi, position c in the tap chain
// j, j+s, j+2s, ..., channel half lo -- so the 4 (6) touches of a line are consecutive K steps (L2 hits)
// instead of up to k*Cin/64 steps apart (with 30+ CUs streaming through an XCD's 4 MB L2 in between: HBM
// re-reads).  Linear layers (k = 1) get the plain order; layouts it does not cover too.  Wave-uniform state
// (SGPRs); advance with next() once per K step.
template <int BK>
struct KOrderT {
    int cin, s, cl, nhi, nlo, j, hi, c, lo;
    bool pair;  // visit only the first tap of each chain (gemm_planes FL_PAIR: the chain is 2 taps)
    __device__ __forceinline__ void init(const GemmArgs& p, bool pr = false) {
        j = hi = c = lo = 0;
        pair = pr;
        const int k = p.a_cin > 0 ? p.K / p.a_cin : 0;
        const int st = p.a_cin > 0 ? p.a_rs / p.a_cin : 0;
        if (p.a_cin % 64 == 0 && k * p.a_cin == p.K && st > 0 && st * p.a_cin == p.a_rs && k % st == 0) {
            cin = p.a_cin;
            s = st;
            cl = k / st;
        } else {  // plain order: one "tap" spanning all of K
            cin = 0;
            s = 1;
            cl = 1;
        }
        const int blk = (cin || p.K % 64 == 0) ? 64 : BK;  // 128-B channel block (or one K step)
        nlo = blk / BK;
        nhi = (cin ? cin : p.K) / blk;
    }
    __device__ __forceinline__ int offset() const { return (j + c * s) * cin + (hi * nlo + lo) * BK; }
    __device__ __forceinline__ void next() {
        if (++lo < nlo) return;
        lo = 0;
        if (!pair && ++c < cl) return;
        c = 0;
        if (++hi < nhi) return;
        hi = 0;
        ++j;
    }
};
using KOrder = KOrderT<32>;

template <int NS>
__device__ __forceinline__ void split_bf16x4(f32x4 v, bf16x4 (&out)[NS]) {
#pragma unroll
    for (int p = 0; p < NS; ++p) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const __bf16 h = (__bf16)v[i];
            out[p][i] = h;
            v[i] = v[i] - (float)h;  // exact in fp32
        }
    }
}

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// one 32x32x16 (MF = 32) or 16x16x32 (MF = 16) MFMA on bf16 or fp16 planes (the planes are carried as bf16x8
// bit patterns either way)
template <bool F16>
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
    if constexpr (F16)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                      0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <bool F16>
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
    if constexpr (F16)
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                      0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// the plane products of one (i, j) tile pair: small terms first, the leading product last
template <int NS, int TM, int TN, bool F16 = false, typename AccT>
__device__ __forceinline__ void mma_split(AccT (&acc)[TM][TN], const bf16x8 (&a)[NS][TM], const bf16x8 (&b)[NS][TN]) {
    auto mf = [](bf16x8 x, bf16x8 y, AccT c) {
        if constexpr (sizeof(AccT) == 64)
            return mfma32<F16>(x, y, c);
        else
            return mfma16<F16>(x, y, c);
    };
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            if (NS == 3) {
                acc[i][j] = mf(a[2 % NS][i], b[0][j], acc[i][j]);
                acc[i][j] = mf(a[1][i], b[1][j], acc[i][j]);
                acc[i][j] = mf(a[0][i], b[2 % NS][j], acc[i][j]);
            }
            acc[i][j] = mf(a[1][i], b[0][j], acc[i][j]);
            acc[i][j] = mf(a[0][i], b[1][j], acc[i][j]);
            acc[i][j] = mf(a[0][i], b[0][j], acc[i][j]);
        }
}

template <int BM, int BN, int WM, int WN, int NS, bool ELU_IN, int PAD, int EPI, int TAG>
__global__ __launch_bounds__(WM* WN * 64) void gemm_bf16x_kernel(GemmArgs p) {
    constexpr int NT = WM * WN * 64;
    constexpr int NW = WM * WN;
    constexpr int BK = 32;
    constexpr int LDB = BK + 8;  // A image: bf16 per row (80 B stride keeps ds_read_b128 conflict-free)
    constexpr int TM = BM / WM / 32;
    constexpr int TN = BN / WN / 32;
    constexpr int A_F4 = BM * (BK / 4) / NT;  // fp32 float4 per thread
    constexpr int BPL = BN * BK;              // B image plane: [BN][32] bf16, 16-B chunks XOR-swizzled
    constexpr int BCH = NS * BN / 16;         // 1 KB LDS-DMA pieces per K slice
    static_assert(NS == 2 || NS == 3, "planes");
    static_assert(TM >= 1 && TN >= 1, "tile");
    static_assert(A_F4 * NT == BM * (BK / 4), "loader");
    static_assert(EPI != EPI_ROPE || (TN % 2 == 0), "rope pairs need even TN");

    // A: activations split in registers, written as NS padded planes; B: weight planes streamed by LDS-DMA
    // (global_load_lds, no VGPRs, no ds_write) into a double-buffered swizzled image.
    __shared__ __attribute__((aligned(16))) __bf16 lds[NS * BM * LDB + 2 * NS * BPL];
    __bf16* As = lds;
    __bf16* Bs0 = lds + NS * BM * LDB;

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
    const __bf16* __restrict__ Wp = reinterpret_cast<const __bf16*>(p.Wsplit);

    const int a_len = (int)p.a_len;
    int aoff[A_F4];
    bool aok[A_F4];
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
        const int idx = tid + i * NT;
        const int m = m0 + (idx >> 3);
        aok[i] = m < M;
        aoff[i] = (int)(p.a_off + (long long)m * p.a_rs) + (idx & 7) * 4;
    }
    // this lane's LDS-DMA source rows: piece j = wave + q*NW covers 16 rows of one plane
    constexpr int NQ = (BCH + NW - 1) / NW;
    int bsrc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int j = wave + q * NW;
        const int pl = j / (BN / 16), rb = j % (BN / 16);
        const int row = rb * 16 + (lane >> 2);
        const int c = (lane & 3) ^ ((row >> 2) & 3);  // logical 16-B chunk stored at physical chunk lane&3
        int n = n0 + row;
        n = n < N ? n : N - 1;  // rows past N only feed columns that are never stored
        bsrc[q] = (pl * N + n) * K + c * 8;
    }
    f32x4 ra[A_F4];
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
    const int kh = (lane >> 5) * 8;

#define MIMI_SPLIT_LOAD_A(k0)                                                                  \
    _Pragma("unroll") for (int i = 0; i < A_F4; ++i) {                                         \
        const int e = aoff[i] + (k0);                                                          \
        f32x4 v;                                                                               \
        if (PAD == PAD_ZERO) {                                                                 \
            const bool ok = aok[i] && e >= 0 && e < a_len;                                     \
            v = *reinterpret_cast<const f32x4*>(Ab + (ok ? e : 0));                            \
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};                                              \
            v = ok ? v : z;                                                                    \
        } else {                                                                               \
            const int cin = p.a_cin;                                                           \
            int t = e >= 0 ? e / cin : -((-e + cin - 1) / cin);                                \
            const int ch = e - t * cin;                                                        \
            const int tmax = a_len / cin - 1;                                                  \
            t = t < 0 ? 0 : (t > tmax ? tmax : t);                                             \
            v = *reinterpret_cast<const f32x4*>(Ab + t * cin + ch);                            \
        }                                                                                      \
        ra[i] = v;                                                                             \
    }
#define MIMI_SPLIT_DMA_B(k0, buf)                                                              \
    _Pragma("unroll") for (int q = 0; q < NQ; ++q) {                                           \
        const int j = wave + q * NW;                                                           \
        if (j < BCH) {                                                                         \
            const int pl = j / (BN / 16), rb = j % (BN / 16);                                  \
            __bf16* dst = Bs0 + (buf) * NS * BPL + pl * BPL + rb * 16 * BK;                    \
            __builtin_amdgcn_global_load_lds((const void*)(Wp + bsrc[q] + (k0)),               \
                (__attribute__((address_space(3))) void*)dst, 16, 0, 0);                       \
        }                                                                                      \
    }
#define MIMI_SPLIT_STORE_A()                                                                   \
    _Pragma("unroll") for (int i = 0; i < A_F4; ++i) {                                         \
        const int idx = tid + i * NT;                                                          \
        f32x4 v = ra[i];                                                                       \
        if (ELU_IN) {                                                                          \
            v.x = elu1(v.x); v.y = elu1(v.y); v.z = elu1(v.z); v.w = elu1(v.w);                \
        }                                                                                      \
        bf16x4 h[NS];                                                                          \
        split_bf16x4<NS>(v, h);                                                                \
        __bf16* dst = As + (idx >> 3) * LDB + (idx & 7) * 4;                                   \
        _Pragma("unroll") for (int pl = 0; pl < NS; ++pl)                                      \
            *reinterpret_cast<bf16x4*>(dst + pl * BM * LDB) = h[pl];                           \
    }

    KOrder ko;
    ko.init(p);
    MIMI_SPLIT_LOAD_A(ko.offset())
    MIMI_SPLIT_DMA_B(ko.offset(), 0)
    MIMI_SPLIT_STORE_A()
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < KT; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < KT) {
            ko.next();
            const int k1 = ko.offset();
            MIMI_SPLIT_LOAD_A(k1)
            MIMI_SPLIT_DMA_B(k1, cur ^ 1)
        }
        const __bf16* Bs = Bs0 + cur * NS * BPL;
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
            bf16x8 af[NS][TM], bf[NS][TN];
#pragma unroll
            for (int pl = 0; pl < NS; ++pl) {
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    af[pl][i] = *reinterpret_cast<const bf16x8*>(As + pl * BM * LDB + (arow + i * 32) * LDB + kk * 16 + kh);
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int row = brow + j * 32;
                    const int phys = ((kk * 2 + (lane >> 5)) ^ ((row >> 2) & 3)) * 8;
                    bf[pl][j] = *reinterpret_cast<const bf16x8*>(Bs + pl * BPL + row * BK + phys);
                }
            }
            mma_split<NS, TM, TN>(acc, af, bf);
        }
        if (kt + 1 < KT) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            MIMI_SPLIT_STORE_A()
            __syncthreads();
        }
    }
#undef MIMI_SPLIT_LOAD_A
#undef MIMI_SPLIT_DMA_B
#undef MIMI_SPLIT_STORE_A

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

}  // namespace mimi
