// Fused SEANet residual block (TF/modeling_mimi.py:408-447, with the ELU that precedes the next down conv):
//   y = ELU( x + b1 + W1 . ELU( b3 + W3 (*) ELU(x) ) )          x, y: [B][T][C] channels-last
// W3: causal k=3 conv C -> C/2 (W'[n][kk*C + ci]), W1: k=1 conv C/2 -> C.  One workgroup owns BM time rows:
//   GEMM1  h[BM][C/2] = ELU(x) window (*) W3   -> ELU(h + b3) kept in LDS (never written to HBM)
//   GEMM2  y[BM][C]   = h . W1^T, in column passes of NP, epilogue + b1 + x (residual), ELU -> HBM
// so the block reads x once and writes y once (the unfused pair moved x, h, h, x, y).
// WINDOW: the (BM+2) x C slab of ELU(x) (rows m0-2 .. m0+BM-1, causal zeros before t=0) is staged in LDS once
//   and GEMM1's im2col rows are overlapping windows of it (row i, tap kk = slab row i+kk): one ELU per element.
// STREAM (large C, where the slab does not fit): GEMM1's A is streamed in 32-wide K slices with ELU on load.
// All MFMAs are v_mfma_f32_32x32x2_f32; LDS rows are padded by 4 floats (row stride = 4 mod 64 dwords), which
// keeps the ds_read_b128 fragment reads conflict-free.
#include <algorithm>
#include <type_traits>

#include "gemm_kernel.h"
#include "resblock_h16.h"

namespace mimi {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float elu_f(float x) { return elu_fast(x); }
__device__ __forceinline__ f32x4 elu4(f32x4 v) {
    v.x = elu_f(v.x); v.y = elu_f(v.y); v.z = elu_f(v.z); v.w = elu_f(v.w);
    return v;
}

// acc[TM][TN] += A[rows][32] . B[cols][32]^T for one 32-wide K slice.  A / B point at the wave's first row /
// first column (row r at A + r*lda); lane (i, h) feeds k = 8*kq + 4*h + s at step s of quad kq.
template <int TM, int TN>
__device__ __forceinline__ void mma_k32(f32x16 (&acc)[TM][TN], const float* A, int lda, const float* B, int ldb,
                                        int lane) {
    const int r = lane & 31;
    const int kh = (lane >> 5) * 4;
#pragma unroll
    for (int kq = 0; kq < 4; ++kq) {
        f32x4 af[TM], bf[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const f32x4*>(A + (i * 32 + r) * lda + kq * 8 + kh);
#pragma unroll
        for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const f32x4*>(B + (j * 32 + r) * ldb + kq * 8 + kh);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    }
}

// Stores one wave's 32 x 64 block of y (v[j][r] in the MFMA C layout: row (r&3) + 8(r>>2) + 4h, column
// 32j + (lane&31)) through an 8 x 68-float wave-private LDS buffer, 8 rows at a time, so that each lane writes
// 8 consecutive values of one row: 2 x 16 B of fp32, or one 16-B bf16x8 per plane -- instead of one scattered
// 4-byte (or per plane 2-byte) store per value.  Same wave writes and reads: LDS order needs no barrier.
constexpr int YSTG_LD = 68;
constexpr int YSTG_FLOATS = 8 * YSTG_LD;
__device__ __forceinline__ void store_y_block(const ResArgs& p, float* stg, const f32x16 (&v)[2], long long ybase,
                                              long long row0, int col0, int C, long long T, int lane, float& mx) {
    const int h = lane >> 5, c = lane & 31;
    const int lr = lane >> 3, lc = (lane & 7) * 8;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) stg[(rr + 4 * h) * YSTG_LD + 32 * j + c] = v[j][4 * g + rr];
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(stg + lr * YSTG_LD + lc);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(stg + lr * YSTG_LD + lc + 4);
        const long long row = row0 + 8 * g + lr;
        if (row < T) {
            const long long idx = ybase + row * C + col0 + lc;
            if (p.yns == 0) {
                *reinterpret_cast<f32x4*>(p.y + idx) = a0;
                *reinterpret_cast<f32x4*>(p.y + idx + 4) = a1;
            } else {
                const float vv[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
                store_act8(p.yp, p.y_pstride, p.yns, idx, vv, p.yscale, &mx);
            }
        }
    }
}

template <int C, int BM, bool WINDOW, bool FIRST, int W1M, int W1N, int W2M, int W2N, int NP>
__global__ __launch_bounds__(256) void resblock_kernel(ResArgs p) {
    constexpr int H = C / 2;
    constexpr int K1 = 3 * C;
    constexpr int LDK = 36;
    constexpr int LDX = C + 4;
    constexpr int LDH = H + 4;
    constexpr int TM1 = BM / W1M / 32, TN1 = H / W1N / 32;
    constexpr int TM2 = BM / W2M / 32, TN2 = NP / W2N / 32;
    static_assert(W1M * W1N == 4 && W2M * W2N == 4, "4 waves");
    static_assert(TM1 >= 1 && TN1 >= 1 && TM2 >= 1 && TN2 >= 1, "tiles");
    static_assert(C % NP == 0 && H % 32 == 0, "shapes");
    // Xs (the ELU(x) slab / streamed A slices) is dead after GEMM1 and doubles as the y staging of store_y_block
    constexpr int XS0 = WINDOW ? (BM + 2) * LDX : BM * LDK;
    constexpr int XS = XS0 > 4 * YSTG_FLOATS ? XS0 : 4 * YSTG_FLOATS;
    constexpr int BST = (H > NP ? H : NP) * LDK;
    constexpr int A_F4 = WINDOW ? 1 : BM * 8 / 256;  // streamed A slice: float4 per thread
    constexpr int B1_F4 = H * 8 / 256 > 0 ? H * 8 / 256 : 1;
    constexpr int B2_F4 = NP * 8 / 256 > 0 ? NP * 8 / 256 : 1;
    static_assert(WINDOW || A_F4 * 256 == BM * 8, "A loader");
    static_assert(!FIRST || (WINDOW && C == 64), "conv0 fusion is for the 64-channel first stage");
    constexpr int AUD = FIRST ? BM + 8 + 64 * 8 : 0;  // audio window + conv0 weights/bias (FIRST)

    __shared__ __attribute__((aligned(16))) float lds[XS + BM * LDH + BST + AUD];
    float* Xs = lds;
    float* Hs = lds + XS;
    float* Bs = Hs + BM * LDH;
    float* Aud = Bs + BST;  // FIRST: audio[m0-8 .. m0+BM), then w0[64][7] (stride 8), b0[64]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long long T = p.T;
    const long long m0 = (long long)blockIdx.x * BM;
    const int b = blockIdx.y;
    const float* __restrict__ xb = p.x + (long long)b * T * C;

    // ---------------- GEMM1: h = ELU(x) (*) W3 ----------------
    if (FIRST) {
        // conv0 (Cin = 1, k = 7, TF/modeling_mimi.py:455) recomputed per tile from the audio: the 24 kHz x0
        // tensor never exists in HBM.  Same arithmetic as conv0_kernel: fmaf chain over taps, then + bias.
        const float* ab = p.audio + (long long)b * T;
        for (int i = tid; i < BM + 8; i += 256) {
            const long long pos = m0 - 8 + i;
            Aud[i] = (pos >= 0 && pos < T) ? ab[pos] : 0.0f;
        }
        for (int i = tid; i < 64 * 7; i += 256) Aud[BM + 8 + (i / 7) * 8 + (i % 7)] = p.w0[i];
        for (int i = tid; i < 64; i += 256) Aud[BM + 8 + i * 8 + 7] = p.b0[i];
        __syncthreads();
        for (int idx = tid; idx < (BM + 2) * 64; idx += 256) {
            const int r = idx >> 6, c = idx & 63;
            const long long pos = m0 - 2 + r;
            float v = 0.0f;  // causal zero padding of x0 before t = 0
            if (pos >= 0) {
                const float* wr = Aud + BM + 8 + c * 8;
                float acc = 0.0f;
#pragma unroll
                for (int k = 0; k < 7; ++k) acc = fmaf(wr[k], Aud[r + k], acc);  // audio[pos - 6 + k]
                v = elu_f(acc + wr[7]);
            }
            Xs[r * LDX + c] = v;
        }
    } else if (WINDOW) {
        constexpr int TOT = (BM + 2) * (C / 4);
        constexpr int NPRO = (TOT + 255) / 256;
        f32x4 pre[NPRO];
#pragma unroll
        for (int i = 0; i < NPRO; ++i) {  // all loads in flight before the first use
            const int idx = tid + i * 256;
            const int r = idx / (C / 4), c = (idx % (C / 4)) * 4;
            const long long pos = m0 - 2 + r;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (idx < TOT && pos >= 0 && pos < T) v = *reinterpret_cast<const f32x4*>(xb + pos * C + c);
            pre[i] = v;
        }
#pragma unroll
        for (int i = 0; i < NPRO; ++i) {
            const int idx = tid + i * 256;
            const int r = idx / (C / 4), c = (idx % (C / 4)) * 4;
            if (idx < TOT) *reinterpret_cast<f32x4*>(Xs + r * LDX + c) = elu4(pre[i]);
        }
    }
    f32x4 ra[A_F4], rb[B1_F4 > B2_F4 ? B1_F4 : B2_F4];
    auto load1 = [&](int k0) {
        if (!WINDOW) {
#pragma unroll
            for (int i = 0; i < A_F4; ++i) {
                const int idx = tid + i * 256;
                const int r = idx >> 3, c = (idx & 7) * 4;
                const long long e = (m0 + r - 2) * C + k0 + c;  // causal pad 2 rows; rows >= T never read
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if (m0 + r < T && e >= 0) v = *reinterpret_cast<const f32x4*>(xb + e);
                ra[i] = v;
            }
        }
#pragma unroll
        for (int i = 0; i < B1_F4; ++i) {
            const int idx = tid + i * 256;
            const int r = idx >> 3, c = (idx & 7) * 4;
            if (r < H) rb[i] = *reinterpret_cast<const f32x4*>(p.w3 + (long long)r * K1 + k0 + c);
        }
    };
    auto store1 = [&]() {
        if (!WINDOW) {
#pragma unroll
            for (int i = 0; i < A_F4; ++i) {
                const int idx = tid + i * 256;
                const int r = idx >> 3, c = (idx & 7) * 4;
                *reinterpret_cast<f32x4*>(Xs + r * LDK + c) = elu4(ra[i]);
            }
        }
#pragma unroll
        for (int i = 0; i < B1_F4; ++i) {
            const int idx = tid + i * 256;
            const int r = idx >> 3, c = (idx & 7) * 4;
            if (r < H) *reinterpret_cast<f32x4*>(Bs + r * LDK + c) = rb[i];
        }
    };

    const int w1m = wave / W1N, w1n = wave % W1N;
    f32x16 acc1[TM1][TN1];
#pragma unroll
    for (int i = 0; i < TM1; ++i)
#pragma unroll
        for (int j = 0; j < TN1; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc1[i][j][r] = 0.f;

    constexpr int NK1 = K1 / 32;
    load1(0);
    store1();
    __syncthreads();
    for (int kc = 0; kc < NK1; ++kc) {
        if (kc + 1 < NK1) load1((kc + 1) * 32);
        const float* Ab;
        int lda;
        if (WINDOW) {
            const int k0 = kc * 32;
            const int kk = k0 / C, ci0 = k0 % C;
            Ab = Xs + (w1m * TM1 * 32 + kk) * LDX + ci0;
            lda = LDX;
        } else {
            Ab = Xs + (w1m * TM1 * 32) * LDK;
            lda = LDK;
        }
        mma_k32<TM1, TN1>(acc1, Ab, lda, Bs + (w1n * TN1 * 32) * LDK, LDK, lane);
        if (kc + 1 < NK1) {
            __syncthreads();
            store1();
            __syncthreads();
        }
    }
    // residual x for the GEMM2 epilogue: FIRST recomputes raw x0 into the (now dead) window slab; the other
    // stages prefetch it from global (L2-hot: just read) into registers so the loads fly under GEMM2
    constexpr int TM2P = BM / W2M / 32, TN2P = NP / W2N / 32;
    const int w2m = wave / W2N, w2n = wave % W2N;
    if (FIRST) {
        __syncthreads();  // every wave is done reading the ELU slab
        for (int idx = tid; idx < BM * 64; idx += 256) {
            const int r = idx >> 6, c = idx & 63;
            const float* wr = Aud + BM + 8 + c * 8;
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < 7; ++k) acc = fmaf(wr[k], Aud[r + 2 + k], acc);
            Xs[r * LDX + c] = acc + wr[7];
        }
    }
    float xres[TM2P][TN2P][16];
    auto prefetch_res = [&](int n0) {
        if (FIRST) return;
        const int rb0 = w2m * TM2P * 32 + 4 * (lane >> 5);
        const int cb0 = n0 + w2n * TN2P * 32 + (lane & 31);
#pragma unroll
        for (int j = 0; j < TN2P; ++j)
#pragma unroll
            for (int i = 0; i < TM2P; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const long long row = m0 + rb0 + i * 32 + (r & 3) + 8 * (r >> 2);
                    xres[i][j][r] = row < T ? xb[row * C + cb0 + j * 32] : 0.0f;
                }
    };
    prefetch_res(0);
    // epilogue 1: Hs = ELU(h + b3)
    {
        const int rb0 = w1m * TM1 * 32 + 4 * (lane >> 5);
        const int cb0 = w1n * TN1 * 32 + (lane & 31);
#pragma unroll
        for (int j = 0; j < TN1; ++j) {
            const int col = cb0 + j * 32;
            const float bias = p.b3[col];
#pragma unroll
            for (int i = 0; i < TM1; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = rb0 + i * 32 + (r & 3) + 8 * (r >> 2);
                    Hs[row * LDH + col] = elu_f(acc1[i][j][r] + bias);
                }
        }
    }

    // ---------------- GEMM2: y = ELU(x + b1 + h . W1^T), NP columns per pass ----------------
    const long long ybase = (long long)b * T * C;
    float ymx = 0.0f;  // max|y| (fp16 planes: the engine's range check)
    for (int n0 = 0; n0 < C; n0 += NP) {
        auto load2 = [&](int k0) {
#pragma unroll
            for (int i = 0; i < B2_F4; ++i) {
                const int idx = tid + i * 256;
                const int r = idx >> 3, c = (idx & 7) * 4;
                if (r < NP) rb[i] = *reinterpret_cast<const f32x4*>(p.w1 + (long long)(n0 + r) * H + k0 + c);
            }
        };
        auto store2 = [&]() {
#pragma unroll
            for (int i = 0; i < B2_F4; ++i) {
                const int idx = tid + i * 256;
                const int r = idx >> 3, c = (idx & 7) * 4;
                if (r < NP) *reinterpret_cast<f32x4*>(Bs + r * LDK + c) = rb[i];
            }
        };
        f32x16 acc2[TM2][TN2];
#pragma unroll
        for (int i = 0; i < TM2; ++i)
#pragma unroll
            for (int j = 0; j < TN2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc2[i][j][r] = 0.f;
        constexpr int NK2 = H / 32;
        load2(0);
        __syncthreads();  // Hs complete; previous readers of Bs done
        store2();
        __syncthreads();
        for (int kc = 0; kc < NK2; ++kc) {
            if (kc + 1 < NK2) load2((kc + 1) * 32);
            mma_k32<TM2, TN2>(acc2, Hs + (w2m * TM2 * 32) * LDH + kc * 32, LDH, Bs + (w2n * TN2 * 32) * LDK, LDK,
                              lane);
            if (kc + 1 < NK2) {
                __syncthreads();
                store2();
                __syncthreads();
            }
        }
        const int rb0 = w2m * TM2 * 32 + 4 * (lane >> 5);
        const int cb0 = n0 + w2n * TN2 * 32 + (lane & 31);
        if constexpr (!FIRST && TM2 == 1 && TN2 == 2) {
            f32x16 v[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const float bias = p.b1[cb0 + j * 32];
#pragma unroll
                for (int r = 0; r < 16; ++r) v[j][r] = elu_f(xres[0][j][r] + (acc2[0][j][r] + bias));
            }
            store_y_block(p, Xs + wave * YSTG_FLOATS, v, ybase, m0 + w2m * 32, n0 + w2n * 64, C, T, lane, ymx);
        } else {
#pragma unroll
        for (int j = 0; j < TN2; ++j) {
            const int col = cb0 + j * 32;
            const float bias = p.b1[col];
#pragma unroll
            for (int i = 0; i < TM2; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const long long row = m0 + rb0 + i * 32 + (r & 3) + 8 * (r >> 2);
                    if (row < T) {
                        const float xr = FIRST ? Xs[(row - m0) * LDX + col] : xres[i][j][r];
                        store_act(p.y, p.yp, p.y_pstride, p.yns, ybase + row * C + col,
                                  elu_f(xr + (acc2[i][j][r] + bias)), p.yscale, &ymx);
                    }
                }
        }
        }
        if (n0 + NP < C) prefetch_res(n0 + NP);
    }
    amax_commit(p.yamax, ymx);
}


// ------------------------------------------------------------------------------------------------
// Stage 0, wave-autonomous: conv0 (1 -> 64, k7) + residual block (64 -> 32 -> 64) + ELU, one WAVE per 32 rows.
// Every wave builds its own 34-row ELU(x0) slab from the audio (lane = channel, 7 taps in registers), runs
// both GEMMs with the weights read straight from L2 in MFMA-fragment order (Wf[ntile][kquad][lane][4]),
// and keeps h in its private LDS: no __syncthreads anywhere, so the two waves sharing a SIMD drift apart
// and overlap one's VALU work (conv0, ELU) with the other's MFMAs.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void resblock0_wave_kernel(ResArgs p) {
    constexpr int C = 64, H = 32;
    constexpr int LDX = C + 4, LDH = H + 4;
    constexpr int AW = 48;  // audio window floats per wave (32 rows + 2 halo + 6 taps, padded)
    constexpr int PERW = 34 * LDX + AW;
    __shared__ __attribute__((aligned(16))) float lds[4 * PERW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float* Xw = lds + wave * PERW;  // [34][LDX]: ELU(x0) rows r0-2 .. r0+31, then h [32][LDH] aliased on it
    float* Hw = Xw;
    float* Aw = Xw + 34 * LDX;      // audio[r0 - 8 .. r0 + 40)
    const long long T = p.T;
    const long long r0 = ((long long)blockIdx.x * 4 + wave) * 32;
    const int b = blockIdx.y;
    if (r0 >= T) return;  // whole wave idle (no barriers in this kernel)
    const float* ab = p.audio + (long long)b * T;
    const f32x4* __restrict__ w3f = reinterpret_cast<const f32x4*>(p.w3);  // [24 kq][64][4]
    const f32x4* __restrict__ w1f = reinterpret_cast<const f32x4*>(p.w1);  // [2 nt][4 kq][64][4]

    // conv0 weights of this lane's channel; the first GEMM1 B fragments fly under the slab work
    float w0[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) w0[k] = p.w0[lane * 7 + k];
    const float b0 = p.b0[lane];
    f32x4 bq[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) bq[q] = w3f[q * 64 + lane];
    if (lane < AW) {
        const long long pos = r0 - 8 + lane;
        Aw[lane] = (pos >= 0 && pos < T) ? ab[pos] : 0.0f;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's audio stores are visible to its reads
    // slab: row i = position r0 - 2 + i; causal zero padding of x0 before t = 0
    const int zero_rows = r0 >= 2 ? 0 : (int)(2 - r0);
#pragma unroll 2
    for (int i = 0; i < 34; ++i) {
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < 7; ++k) acc = fmaf(w0[k], Aw[i + k], acc);  // audio[pos - 6 + k]
        const float v = elu_fast(acc + b0);
        Xw[i * LDX + lane] = i < zero_rows ? 0.0f : v;
    }
    // ---- GEMM1: h[32][32] = slab (*) W3, K = 192 (24 quads of 8)
    f32x16 acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc1[r] = 0.f;
    const int ar = lane & 31;
    const int kh = (lane >> 5) * 4;
#pragma unroll
    for (int g = 0; g < 3; ++g) {
        f32x4 nq[8];
        if (g < 2) {
#pragma unroll
            for (int q = 0; q < 8; ++q) nq[q] = w3f[((g + 1) * 8 + q) * 64 + lane];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int kq = g * 8 + q;  // k = 8*kq + kh + s; tap kk = k / 64, channel = k % 64
            const int kk = (kq * 8) / C, ci = (kq * 8) % C;
            const f32x4 af = *reinterpret_cast<const f32x4*>(Xw + (ar + kk) * LDX + ci + kh);
#pragma unroll
            for (int s = 0; s < 4; ++s) acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bq[q][s], acc1, 0, 0, 0);
        }
        if (g < 2) {
#pragma unroll
            for (int q = 0; q < 8; ++q) bq[q] = nq[q];
        }
    }
    f32x4 b1q[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) b1q[q] = w1f[q * 64 + lane];
    // epilogue 1: ELU(h + b3) over the consumed slab (the wave's own LDS; reads precede writes in order)
    {
        const float bias = p.b3[lane & 31];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            Hw[row * LDH + (lane & 31)] = elu_fast(acc1[r] + bias);
        }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    // ---- GEMM2: y[32][64] = h . W1^T (K = 32), 2 column tiles
    f32x16 acc2[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc2[j][r] = 0.f;
#pragma unroll
    for (int kq = 0; kq < 4; ++kq) {
        const f32x4 af = *reinterpret_cast<const f32x4*>(Hw + ar * LDH + kq * 8 + kh);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], b1q[j * 4 + kq][s], acc2[j], 0, 0, 0);
    }
    // epilogue 2: y = ELU(x0 + (acc + b1)); x0 (the identity skip) recomputed from the audio window; y leaves
    // through the wave's own (now free) slab region
    const long long ybase = (long long)b * T * C;
    f32x16 v[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int col = j * 32 + (lane & 31);
        const float bias = p.b1[col];
        float wc[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) wc[k] = p.w0[col * 7 + k];
        const float bc = p.b0[col];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            float x0 = 0.0f;
#pragma unroll
            for (int k = 0; k < 7; ++k) x0 = fmaf(wc[k], Aw[row + 2 + k], x0);
            x0 = x0 + bc;
            v[j][r] = elu_fast(x0 + (acc2[j][r] + bias));
        }
    }
    static_assert(34 * LDX >= YSTG_FLOATS, "staging fits the slab");
    float ymx = 0.0f;
    store_y_block(p, Xw, v, ybase, r0, 0, C, T, lane, ymx);
    amax_commit(p.yamax, ymx);
}

// ------------------------------------------------------------------------------------------------
// Stage 0 on the fp16 matrix cores (PREC_F16X3): conv0 (1 -> 64, k7) + residual block (64 -> 32 -> 64) + ELU,
// persistent and wave-autonomous.  Every operand is 2 fp16 planes at a power-of-two scale (x s = h0 + h1,
// 22-bit significand) and each GEMM takes the 3 significant plane products, on v_mfma_f32_32x32x16_f16.
//
// Everything is computed TRANSPOSED: the weights are the A operand (rows = output channels) and time is the
// MFMA column, so a lane's accumulator holds one time step x 4 consecutive channels per 4-row group -- the
// layout in which it writes the next operand (8-B LDS rows, 8-B y-plane stores) and in which conv0's output
// is already the identity skip of the block (kept in registers, never re-read).
//
// One wave walks a contiguous range of 32-step tiles (12 waves per CU, one workgroup per CU); per tile:
//   conv0   x0^T[64][32] = W0 . audio-taps^T: K = 16 = 7 taps of the audio's hi plane (lanes 0-31) | 7 of its
//           lo plane (lanes 32-63): 2 MFMAs per 32 channels give w_hi a_hi + w_hi a_lo + w_lo a_hi
//   slab    ELU(x0) -> planes, rows 2..33 of the wave's [34][64] slab; rows 0, 1 (causal halo) are the
//           previous tile's rows 32, 33 (or zeros at t = 0, or conv0 of the preceding tile at a range start:
//           the same arithmetic, so a row never depends on which wave computed it)
//   GEMM1   h^T[32][32] = W3[32][192] . slab-windows^T (K = tap-major 3 x 64)    36 MFMAs
//   h       ELU(h + b3) -> planes [32 t][32 ch] in LDS, over slab rows 2..33 (after the halo is copied)
//   GEMM2   y^T[64][32] = W1[64][32] . h^T                                        12 MFMAs
//   out     y = ELU(x0 + (acc + b1)) -> 2 fp16 planes of y * yscale, staged in LDS -> 1-KB row stores
// No barrier after the weight load: waves drift apart, so one's VALU (ELU, splits) overlaps another's MFMAs.
// LDS: weights 36 KB + biases + 12 x 9.75 KB per-wave slab / audio window = 153.6 KB.  12 waves (3 per SIMD, 168
// VGPRs) beat 8: 0.70 vs 0.75 ms.
// ------------------------------------------------------------------------------------------------

__global__ __launch_bounds__(768) void resblock0_h16_kernel(ResArgs p) {
    using namespace r0h;
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    {
        const uint4* src = reinterpret_cast<const uint4*>(p.wh16);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (int i = tid; i < NFRAG * 64; i += NW * 64) dst[i] = src[i];
        float* bw = reinterpret_cast<float*>(lds + NFRAG * 1024);
        if (tid < 64) {
            bw[tid] = p.b0[tid];
            bw[96 + tid] = p.b1[tid];
        }
        if (tid < 32) bw[64 + tid] = p.b3[tid];
    }
    __syncthreads();
    const f16x8* wf = reinterpret_cast<const f16x8*>(lds);
    const float* bl = reinterpret_cast<const float*>(lds + NFRAG * 1024);
    char* wb = lds + NFRAG * 1024 + BIAS * 4 + wave * WAVE_BYTES;
    _Float16* slab = reinterpret_cast<_Float16*>(wb);
    _Float16* hb = slab + 2 * SLD;  // h plane p, row j at hb + p * SPL + j * SLD (after GEMM1)
    float* aud = reinterpret_cast<float*>(slab + 2 * SPL);

    const long long T = p.T;  // row stride of the audio / y (and every item's length unless ragged)
    // global (not flat) loads: a flat load in flight also holds lgkmcnt, so every LDS drain would wait for HBM
    const __attribute__((address_space(1))) float* __restrict__ audio =
        (const __attribute__((address_space(1))) float*)io_pointer(p.audio_ref, p.audio);
    const unsigned tpi = (unsigned)((T + 31) >> 5);  // tiles per item (host checks B x tpi < 2^32)
    const unsigned long long NT = p.istart ? p.istart[p.batch] : (unsigned long long)tpi * p.batch;
    const unsigned long long W = (unsigned long long)gridDim.x * NW;
    const unsigned long long wid = (unsigned long long)blockIdx.x * NW + wave;
    const unsigned g0 = (unsigned)(wid * NT / W), g1 = (unsigned)((wid + 1) * NT / W);
    // tile g -> (item, first step): items' tiles concatenated (ragged: istart), walked in order from g0
    TileWalk tw(p, tpi, g0);
    const int j = lane & 31, hh = lane >> 5;
    const float sa = p.ascale, sx = p.xscale, sh = p.hscale, sy = p.yscale;
    const float u0 = p.unscale0, u1 = p.unscale1, u2 = p.unscale2;
    float mxa = 0.0f, mxx = 0.0f, mxh = 0.0f, mxy = 0.0f;  // max |audio|, then max |scaled operand|

    // lane's audio-window value of tile (item bb, step t0): audio[t0 - 8 + lane] (lanes < AUD; zero outside the
    // item's [0, T_b))
    auto aload = [&](unsigned bb, long long t0) {
        const long long pos = t0 - 8 + lane;
        return (lane < AUD && pos >= 0 && pos < tw.Tb) ? audio[(long long)bb * T + pos] : 0.0f;  // (bb == tw.b)
    };
    // x0^T for the tile's 32 steps (lane column j = step t0 + j) from its audio window value av, + b0
    auto conv0 = [&](float av, f32x16 (&x0)[2]) {
        if (lane < AUD) {
            mxa = fmaxf(mxa, fabsf(av));
            aud[lane] = av;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        f16x8 bq;  // taps audio[t - 6 + k], k = 0..7 (k = 7 has zero weight): hi plane (hh = 0) | lo plane
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
            unsigned hi2, lo2;  // (fp16(a sa), fp16(a sa - hi): kernels.h split2_f16s, the same bits as the cvt form)
            split2_f16s(aud[j + 2 + k], aud[j + 3 + k], sa, hi2, lo2);
            const f16x2 pair = __builtin_bit_cast(f16x2, hh ? lo2 : hi2);
            bq[k] = pair[0];
            bq[k + 1] = pair[1];
        }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            f32x16 acc;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
            acc = mfma_h(wf[(FR_W0 + 2 * mt + 1) * 64 + lane], bq, acc);  // w_lo a_hi
            acc = mfma_h(wf[(FR_W0 + 2 * mt) * 64 + lane], bq, acc);      // w_hi a_hi + w_hi a_lo
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + 32 * mt + 8 * g + 4 * hh);
#pragma unroll
                for (int q = 0; q < 4; ++q) x0[mt][4 * g + q] = __builtin_fmaf(acc[4 * g + q], u0, bb[q]);  // acc u0 exact
            }
        }
    };
    // ELU(x0) planes -> slab row j + rowoff (rows outside [0, 34) skipped)
    auto slab_put = [&](const f32x16 (&x0)[2], int rowoff) {
        const int row = j + rowoff;
        if (row < 0 || row >= SROWS) return;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float z[4] = {x0[mt][4 * g], x0[mt][4 * g + 1], x0[mt][4 * g + 2], x0[mt][4 * g + 3]};
                float t[4];
                elu_s4(z, sx, t, mxx);
                uint2 hi, lo;
                split4_t(t, hi, lo);
                const int o = row * SLD + 32 * mt + 8 * g + 4 * hh;
                *reinterpret_cast<uint2*>(slab + o) = hi;
                *reinterpret_cast<uint2*>(slab + SPL + o) = lo;
            }
    };
    // 2 slab rows per plane: lane -> (plane, row, 4 halves)
    const int cpl = lane >> 5, crow = (lane >> 4) & 1, cc = (lane & 15) * 4;

    float anext = g0 < g1 ? aload(tw.b, tw.t0) : 0.0f;
    for (unsigned g = g0; g < g1; ++g) {
        const unsigned b = tw.b;
        const long long t0 = tw.t0;
        const long long Tb = tw.Tb;
        if (t0 == 0) {  // causal zero padding of ELU(x0) before t = 0
            *reinterpret_cast<uint2*>(slab + cpl * SPL + crow * SLD + cc) = make_uint2(0u, 0u);
        } else if (g == g0) {  // range start inside an item: halo rows from the preceding tile's conv0
            f32x16 xp[2];
            conv0(aload(b, t0 - 32), xp);
            slab_put(xp, -30);
        }
        const float acur = anext;
        tw.next();
        if (g + 1 < g1) anext = aload(tw.b, tw.t0);  // the next tile's audio flies under this tile
        f32x16 x0[2];
        conv0(acur, x0);
        slab_put(x0, 2);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

        // ---- GEMM1: h^T = W3 . windows^T, k = 16 ks + 8 hh + e -> tap ks / 4, channel 16 (ks % 4) + 8 hh + e
        f32x16 acc1;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc1[r] = 0.0f;
#pragma unroll
        for (int ks = 0; ks < 12; ++ks) {
            const int o = (j + (ks >> 2)) * SLD + (ks & 3) * 16 + 8 * hh;
            const f16x8 bx0 = *reinterpret_cast<const f16x8*>(slab + o);
            const f16x8 bx1 = *reinterpret_cast<const f16x8*>(slab + SPL + o);
            const f16x8 aw0 = wf[(FR_W3 + 2 * ks) * 64 + lane];
            const f16x8 aw1 = wf[(FR_W3 + 2 * ks + 1) * 64 + lane];
            acc1 = mfma_h(aw1, bx0, acc1);
            acc1 = mfma_h(aw0, bx1, acc1);
            acc1 = mfma_h(aw0, bx0, acc1);
        }
        // halo for the next tile: slab rows 32, 33 -> 0, 1 (GEMM1's reads of the slab have been
        // consumed); then h overwrites rows 2..33
        {
            _Float16* sp = slab + cpl * SPL;
            const uint2 v = *reinterpret_cast<const uint2*>(sp + (32 + crow) * SLD + cc);
            *reinterpret_cast<uint2*>(sp + crow * SLD + cc) = v;
        }
        asm volatile("" ::: "memory");
        // ---- h = ELU(acc + b3) -> planes, row j, channels 8g + 4hh .. +3
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
            const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + 64 + 8 * gq + 4 * hh);
            float z[4], t[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) z[q] = __builtin_fmaf(acc1[4 * gq + q], u1, bb[q]);
            elu_s4(z, sh, t, mxh);
            uint2 hi, lo;
            split4_t(t, hi, lo);
            const int o = j * SLD + 8 * gq + 4 * hh;
            *reinterpret_cast<uint2*>(hb + o) = hi;
            *reinterpret_cast<uint2*>(hb + SPL + o) = lo;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

        // ---- GEMM2: y^T = W1 . h^T
        f32x16 acc2[2];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc2[mt][r] = 0.0f;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int o = j * SLD + ks * 16 + 8 * hh;
            const f16x8 bh0 = *reinterpret_cast<const f16x8*>(hb + o);
            const f16x8 bh1 = *reinterpret_cast<const f16x8*>(hb + SPL + o);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                const f16x8 aw0 = wf[(FR_W1 + (mt * 2 + ks) * 2) * 64 + lane];
                const f16x8 aw1 = wf[(FR_W1 + (mt * 2 + ks) * 2 + 1) * 64 + lane];
                acc2[mt] = mfma_h(aw1, bh0, acc2[mt]);
                acc2[mt] = mfma_h(aw0, bh1, acc2[mt]);
                acc2[mt] = mfma_h(aw0, bh0, acc2[mt]);
            }
        }
        // ---- y = ELU(x0 + (acc + b1)) -> 2 fp16 planes of y * yscale, staged in slab rows 2..33 (h has been
        // consumed), then written as whole 128-B rows: each store instruction covers 8 consecutive steps = 1 KB
        float tmy = 0.0f;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + 96 + 32 * mt + 8 * gq + 4 * hh);
                float z[4], t[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) z[q] = x0[mt][4 * gq + q] + __builtin_fmaf(acc2[mt][4 * gq + q], u2, bb[q]);
                elu_s4(z, sy, t, tmy);
                uint2 hi, lo;
                split4_t(t, hi, lo);
                const int o = j * SLD + 32 * mt + 8 * gq + 4 * hh;
                *reinterpret_cast<uint2*>(hb + o) = hi;
                *reinterpret_cast<uint2*>(hb + SPL + o) = lo;
            }
        if (t0 + j < Tb) mxy = fmaxf(mxy, tmy);  // steps past the end are not stored, not in max|y|
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        {
            const int sr = lane >> 3, sc = (lane & 7) * 8;
#pragma unroll
            for (int pl = 0; pl < 2; ++pl)
#pragma unroll
                for (int it = 0; it < 4; ++it) {
                    const int r = it * 8 + sr;
                    const uint4 v = *reinterpret_cast<const uint4*>(hb + pl * SPL + r * SLD + sc);
                    if (t0 + r < Tb)
                        *reinterpret_cast<uint4*>(reinterpret_cast<_Float16*>(p.yp) + pl * p.y_pstride +
                                                  ((long long)b * T + t0 + r) * 64 + sc) = v;
                }
        }
        asm volatile("" ::: "memory");
    }
    amax_commit(p.aamax, mxa);
    amax_commit(p.xamax, mxx * (1.0f / sx));  // exact: the scales are powers of two
    amax_commit(p.hamax, mxh * (1.0f / sh));
    amax_commit(p.yamax, mxy * (1.0f / sy));
}


// ------------------------------------------------------------------------------------------------
// Stage 1 (C = 128, H = 64) on the fp16 matrix cores (PREC_F16X3): residual block + ELU, persistent, workgroups
// walking contiguous ranges of 32-step blocks -- one of 8 waves per CU, or (the default) two of 4 waves per CU
// (template NN below).  W1 (32 KB of 16x16x32 A fragments) is resident in LDS; W3 (96 KB) is register-resident: each
// wave holds the 24 fragments of its M tile (96 VGPRs, loaded once), so GEMM1 reads only the slab from LDS -- with W3
// in LDS every block re-read 192 KB of fragments per CU.  Per block (the 8-wave form's wave roles shown):
//   load    x[t0 .. t0+31][128] fp32, each lane 2 float4 in the GEMM2 output layout (time t = 16n + lane&15,
//           channels 16m + 4(lane>>4) .. +3) -- they stay in registers as the identity skip; the next block's
//           x is prefetched under this one
//   slab    ELU(x) -> 2 fp16 planes, rows 2..33 of the [34][128] slab (rows 0, 1: causal halo, kept in the
//           registers of the lanes that own steps 30, 31 of the previous block, zeros at t = 0, loaded at a
//           range start)                                                                     barrier
//   GEMM1   h^T[64][32] = W3 . windows^T: wave w computes the 16x16 tile (hch 16(w>>1), t 16(w&1)),
//           K = 384 = 12 x 32, 36 MFMAs;  h = ELU(acc + b3) -> planes [32 t][64]                 barrier
//   GEMM2   y^T[128][32] = W1 . h^T: wave w, tiles (ch 16(2(w>>1)+i), t 16(w&1)), 12 MFMAs
//   out     y = ELU(x + (acc + b1)) -> planes staged over slab rows 2..33                     barrier
//           -> 1-KB row stores (256-B rows, 4 per wave instruction)                           barrier
// Slab rows are 288 B (72 dwords = 8 mod 64) and h rows 160 B, 16-B chunks XOR-swizzled by row (r1h_swz): the
// 16x16x32 fragment reads (row lane&15, 16-B chunk lane>>4) are conflict-free, the row writes 2-way.  LDS per
// workgroup: 32 KB W1 + 19.1 KB slab + 10 KB h + biases (+ the compiler's own): 69 KB.
// ------------------------------------------------------------------------------------------------
namespace r1h {
constexpr int C = 128, H = 64, BM = 32, NW = 8;
constexpr int SLD = 144, SROWS = BM + 2, SPL = SROWS * SLD;  // halves
constexpr int HLD = 80, HPL = BM * HLD;
constexpr int FR_W3 = 0, FR_W1 = 96, NFRAG = 128;  // W3 [mt 4][ks 12][pl 2], W1 [mt 8][ks 2][pl 2]
constexpr int BIAS = H + C;                         // b3 | b1
// W3's fragments live in the waves' registers (each wave its M tile's 24: 96 VGPRs), only W1's 32 in LDS
constexpr int LFRAG = NFRAG - FR_W1;
constexpr int LDS_BYTES = LFRAG * 1024 + 2 * SPL * 2 + 2 * HPL * 2 + BIAS * 4;
static_assert(NFRAG == RES1_H16_FRAGS, "fragment count");
static_assert(LDS_BYTES <= 160 * 1024, "LDS");
}  // namespace r1h


// Workgroup barrier for LDS hand-offs only: this wave's LDS operations complete, then s_barrier.  Unlike
// __syncthreads() it does not drain vmcnt, so prefetched global loads and y stores stay in flight across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// 16-B chunk c of slab / h row r at c ^ ((r >> 2) & 1): the 16-lane groups of the ds_write_b64 row writes (16
// consecutive rows, one 8-B piece each) 2-way instead of 4-way on the 288-B / 160-B rows, the 16x16x32 fragment
// reads still conflict-free (MI355X_MICROARCH.md LDS banking; SQ_LDS_BANK_CONFLICT 6.1e7 per launch before)
__device__ __forceinline__ int r1h_swz(int row, int ld, int ch) {
    return row * ld + 8 * ((ch >> 3) ^ ((row >> 2) & 1)) + (ch & 7);
}

// NN = 1: one workgroup of 8 waves per CU, wave w the 16-step N tile w & 1 of M tile w >> 1.  NN = 2: two
// workgroups of 4 waves per CU, wave w both N tiles of M tile w (the W3 fragments it holds serve both), so the two
// workgroups' block chains (barriers, VALU epilogues, MFMA phases) interleave on every SIMD instead of running in
// lockstep; each output element sees the same MFMA sequence and epilogue arithmetic either way (the same bits).
template <int NN>
__global__ __launch_bounds__(512 / NN) __attribute__((amdgpu_waves_per_eu(NN))) void resblock128_h16_kernel(ResArgs p) {
    using namespace r1h;
    constexpr int NWW = NW / NN;  // waves per workgroup
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    _Float16* slab = reinterpret_cast<_Float16*>(lds + LFRAG * 1024);
    _Float16* hb = slab + 2 * SPL;
    float* bl = reinterpret_cast<float*>(hb + 2 * HPL);
    {
        const uint4* src = reinterpret_cast<const uint4*>(p.wh16) + FR_W1 * 64;  // W1's fragments
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (int i = tid; i < LFRAG * 64; i += NWW * 64) dst[i] = src[i];
        if (tid < H) bl[tid] = p.b3[tid];
        if (tid < C) bl[H + tid] = p.b1[tid];
    }
    const f16x8* wf = reinterpret_cast<const f16x8*>(lds) - FR_W1 * 64;  // (indexed by the full image's numbering)

    const long long T = p.T;  // row stride of x / y (and every item's length unless ragged)
    const unsigned tpi = (unsigned)((T + BM - 1) / BM);  // blocks per item (host checks B x tpi < 2^32)
    const unsigned long long NB = p.istart ? p.istart[p.batch] : (unsigned long long)tpi * p.batch;
    const unsigned g0 = (unsigned)((unsigned long long)blockIdx.x * NB / gridDim.x);
    const unsigned g1 = (unsigned)((unsigned long long)(blockIdx.x + 1) * NB / gridDim.x);
    static_assert(BM == 32, "TileWalk steps 32");
    TileWalk tw(p, tpi, g0);
    const int li = lane & 15, lq = lane >> 4;
    const int n0 = NN == 1 ? (wave & 1) : 0;    // this wave's first N tile (16 steps)
    const int mp = NN == 1 ? wave >> 1 : wave;  // its M tile (GEMM1) / M-tile pair (GEMM2)
    auto tof = [&](int nn) { return 16 * (n0 + nn) + li; };  // this lane's step inside a block (E layout), tile nn
    const float sx = p.xscale, sh = p.hscale, sy = p.yscale;
    const float u1 = p.unscale1, u2 = p.unscale2;
    float mxx = 0.0f, mxh = 0.0f, mxy = 0.0f;
    // this wave's W3 fragments (M tile mp: 12 K steps x 2 planes), resident for the whole launch
    f16x8 w3r[12][2];
    {
        const f16x8* wg = reinterpret_cast<const f16x8*>(p.wh16);
#pragma unroll
        for (int ks = 0; ks < 12; ++ks)
#pragma unroll
            for (int pl = 0; pl < 2; ++pl) w3r[ks][pl] = wg[(FR_W3 + (mp * 12 + ks) * 2 + pl) * 64 + lane];
    }

    // x of the block at (item b, step t0), step t0 + off, channels 16(2mp + i) + 4lq .. +3 (zero outside the item's
    // [0, T_b))
    auto xload = [&](unsigned b, long long Tlen, long long t0b, long long off, f32x4 (&xv)[2]) {
        const long long row = t0b + off;
        const bool ok = row >= 0 && row < Tlen;
        const float* xr = p.x + ((long long)b * T + (ok ? row : 0)) * C + 4 * lq;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(xr + 16 * (2 * mp + i));
            xv[i] = ok ? v : (f32x4){0.f, 0.f, 0.f, 0.f};
        }
    };
    // ELU(x) planes of this lane's 2 x 4 channels
    auto xsplit = [&](const f32x4 (&xv)[2], uint2 (&hi)[2], uint2 (&lo)[2]) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const float z[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
            float tt[4];
            elu_s4(z, sx, tt, mxx);
            split4_t(tt, hi[i], lo[i]);
        }
    };
    auto slab_row_put = [&](int row, const uint2 (&hi)[2], const uint2 (&lo)[2]) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int o = r1h_swz(row, SLD, 16 * (2 * mp + i) + 4 * lq);
            *reinterpret_cast<uint2*>(slab + o) = hi[i];
            *reinterpret_cast<uint2*>(slab + SPL + o) = lo[i];
        }
    };

    uint2 hhi[2], hlo[2];  // lanes with t >= 30 (the last N tile): the halo planes for the next block
    f32x4 xn[NN][2];
    if (g0 < g1) {
#pragma unroll
        for (int nn = 0; nn < NN; ++nn) xload(tw.b, tw.Tb, tw.t0, tof(nn), xn[nn]);
    }
    __syncthreads();  // weights and biases resident
    for (unsigned g = g0; g < g1; ++g) {
        const unsigned b = tw.b;
        const long long t0 = tw.t0;
        const long long Tb = tw.Tb;
        f32x4 xc[NN][2];
#pragma unroll
        for (int nn = 0; nn < NN; ++nn) {
            xc[nn][0] = xn[nn][0];
            xc[nn][1] = xn[nn][1];
        }
        tw.next();
        if (g + 1 < g1) {  // flies under this block
#pragma unroll
            for (int nn = 0; nn < NN; ++nn) xload(tw.b, tw.Tb, tw.t0, tof(nn), xn[nn]);
        }
        // ---- slab: halo rows 0, 1 (lanes t = 30, 31), rows 2 + t
        const int tl = tof(NN - 1);  // the last tile's step (the halo lanes live there)
        if (tl >= BM - 2) {
            if (t0 == 0) {
                hhi[0] = hhi[1] = hlo[0] = hlo[1] = make_uint2(0u, 0u);
            } else if (g == g0) {
                f32x4 xh[2];
                xload(b, Tb, t0, tl - BM, xh);  // steps t0 - 2, t0 - 1
                xsplit(xh, hhi, hlo);
            }
            slab_row_put(tl - (BM - 2), hhi, hlo);
        }
#pragma unroll
        for (int nn = 0; nn < NN; ++nn) {
            const int t = tof(nn);
            uint2 hi[2], lo[2];
            xsplit(xc[nn], hi, lo);
            slab_row_put(2 + t, hi, lo);
            if (nn == NN - 1 && t >= BM - 2) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    hhi[i] = hi[i];
                    hlo[i] = lo[i];
                }
            }
        }
        lds_barrier();  // B1: slab complete

        // ---- GEMM1: tile (hch 16 mp, steps 16 n); k = 32 ks + 8 lq + e -> tap ks / 4, channel 32 (ks % 4) + 8 lq + e
        f32x4 acc1[NN];
#pragma unroll
        for (int nn = 0; nn < NN; ++nn) acc1[nn] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 12; ++ks) {
#pragma unroll
            for (int nn = 0; nn < NN; ++nn) {
                const int o = r1h_swz(16 * (n0 + nn) + li + (ks >> 2), SLD, (ks & 3) * 32 + 8 * lq);
                const f16x8 bx0 = *reinterpret_cast<const f16x8*>(slab + o);
                const f16x8 bx1 = *reinterpret_cast<const f16x8*>(slab + SPL + o);
                acc1[nn] = mfma_h16(w3r[ks][1], bx0, acc1[nn]);
                acc1[nn] = mfma_h16(w3r[ks][0], bx1, acc1[nn]);
                acc1[nn] = mfma_h16(w3r[ks][0], bx0, acc1[nn]);
            }
        }
        {  // h = ELU(acc + b3): step t, hch 16 mp + 4 lq .. +3
            const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + 16 * mp + 4 * lq);
#pragma unroll
            for (int nn = 0; nn < NN; ++nn) {
                float z[4], tt[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) z[q] = __builtin_fmaf(acc1[nn][q], u1, bb[q]);
                elu_s4(z, sh, tt, mxh);
                uint2 hi, lo;
                split4_t(tt, hi, lo);
                const int o = r1h_swz(tof(nn), HLD, 16 * mp + 4 * lq);
                *reinterpret_cast<uint2*>(hb + o) = hi;
                *reinterpret_cast<uint2*>(hb + HPL + o) = lo;
            }
        }
        lds_barrier();  // B2: h complete, every wave done reading the slab

        // ---- GEMM2: tiles (channels 16 (2 mp + i), steps 16 n), K = 64
        f32x4 acc2[NN][2];
#pragma unroll
        for (int nn = 0; nn < NN; ++nn) acc2[nn][0] = acc2[nn][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int nn = 0; nn < NN; ++nn) {
                const int o = r1h_swz(16 * (n0 + nn) + li, HLD, ks * 32 + 8 * lq);
                const f16x8 bh0 = *reinterpret_cast<const f16x8*>(hb + o);
                const f16x8 bh1 = *reinterpret_cast<const f16x8*>(hb + HPL + o);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int m = 2 * mp + i;
                    const f16x8 aw0 = wf[(FR_W1 + (m * 2 + ks) * 2) * 64 + lane];
                    const f16x8 aw1 = wf[(FR_W1 + (m * 2 + ks) * 2 + 1) * 64 + lane];
                    acc2[nn][i] = mfma_h16(aw1, bh0, acc2[nn][i]);
                    acc2[nn][i] = mfma_h16(aw0, bh1, acc2[nn][i]);
                    acc2[nn][i] = mfma_h16(aw0, bh0, acc2[nn][i]);
                }
            }
        }
        // ---- y = ELU(x + (acc + b1)) -> planes, staged over slab rows 2..33
#pragma unroll
        for (int nn = 0; nn < NN; ++nn) {
            const int t = tof(nn);
            float tmy = 0.0f;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int ch = 16 * (2 * mp + i) + 4 * lq;
                const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + H + ch);
                float z[4], tt[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) z[q] = xc[nn][i][q] + __builtin_fmaf(acc2[nn][i][q], u2, bb[q]);
                elu_s4(z, sy, tt, tmy);
                uint2 hi, lo;
                split4_t(tt, hi, lo);
                const int o = r1h_swz(2 + t, SLD, ch);
                *reinterpret_cast<uint2*>(slab + o) = hi;
                *reinterpret_cast<uint2*>(slab + SPL + o) = lo;
            }
            if (t0 + t < Tb) mxy = fmaxf(mxy, tmy);  // steps past the end are not stored, not in max|y|
        }
        lds_barrier();  // B3: staging complete
        {  // 2 planes x 32 rows x 16 chunks of 16 B = 1024 chunks, 2 NN per thread
#pragma unroll
            for (int k = 0; k < 2 * NN; ++k) {
                const int idx = tid + k * NWW * 64;
                const int pl = idx >> 9, r = (idx >> 4) & 31, c = (idx & 15) * 8;
                const uint4 v = *reinterpret_cast<const uint4*>(slab + pl * SPL + r1h_swz(2 + r, SLD, c));
                if (t0 + r < Tb)
                    *reinterpret_cast<uint4*>(reinterpret_cast<_Float16*>(p.yp) + pl * p.y_pstride +
                                              ((long long)b * T + t0 + r) * C + c) = v;
            }
        }
        lds_barrier();  // B4: staging consumed before the next slab
    }
    amax_commit(p.xamax, mxx * (1.0f / sx));
    amax_commit(p.hamax, mxh * (1.0f / sh));
    amax_commit(p.yamax, mxy * (1.0f / sy));
}

template <int C, int BM, bool WINDOW, bool FIRST, int W1M, int W1N, int W2M, int W2N, int NP>
static hipError_t run_res(const ResArgs& a, hipStream_t s, const char** kname) {
    static thread_local char name[160];
    if (!name[0])
        snprintf(name, sizeof(name), "mimi::resblock_kernel<%d, %d, %s, %s, %d, %d, %d, %d, %d>", C, BM,
                 WINDOW ? "true" : "false", FIRST ? "true" : "false", W1M, W1N, W2M, W2N, NP);
    if (kname) *kname = name;
    dim3 grid((unsigned)((a.T + BM - 1) / BM), a.batch);
    hipLaunchKernelGGL((resblock_kernel<C, BM, WINDOW, FIRST, W1M, W1N, W2M, W2N, NP>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_resblock(int C, const ResArgs& a, hipStream_t s, const char** kname) {
    if (a.T <= 0 || a.batch <= 0) return hipErrorInvalidValue;
    switch (C) {
        case 64:
            if (a.audio && a.wh16) {
                static const char* nm = "mimi::resblock0_h16_kernel(mimi::ResArgs)";
                if (kname) *kname = nm;
                // persistent: one workgroup (12 waves, 153.6 KB of LDS) per CU, each wave a range of tiles
                int dev = 0, ncu = 256;
                (void)hipGetDevice(&dev);
                (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
                hipLaunchKernelGGL(resblock0_h16_kernel, dim3((unsigned)ncu), dim3(64 * r0h::NW), 0, s, a);
                return hipGetLastError();
            }
            if (a.audio && a.w3frag && a.w1frag) {
                static const char* nm = "mimi::resblock0_wave_kernel(mimi::ResArgs)";
                if (kname) *kname = nm;
                ResArgs f = a;
                f.w3 = a.w3frag;
                f.w1 = a.w1frag;
                hipLaunchKernelGGL(resblock0_wave_kernel, dim3((unsigned)((a.T + 127) / 128), a.batch), dim3(256), 0, s,
                                   f);
                return hipGetLastError();
            }
            if (a.audio) return run_res<64, 128, true, true, 4, 1, 4, 1, 64>(a, s, kname);
            return run_res<64, 128, true, false, 4, 1, 4, 1, 64>(a, s, kname);
        case 128:
            if (a.wh16) {
                // persistent: one workgroup of 8 waves (form 0) or two of 4 waves (form 1) per CU, each workgroup a
                // range of 32-step blocks (62.6 KB of LDS per workgroup)
                int dev = 0, ncu = 256;
                (void)hipGetDevice(&dev);
                (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
                if (a.form == 1) {
                    static const char* nm2 = "mimi::resblock128_h16_kernel<2>(mimi::ResArgs)";
                    if (kname) *kname = nm2;
                    hipLaunchKernelGGL(resblock128_h16_kernel<2>, dim3((unsigned)(2 * ncu)), dim3(64 * r1h::NW / 2), 0,
                                       s, a);
                    return hipGetLastError();
                }
                static const char* nm = "mimi::resblock128_h16_kernel<1>(mimi::ResArgs)";
                if (kname) *kname = nm;
                hipLaunchKernelGGL(resblock128_h16_kernel<1>, dim3((unsigned)ncu), dim3(64 * r1h::NW), 0, s, a);
                return hipGetLastError();
            }
            return run_res<128, 64, true, false, 2, 2, 2, 2, 128>(a, s, kname);
        case 256: return run_res<256, 64, false, false, 2, 2, 2, 2, 128>(a, s, kname);
        case 512: return run_res<512, 32, false, false, 1, 4, 1, 4, 256>(a, s, kname);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mimi
