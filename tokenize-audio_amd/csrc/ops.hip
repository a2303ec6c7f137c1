// Non-GEMM kernels of the Mimi encode path for gfx950: the Cin = 1 input conv, LayerNorm, the
// sliding-window attention and the split residual-VQ argmin.
#include <cstdlib>
#include "kernels.h"
#include "attn_h16.h"

namespace mimi {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------------------------------------
// conv0: causal Conv1d(1 -> 64, k = 7) (TF/modeling_mimi.py:455), channels-last output [B][L][64].
// HBM-bound (7 MACs per 4-byte output): each workgroup stages its 128 + 6 input samples in LDS and
// writes 128 x 64 outputs as coalesced float4 rows.
// ------------------------------------------------------------------------------------------------
template <int COUT, int KS>
__global__ __launch_bounds__(256) void conv0_kernel(const float* __restrict__ x, long long L,
                                                    const float* __restrict__ w, const float* __restrict__ bias,
                                                    float* __restrict__ y) {
    constexpr int TT = 128;
    constexpr int CG = COUT / 4;        // channel groups of 4
    constexpr int TG = 256 / CG;        // time lanes
    __shared__ float xs[TT + KS - 1];
    __shared__ float ws[COUT * KS];
    __shared__ float bs[COUT];
    const int b = blockIdx.y;
    const long long t0 = (long long)blockIdx.x * TT;
    const float* xb = x + (long long)b * L;
    for (int i = threadIdx.x; i < TT + KS - 1; i += 256) {
        const long long t = t0 - (KS - 1) + i;
        xs[i] = (t >= 0 && t < L) ? xb[t] : 0.0f;
    }
    for (int i = threadIdx.x; i < COUT * KS; i += 256) ws[i] = w[i];
    for (int i = threadIdx.x; i < COUT; i += 256) bs[i] = bias[i];
    __syncthreads();
    const int cg = threadIdx.x % CG;
    const int tl = threadIdx.x / CG;
    float* yb = y + (long long)b * L * COUT;
    for (int tt = tl; tt < TT; tt += TG) {
        const long long t = t0 + tt;
        if (t >= L) break;
        float out[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int co = cg * 4 + c;
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < KS; ++k) acc = fmaf(ws[co * KS + k], xs[tt + k], acc);
            out[c] = acc + bs[co];
        }
        *reinterpret_cast<f32x4*>(yb + t * COUT + cg * 4) = f32x4{out[0], out[1], out[2], out[3]};
    }
}

hipError_t launch_conv0(const float* x, long long L, int batch, const float* w, const float* b, float* y,
                        int cout, int ksize, hipStream_t s) {
    if (cout != 64 || ksize != 7) return hipErrorInvalidValue;
    dim3 grid((unsigned)((L + 127) / 128), batch);
    hipLaunchKernelGGL((conv0_kernel<64, 7>), grid, dim3(256), 0, s, x, L, w, b, y);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// LayerNorm(512) (TF/modeling_mimi.py:737-738): one wave per row, two-pass mean / variance in fp32,
// y = (x * rstd + (-mean * rstd)) * gamma + beta as the torch CPU kernel forms it.
// ------------------------------------------------------------------------------------------------
// (wave_sum and the row arithmetic: kernels.h ln_row_coeffs / ln_affine / ln_split4_f16)

// RPW rows per wave, all loads in flight before the first reduction; 8 waves per workgroup.
template <int C, int RPW>
__global__ __launch_bounds__(512) void layernorm_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                        const float* __restrict__ bta, float* __restrict__ y,
                                                        long long rows, float eps, __bf16* __restrict__ yp,
                                                        long long pstride, int yns, float yscale,
                                                        unsigned* __restrict__ yamax, const int* __restrict__ row_len,
                                                        int row_T) {
    constexpr int PER = C / 64;  // floats per lane
    static_assert(PER % 4 == 0, "C multiple of 256");
    const int lane = threadIdx.x & 63;
    const long long row0 = ((long long)blockIdx.x * 8 + (threadIdx.x >> 6)) * RPW;
    float vr[RPW][PER];
    // gamma / beta of this lane's columns, loaded beside the rows (not after each row's reduction: that put two
    // more memory round trips before every row's stores)
    f32x4 gv[PER / 4], bv[PER / 4];
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
        gv[q] = *reinterpret_cast<const f32x4*>(g + q * 256 + lane * 4);
        bv[q] = *reinterpret_cast<const f32x4*>(bta + q * 256 + lane * 4);
    }
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
        const long long row = row0 + rr < rows ? row0 + rr : rows - 1;
        const float* xr = x + row * C;
#pragma unroll
        for (int q = 0; q < PER / 4; ++q) {
            f32x4 t = *reinterpret_cast<const f32x4*>(xr + q * 256 + lane * 4);
            vr[rr][q * 4 + 0] = t.x; vr[rr][q * 4 + 1] = t.y; vr[rr][q * 4 + 2] = t.z; vr[rr][q * 4 + 3] = t.w;
        }
    }
    float mx = 0.0f;
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
    const long long row = row0 + rr;
    if (row >= rows) break;
    if (row_len && row % row_T >= row_len[row / row_T]) continue;  // ragged: past the item's frames
    float (&v)[PER] = vr[rr];
    float sc, bi;
    ln_row_coeffs<C>(v, eps, sc, bi);
    float* yr = y + row * C;
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
        const int c0 = q * 256 + lane * 4;
        const f32x4 gg = gv[q], bb = bv[q];
        f32x4 o;
        o.x = ln_affine(v[q * 4 + 0], sc, bi, gg.x, bb.x);
        o.y = ln_affine(v[q * 4 + 1], sc, bi, gg.y, bb.y);
        o.z = ln_affine(v[q * 4 + 2], sc, bi, gg.z, bb.z);
        o.w = ln_affine(v[q * 4 + 3], sc, bi, gg.w, bb.w);
        if (yns == 0) {
            *reinterpret_cast<f32x4*>(yr + c0) = o;
        } else if (yscale > 0.0f) {
            // fp16 planes of o * yscale (PREC_F16X3)
            _Float16* pr = reinterpret_cast<_Float16*>(yp) + row * C + c0;
            const float ov[4] = {o.x, o.y, o.z, o.w};
            uint2 h0, h1;
            ln_split4_f16(ov, yscale, h0, h1);
            *reinterpret_cast<uint2*>(pr) = h0;
            *reinterpret_cast<uint2*>(pr + pstride) = h1;
            mx = fmaxf(mx, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
        } else {
            // planes for the split-bf16 GEMMs that read this row (q/k/v, fc1)
            typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
            __bf16* pr = yp + row * C + c0;
            f32x4 rem = o;
            for (int pl = 0; pl < yns; ++pl) {
                bf16x4 h;
                h.x = (__bf16)rem.x; h.y = (__bf16)rem.y; h.z = (__bf16)rem.z; h.w = (__bf16)rem.w;
                *reinterpret_cast<bf16x4*>(pr + pl * pstride) = h;
                rem.x -= (float)h.x; rem.y -= (float)h.y; rem.z -= (float)h.z; rem.w -= (float)h.w;
            }
        }
    }
    }
#ifndef MIMI_LN_AMAX
#define MIMI_LN_AMAX 1  // 1: one atomic per workgroup (0.182 vs 0.186 ms per wave, same bits); 0: one per wave; 2: none (timing only)
#endif
#if MIMI_LN_AMAX == 1
    if (yamax) {  // (null: the engine proved the range check cannot fire -- uniform)
        __shared__ float wmx[8];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
        if (lane == 0) wmx[threadIdx.x >> 6] = mx;
        __syncthreads();
        if (threadIdx.x < 64) amax_commit(yamax, lane < 8 ? wmx[lane] : 0.0f);
    }
#elif MIMI_LN_AMAX == 0
    amax_commit(yamax, mx);
#endif
}

hipError_t launch_layernorm(const float* x, const float* g, const float* b, float* y, long long rows, int C,
                            float eps, hipStream_t s, void* yp, long long y_pstride, int yns, float yscale,
                            unsigned* yamax, const int* row_len, int row_T, int rpw) {
    if (row_len && row_T <= 0) return hipErrorInvalidValue;
    if (C != 512 || (yns != 0 && !yp) || (yscale > 0.0f && yns != 2)) return hipErrorInvalidValue;
    // rpw rows per wave (8 waves per workgroup): 2 by default (16 rows per workgroup); 1, 4, 8 for A/B
#define LN_LAUNCH(R_)                                                                                                \
    hipLaunchKernelGGL((layernorm_kernel<512, R_>), dim3((unsigned)((rows + 8 * (R_) - 1) / (8 * (R_)))), dim3(512), 0, \
                       s, x, g, b, y, rows, eps, reinterpret_cast<__bf16*>(yp), y_pstride, yns, yscale, yamax, row_len,  \
                       row_T)
    switch (rpw) {
        case 1: LN_LAUNCH(1); break;
        case 4: LN_LAUNCH(4); break;
        case 8: LN_LAUNCH(8); break;
        default: LN_LAUNCH(2); break;
    }
#undef LN_LAUNCH
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Sliding-window causal attention (window W incl. self: masking_utils.py:76-101), head_dim 64, on fp32 MFMA.
// Workgroup = 128 queries of one (batch, head), 4 waves x 32 queries; 32-key K/V chunks staged in LDS.
// Each wave computes S^T = K . Q^T (keys on rows, queries on lanes), so a query's softmax statistics sit in
// one lane (16 registers + the other lane half), then O^T += V^T . P^T reuses the probabilities straight
// from the S^T accumulator registers as the B operand (no shuffles, no LDS round trip).  Q is pre-scaled
// by 1/sqrt(64) = 1/8 (exact).  Online softmax with running max / sum per query, fp32 throughout.
// ------------------------------------------------------------------------------------------------
// One 32-key chunk of the online-softmax attention for the wave's 32 queries (S^T = K . Q^T with keys on
// rows, queries on lanes; O^T += V^T . P^T).  Ks / Vs: the chunk's K rows (stride D + 4) and V rows (stride D)
// in LDS; keys c0 .. c0 + 31, masked to key <= query, key > query - window, key <= kend.
__device__ __forceinline__ void attn_chunk(f32x16 (&o)[2], float& m, float& l, const f32x4 (&qf)[8],
                                           const float* Ks, const float* Vs, int c0, int qw, int qi, int kend,
                                           int window, int hf, int col) {
    constexpr int D = 64, KC = 32, LDKS = D + 4;
    // S^T[key][query]
    f32x16 st;
#pragma unroll
    for (int r = 0; r < 16; ++r) st[r] = 0.f;
#pragma unroll
    for (int kq = 0; kq < 8; ++kq) {
        const f32x4 kf = *reinterpret_cast<const f32x4*>(Ks + col * LDKS + kq * 8 + hf * 4);
#pragma unroll
        for (int s = 0; s < 4; ++s) st = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[s], qf[kq][s], st, 0, 0, 0);
    }
    // mask + online softmax for this lane's query
    float cmax = -INFINITY;
    // wave-uniform: a chunk wholly inside every query's window needs no mask
    const bool full = c0 + KC - 1 <= qw && c0 > qw + 31 - window && c0 + KC - 1 <= kend;
    if (full) {
#pragma unroll
        for (int r = 0; r < 16; ++r) cmax = fmaxf(cmax, st[r]);
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int key = c0 + (r & 3) + 8 * (r >> 2) + 4 * hf;
            const bool ok = key <= qi && key > qi - window && key <= kend;
            st[r] = ok ? st[r] : -INFINITY;
            cmax = fmaxf(cmax, st[r]);
        }
    }
    cmax = fmaxf(cmax, __shfl_xor(cmax, 32));
    const float mnew = fmaxf(m, cmax);
    const float corr = (m == -INFINITY) ? 0.f : __expf(m - mnew);  // v_exp_f32: ~1 ulp
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float pv = (st[r] == -INFINITY) ? 0.f : __expf(st[r] - mnew);
        st[r] = pv;
        psum += pv;
    }
    psum += __shfl_xor(psum, 32);
    l = l * corr + psum;
    m = mnew;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] *= corr;
    // O^T[d][query] += V^T . P^T : step r pairs key (r&3)+8(r>>2) (half 0) with +4 (half 1)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int key = (r & 3) + 8 * (r >> 2) + 4 * hf;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const float va = Vs[key * D + t * 32 + col];
            o[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(va, st[r], o[t], 0, 0, 0);
        }
    }
}

__global__ __launch_bounds__(256) void attention_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                        int T, int H, int window, float scale,
                                                        void* __restrict__ outp, long long pstride, int outns,
                                                        float oscale, unsigned* __restrict__ oamax) {
    constexpr int D = 64;
    constexpr int KC = 32;
    constexpr int LDKS = D + 4;
    constexpr int LDO = D + 1;
    __shared__ __attribute__((aligned(16))) float Ks[KC * LDKS];
    __shared__ __attribute__((aligned(16))) float Vs[KC * D];
    __shared__ float Os[4][32 * LDO];
    const int b = blockIdx.z, h = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int hf = lane >> 5, col = lane & 31;
    const int q0 = blockIdx.x * 128;
    const int qw = q0 + wave * 32;
    const int qi = qw + col;  // this lane's query (B operand column / S^T column)
    const long long ld = 3LL * H * D;
    const float* base = qkv + (long long)b * T * ld;

    // Q fragment (B operand): lane (q, hf) holds q[8kq + 4hf + s], kq = 0..7, pre-scaled
    f32x4 qf[8];
#pragma unroll
    for (int kq = 0; kq < 8; ++kq) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (qi < T) v = *reinterpret_cast<const f32x4*>(base + (long long)qi * ld + h * D + kq * 8 + hf * 4);
        qf[kq] = v * scale;
    }
    f32x16 o[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
    float m = -INFINITY, l = 0.f;

    const int kstart = max(0, q0 - window + 1);
    const int kend = min(T - 1, q0 + 127);
    // K/V chunks: registers hold chunk c+1 while chunk c is computed (2 float4 of K and of V per thread)
    constexpr int PER = KC * (D / 4) / 256;
    f32x4 kreg[PER], vreg[PER];
    auto fetch = [&](int c0) {
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int idx = tid + q * 256;
            const int r = idx / (D / 4), c = (idx % (D / 4)) * 4;
            const int j = c0 + r;
            f32x4 kv = {0, 0, 0, 0}, vv = {0, 0, 0, 0};
            if (j <= kend) {
                kv = *reinterpret_cast<const f32x4*>(base + (long long)j * ld + H * D + h * D + c);
                vv = *reinterpret_cast<const f32x4*>(base + (long long)j * ld + 2 * H * D + h * D + c);
            }
            kreg[q] = kv;
            vreg[q] = vv;
        }
    };
    fetch(kstart);
    for (int c0 = kstart; c0 <= kend; c0 += KC) {
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int idx = tid + q * 256;
            const int r = idx / (D / 4), c = (idx % (D / 4)) * 4;
            *reinterpret_cast<f32x4*>(Ks + r * LDKS + c) = kreg[q];
            *reinterpret_cast<f32x4*>(Vs + r * D + c) = vreg[q];
        }
        __syncthreads();
        if (c0 + KC <= kend) fetch(c0 + KC);
        // skip chunks entirely outside this wave's band [qw - W + 1, qw + 31]
        if (c0 > qw + 31 || c0 + KC - 1 < qw - window + 1) continue;
        attn_chunk(o, m, l, qf, Ks, Vs, c0, qw, qi, kend, window, hf, col);
    }
    // O^T -> LDS (per wave) -> coalesced rows of out[b][q][h*64 + d]
    const float inv = (l > 0.f) ? 1.0f / l : 0.f;
    float* ow = Os[wave];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
            ow[col * LDO + d] = o[t][r] * inv;
        }
    __syncthreads();
    float mx = 0.0f;
    for (int qq = 0; qq < 32; ++qq) {
        const int q = qw + qq;
        if (q < T)
            store_act(out, outp, pstride, outns, ((long long)b * T + q) * (H * D) + h * D + lane, ow[qq * LDO + lane],
                      oscale, &mx);
    }
    amax_commit(oamax, mx);
}

// T <= 256 (every 10 s clip: T = 250): one workgroup per (head, batch item) with the item's whole K and V
// resident in LDS (loaded once, 128 KiB), 8 waves x 32 queries and no per-chunk barriers.  Wave w takes query
// tile w (w < 4) or 11 - w, so the two waves sharing a SIMD (w, w + 4) own 9 causal chunks between them.
__global__ __launch_bounds__(512) void attention_t256_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                             int T, int H, int window, float scale,
                                                             void* __restrict__ outp, long long pstride, int outns,
                                                             float oscale, unsigned* __restrict__ oamax) {
    constexpr int D = 64, LDKS = D + 4, LDO = D + 1, TM = 256;
    __shared__ __attribute__((aligned(16))) float lds[TM * LDKS + TM * D];
    float* Ks = lds;
    float* Vs = lds + TM * LDKS;
    const int h = blockIdx.x, b = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hf = lane >> 5, col = lane & 31;
    const long long ld = 3LL * H * D;
    const float* base = qkv + (long long)b * T * ld;
    // K / V rows 0 .. 255 (zeros past T): 2 x 16 float4 per thread, all in flight before the first store
    {
        constexpr int PER = TM * (D / 4) / 512;  // 8
        f32x4 kv[PER], vv[PER];
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int idx = tid + q * 512;
            const int r = idx / (D / 4), c = (idx % (D / 4)) * 4;
            const int rr = r < T ? r : T - 1;
            const f32x4 k4 = *reinterpret_cast<const f32x4*>(base + (long long)rr * ld + H * D + h * D + c);
            const f32x4 v4 = *reinterpret_cast<const f32x4*>(base + (long long)rr * ld + 2 * H * D + h * D + c);
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};
            kv[q] = r < T ? k4 : z;
            vv[q] = r < T ? v4 : z;
        }
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int idx = tid + q * 512;
            const int r = idx / (D / 4), c = (idx % (D / 4)) * 4;
            *reinterpret_cast<f32x4*>(Ks + r * LDKS + c) = kv[q];
            *reinterpret_cast<f32x4*>(Vs + r * D + c) = vv[q];
        }
    }
    const int qt = wave < 4 ? wave : 11 - wave;
    const int qw = qt * 32;
    const int qi = qw + col;
    f32x4 qf[8];
#pragma unroll
    for (int kq = 0; kq < 8; ++kq) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (qi < T) v = *reinterpret_cast<const f32x4*>(base + (long long)qi * ld + h * D + kq * 8 + hf * 4);
        qf[kq] = v * scale;
    }
    f32x16 o[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
    float m = -INFINITY, l = 0.f;
    __syncthreads();
    const int kend = min(T - 1, qw + 31);
    if (qw < T) {
        const int kstart = max(0, qw - window + 1) & ~31;
        for (int c0 = kstart; c0 <= kend; c0 += 32)
            attn_chunk(o, m, l, qf, Ks + c0 * LDKS, Vs + c0 * D, c0, qw, qi, kend, window, hf, col);
    }
    __syncthreads();  // K / V dead: the output staging reuses the LDS
    float* ow = lds + wave * 32 * LDO;
    const float inv = (l > 0.f) ? 1.0f / l : 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
            ow[col * LDO + d] = o[t][r] * inv;
        }
    // same wave wrote and reads its staging rows: LDS order, no barrier
    float mx = 0.0f;
    for (int qq = 0; qq < 32; ++qq) {
        const int q = qw + qq;
        if (q < T)
            store_act(out, outp, pstride, outns, ((long long)b * T + q) * (H * D) + h * D + lane, ow[qq * LDO + lane],
                      oscale, &mx);
    }
    amax_commit(oamax, mx);
}

// ------------------------------------------------------------------------------------------------
// T <= 256 attention on the fp16 matrix cores (PREC_F16X3 engines, fp16-plane output).  Same schedule as
// attention_t256_kernel (one workgroup per (batch, head), 8 waves with balanced causal 32-query tiles, fp32
// online softmax), but both products run as 3 fp16 plane products on v_mfma_f32_32x32x16_f16:
//   S^T = K . Q^T   K planes [256 keys][64] in LDS (rows of 144 B), Q planes in registers
//   O^T += V^T . P^T  V^T planes [64][256 keys] in LDS (rows of 528 B), P = softmax numerators in [0, 1]
//                    split at 2^14 straight from the S^T accumulator registers
// The k index of the P . V product runs over a chunk's keys in the order the S^T accumulator holds them
// (lane half h, element e <-> key (e & 3) + 8 (e >> 2) + 4 h of each 16), so V^T is stored with that
// permutation and P needs no shuffle (the banded kernel; the T <= 256 kernel keeps V row-major and reads the same
// V^T fragments with ds_read_b64_tr_b16: attn_vrow_off).  Scales are chosen in-kernel (powers of two): K and V from the head's
// max |.| (workgroup reduction), Q from the wave's max; max |.| s lands in [2^13, 2^14).
// ------------------------------------------------------------------------------------------------
// (pow2_scale, wave_max, split8_h, attn_chunk_h16, the V image layout: attn_h16.h)

// T <= 256 (every clip up to 10.24 s) on the fp16 matrix cores.  A workgroup of 16 waves holds one (item, head)'s
// whole K / V as fp16 planes in LDS (power-of-two scales from the head's max |K|, |V|) and runs the causal 32-query
// tiles as TASKS: tile t's key chunks (t + 1 of them at T = 256) are split into two halves, each run by one wave
// with the online softmax of attn_chunk_h16, and the two partial states are merged once (m = max(m0, m1),
// o = o0 c0 + o1 c1, l = l0 c0 + l1 c1, c_i = exp(m_i - m)).  That halves the longest chain of dependent chunks
// (8 -> 4) and puts 4 waves on every SIMD (VGPRs <= 128) to hide the MFMA / exp latencies the 8-wave, one-tile-per-
// wave form waited out.  qg > 1 (small batches: fewer (item, head) pairs than CUs): workgroup z of qg takes only some
// tiles' tasks -- the SAME tasks, so every output is the same arithmetic whatever qg is (batch-size invariance):
//   qg = 1: all 16 tasks, grouped so the 4 waves sharing a SIMD (w, w + 4, w + 8, w + 12) hold 9 chunks each;
//   qg = 2: tiles {z, 3 - z, 4 + z, 7 - z} on waves 0-7;  qg = 4: tiles {7 - z, z} on waves 0-3.
// Every workgroup still reads all of the head's K / V rows: the plane scales are the maxima over all of them.
#ifndef ATTN_DIAG
#define ATTN_DIAG 0  // tuning diagnostics (tools/attn_check.hip builds only; results garbage): 1 no chunk loop, 2 no K / V
#endif               // plane image, 4 no merge

__global__ __launch_bounds__(1024) void attention_t256_h16_kernel(const float* __restrict__ qkv, int Ts, int H,
                                                                  int window, float scale, void* __restrict__ outp,
                                                                  long long pstride, float oscale,
                                                                  unsigned* __restrict__ oamax,
                                                                  const int* __restrict__ tlen, int qg,
                                                                  const int* __restrict__ toff) {
    constexpr int D = 64, TM = 256, LDO = D + 1, NWV = 16;
    constexpr int KLD = 72, KPL = TM * KLD;  // K planes: [256][72 halves]
    constexpr int VLD = D, VPL = TM * D;     // V planes: [256 keys][64 dims] (attn_vrow_off), read transposed
    __shared__ __attribute__((aligned(16))) _Float16 lds[2 * KPL + 2 * VPL];
    __shared__ float red[2][NWV];
    __shared__ float mlx[8][2][32];  // the half-1 task's m, l per query of each tile
    // after the chunk loops the LDS holds the half-1 tasks' accumulators ([tile][32 regs][64 lanes] fp32, 64 KB)
    // and, behind them, the merged tiles' output staging ([tile][32 queries][LDO] fp32)
    static_assert(8 * 32 * 64 * 4 + 8 * 32 * LDO * 4 <= (2 * KPL + 2 * VPL) * 2, "merge + staging fit the K / V image");
    _Float16* Ks = lds;
    _Float16* Vt = lds + 2 * KPL;
    const int h = blockIdx.x, b = blockIdx.y;
    // Ts: the row stride; T: this item's frames (ragged batches: its own, and items over 256 frames run the banded
    // kernel instead -- what they would run alone)
    const int T = tlen ? tlen[b] : Ts;
    if (T > TM) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hf = lane >> 5, col = lane & 31;
    const long long ld = 3LL * H * D;
    const long long row0 = toff ? (long long)toff[b] : (long long)b * Ts;  // the item's first row (toff: packed rows)
    const float* base = qkv + row0 * ld;
    const int task = attn_task(qg, (int)blockIdx.z, wave);
    const int qt = task >> 1, kh = task & 1;  // (task < 0: no task -- the wave only loads)
    // K / V rows 0 .. 255 (zeros past T) and the task's Q rows -> registers, all loads in flight before the first
    // use (the maxima below wait for K / V, and Q's latency hides under theirs)
    constexpr int PER = TM * (D / 4) / 1024;  // 4
    const int qw = (task < 0 ? 0 : qt) * 32;
    const int qi = qw + col;
    f32x4 kv[PER], vv[PER], qa[4][2];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int idx = tid + q * 1024;
        const int r = idx / (D / 4), c = (idx % (D / 4)) * 4;
        const int rr = r < T ? r : T - 1;
        kv[q] = *reinterpret_cast<const f32x4*>(base + (long long)rr * ld + H * D + h * D + c);
        vv[q] = *reinterpret_cast<const f32x4*>(base + (long long)rr * ld + 2 * H * D + h * D + c);
    }
    // the task's 32 queries: lane (query col, half hf) holds dims 16 ks + 8 hf .. +7 (Q pre-scaled by 1/8)
    const bool qok = task >= 0 && qi < T;
    {
        const float* qr = base + (long long)(qok ? qi : 0) * ld + h * D + 8 * hf;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            qa[ks][0] = *reinterpret_cast<const f32x4*>(qr + 16 * ks);
            qa[ks][1] = *reinterpret_cast<const f32x4*>(qr + 16 * ks + 4);
        }
    }
    float mk = 0.0f, mv = 0.0f;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int r = (tid + q * 1024) / (D / 4);
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        if (r >= T) {
            kv[q] = z;
            vv[q] = z;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            mk = fmaxf(mk, fabsf(kv[q][e]));
            mv = fmaxf(mv, fabsf(vv[q][e]));
        }
    }
    mk = wave_max(mk);
    mv = wave_max(mv);
    if (lane == 0) {
        red[0][wave] = mk;
        red[1][wave] = mv;
    }
    f16x8 qf[4][2];
    {
        float qv[4][8];
        float mq = 0.0f;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                qv[ks][e] = qok ? qa[ks][0][e] * scale : 0.0f;
                qv[ks][4 + e] = qok ? qa[ks][1][e] * scale : 0.0f;
                mq = fmaxf(mq, fmaxf(fabsf(qv[ks][e]), fabsf(qv[ks][4 + e])));
            }
        }
        const float sq = pow2_scale(wave_max(mq));
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) split8_h(qv[ks], sq, qf[ks][0], qf[ks][1]);
        if (lane == 0) mlx[0][0][wave] = sq;  // (read back below: keeps sq out of the chunk loop's registers)
    }
    __syncthreads();
    mk = red[0][0];
    mv = red[1][0];
#pragma unroll
    for (int w = 1; w < NWV; ++w) {
        mk = fmaxf(mk, red[0][w]);
        mv = fmaxf(mv, red[1][w]);
    }
    const float sk = pow2_scale(mk), sv = pow2_scale(mv);
    const float us = 1.0f / (sk * mlx[0][0][wave]);  // S^T accumulator -> scores (exact)
    // K planes (rows as loaded) and V planes (rows as loaded, chunk-swizzled: attn_vrow_off; read transposed)
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        if (ATTN_DIAG & 2) break;
        const int idx = tid + q * 1024;
        const int r = idx / (D / 4), c = (idx % (D / 4)) * 4;
        typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
        f16x4 h0, h1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float t = kv[q][e] * sk;
            h0[e] = (_Float16)t;
            h1[e] = (_Float16)(t - (float)h0[e]);
        }
        *reinterpret_cast<f16x4*>(Ks + r * KLD + c) = h0;
        *reinterpret_cast<f16x4*>(Ks + KPL + r * KLD + c) = h1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float t = vv[q][e] * sv;
            h0[e] = (_Float16)t;
            h1[e] = (_Float16)(t - (float)h0[e]);
        }
        *reinterpret_cast<f16x4*>(Vt + attn_vrow_off(r, c)) = h0;
        *reinterpret_cast<f16x4*>(Vt + VPL + attn_vrow_off(r, c)) = h1;
    }
    const float uo = 1.0f / (16384.0f * sv);  // O^T accumulator -> P V (exact)
    f32x16 o[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
    float m = -INFINITY, l = 0.f;
    __syncthreads();
    const bool active = task >= 0 && qw < T;
    const int kend = min(T - 1, qw + 31);
    const int vlb0 = attn_vlane_base(lane, 0), vlb1 = attn_vlane_base(lane, 1);
    if (active) {
        // the tile's chunks kstart, kstart + 32, .., <= kend: half 0 the first ceil(n / 2), half 1 the rest
        const int kstart = max(0, qw - window + 1) & ~31;
        const int n = (kend - kstart) / 32 + 1, n0 = (n + 1) >> 1;
        const int cb = kstart + (kh ? 32 * n0 : 0), ce = kstart + 32 * (kh ? n : n0);
        for (int c0 = cb; c0 < ce; c0 += 32) {
            if (ATTN_DIAG & 1) break;
            attn_chunk_h16<KLD, KPL, VLD, VPL, true>(o, m, l, qf, Ks + c0 * KLD, Vt, c0, qw, qi, kend, window, hf,
                                                     col, us, 1.0f, 16384.0f, vlb0, vlb1);
        }
    }
    __syncthreads();  // K / V dead: the merge and the output staging reuse the LDS
    float* mo = reinterpret_cast<float*>(lds);
    if (active && kh == 1 && !(ATTN_DIAG & 4)) {
        float* dst = mo + qt * 32 * 64;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) dst[(t * 16 + r) * 64 + lane] = o[t][r];
        if (hf == 0) {
            mlx[qt][0][col] = m;
            mlx[qt][1][col] = l;
        }
    }
    __syncthreads();
    if (active && kh == 0) {
        // merge with the half-1 task (none, or no chunks: m1 = -inf, c1 = 0, c0 = exp(0) = 1 -- o unchanged)
        float m1 = -INFINITY, l1 = 0.0f;
        const int n = (ATTN_DIAG & 4) ? 1 : (kend - (max(0, qw - window + 1) & ~31)) / 32 + 1;
        if (n > 1) {
            m1 = mlx[qt][0][col];
            l1 = mlx[qt][1][col];
        }
        const float mm = fmaxf(m, m1);
        const float c0 = (m == -INFINITY) ? 0.f : __expf(m - mm);
        const float c1 = (m1 == -INFINITY) ? 0.f : __expf(m1 - mm);
        l = l * c0 + l1 * c1;
        const float* src = mo + qt * 32 * 64;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float o1 = n > 1 ? src[(t * 16 + r) * 64 + lane] : 0.0f;
                o[t][r] = o[t][r] * c0 + o1 * c1;
            }
        // staging [tile][32 queries][LDO] behind the merge region
        float* ow = mo + 8 * 32 * 64 + qt * 32 * LDO;
        const float inv = (l > 0.f) ? uo / l : 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int d = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
                ow[col * LDO + d] = o[t][r] * inv;
            }
    }
    __syncthreads();
    // every wave stores 16 queries of a staged tile (wave w: tile w >> 1, queries 16 (w & 1) ..): lane = query
    // 8 s + (lane >> 3) x dims 8 (lane & 7) .. +7, one 16-B store per plane (conflict-free staging reads)
    float mx = 0.0f;
    const int st = wave >> 1;
    if (attn_tile_in_wg(qg, (int)blockIdx.z, st)) {
        const float* ows = mo + 8 * 32 * 64 + st * 32 * LDO;
        const int d8 = (lane & 7) * 8;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const int qq = 16 * (wave & 1) + 8 * s2 + (lane >> 3);
            const int q = st * 32 + qq;
            if (q < T) {
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = ows[qq * LDO + d8 + e];
                store_act8(outp, pstride, 2, (row0 + q) * (H * D) + h * D + d8, v, oscale, &mx);
            }
        }
    }
    amax_commit(oamax, mx);
}

// query-tile groups per (item, head) for the T <= 256 kernel: enough workgroups to cover the CUs
static int attn_qg(int batch, int H) {
    const long long pairs = (long long)batch * H;
    return pairs >= 256 ? 1 : pairs >= 128 ? 2 : 4;
}

// T > 256 (clips over 10.24 s) on the fp16 matrix cores, in a form whose every output is the same arithmetic however
// the work is split across workgroups.  The keys of a 32-query tile's band [q0 - W + 1, q0 + 31] are visited as whole
// 32-key chunks c (keys 32 c .. 32 c + 31), and each chunk's contribution is formed on its own (attn_band_scores,
// attn_band_pv):
//   K / V fp16 planes at power-of-two scales from THAT chunk's max |K|, |V| over its keys < T (never zeroed at a
//   workgroup's band end), S^T = K . Q^T on the planes (Q planes at the tile's own power-of-two scale), the masked
//   chunk max m_c, p = exp(s - m_c), l_c = sum p, O_c^T = V^T . P^T on the planes, unscaled exactly;
// and the tile's state folds the chunks in ascending order (attn_band_coef / _apply: m = max(m, m_c), o = o a + o_c b,
// l = l a + l_c b, a = exp(m_old - m), b = exp(m_c - m)); out = o / l.  Two decompositions of that same arithmetic:
//   SPLIT = false (large grids): a workgroup = 128 queries x 4 waves sharing each chunk image (one chunk per barrier
//                 pair, K / V rows of chunk c + 1 in registers while chunk c is computed), every wave folds the
//                 chunks of its own tile in order;
//   SPLIT = true  (small grids: a batch-1 utterance has 8 x ceil(T / 128) such workgroups for 256 CUs): a workgroup
//                 = ONE 32-query tile x 4 waves; in round r wave w forms chunk cs + 4 r + w into its own LDS image,
//                 waves 1-3 hand their partials to wave 0 through LDS (double-buffered by round), wave 0 folds the
//                 round's chunks in ascending order -- a tile's chain of up to 10 dependent chunk steps becomes 3.
// Every value either form produces is the same bit for bit (tests/test_attention_band.py), so the engine picks the
// form by grid size without an utterance's codes depending on its batch.
namespace {
constexpr int BD = 64, BKC = 32, BLDO = BD + 1;
constexpr int BKLD = 72, BKPL = BKC * BKLD;  // K planes: [32 keys][72 halves] (conflict-free b128 fragment reads)
constexpr int BVLD = 40, BVPL = BD * BVLD;   // V^T planes: [64 dims][40 halves]
constexpr int BCH = 2 * BKPL + 2 * BVPL;     // halves of one chunk image
}  // namespace

// One chunk's scores for the wave's 32 queries (lane: query col, half hf): S^T = K . Q^T on the planes, the mask,
// the chunk's own max mc and p = exp(s - mc) as fp16 planes at 2^14 (pp0 / pp1: keys 16 ks .. of the chunk in the
// S^T accumulator's order), lc = sum p.  us = 1 / (sK sQ).
__device__ __forceinline__ void attn_band_scores(f16x8 (&pp0)[2], f16x8 (&pp1)[2], float& mc, float& lc,
                                                 const f16x8 (&qf)[4][2], const _Float16* Kc, int c0, int qw, int qi,
                                                 int T, int window, int hf, int col, float us) {
    f32x16 st;
#pragma unroll
    for (int r = 0; r < 16; ++r) st[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        const int ko = col * BKLD + 16 * ks + 8 * hf;
        const f16x8 k0 = *reinterpret_cast<const f16x8*>(Kc + ko);
        const f16x8 k1 = *reinterpret_cast<const f16x8*>(Kc + BKPL + ko);
        st = __builtin_amdgcn_mfma_f32_32x32x16_f16(k1, qf[ks][0], st, 0, 0, 0);
        st = __builtin_amdgcn_mfma_f32_32x32x16_f16(k0, qf[ks][1], st, 0, 0, 0);
        st = __builtin_amdgcn_mfma_f32_32x32x16_f16(k0, qf[ks][0], st, 0, 0, 0);
    }
    float cmax = -INFINITY;
    const bool full = c0 + 31 <= qw && c0 > qw + 31 - window && c0 + 31 < T;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        float v = st[r] * us;
        if (!full) {
            const int key = c0 + (r & 3) + 8 * (r >> 2) + 4 * hf;
            const bool ok = key <= qi && key > qi - window && key < T;
            v = ok ? v : -INFINITY;
        }
        st[r] = v;
        cmax = fmaxf(cmax, v);
    }
    cmax = fmaxf(cmax, __shfl_xor(cmax, 32));
    mc = cmax;
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float pv = (st[r] == -INFINITY) ? 0.f : __expf(st[r] - cmax);
        st[r] = pv;
        psum += pv;
    }
    psum += __shfl_xor(psum, 32);
    lc = psum;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        float pe[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) pe[e] = st[8 * ks + e];
        split8_h(pe, 16384.0f, pp0[ks], pp1[ks]);
    }
}

// dims 32 t .. 32 t + 31 of the chunk's O^T = V^T . P^T on the planes (at 2^14 sV)
__device__ __forceinline__ void attn_band_pv(f32x16& oct, const f16x8 (&pp0)[2], const f16x8 (&pp1)[2],
                                             const _Float16* Vc, int t, int hf, int col) {
#pragma unroll
    for (int r = 0; r < 16; ++r) oct[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        const int vo = (32 * t + col) * BVLD + 16 * ks + 8 * hf;
        const f16x8 v0 = *reinterpret_cast<const f16x8*>(Vc + vo);
        const f16x8 v1 = *reinterpret_cast<const f16x8*>(Vc + BVPL + vo);
        oct = __builtin_amdgcn_mfma_f32_32x32x16_f16(v1, pp0[ks], oct, 0, 0, 0);
        oct = __builtin_amdgcn_mfma_f32_32x32x16_f16(v0, pp1[ks], oct, 0, 0, 0);
        oct = __builtin_amdgcn_mfma_f32_32x32x16_f16(v0, pp0[ks], oct, 0, 0, 0);
    }
}

// The tile state after one more chunk, in ascending chunk order: m = max(m, mc), l = l a + lc b, and the factors
// the caller applies to o (o = o a + oc bu with bu = b uo; uo = 1 / (2^14 sV) is a power of two, so oc bu rounds as
// (oc uo) b).  A query with no valid key in the chunk (mc = -inf, oc = 0): a = 1, bu = 0, nothing changes.
__device__ __forceinline__ void attn_band_coef(float& m, float& l, float mc, float lc, float uo, float& a, float& bu) {
    if (mc == -INFINITY) {
        a = 1.0f;
        bu = 0.0f;
        return;
    }
    const float mn = fmaxf(m, mc);
    a = (m == -INFINITY) ? 0.f : __expf(m - mn);
    const float bb = __expf(mc - mn);
    bu = bb * uo;
    l = __builtin_fmaf(lc, bb, l * a);
    m = mn;
}
__device__ __forceinline__ void attn_band_apply(f32x16& ot, const f32x16& oct, float a, float bu) {
#pragma unroll
    for (int r = 0; r < 16; ++r) ot[r] = __builtin_fmaf(oct[r], bu, ot[r] * a);
}

// a chunk's K / V rows as fp16 planes at its own scales: K rows [32][BKLD], V^T [64][BVLD] (keys permuted inside each
// 16 as the S^T accumulator holds them); rows past T hold zeros (loaded as such)
__device__ __forceinline__ void attn_band_planes(_Float16* img, int r, int c, const f32x4& kr, const f32x4& vr,
                                                 float sk, float sv) {
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    f16x4 h0, h1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float t = kr[e] * sk;
        h0[e] = (_Float16)t;
        h1[e] = (_Float16)(t - (float)h0[e]);
    }
    *reinterpret_cast<f16x4*>(img + r * BKLD + c) = h0;
    *reinterpret_cast<f16x4*>(img + BKPL + r * BKLD + c) = h1;
    _Float16* Vt = img + 2 * BKPL;
    const int pr = vt_key_pos(r);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float t = vr[e] * sv;
        const _Float16 a0 = (_Float16)t;
        Vt[(c + e) * BVLD + pr] = a0;
        Vt[BVPL + (c + e) * BVLD + pr] = (_Float16)(t - (float)a0);
    }
}

// Q planes of the wave's 32 queries qw .. qw + 31 (lane: query col, dims 16 ks + 8 hf .. +7), pre-scaled by `scale`,
// at the wave's own power-of-two scale (returned)
__device__ __forceinline__ float attn_band_q(const float* base, long long ld, int h, int qi, int T, float scale, int hf,
                                             f16x8 (&qf)[4][2]) {
    float qv[4][8];
    float mq = 0.0f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        f32x4 a = {0.f, 0.f, 0.f, 0.f}, c = {0.f, 0.f, 0.f, 0.f};
        if (qi < T) {
            const float* qr = base + (long long)qi * ld + h * BD + 16 * ks + 8 * hf;
            a = *reinterpret_cast<const f32x4*>(qr);
            c = *reinterpret_cast<const f32x4*>(qr + 4);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            qv[ks][e] = a[e] * scale;
            qv[ks][4 + e] = c[e] * scale;
            mq = fmaxf(mq, fmaxf(fabsf(qv[ks][e]), fabsf(qv[ks][4 + e])));
        }
    }
    const float sq = pow2_scale(wave_max(mq));
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) split8_h(qv[ks], sq, qf[ks][0], qf[ks][1]);
    return sq;
}

template <bool SPLIT>
__global__ __launch_bounds__(256) void attention_band_h16_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                                 int Ts, int H, int window, float scale,
                                                                 void* __restrict__ outp, long long pstride, int outns,
                                                                 float oscale, unsigned* __restrict__ oamax,
                                                                 const int* __restrict__ tlen,
                                                                 const int* __restrict__ toff) {
    // LDS: SPLIT -- 4 wave-private chunk images, then the partials of waves 1-3 ([2 rounds][3][35][64] fp32: 32
    // O^T values, m, l, the V unscale per lane); else one shared chunk image.  The output staging ([waves][32][BLDO] fp32) reuses
    // the front once the chunks are done.
    constexpr int PARTF = 2 * 3 * 35 * 64;                          // floats
    constexpr int IMGH = SPLIT ? 4 * BCH : BCH;                     // halves
    constexpr int STGH = (SPLIT ? 1 : 4) * 32 * BLDO * 2;           // halves
    constexpr int LDSH = (IMGH > STGH ? IMGH : STGH) + (SPLIT ? 2 * PARTF : 0);
    __shared__ __attribute__((aligned(16))) _Float16 lds[LDSH];
    __shared__ float red[2][4];
    const int b = blockIdx.z, h = blockIdx.y;
    // Ts: the row stride; T: this item's frames (ragged batches: items of <= 256 frames run the T <= 256 kernel)
    const int T = tlen ? tlen[b] : Ts;
    const int q0 = blockIdx.x * (SPLIT ? 32 : 128);
    if (tlen && (T <= 256 || q0 >= T)) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hf = lane >> 5, col = lane & 31;
    const long long ld = 3LL * H * BD;
    const long long row0 = toff ? (long long)toff[b] : (long long)b * Ts;  // the item's first row (toff: packed rows)
    const float* base = qkv + row0 * ld;
    const int qw = SPLIT ? q0 : q0 + 32 * wave, qi = qw + col;
    f16x8 qf[4][2];
    const float sq = attn_band_q(base, ld, h, qi, T, scale, hf, qf);
    // the tile's chunks cs .. ce (every wave of a SPLIT workgroup has the same tile)
    const int cs = max(0, qw - window + 1) >> 5, ce = min(T - 1, qw + 31) >> 5;
    f32x16 o[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
    float m = -INFINITY, l = 0.f;
    float mx = 0.0f;
    if constexpr (SPLIT) {
        f32x16 oc[2];
        _Float16* img = lds + wave * BCH;
        float* part = reinterpret_cast<float*>(lds + (IMGH > STGH ? IMGH : STGH));
        // the wave's chunk of a round: 32 K / V rows, lane -> 16-B column (lane & 15) of rows (lane >> 4) + 4 q; the
        // next round's rows load into the same registers once this round's planes are written
        f32x4 kr[8], vr[8];
        auto fetch = [&](int c) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int j = 32 * c + (lane >> 4) + 4 * q, cc = (lane & 15) * 4;
                const f32x4 z = {0.f, 0.f, 0.f, 0.f};
                kr[q] = z;
                vr[q] = z;
                if (j < T) {
                    kr[q] = *reinterpret_cast<const f32x4*>(base + (long long)j * ld + H * BD + h * BD + cc);
                    vr[q] = *reinterpret_cast<const f32x4*>(base + (long long)j * ld + 2 * H * BD + h * BD + cc);
                }
            }
        };
        if (cs + wave <= ce) fetch(cs + wave);
        for (int r = 0; cs + 4 * r <= ce; ++r) {
            const int c = cs + 4 * r + wave;
            float mc = -INFINITY, lc = 0.f, uo = 0.f;
            if (c <= ce) {
                float ak = 0.0f, av = 0.0f;
#pragma unroll
                for (int q = 0; q < 8; ++q)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        ak = fmaxf(ak, fabsf(kr[q][e]));
                        av = fmaxf(av, fabsf(vr[q][e]));
                    }
                const float sk = pow2_scale(wave_max(ak)), sv = pow2_scale(wave_max(av));
#pragma unroll
                for (int q = 0; q < 8; ++q) attn_band_planes(img, (lane >> 4) + 4 * q, (lane & 15) * 4, kr[q], vr[q], sk, sv);
                if (c + 4 <= ce) fetch(c + 4);
                // the same wave reads its image back: LDS order within a wave (the compiler keeps the writes first)
                asm volatile("" ::: "memory");
                f16x8 pp0[2], pp1[2];
                attn_band_scores(pp0, pp1, mc, lc, qf, img, 32 * c, qw, qi, T, window, hf, col, 1.0f / (sk * sq));
                attn_band_pv(oc[0], pp0, pp1, img + 2 * BKPL, 0, hf, col);
                attn_band_pv(oc[1], pp0, pp1, img + 2 * BKPL, 1, hf, col);
                uo = 1.0f / (16384.0f * sv);
                if (wave > 0) {
                    float* pw = part + ((r & 1) * 3 + wave - 1) * 35 * 64;
#pragma unroll
                    for (int t = 0; t < 2; ++t)
#pragma unroll
                        for (int e = 0; e < 16; ++e) pw[(16 * t + e) * 64 + lane] = oc[t][e];
                    pw[32 * 64 + lane] = mc;
                    pw[33 * 64 + lane] = lc;
                    pw[34 * 64 + lane] = uo;
                }
            }
            __syncthreads();  // the round's partials are in LDS (and the previous round's slots are read)
            if (wave == 0) {
                float a, bu;
                attn_band_coef(m, l, mc, lc, uo, a, bu);  // (mc = -inf when wave 0 had no chunk: no change)
                attn_band_apply(o[0], oc[0], a, bu);
                attn_band_apply(o[1], oc[1], a, bu);
#pragma unroll 1
                for (int w = 1; w < 4; ++w) {
                    if (cs + 4 * r + w > ce) break;
                    const float* pw = part + ((r & 1) * 3 + w - 1) * 35 * 64;
#pragma unroll
                    for (int t = 0; t < 2; ++t)
#pragma unroll
                        for (int e = 0; e < 16; ++e) oc[t][e] = pw[(16 * t + e) * 64 + lane];
                    attn_band_coef(m, l, pw[32 * 64 + lane], pw[33 * 64 + lane], pw[34 * 64 + lane], a, bu);
                    attn_band_apply(o[0], oc[0], a, bu);
                    attn_band_apply(o[1], oc[1], a, bu);
                }
            }
        }
        __syncthreads();  // every image is dead: wave 0 stages the tile's output at the front
        float* ow = reinterpret_cast<float*>(lds);
        if (wave == 0) {
            const float inv = (l > 0.f) ? 1.0f / l : 0.f;
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int d = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
                    ow[col * BLDO + d] = o[t][r] * inv;
                }
        }
        __syncthreads();
        for (int qq = 8 * wave; qq < 8 * wave + 8; ++qq) {  // wave w stores queries 8 w .. 8 w + 7
            const int q = qw + qq;
            if (q < T)
                store_act(out, outp, pstride, outns, (row0 + q) * (H * BD) + h * BD + lane, ow[qq * BLDO + lane],
                          oscale, &mx);
        }
    } else {
        // the workgroup's chunks: the union of its 4 tiles' (rows of chunk c + 1 in registers while c is computed)
        const int kc0 = max(0, q0 - window + 1) >> 5, kc1 = min(T - 1, q0 + 127) >> 5;
        f32x4 kr[2], vr[2];
        auto fetch = [&](int c) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int idx = tid + q * 256, rr = idx >> 4, cc = (idx & 15) * 4, j = 32 * c + rr;
                const f32x4 z = {0.f, 0.f, 0.f, 0.f};
                kr[q] = z;
                vr[q] = z;
                if (j < T) {
                    kr[q] = *reinterpret_cast<const f32x4*>(base + (long long)j * ld + H * BD + h * BD + cc);
                    vr[q] = *reinterpret_cast<const f32x4*>(base + (long long)j * ld + 2 * H * BD + h * BD + cc);
                }
            }
        };
        auto chunk_max = [&]() {
            float a = 0.0f, v = 0.0f;
#pragma unroll
            for (int q = 0; q < 2; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    a = fmaxf(a, fabsf(kr[q][e]));
                    v = fmaxf(v, fabsf(vr[q][e]));
                }
            a = wave_max(a);
            v = wave_max(v);
            if (lane == 0) {
                red[0][wave] = a;
                red[1][wave] = v;
            }
        };
        fetch(kc0);
        chunk_max();
        for (int c = kc0; c <= kc1; ++c) {
            // the previous chunk's fragment reads are done; red holds this chunk's maxima (the explicit wait: no
            // lgkmcnt(0) is emitted before this barrier on the loop's back edge)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __syncthreads();
            const float sk = pow2_scale(fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3])));
            const float sv = pow2_scale(fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3])));
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int idx = tid + q * 256;
                attn_band_planes(lds, idx >> 4, (idx & 15) * 4, kr[q], vr[q], sk, sv);
            }
            __syncthreads();  // the chunk image is complete (and red is read)
            const bool more = c < kc1;
            if (more) fetch(c + 1);
            if (qw < T && c >= cs && c <= ce) {
                float mc, lc, a, bu;
                f16x8 pp0[2], pp1[2];
                attn_band_scores(pp0, pp1, mc, lc, qf, lds, 32 * c, qw, qi, T, window, hf, col, 1.0f / (sk * sq));
                attn_band_coef(m, l, mc, lc, 1.0f / (16384.0f * sv), a, bu);
#pragma unroll
                for (int t = 0; t < 2; ++t) {  // one dim half at a time: 16 accumulator registers, not 32
                    f32x16 oct;
                    attn_band_pv(oct, pp0, pp1, lds + 2 * BKPL, t, hf, col);
                    attn_band_apply(o[t], oct, a, bu);
                }
            }
            if (more) chunk_max();
        }
        __syncthreads();  // the chunk image is dead: the output staging reuses the LDS
        float* ow = reinterpret_cast<float*>(lds) + wave * 32 * BLDO;
        const float inv = (l > 0.f) ? 1.0f / l : 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int d = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
                ow[col * BLDO + d] = o[t][r] * inv;
            }
        // same wave wrote and reads its staging rows: LDS order, no barrier
        for (int qq = 0; qq < 32; ++qq) {
            const int q = qw + qq;
            if (q < T)
                store_act(out, outp, pstride, outns, (row0 + q) * (H * BD) + h * BD + lane, ow[qq * BLDO + lane],
                          oscale, &mx);
        }
    }
    amax_commit(oamax, mx);
}

// the banded kernel's decomposition: SPLIT when the 128-query form would leave most CUs idle (mode: 0 never, 1 when
// it has fewer than 128 workgroups, 2 always -- the same values every way)
static bool band_split(int mode, int batch, int Tmax, int H) {
    if (mode != 1) return mode == 2;
    return (long long)((Tmax + 127) / 128) * H * batch < 128;
}
static hipError_t launch_band(const float* qkv, float* out, int batch, int T, int Tmax, int H, int window,
                              float scale, hipStream_t s, void* outp, long long pstride, int outns, float oscale,
                              unsigned* oamax, const int* tlen, const int* toff, const char** kname, int split) {
    if (band_split(split, batch, Tmax, H)) {
        hipLaunchKernelGGL(attention_band_h16_kernel<true>, dim3((Tmax + 31) / 32, H, batch), dim3(256), 0, s, qkv,
                           out, T, H, window, scale, outp, pstride, outns, oscale, oamax, tlen, toff);
        if (kname) *kname = "mimi::attention_band_h16_kernel<true>";
    } else {
        hipLaunchKernelGGL(attention_band_h16_kernel<false>, dim3((Tmax + 127) / 128, H, batch), dim3(256), 0, s, qkv,
                           out, T, H, window, scale, outp, pstride, outns, oscale, oamax, tlen, toff);
        if (kname) *kname = "mimi::attention_band_h16_kernel<false>";
    }
    return hipGetLastError();
}

hipError_t launch_attention_band(const float* qkv, int batch, int T, int H, int window, float scale,
                                 hipStream_t s, void* outp, long long out_pstride, float oscale, unsigned* oamax,
                                 int split) {
    return launch_band(qkv, nullptr, batch, T, T, H, window, scale, s, outp, out_pstride, 2, oscale, oamax, nullptr,
                       nullptr, nullptr, split);
}

hipError_t launch_attention(const float* qkv, float* out, int batch, int T, int H, int D, int window, float scale,
                            hipStream_t s, void* outp, long long out_pstride, int outns, float oscale,
                            unsigned* oamax, bool h16, const int* tlen, int max_tlen, int min_tlen,
                            const int* toff, const char** kname, int band_split_mode) {
    if (D != 64 || (outns != 0 && !outp) || (outns == 0 && !out) || (oscale > 0.0f && outns != 2)) return hipErrorInvalidValue;
    if (tlen) {  // ragged batch: each item the kernel it would run alone (each exits on the other's items)
        if (!h16 || !(oscale > 0.0f && outns == 2) || max_tlen > T || min_tlen < 1) return hipErrorInvalidValue;
        if (min_tlen <= 256) {
            const int qg = attn_qg(batch, H);
            hipLaunchKernelGGL(attention_t256_h16_kernel, dim3(H, batch, qg), dim3(1024), 0, s, qkv, T, H, window,
                               scale, outp, out_pstride, oscale, oamax, tlen, qg, toff);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        if (max_tlen > 256)
            return launch_band(qkv, out, batch, T, max_tlen, H, window, scale, s, outp, out_pstride, outns, oscale,
                               oamax, tlen, toff, kname, band_split_mode);
        return hipGetLastError();
    }
    // (the banded kernel at T <= 256 measured slower at B = 1 and B = 32: profiles/r2d_ab_attention_band.log)
    if (h16 && T <= 256) {  // fp16-plane output (the engine's plane path at these lengths)
        if (!(oscale > 0.0f && outns == 2)) return hipErrorInvalidValue;
        const int qg = attn_qg(batch, H);
        hipLaunchKernelGGL(attention_t256_h16_kernel, dim3(H, batch, qg), dim3(1024), 0, s, qkv, T, H, window, scale,
                           outp, out_pstride, oscale, oamax, nullptr, qg, nullptr);
        return hipGetLastError();
    }
    if (h16)  // T > 256: fp16-plane output, or fp32 for clips too long for the plane buffers
        return launch_band(qkv, out, batch, T, T, H, window, scale, s, outp, out_pstride, outns, oscale, oamax,
                           nullptr, nullptr, kname, band_split_mode);
    if (T <= 256) {
        hipLaunchKernelGGL(attention_t256_kernel, dim3(H, batch), dim3(512), 0, s, qkv, out, T, H, window, scale,
                           outp, out_pstride, outns, oscale, oamax);
        return hipGetLastError();
    }
    dim3 grid((T + 127) / 128, H, batch);
    hipLaunchKernelGGL(attention_kernel, grid, dim3(256), 0, s, qkv, out, T, H, window, scale, outp, out_pstride,
                       outns, oscale, oamax);
    return hipGetLastError();
}

// one workgroup per (item, edge, 64 output channels): thread (slice sl of 16, group g of 4 consecutive
// channels) sums its C/16 terms with 16-B weight loads all in flight at once; the slices are added in a fixed
// order, then the row and its planes are updated.  T = 1 (F = 1, clips of <= 960 samples): both replicate terms
// land on the one output row, so the edge-0 workgroup adds them both, left edge first (the edge-1 workgroup
// exits) -- two workgroups updating one row would race and lose a term.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void ds_edge_fix_kernel(const float* __restrict__ x, const float* __restrict__ wfix,
                                                          float* __restrict__ out, void* __restrict__ outp,
                                                          long long pstride, float oscale, unsigned* __restrict__ oamax,
                                                          int Ts, int Fs, int C, int N, const int* __restrict__ tlen,
                                                          const int* __restrict__ flen, const int* __restrict__ toff) {
    const int b = blockIdx.x, edge = blockIdx.y;
    const int T = tlen ? tlen[b] : Ts, F = flen ? flen[b] : Fs;  // (Ts, Fs: the row strides)
    const bool right = (T & 1) != 0;                 // a right "extra" row exists
    if (edge == 1 && (!right || F == 1)) return;
    const int last_edge = edge == 0 && right && F == 1 ? 1 : edge;
    const int f = edge == 0 ? 0 : F - 1;
    const int g = threadIdx.x & 15, sl = threadIdx.x >> 4;
    const int n0 = blockIdx.z * 64;
    const int cs = C / 16, c0 = sl * cs;
    __shared__ float part[16][64];
    const long long o = ((long long)b * Fs + f) * N + n0 + (threadIdx.x & 63);
    float v = threadIdx.x < 64 ? out[o] : 0.0f;
    for (int e = edge; e <= last_edge; ++e) {
        const int t = e == 0 ? 0 : T - 1;
        const float* __restrict__ wc = wfix + (long long)e * C * N + n0 + 4 * g;  // [edge][c][n]
        const float* __restrict__ xr = x + ((toff ? (long long)toff[b] : (long long)b * Ts) + t) * C;  // (toff: packed)
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
        // 16 channels per round: all 20 loads issued before the first FMA (a plain loop let the compiler wait out
        // each load's latency in turn: 13.8 us per launch at any batch); same FMA order as the plain loop
        for (int c = c0; c < c0 + cs; c += 16) {
            f32x4 w[16], xv[4];
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = *reinterpret_cast<const f32x4*>(wc + (long long)(c + i) * N);
#pragma unroll
            for (int i = 0; i < 4; ++i) xv[i] = *reinterpret_cast<const f32x4*>(xr + c + 4 * i);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float x1 = xv[i >> 2][i & 3];
                a.x = __builtin_fmaf(w[i].x, x1, a.x);
                a.y = __builtin_fmaf(w[i].y, x1, a.y);
                a.z = __builtin_fmaf(w[i].z, x1, a.z);
                a.w = __builtin_fmaf(w[i].w, x1, a.w);
            }
        }
        if (e != edge) __syncthreads();  // wave 0 has read the previous edge's partials
        part[sl][4 * g] = a.x;
        part[sl][4 * g + 1] = a.y;
        part[sl][4 * g + 2] = a.z;
        part[sl][4 * g + 3] = a.w;
        __syncthreads();
        if (threadIdx.x < 64) {
            float sum = 0.0f;
#pragma unroll
            for (int q = 0; q < 16; ++q) sum += part[q][threadIdx.x];
            v = v + sum;
        }
    }
    if (threadIdx.x >= 64) return;  // (wave-uniform: wave 0 finishes)
    out[o] = v;
    float mx = 0.0f;
    if (outp) store_act(nullptr, outp, pstride, 2, o, v, oscale, &mx);
    if (outp) amax_commit(oamax, mx);
}
hipError_t launch_ds_edge_fix(const float* x, const float* wfix, float* out, void* outp, long long out_pstride,
                              float oscale, unsigned* oamax, int B, int T, int F, int C, int N, hipStream_t s,
                              const int* tlen, const int* flen, const int* toff) {
    if (B <= 0 || T <= 0 || F <= 0 || N % 64 || C % 256 || (outp && !(oscale > 0.0f)) || (!tlen != !flen) ||
        (toff && !tlen))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(ds_edge_fix_kernel, dim3(B, 2, N / 64), dim3(256), 0, s, x, wfix, out, outp, out_pstride,
                       oscale, oamax, T, F, C, N, tlen, flen, toff);
    return hipGetLastError();
}

// ragged batches, packed transformer rows: rpos[toff[b] + t] = t for t < tlen[b] (RoPE positions)
__global__ __launch_bounds__(256) void ragged_rows_kernel(const int* __restrict__ tlen, const int* __restrict__ toff,
                                                          int* __restrict__ rpos) {
    const int b = blockIdx.x, T = tlen[b], o = toff[b];
    for (int t = threadIdx.x; t < T; t += 256) rpos[o + t] = t;
}
hipError_t launch_ragged_rows(const int* tlen, const int* toff, int B, int* rpos, hipStream_t s) {
    if (B <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(ragged_rows_kernel, dim3(B), dim3(256), 0, s, tlen, toff, rpos);
    return hipGetLastError();
}

// Self-check of the fp16 plane split (kernels.h split2_f16s, the form every planes epilogue, LayerNorm and conv0 use)
// against the plain form it replaces (fp16(v s), fp16(v s - hi) by conversions): per value pair, out[4 i .. 4 i + 3]
// = split2_f16s's (hi, lo) words and the plain form's (hi, lo) words.  Diagnostic entry mimi_split_check.
__global__ __launch_bounds__(256) void split_check_kernel(const float* __restrict__ in, long long npairs, float s,
                                                          unsigned* __restrict__ out) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < npairs; i += (long long)gridDim.x * 256) {
        const float v0 = in[2 * i], v1 = in[2 * i + 1];
        unsigned hi, lo;
        split2_f16s(v0, v1, s, hi, lo);
        const float t0 = v0 * s, t1 = v1 * s;
        h2 a, b;
        a[0] = (_Float16)t0;
        a[1] = (_Float16)t1;
        b[0] = (_Float16)(t0 - (float)a[0]);
        b[1] = (_Float16)(t1 - (float)a[1]);
        out[4 * i] = hi;
        out[4 * i + 1] = lo;
        out[4 * i + 2] = __builtin_bit_cast(unsigned, a);
        out[4 * i + 3] = __builtin_bit_cast(unsigned, b);
    }
}
hipError_t launch_split_check(const float* in, long long npairs, float s, unsigned* out, hipStream_t st) {
    if (npairs <= 0) return hipSuccess;
    const long long blocks = std::min<long long>((npairs + 255) / 256, 4096);
    hipLaunchKernelGGL(split_check_kernel, dim3((unsigned)blocks), dim3(256), 0, st, in, npairs, s, out);
    return hipGetLastError();
}

// (+ zeroes the replay's RVQ chain flag and granules, n16 16-B units from zero: the memset node a graph would hold)
__global__ __launch_bounds__(256) void set_io_kernel(void** io, const float* audio, int32_t* codes, unsigned* hamax,
                                                     unsigned* hflag, uint4* zero, long long n16) {
    if (threadIdx.x == 0) {
        io[0] = const_cast<float*>(audio);
        io[1] = codes;
        io[2] = hamax;
        io[3] = hflag;
    }
    const uint4 z = {0u, 0u, 0u, 0u};
    for (long long i = threadIdx.x; i < n16; i += 256) zero[i] = z;
}
hipError_t launch_set_io(void** io, const float* audio, int32_t* codes, hipStream_t s, unsigned* hamax,
                         unsigned* hflag, void* zero, size_t zero_bytes) {
    if (zero_bytes % 16 || (zero_bytes && (!zero || reinterpret_cast<uintptr_t>(zero) % 16))) return hipErrorInvalidValue;
    hipLaunchKernelGGL(set_io_kernel, dim3(1), dim3(256), 0, s, io, audio, codes, hamax, hflag,
                       static_cast<uint4*>(zero), (long long)(zero_bytes / 16));
    return hipGetLastError();
}

// Each sub-slot is read AND reset to 0 by one device-scope atomic exchange (at the memory side, like the
// producers' atomicMax): no XCD's L2 can hand this fold a stale line, and the next encode (or graph replay)
// starts from zeros without a memset.
// With a ticket (hamax: pinned host words) the folded maxima also go straight to the host, and workgroup 0 copies the
// persistent RVQ chain's give-up flag beside them -- in place of two D2H copy launches after the encode (~7 us each
// at batch 1).  io != null: a graph replay's destinations, io[2] / io[3] as set_io_kernel wrote them before it.
__global__ __launch_bounds__(64) void amax_reduce_kernel(unsigned* __restrict__ amax, unsigned* __restrict__ out,
                                                         unsigned* hamax, const unsigned* __restrict__ flag,
                                                         unsigned* hflag, void* const* __restrict__ io) {
    if (io) {
        hamax = static_cast<unsigned*>(io[2]);
        hflag = static_cast<unsigned*>(io[3]);
    }
    unsigned* a = amax + (long long)blockIdx.x * AMAX_SLOT_WORDS;
    unsigned v = threadIdx.x < AMAX_SUB ? atomicExch(a + threadIdx.x * AMAX_STRIDE, 0u) : 0u;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, (unsigned)__shfl_xor((int)v, o));
    if (threadIdx.x == 0) {
        out[blockIdx.x] = v;
        if (hamax) hamax[blockIdx.x] = v;
        if (blockIdx.x == 0 && flag && hflag) hflag[0] = *flag;
    }
}

hipError_t launch_amax_reduce(unsigned* amax, int nslots, unsigned* out, hipStream_t s, unsigned* hamax,
                              const unsigned* flag, unsigned* hflag, void* const* io) {
    if (nslots <= 0) return hipSuccess;
    static_assert(AMAX_SUB <= 64, "one wave per slot");
    hipLaunchKernelGGL(amax_reduce_kernel, dim3(nslots), dim3(64), 0, s, amax, out, hamax, flag, hflag, io);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void planes_to_f32_kernel(const __bf16* __restrict__ pl, long long pstride, int ns,
                                                            float* __restrict__ out, long long n, float hscale) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    if (hscale > 0.0f) {
        const _Float16* hp = reinterpret_cast<const _Float16*>(pl);
        out[i] = ((float)hp[i] + (float)hp[i + pstride]) / hscale;
        return;
    }
    float v = (float)pl[i] + (float)pl[i + pstride];
    if (ns == 3) v = v + (float)pl[i + 2 * pstride];
    out[i] = v;
}

hipError_t launch_planes_to_f32(const void* planes, long long pstride, int ns, float* out, long long n,
                                hipStream_t s, float hscale) {
    if (n <= 0) return hipSuccess;
    if ((ns != 2 && ns != 3) || (hscale > 0.0f && ns != 2)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(planes_to_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const __bf16*>(planes), pstride, ns, out, n, hscale);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Split residual VQ (TF/modeling_mimi.py:964-1126) on fp32 MFMA, bit-exact with the reference:
//   dist = sqrt(clamp_min( sum_k(-2 r_k) e_k  (+ |r|^2) (+ |e|^2), 0 ))
// is torch's cdist 'mm' form (torch/_decomp/decompositions.py:691-703), whose CPU matmul is ONE in-order
// FMA chain over k = 0..255, then + |r|^2, then + |e|^2 (verified bitwise in the survey container).
// v_mfma_f32_32x32x2_f32 is an in-order fmaf chain over its two k (k0 then k1), so feeding k = 2t (lane
// half 0) and 2t+1 (half 1) at step t reproduces the chain exactly.  |r|^2 follows torch's
// x.pow(2).sum(-1) order (4 accumulators x 8 lanes, then lanes in order).  argmin keeps the first index.
// One workgroup = 32 frames; its 8 waves split the 2048 codes; levels are chained in LDS.
// ------------------------------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ float torch_sqsum(const float* r) {
    // 4 vector accumulators of 8 lanes over blocks of 8, combined acc0+acc1+acc2+acc3, lanes summed in order
    float tot = 0.f;
    float lanes[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        float a[4] = {0.f, 0.f, 0.f, 0.f};
        for (int blk = 0; blk < D / 8; ++blk) {
            const float v = r[blk * 8 + l];
            a[blk & 3] = a[blk & 3] + v * v;
        }
        lanes[l] = ((a[0] + a[1]) + a[2]) + a[3];
    }
    tot = lanes[0];
#pragma unroll
    for (int l = 1; l < 8; ++l) tot = tot + lanes[l];
    return tot;
}

// Level-parallel form.  One launch per level L over (frame tiles of RVQ_FT) x (code slices of RVQ_CS): every
// workgroup computes the distances of its RVQ_FT frames to its 256 codes (8 waves x 32 codes, RVQ_FT / 32
// MFMA tiles per wave) and writes the slice's (min distance, first index) per frame.  The NEXT launch's prologue
// merges the slices of level L-1 (lexicographic (d, idx): the global first-index argmin), writes those codes
// (slice-0 workgroups), and forms r_L = r_{L-1} - embed_{L-1}[idx] (bitwise the same in every slice's
// workgroup); a last launch merges level K-1.  8 + 1 launches of F/64 x 8 = 504 workgroups (B = 32 x 10 s)
// instead of one launch of F/32 = 125 workgroups that left half the CUs idle.  Distances: identical arithmetic and k order to the
// reference chain above (|r|^2 from the (-2r)^2 image: scaling by 4 is exact).
constexpr int RVQ_FT = 64;  // 64 frames: 68 KiB of LDS, two workgroups per CU overlap prologue / MFMA / argmin
constexpr int RVQ_CS = 256;

size_t rvq_work_bytes(long long frames) {
    const long long fp = (frames + RVQ_FT - 1) / RVQ_FT * RVQ_FT;
    const int nsl = 32;  // the most code slices any rvq_level_h16_kernel form may use (NWV = 2: 64-code slices)
    return (size_t)(2 * fp * 256 * 4 + 2 * 3 * fp * nsl * 4);
}

// work layout: res[2][Fp][D] | pd[3][Fp][nsl] | pi[3][Fp][nsl]; residual parity = level & 1, partial-argmin slot =
// rvq_slot (selected by arithmetic, not by indexing a pointer array, which would live in scratch)
struct RvqWork {
    float* base;
    long long fp;
    int D, nsl;
    __device__ float* res(int par) const { return base + (par ? fp * D : 0); }
    __device__ float* pd(int slot) const { return base + 2 * fp * D + slot * fp * nsl; }
    __device__ int* pi(int slot) const {
        return reinterpret_cast<int*>(base + 2 * fp * D + 3 * fp * nsl) + slot * fp * nsl;
    }
};

// The split quantizer's semantic level (nsem = 1) and first acoustic level both start from the projection, so
// they run as ONE launch (grid.z = 2, rvq_level_h16_kernel); the semantic level's partial argmins then go to a
// third slot that no later level overwrites, and rvq_final_kernel writes code 0 from it.
__device__ __forceinline__ bool rvq_sem_split(const RvqArgs& p) { return p.sem_split != 0; }
__device__ __forceinline__ int rvq_slot(const RvqArgs& p, int L) { return (L == 0 && rvq_sem_split(p)) ? 2 : (L & 1); }

__device__ __forceinline__ RvqWork rvq_work(const RvqArgs& p, int nsl) {
    RvqWork r;
    r.base = reinterpret_cast<float*>(p.work);
    r.fp = (p.frames + RVQ_FT - 1) / RVQ_FT * RVQ_FT;
    r.D = p.D;
    r.nsl = nsl;
    return r;
}

// frame f holds data: inside the frames and, for a ragged batch, inside its item's valid frames
__device__ __forceinline__ bool rvq_valid(const RvqArgs& p, long long f) {
    if (f >= p.frames) return false;
    if (!p.flen) return true;
    const long long bb = f / p.frames_per_item;
    return f - bb * p.frames_per_item < p.flen[bb];
}

__device__ __forceinline__ void rvq_store_code(const RvqArgs& p, int level, long long f, int ix) {
    int32_t* codes = io_pointer(p.codes_ref, p.codes);
    if (p.frames_per_item > 0) {
        const long long bb = f / p.frames_per_item, t = f % p.frames_per_item;
        codes[(bb * p.levels + level) * p.frames_per_item + t] = ix;
    } else {
        codes[(long long)level * p.frames + f] = ix;
    }
}

// merged argmin of level L over its slices (ties -> lower index; an all-NaN row keeps index 0).  All NSL
// (distance, index) pairs are loaded as 16-B vectors before the first compare: a runtime-length loop waited out
// one memory round trip per slice, on the critical path of every level's prologue.
template <int NSL>
__device__ __forceinline__ int rvq_merge(const RvqWork& w, int slot, long long f, int ncodes) {
    static_assert(NSL % 4 == 0, "slices in 16-B groups");
    const float* pd = w.pd(slot) + f * NSL;  // 16-B aligned: the work layout's offsets are multiples of 4 floats
    const int* pi = w.pi(slot) + f * NSL;
    float dv[NSL];
    int iv[NSL];
#pragma unroll
    for (int q = 0; q < NSL; q += 4) {
        const float4 a = *reinterpret_cast<const float4*>(pd + q);
        const int4 b = *reinterpret_cast<const int4*>(pi + q);
        dv[q] = a.x; dv[q + 1] = a.y; dv[q + 2] = a.z; dv[q + 3] = a.w;
        iv[q] = b.x; iv[q + 1] = b.y; iv[q + 2] = b.z; iv[q + 3] = b.w;
    }
    float d = dv[0];
    int ix = iv[0];
#pragma unroll
    for (int q = 1; q < NSL; ++q)
        if (dv[q] < d || (dv[q] == d && iv[q] < ix)) { d = dv[q]; ix = iv[q]; }
    return (ix < 0 || ix >= ncodes) ? 0 : ix;
}

// FT: frames per workgroup -- RVQ_FT, or 32 for small batches (more workgroups; the work layout stays padded
// to RVQ_FT, and each (frame, code) distance is the same fmaf chain either way)
template <int D, int FT>
__global__ __launch_bounds__(512) void rvq_level_kernel(RvqArgs p, int L) {
    constexpr int LDH = D / 2 + 4;
    static_assert(FT % 32 == 0 && RVQ_FT % FT == 0, "frame tile");
    constexpr int NSL = 2048 / RVQ_CS;
    __shared__ __attribute__((aligned(16))) float img[2][FT][LDH];  // -2 r, split by k parity
    __shared__ float xn[FT];
    __shared__ int prev[FT];
    __shared__ float redd[8][FT];
    __shared__ int redi[8][FT];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
    const long long f0 = (long long)blockIdx.x * FT;
    const int slice = blockIdx.y;
    const RvqWork w = rvq_work(p, NSL);

    // ---- prologue: finish level L-1, form r_L
    if (L >= 1 && tid < FT) {
        const long long f = f0 + tid;
        int ix = 0;
        if (f < p.frames) {
            ix = rvq_merge<NSL>(w, rvq_slot(p, L - 1), f, p.ncodes);
            if (slice == 0) rvq_store_code(p, L - 1, f, ix);
        }
        prev[tid] = ix;
    }
    __syncthreads();
    const bool fresh = (L == 0 || L == p.nsem);  // semantic start / acoustic start: r = projection
    const int coff = (L < p.nsem) ? 0 : D;
    const float* rows_prev = p.cb_rows + (long long)(L - 1) * p.ncodes * D;
    const float* rin = w.res((L + 1) & 1);  // residual entering level L-1
    float* rout = w.res(L & 1);
    // float4 chunks, 16 per thread, loads batched 8 at a time (a serial load->use loop here is latency-bound)
#pragma unroll 8
    for (int idx = tid; idx < FT * D / 4; idx += 512) {
        const int i = idx / (D / 4), k = (idx % (D / 4)) * 4;
        const long long f = f0 + i;
        f32x4 r = {0.f, 0.f, 0.f, 0.f};
        if (rvq_valid(p, f)) {
            if (fresh) {
                r = *reinterpret_cast<const f32x4*>(p.proj + f * (2 * D) + coff + k);
            } else {
                const f32x4 a = *reinterpret_cast<const f32x4*>(rin + f * D + k);
                const f32x4 e = *reinterpret_cast<const f32x4*>(rows_prev + (long long)prev[i] * D + k);
                r = a - e;
            }
            if (slice == 0) *reinterpret_cast<f32x4*>(rout + f * D + k) = r;
        }
        img[0][i][k >> 1] = -2.0f * r.x;
        img[1][i][k >> 1] = -2.0f * r.y;
        img[0][i][(k >> 1) + 1] = -2.0f * r.z;
        img[1][i][(k >> 1) + 1] = -2.0f * r.w;
    }
    __syncthreads();
    // torch x.pow(2).sum(-1) order (8 lanes x 4 accumulators, accumulators combined, lanes summed in order) on
    // (-2r)^2 = 4 r^2, then * 0.25 (power-of-two scaling: exact); 8 threads per frame, one per lane
    for (int fi = tid >> 3; fi < FT; fi += 64) {
        const int l = tid & 7;
        float a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
        for (int blk = 0; blk < D / 8; ++blk) {
            const int k = blk * 8 + l;
            const float v = img[k & 1][fi][k >> 1];
            a[blk & 3] = a[blk & 3] + v * v;
        }
        const float part = ((a[0] + a[1]) + a[2]) + a[3];
        float tot = __shfl(part, (lane & ~7));
#pragma unroll
        for (int q = 1; q < 8; ++q) tot = tot + __shfl(part, (lane & ~7) + q);
        if (l == 0) xn[fi] = tot * 0.25f;
    }
    __syncthreads();

    // ---- distances of FT frames x this wave's 32 codes (8 waves: 2 per SIMD)
    const int code0 = slice * RVQ_CS + wave * 32;
    const int nu = D / 8;
    const float* cbf = p.cb_frag + (long long)L * (p.ncodes / 32) * nu * 256;
    constexpr int RT = FT / 32;  // row tiles per wave
    f32x16 acc[RT];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.0f;
    const f32x4* bp = reinterpret_cast<const f32x4*>(cbf + (long long)(code0 / 32) * nu * 256) + lane;
    // codebook fragments 4 k-quads ahead (an L2 hit takes longer than one quad's 8 MFMAs)
    constexpr int PF = 4;
    f32x4 bq[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) bq[q] = bp[q * 64];
#pragma unroll PF
    for (int u = 0; u < nu; ++u) {
        const f32x4 bv = bq[u % PF];
        if (u + PF < nu) bq[u % PF] = bp[(u + PF) * 64];
        f32x4 av[RT];
#pragma unroll
        for (int i = 0; i < RT; ++i) av[i] = *reinterpret_cast<const f32x4*>(&img[h][i * 32 + (lane & 31)][u * 4]);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < RT; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][s], bv[s], acc[i], 0, 0, 0);
    }
    const float yn = p.cb_norm[(long long)L * p.ncodes + code0 + (lane & 31)];
#pragma unroll
    for (int i = 0; i < RT; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            float d2 = acc[i][r] + xn[row];
            d2 = d2 + yn;
            float d = __builtin_sqrtf(fmaxf(d2, 0.0f));
            int ix = code0 + (lane & 31);
#pragma unroll
            for (int o = 16; o >= 1; o >>= 1) {
                const float od = __shfl_xor(d, o);
                const int oi = __shfl_xor(ix, o);
                if (od < d || (od == d && oi < ix)) { d = od; ix = oi; }
            }
            if ((lane & 31) == 0) {
                redd[wave][row] = d;
                redi[wave][row] = ix;
            }
        }
    }
    __syncthreads();
    if (tid < FT && f0 + tid < p.frames) {
        float d = redd[0][tid];
        int ix = redi[0][tid];
        for (int q = 1; q < 8; ++q) {
            const float od = redd[q][tid];
            const int oi = redi[q][tid];
            if (od < d || (od == d && oi < ix)) { d = od; ix = oi; }
        }
        const long long f = f0 + tid;
        w.pd(rvq_slot(p, L))[f * NSL + slice] = d;
        w.pi(rvq_slot(p, L))[f * NSL + slice] = ix;
    }
}

template <int NSL = 2048 / RVQ_CS>
__global__ __launch_bounds__(256) void rvq_final_kernel(RvqArgs p, int L) {
    const long long f = (long long)blockIdx.x * 256 + threadIdx.x;
    if (f >= p.frames) return;
    const RvqWork w = rvq_work(p, NSL);
    rvq_store_code(p, L, f, rvq_merge<NSL>(w, rvq_slot(p, L), f, p.ncodes));
    if (rvq_sem_split(p) && L > 0) rvq_store_code(p, 0, f, rvq_merge<NSL>(w, rvq_slot(p, 0), f, p.ncodes));
}

// Approximate-then-exact form (default).  The distances above are exact only for the code that wins: per frame
// and code slice, an approximate -2 r.e on the fp16 matrix cores (r and the codebook as 2 fp16 planes each, 3
// products, v_mfma_f32_32x32x16_f16: 1/5 of the fp32-MFMA time) selects the codes whose approximate squared
// distance lies within a window of the slice's approximate minimum, and only those are re-scored with the
// reference's exact chain (the fmaf chain over k = 0..255, + |r|^2, + |e|^2, clamp, sqrt -- the same operations
// as rvq_level_kernel, so the same bits).  The window is rigorous: both the fp32 chain and the fp16-plane sum
// lie within gamma_256 * 2|r||e| + O(2^-21 |r||e|) of the true dot product, i.e. within 2^-14 |r| |e| of each
// other; the window is 2 x 2^-12 (|r| + max|e|)^2 plus a slack for the final adds and the sqrt rounding, so
// the slice's exact argmin (first index on ties) is always a candidate.  Typical: 1.0-1.1 candidates per frame
// and slice (measured on the golden embeddings with a 4x narrower window).  If a workgroup's candidates
// overflow the LDS list (degenerate codebooks, e.g. all-equal entries), it scores every code exactly.
// Per level one launch of (frames / 32) x 8 slices: each level's work is spread over ~1000 workgroups (a
// single launch chaining all levels per 32-frame workgroup measured 25 % slower: too few, too serial).
constexpr int RVQ_CAND = 2048;

// 32 frames per workgroup (64-frame tiles, which halve the per-CU codebook stream, were slower: 1 workgroup per CU,
// profiles/r2d_rvq_ft64.log).  PF: codebook k-steps in flight per wave (4: two workgroups per CU; 16 = all of them, for small batches whose few
// workgroups wait on L2 / Infinity-Cache latency); EX: float4 of a code row in flight per exact re-score round
// CW: codes per wave (32, or 64 as two 32-code MFMA tiles): a slice of 8 CW codes, NSL = 2048 / (8 CW) slices.  The
// large-batch form takes 64 (4 slices: 500 workgroups at B = 32 x 10 s -- one round of two per CU -- instead of 1000
// in two rounds, each round paying the whole merge / residual / |r|^2 / plane prologue chain again).
// NWV: waves per workgroup (8; 2 and 4 were timed for small grids, not kept: launch_rvq)
// FT: frames per workgroup (32, or 64: a workgroup streams its codebook slice once for twice the frames -- half the
// L2 -> CU codebook bytes per level).  P1 (round 4): the approximate distance is ONE fp16 product (hi planes of r and
// of the codebook, v_mfma_f32_32x32x16_f16) instead of three, with the window widened to that product's rigorous
// error bound (below): a third of the MFMAs and half the codebook bytes; the exact re-score decides, so the codes are
// the same bits.
// |r|^2 in torch's order (x.pow(2).sum(-1): 8 lanes x 4 accumulators, each accumulator over blocks blk = j, j + 4, ..,
// the 4 combined as ((a0 + a1) + a2) + a3, the 8 lanes summed in order) and the fp16 scale of max |r|, from the -2 r
// image (4 r^2 summed, then * 0.25: power-of-two scalings, exact).  32 threads per frame, one accumulator chain of 8
// each (round 4; 16 threads per frame with chains of 32 before: the same sums in the same order).  NT >= 32 threads.
template <int FT, int D, int LDH, int NT>
__device__ __forceinline__ void rvq_norms(const float (*img)[FT][LDH], float* xn, float* rus, float* win, int tid) {
    static_assert(D == 256, "8 lanes x 4 accumulators x 8 blocks");
    const int lane = tid & 63, sub = tid & 31, l = sub & 7, j = sub >> 3, gb = lane & 32;
    for (int fi = tid >> 5; fi < FT; fi += NT / 32) {
        float a = 0.0f, mx = 0.0f;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int k = 8 * (j + 4 * t) + l;
            const float v = img[k & 1][fi][k >> 1];
            a = a + v * v;
            mx = fmaxf(mx, fabsf(v));
        }
        const float part = ((__shfl(a, gb + l) + __shfl(a, gb + l + 8)) + __shfl(a, gb + l + 16)) + __shfl(a, gb + l + 24);
        float tot = __shfl(part, gb);
#pragma unroll
        for (int q = 1; q < 8; ++q) tot = tot + __shfl(part, gb + q);
#pragma unroll
        for (int o = 16; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
        if (sub == 0) {
            xn[fi] = tot * 0.25f;
            mx *= 0.5f;  // max |r|
            const float rs = mx > 0.0f && mx < INFINITY ? ldexpf(1.0f, 13 - ilogbf(mx)) : 1.0f;
            rus[fi] = 1.0f / rs;
            win[fi] = rs;  // (the scale, until the window replaces it)
        }
    }
}

// Exact re-score of the candidates (the reference's fp32 chain: fmaf over k = 0..255 in order of -2 r_k e_k, + |r|^2,
// + |e|^2, clamp, sqrt; (distance, code) minimum per frame by a 64-bit LDS atomicMin), one thread per candidate with EX
// float4 of its code row in flight, or every code of the slice when the list overflowed (degenerate codebooks).  (Staging
// the rows in LDS 32 at a time -- one memory round trip per 32 candidates -- was slower: the chains then wait on an LDS
// read per 4 FMAs, rvq 0.21 -> 0.36 ms per B = 32 step, 0.50 -> 0.58 ms at batch 1 K = 32.)
template <int FT, int D, int LDH, int NT, int SLC, int EX>
__device__ __forceinline__ void rvq_exact(const float (*img)[FT][LDH], const float* xn, const unsigned* cand,
                                          unsigned nc, unsigned long long* best, const float* cbr, const float* cnorm,
                                          int cbase, long long f0, long long frames, int tid) {
    const bool all = nc > RVQ_CAND;
    const unsigned total = all ? FT * SLC : nc;
    for (unsigned i = tid; i < total; i += NT) {
        const int row = all ? (int)(i % FT) : (int)(cand[i] >> 16);
        const int c = cbase + (all ? (int)(i / FT) : (int)(cand[i] & 0xffff));
        if (f0 + row >= frames) continue;
        const f32x4* e = reinterpret_cast<const f32x4*>(cbr + (long long)c * D);
        float a = 0.0f;
        // (not unrolled: unrolled, hipcc hoisted every round's loads -- the whole 1-KB row in 256 VGPRs -- and spilled)
#pragma unroll 1
        for (int k0 = 0; k0 < D / 4; k0 += EX) {  // EX float4 of the code row in flight, then the in-order chain
            f32x4 ev[EX];
#pragma unroll
            for (int j = 0; j < EX; ++j) ev[j] = e[k0 + j];
#pragma unroll
            for (int j = 0; j < EX; ++j) {
                const int k4 = k0 + j;
                a = __builtin_fmaf(img[0][row][2 * k4], ev[j].x, a);
                a = __builtin_fmaf(img[1][row][2 * k4], ev[j].y, a);
                a = __builtin_fmaf(img[0][row][2 * k4 + 1], ev[j].z, a);
                a = __builtin_fmaf(img[1][row][2 * k4 + 1], ev[j].w, a);
            }
        }
        float d2 = a + xn[row];
        d2 = d2 + cnorm[c];
        const float d = __builtin_sqrtf(fmaxf(d2, 0.0f));
        atomicMin(&best[row], ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)c);
    }
}

// rvq_exact with every candidate's code row staged in LDS first (the persistent chain, whose workgroup has the LDS):
// wave w issues the rows of candidates w, w + 8, .. as LDS-DMA (one 1-KB row per wave-instruction, all in flight at
// once), so the exact chains read LDS instead of waiting out D / 4 / EX global round trips each.  Same chain, same
// order, same values as rvq_exact (|e|^2 from the slice's ynl copy of cnorm).  nc <= NSTG.
template <int FT, int D, int LDH, int NT, int NSTG>
__device__ __forceinline__ void rvq_exact_staged(const float (*img)[FT][LDH], const float* xn, const unsigned* cand,
                                                 unsigned nc, unsigned long long* best, const float* cbr,
                                                 const float* ynl, int cbase, long long f0, long long frames, int tid,
                                                 float* rowbuf) {
    [[maybe_unused]] constexpr int NWV = NT / 64, RS = D + 4;  // (row stride: + 16 B, conflict-free b128 reads)
    static_assert(D == 256, "one 16-B piece per lane per row");
    [[maybe_unused]] const int lane = tid & 63, wave = tid >> 6;
#if defined(__HIP_DEVICE_COMPILE__)
    // LDS-DMA: no registers held; candidate i's 1-KB row lands at rowbuf + i RS (lane l: floats 4 l .. 4 l + 3)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(cbr), (short)0, 0x7fffffff,
                                                                         0x00020000);
    for (unsigned i = wave; i < nc; i += NWV) {  // (wave-uniform)
        const int c = cbase + (int)(cand[i] & 0xffff);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(rowbuf + i * RS), 16,
                                                 (c * D + 4 * lane) * 4, 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    __syncthreads();
    for (unsigned i = tid; i < nc; i += NT) {
        const int row = (int)(cand[i] >> 16), cl = (int)(cand[i] & 0xffff);
        if (f0 + row >= frames) continue;
        const float* e = rowbuf + i * RS;
        float a = 0.0f;
#pragma unroll 4
        for (int k4 = 0; k4 < D / 4; ++k4) {
            const f32x4 ev = *reinterpret_cast<const f32x4*>(e + 4 * k4);
            a = __builtin_fmaf(img[0][row][2 * k4], ev.x, a);
            a = __builtin_fmaf(img[1][row][2 * k4], ev.y, a);
            a = __builtin_fmaf(img[0][row][2 * k4 + 1], ev.z, a);
            a = __builtin_fmaf(img[1][row][2 * k4 + 1], ev.w, a);
        }
        float d2 = a + xn[row];
        d2 = d2 + ynl[cl];
        const float d = __builtin_sqrtf(fmaxf(d2, 0.0f));
        atomicMin(&best[row], ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)(cbase + cl));
    }
}

template <int D, int PF = 4, int EX = 16, bool RG = false, int CW = 32, int NWV = 8, int FT = 32, bool P1 = false>
// (HIP's second launch bound is waves per SIMD: 4 = two 8-wave workgroups per CU, i.e. <= 128 VGPRs)
__global__ __launch_bounds__(64 * NWV, (PF <= 4 && FT == 32) ? 4 : 2) void rvq_level_h16_kernel(RvqArgs p, int L0) {
    constexpr int NT = 64 * NWV;          // threads
    constexpr int TNC = CW / 32;          // 32-code MFMA tiles per wave
    constexpr int RT = FT / 32;           // 32-frame MFMA row tiles
    constexpr int SLC = NWV * CW;         // codes per slice
    constexpr int NSL = 2048 / SLC;       // slices
    constexpr int NPL = P1 ? 1 : 2;       // fp16 planes of r and of the codebook the approximation reads
    static_assert(NSL <= 32 && NSL % 4 == 0, "slices: rvq_work_bytes, rvq_merge");
    static_assert(FT == 32 || FT == 64, "frame tile (RVQ_FT pads the work layout to 64)");
    // RG (a ragged batch: p.flen): a workgroup none of whose frames is valid has nothing to do -- no later level
    // reads what it would write (only valid frames' residuals and partial argmins are ever read)
    // p.xcd_group (large grids, round 4): a 1-D grid whose workgroup b runs slice (b >> 3) % NSL of frame tile
    // (b & 7) + 8 ((b >> 3) / NSL) -- the slices of a frame tile land on one XCD (workgroups are dealt round-robin over
    // the 8 XCDs; speed only), so its L2 serves the residual and code-row reads the NSL slices share
    unsigned ftile = blockIdx.x, slc = blockIdx.y;
    if (p.xcd_group) {
        const unsigned q = blockIdx.x >> 3;
        slc = q % NSL;
        ftile = (blockIdx.x & 7) + 8 * (q / NSL);
        if ((long long)ftile * FT >= p.frames) return;  // (padding of the grid to whole groups of 8 frame tiles)
    }
    if constexpr (RG) {
        if (!__syncthreads_or((int)threadIdx.x < FT && rvq_valid(p, (long long)ftile * FT + threadIdx.x))) return;
    }
    const int L = L0 + (int)blockIdx.z;  // (grid.z = 2: the semantic and first acoustic levels together)
    constexpr int LDH = D / 2 + 4;
    constexpr int RLD = D + 8;  // fp16 plane rows: 528 B = 132 dwords (conflict-free b128 fragment reads)
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    __shared__ __attribute__((aligned(16))) float img[2][FT][LDH];  // -2 r, split by k parity (exact chain)
    __shared__ __attribute__((aligned(16))) _Float16 rpl[NPL][FT][RLD];  // fp16 planes of r * rs
    __shared__ float xn[FT], rus[FT], win[FT], smin[FT];
    __shared__ int prev[FT];
    __shared__ float redd[NWV][FT];
    __shared__ unsigned cand[RVQ_CAND];
    __shared__ unsigned ncand;
    __shared__ unsigned long long best[FT];
    __shared__ float ynl[SLC];  // |e|^2 of the slice's codes
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
    const long long f0 = (long long)ftile * FT;
    const int slice = (int)slc;
    const RvqWork w = rvq_work(p, NSL);
    // the level's scalars and this lane's code norms, loaded here so the barriers below wait for them (used after the
    // MFMA loop, where a load is a whole exposed memory round trip)
    const int code0 = slice * SLC + wave * CW;
    const float cus = p.cb_unscale[L], emax_l = p.cb_emax[L];
    for (int c = tid; c < SLC; c += NT) ynl[c] = p.cb_norm[(long long)L * p.ncodes + slice * SLC + c];

    // ---- prologue (as rvq_level_kernel): finish level L-1, form r_L
    // (the first acoustic level of a combined launch, blockIdx.z = 1, does not merge the semantic level running beside
    // it: rvq_final_kernel does.  The test sits inside the merge branch: on the outer branch it cost 28 VGPRs)
    if (L >= 1 && tid < FT) {
        const long long f = f0 + tid;
        int ix = 0;
        if (f < p.frames && blockIdx.z == 0) {
            ix = rvq_merge<NSL>(w, rvq_slot(p, L - 1), f, p.ncodes);
            if (slice == 0) rvq_store_code(p, L - 1, f, ix);
        }
        prev[tid] = ix;
    }
    if (tid < FT) best[tid] = ~0ull;
    if (tid == 0) ncand = 0;
    __syncthreads();
    const bool fresh = (L == 0 || L == p.nsem);
    const int coff = (L < p.nsem) ? 0 : D;
    const float* rows_prev = p.cb_rows + (long long)(L - 1) * p.ncodes * D;
    const float* rin = w.res((L + 1) & 1);
    float* rout = w.res(L & 1);
#pragma unroll 4
    for (int idx = tid; idx < FT * D / 4; idx += NT) {
        const int i = idx / (D / 4), k = (idx % (D / 4)) * 4;
        const long long f = f0 + i;
        f32x4 r = {0.f, 0.f, 0.f, 0.f};
        if (rvq_valid(p, f)) {
            if (fresh) {
                r = *reinterpret_cast<const f32x4*>(p.proj + f * (2 * D) + coff + k);
            } else {
                const f32x4 a = *reinterpret_cast<const f32x4*>(rin + f * D + k);
                const f32x4 e = *reinterpret_cast<const f32x4*>(rows_prev + (long long)prev[i] * D + k);
                r = a - e;
            }
            if (slice == 0) *reinterpret_cast<f32x4*>(rout + f * D + k) = r;
        }
        img[0][i][k >> 1] = -2.0f * r.x;
        img[1][i][k >> 1] = -2.0f * r.y;
        img[0][i][(k >> 1) + 1] = -2.0f * r.z;
        img[1][i][(k >> 1) + 1] = -2.0f * r.w;
    }
    __syncthreads();
    rvq_norms<FT, D, LDH, NT>(img, xn, rus, win, tid);
    __syncthreads();
    // fp16 planes of r * rs (P1: the hi plane only)
    for (int idx = tid; idx < FT * D / 2; idx += NT) {
        const int i = idx / (D / 2), k = (idx % (D / 2)) * 2;
        const float rs = -0.5f * win[i];
        const float t0 = img[0][i][k >> 1] * rs, t1 = img[1][i][k >> 1] * rs;
        const _Float16 a0 = (_Float16)t0, a1 = (_Float16)t1;
        rpl[0][i][k] = a0;
        rpl[0][i][k + 1] = a1;
        if constexpr (!P1) {
            rpl[NPL - 1][i][k] = (_Float16)(t0 - (float)a0);
            rpl[NPL - 1][i][k + 1] = (_Float16)(t1 - (float)a1);
        }
    }
    __syncthreads();

    // ---- approximate r.e for FT frames x this wave's CW codes; the wave's codebook planes stream from L2 with PF
    // k-steps in flight
    const h8* bp = reinterpret_cast<const h8*>(p.cb_h16) +
                   ((long long)L * (p.ncodes / 32) + code0 / 32) * (D / 16) * 2 * 64 + lane;
    constexpr int TST = (D / 16) * 2 * 64;  // h8 per 32-code block of the fragment image
    f32x16 acc[RT][TNC];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int t = 0; t < TNC; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][t][r] = 0.0f;
    h8 bq[PF][TNC][NPL];
#pragma unroll
    for (int q = 0; q < PF; ++q)
#pragma unroll
        for (int t = 0; t < TNC; ++t)
#pragma unroll
            for (int pl = 0; pl < NPL; ++pl) bq[q][t][pl] = bp[t * TST + q * 128 + pl * 64];
    auto kstep = [&](int ks) {
        const int cur = ks % PF;
        h8 bb[TNC][NPL];
#pragma unroll
        for (int t = 0; t < TNC; ++t)
#pragma unroll
            for (int pl = 0; pl < NPL; ++pl) bb[t][pl] = bq[cur][t][pl];
        if (ks + PF < D / 16) {
#pragma unroll
            for (int t = 0; t < TNC; ++t)
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl) bq[cur][t][pl] = bp[t * TST + (ks + PF) * 128 + pl * 64];
        }
#pragma unroll
        for (int i = 0; i < RT; ++i) {
            const h8 a0 = *reinterpret_cast<const h8*>(&rpl[0][i * 32 + (lane & 31)][ks * 16 + 8 * h]);
            // transposed: the codebook fragment is the A operand (rows = codes), r the B operand (columns = frames), so
            // a lane holds ONE frame and 16 codes per tile -- the minimum over codes is in-register, not 5 shuffles per
            // frame row (a fragment serves as either operand: lane (j, h) holds row / column j, k = 8 h .. 8 h + 7)
            if constexpr (P1) {
#pragma unroll
                for (int t = 0; t < TNC; ++t)
                    acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bb[t][0], a0, acc[i][t], 0, 0, 0);
            } else {
                const h8 a1 = *reinterpret_cast<const h8*>(&rpl[NPL - 1][i * 32 + (lane & 31)][ks * 16 + 8 * h]);
#pragma unroll
                for (int t = 0; t < TNC; ++t) {
                    acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bb[t][0], a1, acc[i][t], 0, 0, 0);
                    acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bb[t][NPL - 1], a0, acc[i][t], 0, 0, 0);
                    acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bb[t][0], a0, acc[i][t], 0, 0, 0);
                }
            }
        }
        // P1 with PF k-steps in flight: keep the scheduler from hoisting later k-steps' codebook loads above these
        // MFMAs (with one product per k-step it did, holding every k-step's fragments live: 128-256 VGPRs, spills)
        if constexpr (P1 && PF < 16) __builtin_amdgcn_sched_barrier(0);
    };
    // (a template-dependent `#pragma unroll PF` is not honoured by hipcc -- the loop is then fully unrolled and
    // the prefetch loads sunk to their uses -- so the depths spell their unroll factor out)
    if constexpr (PF == 4) {
#pragma unroll 4
        for (int ks = 0; ks < D / 16; ++ks) kstep(ks);
    } else if constexpr (PF == 2) {
#pragma unroll 2
        for (int ks = 0; ks < D / 16; ++ks) kstep(ks);
    } else {
        __builtin_amdgcn_sched_barrier(0);  // all PF k-steps' loads issued before the first MFMA
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) kstep(ks);
    }
    // approximate d^2 (transposed layout: frame i * 32 + (lane & 31), code 32 t + (r & 3) + 8 (r >> 2) + 4 h of the
    // wave's CW) and each frame's minimum over the wave's codes
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        const int fr = i * 32 + (lane & 31);
        const float ur = rus[fr] * cus, xr = xn[fr];
        float m = INFINITY;
#pragma unroll
        for (int t = 0; t < TNC; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float yn = ynl[wave * CW + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h];
                acc[i][t][r] = (-2.0f * (acc[i][t][r] * ur) + xr) + yn;
                m = fminf(m, acc[i][t][r]);
            }
        m = fminf(m, __shfl_xor(m, 32));
        if (h == 0) redd[wave][fr] = m;
    }
    __syncthreads();
    if (tid < FT) {
        float m = redd[0][tid];
#pragma unroll
        for (int q = 1; q < NWV; ++q) m = fminf(m, redd[q][tid]);
        smin[tid] = m;
        const float emax = emax_l;
        const float rnorm = __builtin_sqrtf(fmaxf(xn[tid], 0.0f));
        const float rn = rnorm + emax;
        if constexpr (P1) {
            // one fp16 product: per element |r_k e_k - rh_k eh_k| <= (2 2^-11 + 2^-22) |r_k e_k| (fp16 unit roundoff; a
            // subnormal rounding adds at most 2^-25 / scale per element, far below), so the approximate dot product is
            // within (2^-10 + 2^-22) sum |r_k e_k| <= 1.0001 2^-10 |r| |e| of the true one, the MFMA's fp32 accumulation
            // within 2^-19 |r| |e| more and the reference's fp32 chain within gamma_256 < 2^-15.9 |r| |e|.  A d^2 moves
            // by twice the dot-product error: both the candidate and the slice minimum by <= 1.04 2^-9 |r| emax, so the
            // exact argmin lies within 1.04 2^-8 |r| emax of the approximate minimum; plus the final adds' rounding
            // (<= 2^-22 (|r| + emax)^2 each) and the sqrt / compare slack.
            win[tid] = ldexpf(1.06f * rnorm * emax, -8) + ldexpf(rn * rn, -18) + ldexpf(fabsf(m), -20) + 1e-30f;
        } else {
            win[tid] = ldexpf(rn * rn, -11) + ldexpf(fabsf(m), -20) + 1e-30f;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        const int fr = i * 32 + (lane & 31);
        const float lim = smin[fr] + win[fr];
        const bool fin = f0 + fr < p.frames;
#pragma unroll
        for (int t = 0; t < TNC; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                // NaN distances (a non-finite residual) are candidates too: the exact path decides
                if (!(acc[i][t][r] > lim) && fin) {
                    const unsigned slot = atomicAdd(&ncand, 1u);
                    if (slot < RVQ_CAND)
                        cand[slot] = ((unsigned)fr << 16) | (unsigned)(wave * CW + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h);
                }
            }
    }
    __syncthreads();
    // ---- exact re-scoring (rvq_exact): the candidates, or every code of the slice when the list overflowed
    rvq_exact<FT, D, LDH, NT, SLC, EX>(img, xn, cand, ncand, best, p.cb_rows + (long long)L * p.ncodes * D,
                                       p.cb_norm + (long long)L * p.ncodes, slice * SLC, f0, p.frames, tid);
    __syncthreads();
    if (tid < FT && f0 + tid < p.frames) {
        const unsigned long long b = best[tid];
        const long long f = f0 + tid;
        w.pd(rvq_slot(p, L))[f * NSL + slice] = __uint_as_float((unsigned)(b >> 32));
        w.pi(rvq_slot(p, L))[f * NSL + slice] = (int)(b & 0xffffffffu);
    }
}

// ---- Persistent all-levels RVQ for small grids (round 4: the per-utterance callers at K = 32) ----
// rvq_level_h16_kernel runs one launch per level; at batch 1 a level is a chain of dependent memory round trips (merge
// of the slices' minima, residual and code-row gathers, the codebook stream, the exact re-score) plus a launch: 17 us
// per level, 0.53 of a 1.51 ms K = 32 encode.  Here one launch runs every level.  Grid (frame tiles, 8 slices, chains):
// chain 0 the acoustic levels [nsem, K), chain 1 the semantic levels [0, nsem).  A workgroup keeps its 32 frames'
// residual in LDS across levels (as -2 r, the image the exact chain reads: r = -0.5 img and -2 (r - e) are exact) and
// per level scores its 256-code slice with rvq_level_h16_kernel<..., P1>'s arithmetic (same approximate window, same
// exact chain and (distance, code) minimum), publishes its 32 minima as tagged 8-byte granules (the data is the flag:
// MI355X_MICROARCH.md / cdna_hip_programming.md Guideline 16 R2, tag = level + 1, two parity slots zeroed before the
// launch), sweeps the granules of the frame tile's other 7 slices, merges the 8 slices in slice order with
// rvq_merge's rule, stores the codes (slice 0) and subtracts the winning code rows.  The next level's codebook
// fragments are loaded before the sweep, so they fly under it.  Same codes as the per-level launches.
// Every workgroup of a launch must be resident at once: the host takes this kernel only when the occupancy query admits
// the whole grid (<= 128 workgroups, 2 per CU), and every spin is bounded.  A sweep that gives up (other work -- another
// process's kernels -- kept a peer off the CUs for the whole budget) never merges what it has: the workgroup raises the
// launch's flag word (the 16 bytes in front of the granules, zeroed by the same memset node) and leaves, every other
// workgroup leaves at its next sweep once it sees the flag, and the host, which reads the flag back behind the encode,
// re-runs the encode without the chain (engine.cpp encode_wait).  So a give-up costs time, never codes.
constexpr int RVQC_MAX_WG = 128;
#ifndef MIMI_RVQC_XCD
#define MIMI_RVQC_XCD 1  // (A/B knob) 1: a group's 8 slice workgroups on one XCD (1-D grid); 0: the 3-D grid
#endif
constexpr int RVQC_SPIN = 1 << 20;
constexpr int RVQC_HDR = 2;  // u64 words in front of the granules: [0] the give-up flag (u32), [1] padding
constexpr int RVQC_NSTG = 64;  // candidates whose code rows the exact re-score stages in LDS (more: global reads)

__device__ __forceinline__ unsigned long long rvqc_granule(unsigned epoch, unsigned long long best) {
    // best = (distance bits << 32) | code (code 0xffffffff: none): tag 16 bits | code 16 bits | distance 32 bits
    return ((unsigned long long)epoch << 48) | ((best & 0xffffull) << 32) | (best >> 32);
}

#if RVQC_STAMP  // tuning: per-phase cycle sums of wave 0 of workgroup (0, 0, 0), printed at its end
#define RVQC_T0() unsigned long long st_last = __builtin_readcyclecounter(), st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define RVQC_T(i)                                                     \
    do {                                                              \
        const unsigned long long now_ = __builtin_readcyclecounter(); \
        st_acc[i] += now_ - st_last;                                  \
        st_last = now_;                                               \
    } while (0)
#define RVQC_TPRINT()                                                                                              \
    if (ftile == 0 && slice == 0 && chain == 0 && tid == 0)                                                      \
    printf("rvqc levels %d: r2 %llu planes %llu mfma %llu cand %llu exact %llu sweep %llu merge %llu resid %llu\n", \
           Le - Lb, st_acc[0], st_acc[1], st_acc[2], st_acc[3], st_acc[4], st_acc[5], st_acc[6], st_acc[7])
#else
#define RVQC_T0()
#define RVQC_T(i)
#define RVQC_TPRINT()
#endif
template <int D, int EX>
__global__ __launch_bounds__(512, 2) void rvq_chain_h16_kernel(RvqArgs p, unsigned long long* __restrict__ gbase) {
    constexpr int NWV = 8, NT = 512, FT = 32, CW = 32, SLC = NWV * CW, NSL = 2048 / SLC;
    constexpr int LDH = D / 2 + 4, RLD = D + 8, KS = D / 16;
    static_assert(NSL == 8, "8 slices of 256 codes");
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    typedef __attribute__((address_space(1))) unsigned long long gu64;
    __shared__ __attribute__((aligned(16))) float img[2][FT][LDH];  // -2 r (the residual, kept across levels)
    __shared__ __attribute__((aligned(16))) _Float16 rpl[FT][RLD];  // hi fp16 plane of r * rs
    __shared__ float xn[FT], rus[FT], win[FT], smin[FT];
    __shared__ float redd[NWV][FT];
    __shared__ unsigned cand[RVQ_CAND];
    __shared__ unsigned ncand;
    __shared__ unsigned long long best[FT];
    __shared__ int prev[FT];
    __shared__ float gd[NSL][FT];
    __shared__ int gi[NSL][FT];
    __shared__ int tmo;
    __shared__ int codes_l[FT][32];  // this tile's codes per level, stored at the end (slice 0)
    __shared__ float ynl[SLC];       // |e|^2 of the slice's codes at this level
    __shared__ __attribute__((aligned(16))) float rowbuf[RVQC_NSTG * (D + 4)];  // candidates' code rows (exact)
#if MIMI_RVQC_XCD
    // a 1-D grid whose 8 slices of one (frame tile, chain) group share an XCD (workgroups are dealt round-robin over
    // the 8 XCDs): workgroup b runs slice (b >> 3) & 7 of group (b & 7) + 8 (b >> 6), so the winning code rows the
    // residual update gathers were staged by a peer on the same XCD (its L2), as were the group's projection rows.
    // Groups past 2 x ftiles (grid padding to whole 64s) leave at once; they join no sweep.
    const unsigned ftiles = (unsigned)((p.frames + FT - 1) / FT);
    const unsigned group = (blockIdx.x & 7u) + 8u * (blockIdx.x >> 6);
    if (group >= 2u * ftiles) return;  // (workgroup-uniform)
    const int chain = (int)(group / ftiles);
    const unsigned ftile = group % ftiles;
    const int slice = (int)((blockIdx.x >> 3) & 7u);
#else
    const int chain = blockIdx.z;
    const unsigned ftile = blockIdx.x;
    const int slice = blockIdx.y;
    const unsigned ftiles = gridDim.x;
#endif
    const int Lb = chain ? 0 : p.nsem, Le = chain ? min(p.nsem, p.levels) : p.levels;
    if (Lb >= Le) return;  // (workgroup-uniform)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
    const long long f0 = (long long)ftile * FT;
    const int code0 = slice * SLC + wave * CW;
    typedef __attribute__((address_space(1))) unsigned gu32;
    gu32* const flag = (gu32*)gbase;  // the launch's give-up flag
    unsigned long long* const gran = gbase + RVQC_HDR;
    const unsigned spin_limit = p.chain_fault == 1 ? 0u : (unsigned)RVQC_SPIN;
    // granules [parity 2][chain 2][frame tile][slice 8][32 frames]
    auto gslot = [&](int par, int sl) {
        return gran + ((((long long)par * 2 + chain) * ftiles + ftile) * NSL + sl) * FT;
    };
    // the chain's first residual: the projection (as rvq_level_h16_kernel's fresh levels), zero for invalid frames
    const int coff = chain ? 0 : D;
#pragma unroll 4
    for (int idx = tid; idx < FT * D / 4; idx += NT) {
        const int i = idx / (D / 4), k = (idx % (D / 4)) * 4;
        const long long f = f0 + i;
        f32x4 r = {0.f, 0.f, 0.f, 0.f};
        if (rvq_valid(p, f)) r = *reinterpret_cast<const f32x4*>(p.proj + f * (2 * D) + coff + k);
        img[0][i][k >> 1] = -2.0f * r.x;
        img[1][i][k >> 1] = -2.0f * r.y;
        img[0][i][(k >> 1) + 1] = -2.0f * r.z;
        img[1][i][(k >> 1) + 1] = -2.0f * r.w;
    }
    h8 bq[KS];  // this wave's 32 codes' hi-plane fragments of the level's codebook, every k-step
    float yn = 0.0f, cus = 0.0f, emax = 0.0f;  // ... and the norm of the slice's code tid, the level's scalars
    auto load_cb = [&](int L) {
        const h8* bp = reinterpret_cast<const h8*>(p.cb_h16) +
                       ((long long)L * (p.ncodes / 32) + code0 / 32) * KS * 2 * 64 + lane;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) bq[ks] = bp[ks * 128];
        if (tid < SLC) yn = p.cb_norm[(long long)L * p.ncodes + slice * SLC + tid];
        cus = p.cb_unscale[L];
        emax = p.cb_emax[L];
    };
    load_cb(Lb);
    if (tid == 0) tmo = 0;
    RVQC_T0();
    for (int L = Lb; L < Le; ++L) {
        if (tid < FT) best[tid] = ~0ull;
        if (tid == 0) ncand = 0;
        if (tid < SLC) ynl[tid] = yn;
        __syncthreads();  // the residual image is complete
        RVQC_T(7);
        rvq_norms<FT, D, LDH, NT>(img, xn, rus, win, tid);
        __syncthreads();
        RVQC_T(0);
        for (int idx = tid; idx < FT * D / 2; idx += NT) {
            const int i = idx / (D / 2), k = (idx % (D / 2)) * 2;
            const float rs = -0.5f * win[i];
            rpl[i][k] = (_Float16)(img[0][i][k >> 1] * rs);
            rpl[i][k + 1] = (_Float16)(img[1][i][k >> 1] * rs);
        }
        __syncthreads();
        RVQC_T(1);
        // approximate r.e: one fp16 product per k-step (P1)
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const h8 a0 = *reinterpret_cast<const h8*>(&rpl[lane & 31][ks * 16 + 8 * h]);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bq[ks], a0, acc, 0, 0, 0);  // transposed (level kernel)
        }
        {  // lane: frame lane & 31, codes (r & 3) + 8 (r >> 2) + 4 h of the wave's 32
            const int fr = lane & 31;
            const float ur = rus[fr] * cus, xr = xn[fr];
            float m = INFINITY;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[r] = (-2.0f * (acc[r] * ur) + xr) + ynl[wave * CW + (r & 3) + 8 * (r >> 2) + 4 * h];
                m = fminf(m, acc[r]);
            }
            m = fminf(m, __shfl_xor(m, 32));
            if (h == 0) redd[wave][fr] = m;
        }
        __syncthreads();
        RVQC_T(2);
        if (tid < FT) {
            float m = redd[0][tid];
#pragma unroll
            for (int q = 1; q < NWV; ++q) m = fminf(m, redd[q][tid]);
            smin[tid] = m;
            const float rnorm = __builtin_sqrtf(fmaxf(xn[tid], 0.0f));
            const float rn = rnorm + emax;
            // rvq_level_h16_kernel's P1 window (its derivation is there)
            win[tid] = ldexpf(1.06f * rnorm * emax, -8) + ldexpf(rn * rn, -18) + ldexpf(fabsf(m), -20) + 1e-30f;
        }
        __syncthreads();
        {
            const int fr = lane & 31;
            const float lim = smin[fr] + win[fr];
            const bool fin = f0 + fr < p.frames;
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (!(acc[r] > lim) && fin) {
                    const unsigned sl = atomicAdd(&ncand, 1u);
                    if (sl < RVQ_CAND) cand[sl] = ((unsigned)fr << 16) | (unsigned)(wave * CW + (r & 3) + 8 * (r >> 2) + 4 * h);
                }
        }
        __syncthreads();
        RVQC_T(3);
        // exact re-score (the reference's fp32 chain), rvq_exact as in rvq_level_h16_kernel; with the candidates'
        // code rows staged in LDS when they fit (one global round trip instead of D / 4 / EX)
        if (ncand <= RVQC_NSTG)
            rvq_exact_staged<FT, D, LDH, NT, RVQC_NSTG>(img, xn, cand, ncand, best,
                                                        p.cb_rows + (long long)L * p.ncodes * D, ynl, slice * SLC,
                                                        f0, p.frames, tid, rowbuf);
        else
            rvq_exact<FT, D, LDH, NT, SLC, EX>(img, xn, cand, ncand, best, p.cb_rows + (long long)L * p.ncodes * D,
                                               p.cb_norm + (long long)L * p.ncodes, slice * SLC, f0, p.frames, tid);
        __syncthreads();
        RVQC_T(4);
        // publish this slice's 32 minima (one 8-byte agent-scope store each: the granule is its own flag)
        const unsigned epoch = (unsigned)L + 1;
        if (tid < FT)
            __hip_atomic_store((gu64*)(gslot(L & 1, slice) + tid), rvqc_granule(epoch, best[tid]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (L + 1 < Le) load_cb(L + 1);  // the next level's codebook: in flight under the sweep
        // sweep the frame tile's 8 slices (wave 0, 4 granules per lane) until every tag is this level's; give up when
        // the budget runs out or another workgroup already gave up (the flag, polled every 64th pass)
        if (wave == 0) {
            unsigned long long v[4];
            bool fail = p.chain_fault == 2;
            for (unsigned spins = 0; !fail; ++spins) {
                bool ok = true;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int j = lane + 64 * q;
                    v[q] = __hip_atomic_load((gu64*)(gslot(L & 1, j >> 5) + (j & 31)), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
                    ok = ok && (unsigned)(v[q] >> 48) == epoch;
                }
                if (__all(ok)) break;
                if (spins >= spin_limit ||
                    ((spins & 63) == 63 &&
                     __any(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u))) {
                    fail = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (fail) {
                if (lane == 0) {
                    __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    tmo = 1;
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int j = lane + 64 * q;
                    gd[j >> 5][j & 31] = __uint_as_float((unsigned)(v[q] & 0xffffffffu));
                    gi[j >> 5][j & 31] = (int)(short)(unsigned short)((v[q] >> 32) & 0xffffu);
                }
            }
        }
        __syncthreads();
        if (tmo) return;  // (workgroup-uniform: LDS, behind the barrier) nothing of this launch is kept
        RVQC_T(5);
        if (tid < FT) {  // rvq_merge's rule over the slices in order
            float d = gd[0][tid];
            int ix = gi[0][tid];
#pragma unroll
            for (int q = 1; q < NSL; ++q)
                if (gd[q][tid] < d || (gd[q][tid] == d && gi[q][tid] < ix)) {
                    d = gd[q][tid];
                    ix = gi[q][tid];
                }
            ix = (ix < 0 || ix >= p.ncodes) ? 0 : ix;
            codes_l[tid][L] = ix;
            prev[tid] = ix;
        }
        __syncthreads();
        RVQC_T(6);
        if (L + 1 < Le) {  // r_{L+1} = r_L - embed_L[idx] (fp32), kept as -2 r; invalid frames stay 0
            const float* rows = p.cb_rows + (long long)L * p.ncodes * D;
#pragma unroll 4
            for (int idx = tid; idx < FT * D / 4; idx += NT) {
                const int i = idx / (D / 4), k = (idx % (D / 4)) * 4;
                if (!rvq_valid(p, f0 + i)) continue;
                const f32x4 e = *reinterpret_cast<const f32x4*>(rows + (long long)prev[i] * D + k);
                const float r0 = -0.5f * img[0][i][k >> 1], r1 = -0.5f * img[1][i][k >> 1];
                const float r2 = -0.5f * img[0][i][(k >> 1) + 1], r3 = -0.5f * img[1][i][(k >> 1) + 1];
                img[0][i][k >> 1] = -2.0f * (r0 - e.x);
                img[1][i][k >> 1] = -2.0f * (r1 - e.y);
                img[0][i][(k >> 1) + 1] = -2.0f * (r2 - e.z);
                img[1][i][(k >> 1) + 1] = -2.0f * (r3 - e.w);
            }
        }
    }
    RVQC_TPRINT();
    if (slice == 0) {  // the tile's codes, every level (stores deferred: a barrier after each would wait for them)
        __syncthreads();
        for (int i = tid; i < FT * (Le - Lb); i += NT) {
            const int fr = i % FT, L = Lb + i / FT;
            const long long f = f0 + fr;
            if (f < p.frames) rvq_store_code(p, L, f, codes_l[fr][L]);
        }
    }
}

// whether the chain's whole grid is resident at once by the occupancy query (this process's view: other processes'
// kernels can still hold CUs for a while, which the bounded sweeps and the give-up flag cover)
static bool rvq_chain_fits(unsigned grid) {
    static const int cap = [] {  // (once; thread-safe initialisation)
        int dev = 0, ncu = 0, nb = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rvq_chain_h16_kernel<256, 16>, 512, 0) != hipSuccess) {
            (void)hipGetLastError();
            nb = ncu = 0;
        }
        return nb * ncu;
    }();
    return grid <= (unsigned)cap;
}

hipError_t launch_rvq(const RvqArgs& args, hipStream_t s, const char** kname, unsigned** chain_flag,
                      size_t* clear_bytes) {
    const char* kn_dummy = nullptr;
    if (!kname) kname = &kn_dummy;
    if (chain_flag) *chain_flag = nullptr;
    if (args.D != 256 || args.ncodes != 2048 || !args.work) return hipErrorInvalidValue;
    RvqArgs a = args;
    a.sem_split = (a.nsem == 1 && a.levels > 1 && a.cb_h16 && a.cb_unscale && a.cb_emax) ? 1 : 0;
    if (a.frames <= 0) return hipSuccess;
    if (a.cb_h16 && a.cb_unscale && a.cb_emax) {
        // (64-frame tiles, which halve the per-CU codebook stream, measured slower at B = 32: 0.56 vs 0.42 ms for 8
        // levels -- one workgroup per CU and 16 spilled VGPRs; profiles/r2d_rvq_ft64.log)
        // small batches (fewer 256-code-slice workgroups than CUs): 8 slices, every codebook k-step in flight at once
        // and half a code row per exact round -- the same arithmetic, latency-bound waves wait once instead of four
        // times; large batches: 4 slices of 512 codes (64 per wave, 2 k-steps in flight per 32-code tile)
        const unsigned ftiles32 = (unsigned)((a.frames + 31) / 32);
        const bool small = ftiles32 * 8 < 256;
        const bool split = a.sem_split != 0;  // levels 0 and 1 in one launch (rvq_sem_split)
        // (2- and 4-wave workgroups on small grids -- 32 / 16 slices, 4x / 2x the workgroups, each streaming a quarter /
        // half of the codebook bytes -- were slower at batch 1 and 4: rvq 0.14 -> 0.21 / 0.16 ms per batch-1 encode,
        // the per-workgroup prologue chain on fewer threads outweighs the shorter stream; profiles/r3j_ab_*)
        // form: 1 = three fp16 products (round 3); one product (P1): 2 = 2 k-steps in flight per 32-code tile, 3 = the
        // same on 64-frame tiles, 4 / 5 = 4 / 8 k-steps in flight, 6 = the small-batch form (8 slices of 256 codes,
        // every k-step in flight) at every batch size; 0 = the default.  Small batches: the small-batch form, P1 from 2 on
        const int form = a.form == 0 ? 5 : a.form;
        // small grids: every level in one persistent launch (rvq_chain_h16_kernel), unless the form asks otherwise
        const int nchain = (a.levels > a.nsem ? 1 : 0) + (a.nsem > 0 ? 1 : 0);
        // (only for a caller that reads the give-up flag back: chain_flag non-null)
        // (MIMI_RVQC_XCD: the 1-D grid of 8-slice groups on one XCD each, padded to whole 64s)
        const unsigned cgrid = MIMI_RVQC_XCD ? 64u * ((2u * ftiles32 + 7u) / 8u) : ftiles32 * 8u * 2u;
        if (small && a.chain && chain_flag && form != 1 && cgrid <= (unsigned)RVQC_MAX_WG && a.nsem <= 1 &&
            rvq_chain_fits(cgrid)) {
            const size_t gbytes = (size_t)RVQC_HDR * 8 + (size_t)2 * 2 * ftiles32 * 8 * 32 * 8;
            const size_t pd_off = (size_t)2 * ((a.frames + RVQ_FT - 1) / RVQ_FT * RVQ_FT) * a.D * 4;
            if (gbytes > rvq_work_bytes(a.frames) - pd_off) return hipErrorInvalidValue;
            unsigned long long* gbase = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(a.work) + pd_off);
            // flag + granules zeroed before every launch: by a memset here, or (clear_bytes: a captured graph) by the
            // caller before each replay (set_io_kernel), *clear_bytes bytes from the returned flag's address
            if (clear_bytes) {
                *clear_bytes = gbytes;
            } else {
                const hipError_t me = hipMemsetAsync(gbase, 0, gbytes, s);
                if (me != hipSuccess) return me;
            }
            static thread_local char knc[96];
            snprintf(knc, sizeof knc, "mimi::rvq_chain_h16_kernel<256, 16>");
            *kname = knc;
            (void)nchain;
            if (MIMI_RVQC_XCD)
                hipLaunchKernelGGL((rvq_chain_h16_kernel<256, 16>), dim3(cgrid), dim3(512), 0, s, a, gbase);
            else
                hipLaunchKernelGGL((rvq_chain_h16_kernel<256, 16>), dim3(ftiles32, 8, 2), dim3(512), 0, s, a, gbase);
            *chain_flag = reinterpret_cast<unsigned*>(gbase);
            return hipGetLastError();
        }
        const bool p1 = form >= 2;
        const bool scfg = small || form == 6;
        const int ft = (!scfg && form == 3) ? 64 : 32;
        const int pf = scfg ? 16 : form == 4 ? 4 : form == 5 ? 8 : 2;
        const unsigned ftiles = (unsigned)((a.frames + ft - 1) / ft);
        constexpr int nwv = 8;
        const unsigned nsl = 2048 / (scfg ? nwv * 32 : 8 * 64);
        static thread_local char kn[112];
        snprintf(kn, sizeof kn, "mimi::rvq_level_h16_kernel<256, %d, %d, %s, %d, %d, %d, %s>", pf, scfg ? 32 : 16,
                 a.flen ? "true" : "false", scfg ? 32 : 64, nwv, ft, p1 ? "true" : "false");
        *kname = kn;
        for (int L = 0; L < a.levels; L += (split && L == 0) ? 2 : 1) {
            a.xcd_group = (!scfg && a.xcd_group_ok) ? 1 : 0;
            const dim3 g = a.xcd_group ? dim3((ftiles + 7) / 8 * 8 * nsl, 1, (split && L == 0) ? 2 : 1)
                                       : dim3(ftiles, nsl, (split && L == 0) ? 2 : 1);
            const dim3 blk(64 * nwv);
            // (ragged, RG: workgroups of invalid frames exit)
#define RVQ_LAUNCH(PF_, EX_, CW_, NWV_, FT_, P1_)                                                                   \
    do {                                                                                                            \
        if (a.flen)                                                                                                 \
            hipLaunchKernelGGL((rvq_level_h16_kernel<256, PF_, EX_, true, CW_, NWV_, FT_, P1_>), g, blk, 0, s, a, L);  \
        else                                                                                                        \
            hipLaunchKernelGGL((rvq_level_h16_kernel<256, PF_, EX_, false, CW_, NWV_, FT_, P1_>), g, blk, 0, s, a, L); \
    } while (0)
            if (scfg) {
                if (p1)
                    RVQ_LAUNCH(16, 32, 32, 8, 32, true);
                else
                    RVQ_LAUNCH(16, 32, 32, 8, 32, false);
            } else if (!p1) {
                RVQ_LAUNCH(2, 16, 64, 8, 32, false);
            } else if (ft == 64) {
                RVQ_LAUNCH(2, 16, 64, 8, 64, true);
            } else if (pf == 4) {
                RVQ_LAUNCH(4, 16, 64, 8, 32, true);
            } else if (pf == 8) {
                RVQ_LAUNCH(8, 16, 64, 8, 32, true);
            } else {
                RVQ_LAUNCH(2, 16, 64, 8, 32, true);
            }
#undef RVQ_LAUNCH
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        const dim3 gf((unsigned)((a.frames + 255) / 256));
        if (nsl == 4)
            hipLaunchKernelGGL(rvq_final_kernel<4>, gf, dim3(256), 0, s, a, a.levels - 1);
        else
            hipLaunchKernelGGL(rvq_final_kernel<8>, gf, dim3(256), 0, s, a, a.levels - 1);
        return hipGetLastError();
    }
    // small batches (fewer 64-frame workgroups than CUs, B < 16 x 10 s): 32-frame tiles
    const bool small = (a.frames + RVQ_FT - 1) / RVQ_FT * (2048 / RVQ_CS) < 256;
    const int ft = small ? 32 : RVQ_FT;
    *kname = small ? "mimi::rvq_level_kernel<256, 32>" : "mimi::rvq_level_kernel<256, 64>";
    const dim3 grid((unsigned)((a.frames + ft - 1) / ft), 2048 / RVQ_CS);
    for (int L = 0; L < a.levels; ++L) {
        if (small)
            hipLaunchKernelGGL((rvq_level_kernel<256, 32>), grid, dim3(512), 0, s, a, L);
        else
            hipLaunchKernelGGL((rvq_level_kernel<256, RVQ_FT>), grid, dim3(512), 0, s, a, L);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(rvq_final_kernel<>, dim3((unsigned)((a.frames + 255) / 256)), dim3(256), 0, s, a, a.levels - 1);
    return hipGetLastError();
}

}  // namespace mimi
