// o_proj + layer scale + residual, then the post-attention LayerNorm, in one kernel for the large-batch transformer
// (TF/modeling_mimi.py MimiTransformerLayer.forward :851-869: residual + self_attn_layer_scale(o_proj(attn)), then
// post_attention_layernorm).  The two-kernel form runs the o_proj planes GEMM (128x128 tiles, EPI_SCALE_RES) and a
// LayerNorm launch that reads the 16 MB residual stream back and writes its fp16 planes (0.025 + 0.012 ms per layer
// at B = 32).  A LayerNorm needs whole 512-wide rows, so here a workgroup owns 32 rows x all 512 output columns:
//   GEMM: 8 waves = 2 row groups x 4 column groups (16 rows x 128 columns, 8 tiles of 16x16 each); A (the attention
//   output planes) loads straight into registers in the MFMA operand layout two K steps ahead; W_o's planes stream
//   through a 2-deep LDS-DMA ring of 64 KiB stages.  The per-element sequence is the planes GEMM's (16x16x32 MFMAs,
//   K steps in order, mma_split's product order, unscale then layer scale), so t0 is bitwise the o_proj GEMM's.
//   Epilogue: scale x acc into an fp32 LDS image of the 32 rows; then wave w takes rows 4 w .. 4 w + 3 with
//   layernorm_kernel's lane layout (lane l: columns 256 q + 4 l + e): t0 = R + v stored, and ln_row_coeffs /
//   ln_affine / ln_split4_f16 on exactly those values -- the LayerNorm planes are bitwise the LayerNorm kernel's.
#include "gemm_rows.h"

namespace mimi {

template <int K, int N>
__global__ __launch_bounds__(512) void oproj_ln_h16_kernel(OprojLnArgs p) {
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr int BK = 32, KT = K / BK, BM = 32, NCG = 4, TN = N / NCG / 16, PA = 2, S = 2;
    constexpr int BIMG = N * BK, BSTG = 2 * BIMG;  // halves per W plane image / ring stage (N rows x 32)
    constexpr int NPB = 2 * N / 16, PPW = NPB / 8;  // DMA pieces per stage / per wave
    constexpr int LDV = N + 4;                      // fp32 row of the epilogue image
    static_assert(NPB % 8 == 0 && TN * 16 * NCG == N && N == 512, "shape");
    static_assert(BM * LDV * 2 <= S * BSTG, "the epilogue image inside the ring");
    __shared__ __attribute__((aligned(16))) _Float16 lds[S * BSTG];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hsel = lane >> 4, l16 = lane & 15;
    const int g = wave & 1, cg = wave >> 1;  // row group, column group
    const int M = p.M;
    const int m0 = (int)blockIdx.x * BM;
    const long long abytes = (long long)M * K * 2;
    const __amdgpu_buffer_rsrc_t ars0 = make_rsrc(p.Ap, abytes);
    const __amdgpu_buffer_rsrc_t ars1 = make_rsrc(reinterpret_cast<const _Float16*>(p.Ap) + p.a_pstride, abytes);
    const int aoff = (int)(((long long)(m0 + g * 16 + l16) * K + hsel * 8) * 2);
    auto loadA = [&](int kt, bf16x8 (&a)[2]) {
        a[0] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ars0, aoff + kt * BK * 2, 0, 0));
        a[1] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ars1, aoff + kt * BK * 2, 0, 0));
    };
    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(p.Wp, 2LL * N * K * 2);
    const int prow = lane >> 2, pch = lane & 3;
    int woff[PPW];
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
        const int j = wave + q * 8;
        const int pl = j / (N / 16), nl = (j % (N / 16)) * 16 + prow;
        woff[q] = (int)((((long long)pl * N + nl) * K + (pch ^ chunk_swz<BK, 16>(nl)) * 8) * 2);
    }
    auto issueB = [&](int kt) {
        _Float16* st = lds + (kt % S) * BSTG;
#pragma unroll
        for (int q = 0; q < PPW; ++q) {
            const int j = wave + q * 8;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                wrs, (__attribute__((address_space(3))) void*)(st + (j / (N / 16)) * BIMG + (j % (N / 16)) * 16 * BK),
                16, woff[q], kt * BK * 2, 0, 0);
        }
    };

    f32x4 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a[PA + 1][2];
    issueB(0);
#pragma unroll
    for (int k = 0; k < PA; ++k) loadA(k, a[k]);
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
        vm_wait(rows_dma_after<S, KT, PPW>(kt));  // (S = 2: W(kt), the only stage in flight)
        __builtin_amdgcn_s_barrier();  // every wave's pieces of W(kt) landed; stage kt - 1 is free
        if (kt + 1 < KT) issueB(kt + 1);
        if (kt + PA < KT) loadA(kt + PA, a[(kt + PA) % (PA + 1)]);
        const __bf16* Bs = reinterpret_cast<const __bf16*>(lds + (kt % S) * BSTG);
        const bf16x8(&ak)[2] = a[kt % (PA + 1)];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int nl = cg * (N / NCG) + j * 16 + l16;
            const int off = nl * BK + (hsel ^ chunk_swz<BK, 16>(nl)) * 8;
            const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(Bs + off);
            const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(Bs + BIMG + off);
            acc[j] = mfma16<true>(ak[1], b0, acc[j]);  // mma_split<2, ..., true>'s order
            acc[j] = mfma16<true>(ak[0], b1, acc[j]);
            acc[j] = mfma16<true>(ak[0], b0, acc[j]);
        }
    }
    __syncthreads();  // the ring is free: the epilogue image

    // ---- phase 1: scale * (acc * unscale) (the planes GEMM's EPI_SCALE_RES before its residual add)
    float* img = reinterpret_cast<float*>(lds);  // [32][LDV]
    const float us = p.unscale;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int col = cg * (N / NCG) + j * 16 + l16;
        const float sc = p.scale[col];
#pragma unroll
        for (int r = 0; r < 4; ++r) img[(g * 16 + 4 * hsel + r) * LDV + col] = sc * (acc[j][r] * us);
    }
    __syncthreads();
    // ---- phase 2: rows 4 wave .. +3, layernorm_kernel's lane layout: residual add + store, then the LayerNorm
    f32x4 gv[2], bv[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        gv[q] = *reinterpret_cast<const f32x4*>(p.ln_g + q * 256 + lane * 4);
        bv[q] = *reinterpret_cast<const f32x4*>(p.ln_b + q * 256 + lane * 4);
    }
    float mx = 0.0f;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
        const int lr = wave * 4 + rr, row = m0 + lr;
        if (row >= M) break;  // (wave-uniform)
        float v[8];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int c0 = q * 256 + lane * 4;
            const long long off = (long long)row * N + c0;
            const f32x4 rv = *reinterpret_cast<const f32x4*>(p.R + off);
            const f32x4 sv = *reinterpret_cast<const f32x4*>(img + lr * LDV + c0);
            const f32x4 t = rv + sv;  // R + scale * acc: the reference's operation order
            *reinterpret_cast<f32x4*>(p.C + off) = t;
            v[q * 4 + 0] = t.x; v[q * 4 + 1] = t.y; v[q * 4 + 2] = t.z; v[q * 4 + 3] = t.w;
        }
        float sc, bi;
        ln_row_coeffs<N>(v, p.ln_eps, sc, bi);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int c0 = q * 256 + lane * 4;
            const float o[4] = {ln_affine(v[q * 4 + 0], sc, bi, gv[q].x, bv[q].x),
                                ln_affine(v[q * 4 + 1], sc, bi, gv[q].y, bv[q].y),
                                ln_affine(v[q * 4 + 2], sc, bi, gv[q].z, bv[q].z),
                                ln_affine(v[q * 4 + 3], sc, bi, gv[q].w, bv[q].w)};
            uint2 h0, h1;
            ln_split4_f16(o, p.ln_scale, h0, h1);
            _Float16* pr = reinterpret_cast<_Float16*>(p.ln_out) + (long long)row * N + c0;
            *reinterpret_cast<uint2*>(pr) = h0;
            *reinterpret_cast<uint2*>(pr + p.ln_pstride) = h1;
            mx = fmaxf(mx, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
        }
    }
    amax_commit(p.ln_amax, mx);
#endif
}

hipError_t launch_oproj_ln(const OprojLnArgs& a, hipStream_t s, const char** kname) {
    if (a.K != 512 || a.N != 512 || a.M <= 0 || !a.Ap || !a.Wp || !a.scale || !a.R || !a.C || !a.ln_g || !a.ln_b ||
        !a.ln_out || !(a.unscale > 0.0f) || !(a.ln_scale > 0.0f))
        return hipErrorInvalidValue;
    if ((long long)a.M * a.K * 2 + 32LL * a.K * 2 > 0x7fffffffLL) return hipErrorInvalidValue;  // 32-bit offsets
    hipLaunchKernelGGL((oproj_ln_h16_kernel<512, 512>), dim3((unsigned)((a.M + 31) / 32)), dim3(512), 0, s, a);
    if (kname) *kname = "mimi::oproj_ln_h16_kernel<512, 512>";
    return hipGetLastError();
}

}  // namespace mimi
