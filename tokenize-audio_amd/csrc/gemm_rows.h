// Row-slab GEMM over fp16 planes for the large-batch transformer linears (fc1, fc2, o_proj): C = epi(A . W^T), A the
// [M][K] activation planes, W the [N][K] weight planes, both 2 fp16 planes at power-of-two scales (PREC_F16X3).
//
// The planes kernel (gemm_planes.h) stages BOTH operands through LDS by LDS-DMA; on these shapes its 128x128 tiles
// keep ~32-64 KiB per CU in flight and ingest ~25 GB/s per CU, so they run at 0.2-0.3 of the fp16 MFMA peak
// (profiles/r3c_gemm_bench_transformer_diag.log).  The fused q/k/v + attention kernel (qkv_attn.hip) showed the other
// arrangement: each wave owns 16 rows x all BN columns of the tile, loads its A fragments straight from global memory
// into registers (lane: row lane % 16, 16-B chunk lane / 16 of the 32-wide K step -- the operand layout of
// v_mfma_f32_16x16x32_f16) two K steps ahead, and only W goes through LDS, by LDS-DMA into an S-deep ring.  The A
// bytes then cost no LDS traffic and the W stage is shared by all the tile's rows.
//
// Every output element is formed by the same instruction sequence as in the planes kernel and the small-grid tiles
// (16x16x32 MFMAs, K steps of 32 in order, mma_split's product order, the same epilogue expressions), so an
// utterance's bits do not depend on which form its batch ran (batch 1 keeps the small-grid planes tiles).
//
// K is a template parameter: the K loop unrolls completely, every wave issues the same loads at every step, and the
// compiler's wait counts for the A registers stay exact (a data-dependent trip count or per-wave issue count made it
// wait for all loads, s_waitcnt vmcnt(0), after each step's refills -- qkv_attn.hip).
#pragma once
#include "gemm_planes.h"

namespace mimi {

// s_waitcnt vmcnt(n) for a run-time n that folds to a constant once the K loop is unrolled (n > 31: waits for more)
__device__ __forceinline__ void vm_wait(int n) {
#define MIMI_VMW(c) \
    case c: asm volatile("s_waitcnt vmcnt(" #c ")" ::: "memory"); break;
    switch (n) {
        MIMI_VMW(1) MIMI_VMW(2) MIMI_VMW(3) MIMI_VMW(4) MIMI_VMW(5) MIMI_VMW(6) MIMI_VMW(7) MIMI_VMW(8)
        MIMI_VMW(9) MIMI_VMW(10) MIMI_VMW(11) MIMI_VMW(12) MIMI_VMW(13) MIMI_VMW(14) MIMI_VMW(15) MIMI_VMW(16)
        MIMI_VMW(17) MIMI_VMW(18) MIMI_VMW(19) MIMI_VMW(20) MIMI_VMW(21) MIMI_VMW(22) MIMI_VMW(23) MIMI_VMW(24)
        MIMI_VMW(25) MIMI_VMW(26) MIMI_VMW(27) MIMI_VMW(28) MIMI_VMW(29) MIMI_VMW(30) MIMI_VMW(31)
        default:
            if (n > 31)
                asm volatile("s_waitcnt vmcnt(31)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#undef MIMI_VMW
}

constexpr int rows_lcm(int x, int y) {
    int l = x;
    while (l % y) l += x;
    return l;
}

// LDS-DMA pieces a wave may leave in flight at the top of K step kt so that W(kt) has landed: those of W(kt + 1) ..
// W(kt + S - 2), issued after it (step i issues W(i + S - 1), PPW pieces).  Only the DMA pieces are counted: the
// compiler keeps them in program order against the waits (inline asm with a memory clobber), but it moves the A
// register loads freely (it hoisted them above the wait of their step), so an A load may sit anywhere in the
// queue -- counting only what is certainly behind W(kt) is safe wherever they land, and the compiler inserts the
// waits for the A registers itself.
template <int S, int KT, int PPW>
__host__ __device__ constexpr int rows_dma_after(int kt) {
    int n = 0;
    for (int w = kt + 1; w <= kt + S - 2; ++w) n += w < KT ? PPW : 0;
    return n;
}

template <int K, int BN, int NW, int S, int EPI, int OUTP, int PA = 2>
__global__ __launch_bounds__(NW * 64) void gemm_rows_kernel(GemmArgs p) {
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr int BK = 32, KT = K / BK, BM = 16 * NW, TN = BN / 16;
    constexpr int BIMG = BN * BK, BSTG = 2 * BIMG;  // halves per W plane image / ring stage
    constexpr int NPB = 2 * BN / 16;                // 1-KiB DMA pieces per stage (16 rows x 64 B)
    constexpr int PPW = (NPB + NW - 1) / NW;        // pieces per wave per stage (extra ones go to a dummy slot)
    constexpr int ONS = OUTP & 7;
    constexpr int CWC = 64, LDE = CWC + 4;          // epilogue: 64-column passes through LDS, [16 rows][68] per wave
    static_assert(K % BK == 0 && BN % 64 == 0 && KT >= S, "shape");
    static_assert(ONS == 0 || ONS == 2, "fp16 output planes: 2");
    static_assert(EPI == EPI_GELU || EPI == EPI_SCALE_RES, "epilogues built: fc1, o_proj / fc2");
    constexpr int RING = S * BSTG, STAGE_EL = NW * 16 * LDE * 2;  // halves
    constexpr int LDS_EL = (RING > STAGE_EL ? RING : STAGE_EL) + 512;
    static_assert(LDS_EL * 2 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) _Float16 lds[LDS_EL];
    _Float16* const dummy = lds + LDS_EL - 512;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hsel = lane >> 4;
    const int M = p.M, N = p.N;
    const int MT = (M + BM - 1) / BM, NTn = N / BN;
    const int logical = xcd_remap((int)blockIdx.x, MT * NTn);  // the N tiles of an M slab on one XCD (n fastest)
    const int nt = logical % NTn, mt = logical / NTn;
    const int m0 = mt * BM, n0 = nt * BN;

    // A: this wave's 16 rows (rows past the planes' end load 0; rows in [M, end) only feed unstored outputs)
    const long long abytes = (long long)M * K * 2;
    const __amdgpu_buffer_rsrc_t ars0 = make_rsrc(p.Ap, abytes);
    const __amdgpu_buffer_rsrc_t ars1 = make_rsrc(reinterpret_cast<const _Float16*>(p.Ap) + p.a_pstride, abytes);
    const int aoff = (int)(((long long)(m0 + wave * 16 + (lane & 15)) * K + hsel * 8) * 2);
    auto loadA = [&](int kt, bf16x8 (&a)[2]) {
        a[0] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ars0, aoff + kt * BK * 2, 0, 0));
        a[1] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ars1, aoff + kt * BK * 2, 0, 0));
    };
    // W: piece j of a stage = plane j / (BN / 16), rows 16 (j % (BN / 16)) ..; wave w issues pieces w + q NW
    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(p.Wsplit, 2LL * N * K * 2);
    const int prow = lane >> 2, pch = lane & 3;
    int woff[PPW], wdst[PPW];
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
        const int j0 = wave + q * NW, j = j0 < NPB ? j0 : wave;
        const int pl = j / (BN / 16), nl = (j % (BN / 16)) * 16 + prow;
        const int c = pch ^ chunk_swz<BK, 16>(nl);
        woff[q] = (int)((((long long)pl * N + n0 + nl) * K + c * 8) * 2);
        wdst[q] = j0 < NPB ? pl * BIMG + (j % (BN / 16)) * 16 * BK : -1;  // (wave-uniform)
    }
    auto issueB = [&](int kt, int slot) {
        _Float16* st = lds + slot * BSTG;
#pragma unroll
        for (int q = 0; q < PPW; ++q)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                wrs, (__attribute__((address_space(3))) void*)(wdst[q] >= 0 ? st + wdst[q] : dummy), 16,
                woff[q] + kt * BK * 2, 0, 0, 0);
    };

    f32x4 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a[PA + 1][2];  // A fragments of K steps kt .. kt + PA (slot kt % (PA + 1))
    // step i issues A(i + PA) and W(i + S - 1); the prologue is steps -max(PA, S - 1) .. -1 of the same rule
#pragma unroll
    for (int i = -(PA > S - 1 ? PA : S - 1); i < 0; ++i) {
        if (i + PA >= 0) loadA(i + PA, a[(i + PA) % (PA + 1)]);
        if (i + S - 1 >= 0) issueB(i + S - 1, (i + S - 1) % S);
    }
    // one K step: W ring slot sw, A slot sa (the refill of A(kt + PA) goes to slot san)
    auto step = [&](int kt, int sw, int sa, int san, int nwait, bool refA, bool refW) __attribute__((always_inline)) {
        vm_wait(nwait);
        __builtin_amdgcn_s_barrier();  // every wave's W pieces of step kt landed; stage kt - 1 is free
        if (refA) loadA(kt + PA, a[san]);
        if (refW) issueB(kt + S - 1, sw == 0 ? S - 1 : sw - 1);
        const __bf16* Bs = reinterpret_cast<const __bf16*>(lds + sw * BSTG);
        const bf16x8(&ak)[2] = a[sa];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int nl = j * 16 + (lane & 15);
            const int off = nl * BK + (hsel ^ chunk_swz<BK, 16>(nl)) * 8;
            const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(Bs + off);
            const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(Bs + BIMG + off);
            acc[j] = mfma16<true>(ak[1], b0, acc[j]);  // mma_split<2, ..., true>'s order
            acc[j] = mfma16<true>(ak[0], b1, acc[j]);
            acc[j] = mfma16<true>(ak[0], b0, acc[j]);
        }
    };
    // steady state: a loop over U = lcm(S, PA + 1) steps whose slots are compile-time, every step refilling both
    // operands with the same wait count; then the last steps unrolled with their own counts.  (A fully unrolled
    // K = 2048 loop is past the unroller's budget, and a partially unrolled one with per-step conditions lost the
    // compiler's exact A-register waits.)
    constexpr int TAIL = PA > S - 1 ? PA : S - 1;
    constexpr int U = rows_lcm(S, PA + 1);
    constexpr int NSTEADY = KT > TAIL ? (KT - TAIL) / U * U : 0;
    constexpr int NSS = rows_dma_after<S, 1 << 20, PPW>(0);  // (every refill present)
    for (int base = 0; base < NSTEADY; base += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) step(base + u, u % S, u % (PA + 1), (u + PA) % (PA + 1), NSS, true, true);
    }
#pragma unroll
    for (int kt = NSTEADY; kt < KT; ++kt)
        step(kt, kt % S, kt % (PA + 1), (kt + PA) % (PA + 1), rows_dma_after<S, KT, PPW>(kt), kt + PA < KT,
             kt + S - 1 < KT);
    __syncthreads();  // the ring is free: epilogue staging

    // ---- epilogue (gemm_planes_kernel's expressions): phase 1 in the MFMA layout into a wave-private [16][LDE] fp32
    // tile per 64-column pass; phase 2: lane -> row lane / 8 (+ 8 per half), 8 columns 8 (lane % 8) .. of the pass,
    // the residual add, fp32 and planes stores of 16 B
    float* stg = reinterpret_cast<float*>(lds) + wave * 16 * LDE;
    const float us = p.unscale;
    float omx = 0.0f;
    const int rbase = m0 + wave * 16;
#pragma unroll
    for (int jp = 0; jp < BN / CWC; ++jp) {
#pragma unroll
        for (int jj = 0; jj < CWC / 16; ++jj) {
            const int j = jp * (CWC / 16) + jj;
            const int col = n0 + j * 16 + (lane & 15);
            const float scale = EPI == EPI_SCALE_RES ? p.scale[col] : 0.0f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float v = acc[j][r] * us;
                if (EPI == EPI_GELU) v = gelu_erf(v);
                if (EPI == EPI_SCALE_RES) v = scale * v;  // + R in phase 2
                stg[(4 * hsel + r) * LDE + jj * 16 + (lane & 15)] = v;
            }
        }
        asm volatile("" ::: "memory");  // (the same wave writes and reads its staging tile: LDS keeps a wave's order)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int lr = (lane >> 3) + 8 * h, lc = (lane & 7) * 8;
            f32x4 v0 = *reinterpret_cast<const f32x4*>(stg + lr * LDE + lc);
            f32x4 v1 = *reinterpret_cast<const f32x4*>(stg + lr * LDE + lc + 4);
            const int row = rbase + lr, col = n0 + jp * CWC + lc;
            if (row >= M) continue;
            const long long off = (long long)row * p.ldc + col;
            if (EPI == EPI_SCALE_RES) {
                const f32x4 r0 = *reinterpret_cast<const f32x4*>(p.R + off);
                const f32x4 r1 = *reinterpret_cast<const f32x4*>(p.R + off + 4);
                v0 = r0 + v0;  // R + scale * acc: the reference's operation order
                v1 = r1 + v1;
            }
            if (ONS) {
                const float pv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
                store_act8(p.Cp, p.c_pstride, ONS, off, pv, p.out_scale, &omx);
            }
            if (p.C) {
                *reinterpret_cast<f32x4*>(p.C + off) = v0;
                *reinterpret_cast<f32x4*>(p.C + off + 4) = v1;
            }
        }
        asm volatile("" ::: "memory");  // this pass's staging reads precede the next pass's writes
    }
    if (ONS) amax_commit(p.out_amax, omx);
#endif
}

}  // namespace mimi
