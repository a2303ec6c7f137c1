// Fused q/k/v projection + RoPE + causal sliding-window attention of one transformer layer for items of at most
// 256 frames (TF/modeling_mimi.py:657-726 q/k/v + RoPE + softmax(QK^T / 8) V, `sliding_window` band), large
// batches.  The unfused path runs the q/k/v GEMM (gemm_planes.h, EPI_ROPE) into an fp32 [rows][3 H 64] tensor
// and attention_t256_h16_kernel (ops.hip) reads it back: at B = 32 x 10 s that is 49 MB written and read per
// layer and a launch boundary, and the GEMM itself runs 128x128 tiles whose A / W re-reads bound it.
//
// One workgroup (16 waves) per (item, head):
//   1. GEMM: the head's 192 q/k/v columns of the item's 256 rows, K = hidden, on the same fp16 planes with the same
//      instruction sequence per output element as the q/k/v GEMM (v_mfma_f32_16x16x32_f16, K steps of 32 in
//      order, the 3 plane products in mma_split's order), so every fp32 q/k/v value is bitwise the one the GEMM
//      stores.  Wave w owns 16 rows and all 192 columns, the RoPE pairs (d, d + 32) in one lane (gemm_kernel.h
//      rope_lo / rope_hi).  A fragments load straight into registers two K steps ahead; the W planes stream through
//      a 5-deep LDS-DMA ring (the first form, both operands through a 2-stage ring of 56 KiB, kept one stage in
//      flight: ~13 GB/s per CU of ingest and 0.87 ms per B = 32 step, slower than the two kernels' 0.74).
//   2. Epilogue in registers: unscale, RoPE on q and k; q goes to an fp32 LDS image (the attention tasks' queries
//      belong to other waves), k / v stay in the accumulators; the head's max |k|, |v| over the item's frames.
//   3. attention_t256_h16_kernel's arithmetic from there on (qg = 1 tasks): K / V fp16 planes in LDS at the
//      head's power-of-two scales, per-task Q planes, the chunk loops, the two-half merge and the planes store.
// Every value is computed as on the unfused path, so an item's codes do not depend on which path its batch took
// (the engine runs this kernel only for large batches; batch 1 keeps the small-grid GEMM + attention).
#include "ring_wait.h"
#include "attn_h16.h"

#ifndef QA_DIAG
#define QA_DIAG 0  // timing diagnostics (tools/qa_diag.sh builds only; results garbage): 1 return after the q/k/v
#endif             // epilogue, 2 no DMA refills in the K loop, 4 no MFMAs in the K loop, 8 no chunk loop, 16 no K / V
                   // plane writes

#ifndef QA_KG
#define QA_KG 1  // W ring stages retired per barrier (2: 0.468 -> 0.494 ms per B = 32 step, profiles/r4w_ab_kg.txt)
#endif

namespace mimi {

template <int K>
__global__ __launch_bounds__(1024) void qkv_attention_h16_kernel(QkvAttnArgs p, int items) {
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr int D = 64, TM = 256, LDO = D + 1, NWV = 16;
    constexpr int KLD = 72, KPL = TM * KLD;  // K planes: [256][72 halves]
    constexpr int VPL = TM * D;              // V planes: [256 keys][64 dims] (attn_vrow_off)
    constexpr int BK = 32, NC = 3 * D;       // K step; the head's q/k/v columns
    constexpr int S = 5;                                 // W ring stages
    constexpr int KG = QA_KG;                            // ring stages retired per barrier
    static_assert(S >= 2 * KG + 1 && KG >= 1, "ring");
    constexpr int BIMG = NC * BK, BSTG = 2 * BIMG;       // halves per W plane image / stage
    constexpr int NPB = 2 * NC / 16;                     // 1-KiB DMA pieces per stage: 24
    constexpr int QLD = D + 4;                           // q image row (floats)
    static_assert(S * BSTG <= 2 * KPL + 2 * VPL, "ring inside the K / V image");
    static_assert(TM * QLD * 2 <= 2 * KPL + 2 * VPL, "q image");
    static_assert(8 * 32 * 64 * 2 + 8 * 32 * LDO * 2 <= 2 * KPL + 2 * VPL, "merge + staging");
    __shared__ __attribute__((aligned(16))) _Float16 lds[2 * KPL + 2 * VPL + 512];  // (+ the dummy DMA piece's 1 KiB)
    __shared__ float red[2][NWV];
    __shared__ float mlx[8][2][32];

    const int H = p.H;
    int h, b;
    if (p.xcd) {  // workgroups are dealt round-robin over the 8 XCDs: item b's heads all land on XCD b & 7
        const int id = (int)blockIdx.x, s = id >> 3;
        b = (id & 7) + 8 * (s / H);
        h = s % H;
    } else {
        h = (int)blockIdx.x % H;
        b = (int)blockIdx.x / H;
    }
    if (b >= items) return;
    const int T = p.tlen ? p.tlen[b] : p.Ts;
    if (T > TM || T < 1) return;  // (the engine routes such batches to the unfused path)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    constexpr int KT = K / BK;  // (compile-time: the K loop unrolls, so the compiler counts the A loads exactly)
    const long long row0 = p.toff ? (long long)p.toff[b] : (long long)b * p.Ts;

    // ---- 1. GEMM ------------------------------------------------------------------------------------------------
    // Wave w owns rows 16 w .. +15 and all 192 columns (12 16x16 tiles: tile j = block j / 4 (q, k, v), dims
    // 16 (j % 4) ..; RoPE pairs j, j + 2 in one lane).  A fragments come straight from global memory into registers
    // (lane: row lane % 16, 16-B chunk lane / 16 of the K step -- the MFMA operand layout), two K steps ahead; only
    // the W planes go through LDS, by LDS-DMA into an S-deep ring (192 x 32 x 2 planes = 24 KiB per stage, pieces of
    // 16 rows x 64 B, chunk-swizzled as gemm_planes' 16x16x32 images: chunk_swz<32, 16>).  Bytes in flight per CU
    // while a K step computes: 2 A steps (64 KiB) + S - 1 W stages.
    const int hsel = lane >> 4;
    const long long abytes = p.a_rows * K * 2;
    const __amdgpu_buffer_rsrc_t ars0 = make_rsrc(p.Ap, abytes);
    const __amdgpu_buffer_rsrc_t ars1 = make_rsrc(reinterpret_cast<const _Float16*>(p.Ap) + p.a_pstride, abytes);
    const int aoff = (int)(((row0 + wave * 16 + (lane & 15)) * K + hsel * 8) * 2);  // (rows past the buffer load 0)
    const long long N = 3LL * H * D;
    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(p.Wp, 2 * N * K * 2);
    // W piece j (0 .. 23) of a stage: plane j / 12, local columns 16 (j % 12) ..; wave w issues pieces w and w + 16.
    // Waves 8 .. 15 have no second piece: they issue a copy of their first into a dummy LDS slot, so every wave
    // issues the same loads and the compiler's wait counts for the A registers stay exact (a wave-dependent count
    // made it wait for everything, vmcnt(0), after each step's refills)
    const int prow = lane >> 2, pch = lane & 3;
    int woff[2], wdst[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int j0 = wave + 16 * q, j = j0 < NPB ? j0 : wave;
        const int pl = j / 12, nl = (j % 12) * 16 + prow;
        const int c = pch ^ chunk_swz<BK, 16>(nl);
        const long long wrow = (long long)(nl >> 6) * H * D + h * D + (nl & 63);
        woff[q] = (int)(((pl * N + wrow) * K + c * 8) * 2);
        wdst[q] = j0 < NPB ? (j / 12) * BIMG + (j % 12) * 16 * BK : -1;  // (wave-uniform)
    }
    auto issueB = [&](int kt) {
        _Float16* st = lds + (kt % S) * BSTG;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            _Float16* dst = wdst[q] >= 0 ? st + wdst[q] : lds + 2 * KPL + 2 * VPL;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)dst, 16,
                                                     woff[q] + kt * BK * 2, 0, 0, 0);
        }
    };
    auto loadA = [&](int kt, bf16x8 (&a)[2]) {
        a[0] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ars0, aoff + kt * BK * 2, 0, 0));
        a[1] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ars1, aoff + kt * BK * 2, 0, 0));
    };

    f32x4 acc[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // A fragments of K steps kt .. kt + PA (slot kt % (PA + 1))
    constexpr int PA = 2;
    bf16x8 a[PA + 1][2];
    // W(0) .. W(S - KG - 1) and A(0) .. A(PA - 1) ahead; per K step kt: A(kt + PA); per group of KG steps the W refills
    // (below).  The compiler keeps the DMA issues in order against the waits but places the A register loads freely
    // (and inserts their waits itself), so the ring waits count DMA pieces only (dma_after_group below, ring_wait.h
    // vm_wait)
#pragma unroll
    for (int k = 0; k < S - KG; ++k)
        if (k < KT) issueB(k);
#pragma unroll
    for (int k = 0; k < PA; ++k)
        if (k < KT) loadA(k, a[k]);
    // one K step with the A fragments in `a`; refills go to `an` (the step PA ahead).  The W ring is retired KG
    // stages per barrier: before group kt0's barrier every wave waits for its pieces of W(kt0 .. kt0 + KG - 1) (the
    // DMA pieces certainly behind them: W(kt0 + KG .. kt0 + S - KG - 1), 2 per wave each), after it refills the KG
    // slots the previous group freed
    auto step = [&](int kt, bf16x8 (&a)[2], bf16x8 (&an)[2]) __attribute__((always_inline)) {
        if (!(QA_DIAG & 2) && kt + PA < KT) loadA(kt + PA, an);
        const __bf16* Bs = reinterpret_cast<const __bf16*>(lds + (kt % S) * BSTG);
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const int nl = (j >> 2) * 64 + (j & 3) * 16 + (lane & 15);
            const int off = nl * BK + (hsel ^ chunk_swz<BK, 16>(nl)) * 8;
            const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(Bs + off);
            const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(Bs + BIMG + off);
            if (!(QA_DIAG & 4)) {  // mma_split<2, ..., true>'s order: lo x hi, hi x lo, hi x hi
                acc[j] = mfma16<true>(a[1], b0, acc[j]);
                acc[j] = mfma16<true>(a[0], b1, acc[j]);
                acc[j] = mfma16<true>(a[0], b0, acc[j]);
            }
        }
    };
    auto dma_after_group = [&](int kt0) {
        int n = 0;
        for (int w = kt0 + KG; w <= kt0 + S - KG - 1; ++w) n += w < KT ? 2 : 0;
        return n;
    };
#pragma unroll
    for (int kt0 = 0; kt0 < KT; kt0 += KG) {
        vm_wait(dma_after_group(kt0));
        __builtin_amdgcn_s_barrier();  // every wave's W pieces of stages kt0 .. kt0 + KG - 1 landed; the previous
                                       // group's slots are free
        if (!(QA_DIAG & 2)) {
#pragma unroll
            for (int i = 0; i < KG; ++i)
                if (kt0 + S - KG + i < KT) issueB(kt0 + S - KG + i);
        }
#pragma unroll
        for (int i = 0; i < KG; ++i) {
            const int kt = kt0 + i;
            if (kt < KT) step(kt, a[kt % (PA + 1)], a[(kt + PA) % (PA + 1)]);
        }
    }
    __syncthreads();  // every wave is done with the ring

    // ---- 2. epilogue: unscale + RoPE (the GEMM's EPI_ROPE), q -> LDS, the head's max |k|, |v| -----------------
    float* Qs = reinterpret_cast<float*>(lds);  // [256][QLD]
    const float us = p.unscale;
    float mk = 0.0f, mv = 0.0f;
    const long long ldq = 3LL * H * D;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int row = wave * 16 + 4 * hsel + r;
        const int pos = row < T ? row : T - 1;  // (rows past T are never used: any table entry will do)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int dl = q * 16 + (lane & 15);  // dims dl, dl + 32: tiles 4 blk + q, 4 blk + q + 2
            const float c = p.rope_cos[(long long)pos * 32 + dl];
            const float sn = p.rope_sin[(long long)pos * 32 + dl];
#pragma unroll
            for (int blk = 0; blk < 3; ++blk) {
                const int j1 = 4 * blk + q, j2 = j1 + 2;
                const float x1 = acc[j1][r] * us, x2 = acc[j2][r] * us;
                acc[j1][r] = blk < 2 ? rope_lo(x1, x2, c, sn) : x1;
                acc[j2][r] = blk < 2 ? rope_hi(x2, x1, c, sn) : x2;
            }
        }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) Qs[row * QLD + jj * 16 + (lane & 15)] = acc[jj][r];
        if (row < T) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                mk = fmaxf(mk, fabsf(acc[4 + jj][r]));
                mv = fmaxf(mv, fabsf(acc[8 + jj][r]));
            }
            if (p.qkv) {
                float* qr = p.qkv + (row0 + row) * ldq + h * D + (lane & 15);
#pragma unroll
                for (int j = 0; j < 12; ++j) qr[(j >> 2) * H * D + (j & 3) * 16] = acc[j][r];
            }
        }
    }
    mk = wave_max(mk);
    mv = wave_max(mv);
    if (QA_DIAG & 1) {
        if (mk == 12345.0f) p.oamax[0] = 0u;  // (keeps the GEMM and the epilogue live)
        return;
    }
    if (lane == 0) {
        red[0][wave] = mk;
        red[1][wave] = mv;
    }
    __syncthreads();

    // ---- 3. attention_t256_h16_kernel (qg = 1) ------------------------------------------------------------------
    const int hf = lane >> 5, col = lane & 31;
    const int task = attn_task(1, 0, wave);
    const int qt = task >> 1, kh = task & 1;
    const int qw = qt * 32, qi = qw + col;
    const bool qok = qi < T;
    f16x8 qf[4][2];
    float sq;
    {
        float qv[4][8];
        float mq = 0.0f;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const float* qr = Qs + (qok ? qi : 0) * QLD + 16 * ks + 8 * hf;
            const f32x4 q0 = *reinterpret_cast<const f32x4*>(qr);
            const f32x4 q1 = *reinterpret_cast<const f32x4*>(qr + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                qv[ks][e] = qok ? q0[e] * p.scale : 0.0f;
                qv[ks][4 + e] = qok ? q1[e] * p.scale : 0.0f;
                mq = fmaxf(mq, fmaxf(fabsf(qv[ks][e]), fabsf(qv[ks][4 + e])));
            }
        }
        sq = pow2_scale(wave_max(mq));
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) split8_h(qv[ks], sq, qf[ks][0], qf[ks][1]);
    }
    mk = red[0][0];
    mv = red[1][0];
#pragma unroll
    for (int w = 1; w < NWV; ++w) {
        mk = fmaxf(mk, red[0][w]);
        mv = fmaxf(mv, red[1][w]);
    }
    const float sk = pow2_scale(mk), sv = pow2_scale(mv);
    const float usa = 1.0f / (sk * sq);  // S^T accumulator -> scores (exact)
    __syncthreads();                     // the q image is dead: K / V planes over it
    _Float16* Ks = lds;
    _Float16* Vt = lds + 2 * KPL;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        if (QA_DIAG & 16) break;
        const int row = wave * 16 + 4 * hsel + r;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int d = jj * 16 + (lane & 15);
            const float kv = row < T ? acc[4 + jj][r] : 0.0f, vv = row < T ? acc[8 + jj][r] : 0.0f;
            const float tk = kv * sk, tv = vv * sv;
            const _Float16 k0 = (_Float16)tk, v0 = (_Float16)tv;
            Ks[row * KLD + d] = k0;
            Ks[KPL + row * KLD + d] = (_Float16)(tk - (float)k0);
            Vt[attn_vrow_off(row, d)] = v0;
            Vt[VPL + attn_vrow_off(row, d)] = (_Float16)(tv - (float)v0);
        }
    }
    const float uo = 1.0f / (16384.0f * sv);  // O^T accumulator -> P V (exact)
    f32x16 o[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
    float m = -INFINITY, l = 0.f;
    __syncthreads();
    const bool active = qw < T;
    const int kend = min(T - 1, qw + 31);
    const int vlb0 = attn_vlane_base(lane, 0), vlb1 = attn_vlane_base(lane, 1);
    if (active) {
        const int kstart = max(0, qw - p.window + 1) & ~31;
        const int n = (kend - kstart) / 32 + 1, n0 = (n + 1) >> 1;
        const int cb = kstart + (kh ? 32 * n0 : 0), ce = kstart + 32 * (kh ? n : n0);
        for (int c0 = cb; c0 < ce; c0 += 32) {
            if (QA_DIAG & 8) break;
            attn_chunk_h16<KLD, KPL, D, VPL, true>(o, m, l, qf, Ks + c0 * KLD, Vt, c0, qw, qi, kend, p.window, hf, col,
                                                   usa, 1.0f, 16384.0f, vlb0, vlb1);
        }
    }
    __syncthreads();  // K / V dead: the merge and the output staging reuse the LDS
    float* mo = reinterpret_cast<float*>(lds);
    if (active && kh == 1) {
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
        float m1 = -INFINITY, l1 = 0.0f;
        const int n = (kend - (max(0, qw - p.window + 1) & ~31)) / 32 + 1;
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
    float mx = 0.0f;
    {
        const int st = wave >> 1;
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
                store_act8(p.outp, p.out_pstride, 2, (row0 + q) * (H * D) + h * D + d8, v, p.oscale, &mx);
            }
        }
    }
    amax_commit(p.oamax, mx);
#endif
}

hipError_t launch_qkv_attention(const QkvAttnArgs& a, int items, hipStream_t s) {
    if (items <= 0 || a.H <= 0 || a.K != 512 || !a.Ap || !a.Wp || !a.rope_cos || !a.rope_sin || !a.outp ||
        !(a.oscale > 0.0f) || !(a.unscale > 0.0f) || a.a_rows <= 0 || (!a.tlen && (a.Ts < 1 || a.Ts > 256)) ||
        (!a.tlen != !a.toff))
        return hipErrorInvalidValue;
    // 32-bit byte offsets of the buffer loads
    if (a.a_rows * a.K * 2 + 256LL * a.K * 2 > 0x7fffffffLL || 2LL * 3 * a.H * 64 * a.K * 2 > 0x7fffffffLL)
        return hipErrorInvalidValue;
    const long long nwg = a.xcd ? (long long)(items + 7) / 8 * 8 * a.H : (long long)items * a.H;
    hipLaunchKernelGGL((qkv_attention_h16_kernel<512>), dim3((unsigned)nwg), dim3(1024), 0, s, a, items);
    return hipGetLastError();
}

}  // namespace mimi
