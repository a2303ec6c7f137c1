// Split-bf16 GEMM over pre-split operands ("planes"): both A (activations) and W are stored in HBM as NS
// bf16 planes (x = x0 + x1 [+ x2], see gemm_kernel.h), so the main loop moves bytes only with LDS-DMA and
// does no VALU conversion work.  Included by gemm.hip and tools/gemm_bench.hip.
//
// Structure (MI355X_MICROARCH.md / cdna_hip_programming.md "pipelining across barriers"):
//   * one LDS array holding a STAGES-deep ring of {A planes, B planes} images; per stage the workgroup
//     issues (NS*BM + NS*BN)/16 1-KiB `buffer_load_dwordx4 ... lds` / `global_load_lds_dwordx4` pieces,
//     split evenly over the waves;
//   * per K step: counted `s_waitcnt vmcnt(N)` (never 0 while later stages are in flight), ONE barrier,
//     refill of the stage consumed in the previous step, then the MFMAs of this step;
//   * each image row is BK = 32 bf16 = 64 B = four 16-B chunks, stored at chunk (c ^ ((row >> 2) & 3)) so the
//     MFMA fragment reads (ds_read_b128, 16 rows x one chunk per quarter-wave) are conflict-free; the swizzle
//     is applied on the SOURCE address of each DMA lane (the LDS destination of a DMA is lane-linear);
//   * A rows come from the implicit im2col view of a channels-last activation (row m = span
//     a_off + m*a_rs); causal zero padding and the right edge come from the buffer resource's range check
//     (an out-of-range offset, including a negative one, loads 0) -- no per-element branches;
//   * workgroup -> tile map is XCD-aware: the 8 XCDs each take a contiguous run of the (m, n) tile order
//     with n fastest, so the N tiles sharing an A tile hit the same L2.
#pragma once
#include <type_traits>

#include "gemm_kernel.h"

namespace mimi {

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const long long lim = bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)lim, 0x00020000);
}
#endif

// s_waitcnt vmcnt(later * PM) for a run-time later in [0, L] (the immediate must be a constant): retires the oldest
// stage of a loading wave while `later` stages of PM pieces each stay in flight
template <int PM, int L>
__device__ __forceinline__ void wait_stages(int later) {
    if constexpr (L == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        if (later >= L)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L * PM) : "memory");
        else
            wait_stages<PM, L - 1>(later);
    }
}

// (XCD-aware) linear workgroup index -> logical tile index; bijective for any count.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// 16-B chunk position of an LDS image row (applied on the DMA source and on the fragment read: an involution),
// chosen so that every ds_read_b128 lane group of the fragment reads (MI355X_MICROARCH.md §LDS) hits 16
// distinct 16-B bank slots:
//   BK = 32 (64-B rows), 32x32x16 reads (row lane&31, chunk 2ks + lane>>5): chunk ^ ((row >> 2) & 3)
//   BK = 32 (64-B rows), 16x16x32 reads (row lane&15, chunk lane>>4):        chunk ^ 3 * ((row >> 3) & 1)
//   BK = 16 (32-B rows), 32x32x16 reads (row lane&31, chunk lane>>5):        chunk ^ ((row >> 3) & 1)
template <int BK, int MF>
__device__ __forceinline__ int chunk_swz(int row) {
    if (BK == 16) return (row >> 3) & 1;
    if (MF == 16) return ((row >> 3) & 1) * 3;
    return (row >> 2) & 3;
}


// Template knobs beyond the tile (BM x BN, WM x WN compute waves, NS planes, STAGES-deep ring):
//   LW > 0: warp-specialised -- LW extra loader waves issue every LDS-DMA piece and do the counted waits, the
//           compute waves only ds_read and MFMA (an LDS-DMA piece costs its issuing wave ~60-185 cycles,
//           MI355X_MICROARCH.md; with LW = 0 the compute waves pay it between their MFMAs).  Both kinds meet at
//           the one barrier per K step.
//   BK:     K per step, 32 (64-B image rows, 16 rows x 4 chunks per DMA piece) or 16 (32-B rows, 32 x 2):
//           BK = 16 halves the stage so a 256-row tile fits a 4-deep ring.
//   MF:     MFMA shape, 32 (v_mfma_f32_32x32x16_bf16) or 16 (v_mfma_f32_16x16x32_bf16, BK = 32).
//   F16:    the planes are fp16 (2 planes, 3 products, PREC_F16X3) scaled by powers of two; the accumulator is
//           multiplied by p.unscale before the epilogue; fp16 output planes hold out * p.out_scale.
//   FL:     FL_PRIO -- s_setprio(1) over the MFMA section;
//           FL_PAIR -- tap pairs of a k = 2s conv (the down convs): taps j and j+s of row m read the same
//           input line (A(m, (j+s)Cin + c) = A(m+1, j Cin + c)), so a stage holds ONE A image of BM + RPP rows
//           and the B images of both taps, and the second K step reads the A image one row down.  A's
//           LDS-DMA bytes halve (stage = 2 K steps; KOrder visits the chains' first taps only).
//           FL_KG2 / FL_KG4 -- 2 / 4 ring stages per barrier (below);
//           FL_PERSIST -- a grid of (CUs x resident workgroups) loops over the tiles (tile = blockIdx.x + i *
//           gridDim.x, the XCD map applied to the tile index): a tile's epilogue stores drain while the same
//           workgroup already streams its next tile's first stages (the barrier between them waits for LDS
//           only, never for the stores), and no workgroup launch / ring fill per tile.
//           FL_PF -- (with FL_PERSIST and loader waves) the loaders issue the next tile's first ring stages while
//           the compute waves run this tile's epilogue (the staging moves past those slots, in more passes if
//           needed).
//           FL_RAGGED -- per-item valid rows (GemmArgs a_rows / m_rows: ragged batches); a separate instantiation so
//           the uniform batches' kernels carry none of its bookkeeping (it cost them 2-7 % when it was run-time)
//           FL_LNA -- A = LayerNorm(p.ln_x) for the tile's BM rows, computed by every wave before the K loop with
//           layernorm_kernel's arithmetic (kernels.h ln_row_coeffs), its fp16 planes written straight into an LDS
//           image of the whole K = 512 (same rows, chunk swizzle and K-step layout as the DMA'd A images): the ring
//           carries B only and the LayerNorm launch + its planes' HBM round trip are gone.  Small grids only (the
//           LayerNorm is recomputed per N tile; a 512-wide A image is BM x 2 KiB of LDS).
//           FL_SC1OUT -- the epilogue's output stores are `sc1` buffer stores (MI355X_MICROARCH.md: an sc1 store drops
//           the line from the XCD's L2, a plain one keeps it): a large output stream then no longer evicts the weight
//           planes every tile of the XCD re-reads from its L2.  Byte offsets from the item's C / planes base are 32-bit
//           (run_planes checks).
enum : int { FL_PRIO = 2, FL_PAIR = 4, FL_PERSIST = 8, FL_KG2 = 16, FL_KG4 = 32, FL_PF = 256, FL_RAGGED = 512,
             FL_LNA = 2048, FL_SC1OUT = 4096 };
// tuning diagnostics (tools/gemm_bench.hip only; results are garbage): no DMA refills after the prologue / no MFMAs
enum : int { FL_DIAG_NODMA = 64, FL_DIAG_NOMMA = 128 };
// timing probe of an interleaved plane layout (tools/gemm_bench.hip only, results garbage): the loader waves fetch
// 8 rows x 128 B per piece (the hi and lo 64-B segments of a row adjacent, as if stored [row][k / 32][plane][32])
// instead of 16 rows x 64 B of one plane; same pieces per stage, same LDS writes
enum : int { FL_DIAG_ILV = 1024 };

template <int BM, int BN, int WM, int WN, int NS, int STAGES, int EPI, int OUTP, int TAG, int LW = 0, int BK = 32,
          int MF = 32, int FL = 0, bool F16 = false>
__global__ __launch_bounds__((WM * WN + LW) * 64) void gemm_planes_kernel(GemmArgs p) {
#if defined(__HIP_DEVICE_COMPILE__)  // buffer-resource builtins exist only in the device pass
    constexpr int NW = WM * WN;
    constexpr int NLD = LW > 0 ? LW : NW;        // waves issuing DMA
    constexpr int CPR = BK / 8;                  // 16-B chunks per image row
    constexpr int RPP = 64 / CPR;                // image rows per 1-KiB DMA piece
    constexpr int TM = BM / WM / MF;
    constexpr int TN = BN / WN / MF;
    constexpr int KSUB = MF == 32 ? BK / 16 : BK / 32;  // MFMA k-steps per K step
    constexpr bool PAIR = (FL & FL_PAIR) != 0;
    constexpr int KG = (FL & FL_KG4) ? 4 : (FL & FL_KG2) ? 2 : 1;  // ring stages per barrier
    constexpr int XR = PAIR ? RPP : 0;           // extra A image rows (PAIR: row BM, rounded to a piece)
    constexpr int NB = PAIR ? 2 : 1;             // B images (K steps) per stage
    constexpr int AR = BM + XR;                  // A image rows
    constexpr int APL = AR * BK, BPL = BN * BK;  // bf16 per plane image
    constexpr bool LNA = (FL & FL_LNA) != 0;     // A from the LayerNorm prologue (LDS-resident, not in the ring)
    constexpr int BOFF = LNA ? 0 : NS * APL;     // B images' offset in a stage
    constexpr int STG = BOFF + NS * NB * BPL;    // bf16 per stage
    // DMA pieces of a stage: A planes [0, TPA), then B [plane][image] images; piece j is issued by loading wave
    // j % NLD
    constexpr int TPA = LNA ? 0 : NS * AR / RPP, TP = TPA + NS * NB * BN / RPP;
    constexpr int PMAX = (TP + NLD - 1) / NLD;   // pieces per loading wave per stage (the first TP % NLD waves)
    constexpr int PMIN = TP / NLD;               // (the others)
    static_assert(BK == 32 || (BK == 16 && MF == 32), "BK");
    static_assert(MF == 32 || MF == 16, "MFMA shape");
    static_assert(TM >= 1 && TN >= 1 && KSUB >= 1, "tile");
    static_assert(NS * BM % RPP == 0 && NS * BN % RPP == 0, "whole pieces");
    static_assert(STAGES >= 2 * KG && STAGES <= 16, "stages");
    static_assert(PMAX * (STAGES - 2 * KG) <= 63, "vmcnt range");
    static_assert(EPI != EPI_ROPE || (MF == 32 ? TN % 2 == 0 : TN % 4 == 0), "rope pairs (d, d+32) in one lane");
    static_assert(!F16 || NS == 2, "fp16 planes: 2 planes, 3 products");
    static_assert(!LNA || (F16 && !PAIR && !(FL & (FL_PERSIST | FL_RAGGED | FL_DIAG_ILV))), "LayerNorm prologue");
    constexpr int LNK = 512;                     // (FL_LNA) the LayerNorm width = K
    constexpr int LNE = LNA ? LNK / BK * NS * APL : 0;  // bf16 of the LDS A image [K step][plane][row][BK]
    // OUTP: 0 = fp32 C only; 2/3 = that many bf16 planes of the output (+ fp32 C when p.C is set);
    // | 8 = the planes hold ELU(output) (fp32 C keeps the raw value)
    constexpr int ONS = OUTP & 7;
    constexpr bool OELU = (OUTP & 8) != 0;
    typedef typename std::conditional<MF == 32, f32x16, f32x4>::type accT;
    constexpr int NACC = MF == 32 ? 16 : 4;

    // epilogue staging (wave-private fp32 tiles) reuses the ring; a wave's CW columns go through it in JH
    // passes of CWC when the whole tile would not fit (256x256 tiles).  PF (FL_PF): the loaders issue the next
    // tile's first STAGES - KG stages while the compute waves run this tile's epilogue, so the staging sits
    // past those ring slots (PFS halves in)
    constexpr int CW = TN * MF, RW = TM * MF;
    constexpr int PFS0 = (STAGES - KG) * STG;
    constexpr bool PFIT1 = PFS0 * 2 + NW * RW * (CW + 4) * 4 <= 160 * 1024;
    constexpr bool PFIT2 = TN % 2 == 0 && PFS0 * 2 + NW * RW * (CW / 2 + 4) * 4 <= 160 * 1024;
    constexpr bool PFIT4 = TN % 4 == 0 && PFS0 * 2 + NW * RW * (CW / 4 + 4) * 4 <= 160 * 1024;
    constexpr bool PF = (FL & FL_PF) && (FL & FL_PERSIST) && LW > 0 && (PFIT1 || PFIT2 || PFIT4);
    constexpr int PFS = PF ? PFS0 : 0;
    constexpr int JH = PF ? (PFIT1 ? 1 : PFIT2 ? 2 : 4) : (NW * RW * (CW + 4) * 4 <= 160 * 1024 ? 1 : 2);
    constexpr int TNC = TN / JH, CWC = TNC * MF, LDE = CWC + 4;
    static_assert(TNC * JH == TN, "epilogue passes");  // (RoPE pairs are read from acc, not from the staging)
    constexpr int LDS_EL = STAGES * STG > PFS + NW * RW * LDE * 2 ? STAGES * STG : PFS + NW * RW * LDE * 2;
    static_assert((LDS_EL + LNE) * 2 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) __bf16 lds[LDS_EL + LNE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: keeps rsrc/LDS bases in SGPRs
    const bool loader = LW == 0 || wave >= NW;
    const bool compute = LW == 0 || wave < NW;
    const int ldw = LW > 0 ? (loader ? wave - NW : 0) : wave;  // index among the loading waves
    const int wm = compute ? wave / WN : 0;
    const int wn = compute ? wave % WN : 0;
    const int M = p.M, N = p.N, K = p.K;
    const int MT = (M + BM - 1) / BM, NTn = (N + BN - 1) / BN;
    // ragged batches (FL_RAGGED): the tile space is only the items' valid M tiles (item b: ceil(m_rows[b] / BM),
    // items concatenated) x the N tiles, so the XCD-contiguous blocks of xcd_remap and the persistent round-robin
    // share VALID work evenly (a skip of invalid tiles would leave whole XCDs idle beside long items)
    constexpr bool RG = (FL & FL_RAGGED) != 0;
    int ntiles = MT * NTn * p.batch;
    if constexpr (RG) {
        int v = 0;
        for (int bb = 0; bb < p.batch; ++bb) v += (p.m_rows[bb] + BM - 1) / BM;
        ntiles = v * NTn;
    }
    float omx = 0.0f;  // max|planes value| (fp16 planes: the engine's range check), over this workgroup's tiles
    const int KT = K / BK / NB;
    // tile -> (item, M tile, N tile).  p.ncg > 1 (XCD column groups): the logical order is column group outermost, so
    // the XCD-contiguous runs of xcd_remap cover 8 / ncg of the M tiles x N / ncg of the N tiles each -- an XCD's L2
    // then re-serves 1 / ncg of W to all its M tiles instead of streaming all of W past its 4 MB once per M-tile wave
    const int ncg = (p.ncg > 1 && NTn % p.ncg == 0) ? p.ncg : 1;
    auto decode = [&](int tile, int& b, int& mt, int& nt) {
        const int logical = xcd_remap(tile, ntiles);
        int rest;
        if (ncg > 1) {
            const int NG = NTn / ncg, per = ntiles / ncg;
            const int cg = logical / per, w = logical - cg * per;
            nt = cg * NG + w % NG;
            rest = w / NG;
        } else {
            nt = logical % NTn;
            rest = logical / NTn;
        }
        if constexpr (RG) {
            b = 0;
            for (; b < p.batch - 1; ++b) {
                const int nb = (p.m_rows[b] + BM - 1) / BM;
                if (rest < nb) break;
                rest -= nb;
            }
            mt = rest;
        } else {
            mt = rest % MT;
            b = rest / MT;
        }
    };
    auto a_len_of = [&](int b) { return RG ? (long long)p.a_rows[b] * p.a_cin : p.a_len; };
    // item b's first A / C element (ragged batches with packed rows: a_boff / c_boff)
    auto a_base_of = [&](int b) {
        return (RG && p.a_boff) ? (long long)p.a_boff[b] * p.a_cin : (long long)b * p.a_bstride;
    };
    auto c_base_of = [&](int b) {
        return (RG && p.c_boff) ? (long long)p.c_boff[b] * p.ldc : (long long)b * p.c_bstride;
    };

    // LayerNorm prologue (FL_LNA; one tile per workgroup): the tile's rows over all waves, one wave per row, all of
    // a wave's rows loaded before the first reduction.  Loader waves run it after issuing their first ring stages;
    // the barrier behind it (one extra on both sides) publishes the A image.
    float ln_mx = 0.0f;  // max|LayerNorm output| of this wave's rows, committed at the wave's end (not before the barrier)
    auto ln_prologue = [&]() __attribute__((always_inline)) {
        int b, mt, nt;
        decode((int)blockIdx.x, b, mt, nt);
        constexpr int PER = LNK / 64, NWA = NW + LW, LRW = (BM + NWA - 1) / NWA;
        float mx = 0.0f;
        const float* __restrict__ xb = p.ln_x + a_base_of(b) + p.a_off;
        // gamma / beta of this lane's columns beside the rows (not after the reductions: one more memory round trip)
        f32x4 gv[PER / 4], bv[PER / 4];
#pragma unroll
        for (int q = 0; q < PER / 4; ++q) {
            gv[q] = *reinterpret_cast<const f32x4*>(p.ln_g + q * 256 + lane * 4);
            bv[q] = *reinterpret_cast<const f32x4*>(p.ln_b + q * 256 + lane * 4);
        }
        float v[LRW][PER];
#pragma unroll
        for (int i = 0; i < LRW; ++i) {
            const int m = mt * BM + wave + i * NWA;
            if (wave + i * NWA < BM && m < M) {
                const float* xr = xb + (long long)m * p.a_rs;
#pragma unroll
                for (int q = 0; q < PER / 4; ++q) {
                    const f32x4 t = *reinterpret_cast<const f32x4*>(xr + q * 256 + lane * 4);
                    v[i][q * 4 + 0] = t.x; v[i][q * 4 + 1] = t.y; v[i][q * 4 + 2] = t.z; v[i][q * 4 + 3] = t.w;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < LRW; ++i) {
            const int r = wave + i * NWA, m = mt * BM + r;
            if (r >= BM) continue;  // (wave-uniform)
            float sc = 0.0f, bi = 0.0f;
            if (m < M) ln_row_coeffs<LNK>(v[i], p.ln_eps, sc, bi);  // (m is wave-uniform: whole-wave shuffles)
#pragma unroll
            for (int q = 0; q < PER / 4; ++q) {
                const int c0 = q * 256 + lane * 4;  // 4 columns inside one 16-B chunk of K step c0 / BK
                uint2 hi = make_uint2(0u, 0u), lo = make_uint2(0u, 0u);
                if (m < M) {
                    float o[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] = ln_affine(v[i][q * 4 + e], sc, bi, gv[q][e], bv[q][e]);
                    ln_split4_f16(o, p.ln_scale, hi, lo);
                    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
                }
                const int ks = c0 / BK, ch = (c0 % BK) / 8;
                __bf16* d = lds + LDS_EL + ks * NS * APL + r * BK + (ch ^ chunk_swz<BK, MF>(r)) * 8 + (c0 % 8);
                *reinterpret_cast<uint2*>(d) = hi;
                *reinterpret_cast<uint2*>(d + APL) = lo;
            }
        }
        ln_mx = mx;
        __syncthreads();
    };
    if constexpr (LNA && LW == 0) ln_prologue();

    if constexpr (LW > 0) {
        // Warp-specialised: the loading waves run their own tile loop, meeting the compute waves at the same
        // barriers (one per ring group, the epilogue's __syncthreads, the persistent tiles' barrier), so neither
        // keeps the other's registers live.  Loading wave W issues the pieces j = W + q LW of every stage --
        // compile-time once unrolled (no per-piece branches) -- from two 32-bit lane offsets into buffer
        // resources (A planes per batch item, all weight planes), plus wave-uniform piece and K offsets.  Rows
        // past M / N read data that only feeds never-stored outputs, or 0 past a buffer's end.
        if (loader) {
            const int prow = lane / CPR, pch = lane % CPR;
            const int c = pch ^ chunk_swz<BK, MF>(prow);  // the swizzle depends on the row's low bits only
            const __bf16* __restrict__ Wp = reinterpret_cast<const __bf16*>(p.Wsplit);
            const __amdgpu_buffer_rsrc_t wrsrc = make_rsrc(Wp, (long long)NS * N * K * 2);
            constexpr bool ILV = (FL & FL_DIAG_ILV) != 0;
            const int a_rb = ILV ? 8 * p.a_rs * 4 : RPP * p.a_rs * 2, b_rb = ILV ? 8 * K * 4 : RPP * K * 2,
                      b_pl = N * K * 2;
            auto run_loader = [&](auto Wc) {
                constexpr int W = decltype(Wc)::value;
                constexpr int PW = (TP - W + NLD - 1) / NLD;  // this wave's pieces per stage
                __amdgpu_buffer_rsrc_t arsrc[NS];
                int a_lane = 0, b_lane = 0, kimg = 0;
                KOrderT<BK> ko;  // K steps are issued in order: the cursor follows the issues
                auto setup = [&](int tile) {  // this wave's sources for `tile`, K cursor at its first step
                    int b, mt, nt;
                    decode(tile, b, mt, nt);
                    const int m0 = mt * BM, n0 = nt * BN;
                    const __bf16* __restrict__ Abase = reinterpret_cast<const __bf16*>(p.Ap) + a_base_of(b);
#pragma unroll
                    for (int pl = 0; pl < NS; ++pl)
                        arsrc[pl] = make_rsrc(Abase + (long long)pl * p.a_pstride, a_len_of(b) * 2 * (ILV ? 2 : 1));
                    if constexpr (ILV) {
                        const int r8 = lane / 8, c8 = lane % 8;
                        a_lane = (int)(((p.a_off + (long long)(m0 + r8) * p.a_rs) * 2 + c8 * 8) * 2);
                        b_lane = ((n0 + r8) * K * 2 + c8 * 8) * 2;
                    } else {
                        a_lane = (int)((p.a_off + (long long)(m0 + prow) * p.a_rs + c * 8) * 2);
                        b_lane = ((n0 + prow) * K + c * 8) * 2;
                    }
                    ko.init(p, PAIR);
                    kimg = PAIR ? ko.s * ko.cin : 0;  // K offset of a stage's second tap
                };
                auto issue_w = [&](int stage) {
                    __bf16* st = lds + stage * STG;
                    const int kb = ko.offset() * 2 * (ILV ? 2 : 1);
                    ko.next();
#pragma unroll
                    for (int q = 0; q < PW; ++q) {
                        const int j = W + q * NLD;
                        if (ILV) {
                            // DIAG: pieces of 8 rows x 128 B (both planes of a row), A then B, same LDS destinations
                            if (j < TPA) {
                                const int pl = j / (AR / RPP), rb = j % (AR / RPP);
                                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                                    arsrc[0], (__attribute__((address_space(3))) void*)(st + pl * APL + rb * RPP * BK),
                                    16, a_lane + j * a_rb + kb, 0, 0, 0);
                            } else {
                                const int jb = j - TPA;
                                const int pi = jb / (BN / RPP), rb = jb % (BN / RPP);
                                const int img = jb / (2 * BN / RPP), r8 = jb % (2 * BN / RPP);
                                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                                    wrsrc,
                                    (__attribute__((address_space(3))) void*)(st + BOFF + pi * BPL + rb * RPP * BK),
                                    16, b_lane + r8 * b_rb + kb + img * kimg * 4, 0, 0, 0);
                            }
                            continue;
                        }
                        if (j < TPA) {
                            const int pl = j / (AR / RPP), rb = j % (AR / RPP);
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                                arsrc[pl], (__attribute__((address_space(3))) void*)(st + pl * APL + rb * RPP * BK),
                                16, a_lane + rb * a_rb + kb, 0, 0, 0);
                        } else {
                            const int jb = j - TPA;
                            const int pi = jb / (BN / RPP), rb = jb % (BN / RPP);  // pi = plane * NB + image
                            const int pl = pi / NB, img = pi % NB;
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                                wrsrc,
                                (__attribute__((address_space(3))) void*)(st + BOFF + pi * BPL + rb * RPP * BK),
                                16, b_lane + pl * b_pl + rb * b_rb + kb + img * kimg * 2, 0, 0, 0);
                        }
                    }
                };
                auto prologue = [&](int tile) {
                    setup(tile);
#pragma unroll
                    for (int s2 = 0; s2 < STAGES - KG; ++s2)
                        if (s2 < KT) issue_w(s2);
                };
                const int first = (int)blockIdx.x;
                if (first < ntiles) prologue(first);
                if constexpr (LNA) ln_prologue();  // (after this wave's first ring stages are in flight)
                for (int tile = first; tile < ntiles;) {
                    for (int kt = 0; kt < KT; kt += KG) {
                        const int ng = min(KG, KT - kt);
                        wait_stages<PW, STAGES - 2 * KG>(min(KT, kt + STAGES - KG) - (kt + ng));
                        __builtin_amdgcn_s_barrier();
                        if (!(FL & FL_DIAG_NODMA)) {
#pragma unroll
                            for (int q = 0; q < KG; ++q)
                                if (kt + STAGES - KG + q < KT) issue_w((kt + STAGES - KG + q) % STAGES);
                        }
                    }
                    __syncthreads();  // the compute waves' epilogue starts (the ring is free)
                    const int next = tile + (int)gridDim.x;
                    if (PF && next < ntiles) prologue(next);  // lands in slots [0, STAGES - KG) under the epilogue
                    if (FL & FL_PERSIST) {
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        __builtin_amdgcn_s_barrier();
                    }
                    if (!PF && next < ntiles) prologue(next);
                    tile = next;
                }
            };
            static_assert(LW <= 8, "loader waves");
            switch (ldw) {
                case 0: run_loader(std::integral_constant<int, 0>()); break;
                case 1: if constexpr (LW > 1) run_loader(std::integral_constant<int, 1>()); break;
                case 2: if constexpr (LW > 2) run_loader(std::integral_constant<int, 2>()); break;
                case 3: if constexpr (LW > 3) run_loader(std::integral_constant<int, 3>()); break;
                case 4: if constexpr (LW > 4) run_loader(std::integral_constant<int, 4>()); break;
                case 5: if constexpr (LW > 5) run_loader(std::integral_constant<int, 5>()); break;
                case 6: if constexpr (LW > 6) run_loader(std::integral_constant<int, 6>()); break;
                default: if constexpr (LW > 7) run_loader(std::integral_constant<int, 7>()); break;
            }
            if constexpr (LNA) amax_commit(p.ln_amax, ln_mx);
            return;  // (no barrier follows in the compute waves)
        }
    }

    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    int b, mt, nt;
    decode(tile, b, mt, nt);
    const int m0 = mt * BM, n0 = nt * BN;

    // ---- DMA sources for this lane (RPP rows x CPR chunks per piece; lane -> row lane/CPR, chunk lane%CPR)
    const int prow = lane / CPR, pch = lane % CPR;
    const __bf16* __restrict__ Abase = reinterpret_cast<const __bf16*>(p.Ap) + a_base_of(b);
    __amdgpu_buffer_rsrc_t arsrc[NS];
#pragma unroll
    for (int pl = 0; pl < NS; ++pl) arsrc[pl] = make_rsrc(Abase + (long long)pl * p.a_pstride, a_len_of(b) * 2);
    // per piece slot q of this wave: piece j = ldw + q * NLD (wave-uniform), its LDS destination within a stage
    // (elements) and this lane's source: a byte offset into A plane pl (may be negative or past the end: the
    // buffer range check loads 0 -- the causal padding) or an element offset into the weight planes.
    const __bf16* __restrict__ Wp = reinterpret_cast<const __bf16*>(p.Wsplit);
    int soff[PMAX];
#pragma unroll
    for (int q = 0; q < PMAX; ++q) {
        const int j = ldw + q * NLD;
        soff[q] = 0;
        if (j < TPA) {
            const int rb = j % (AR / RPP);
            const int row = rb * RPP + prow;
            const int c = pch ^ chunk_swz<BK, MF>(row);
            const int m = m0 + row;
            const long long e = p.a_off + (long long)m * p.a_rs + c * 8;
            // rows past M load 0 or stale data (never stored) -- except row M in PAIR mode, the second tap of
            // row M - 1 (its address is the real one; the buffer range check zeroes what lies past the input)
            soff[q] = (m < M + (PAIR ? 1 : 0)) ? (int)(e * 2) : -16;
        } else if (j < TP) {
            const int jb = j - TPA;
            const int pl = jb / (NB * BN / RPP), rb = jb % (BN / RPP);
            const int row = rb * RPP + prow;
            const int c = pch ^ chunk_swz<BK, MF>(row);
            int n = n0 + row;
            n = n < N ? n : N - 1;  // rows past N only feed columns that are never stored
            soff[q] = (int)(((long long)pl * N + n) * K + c * 8);
        }
    }
    const int npieces = ldw < TP % NLD ? PMAX : PMIN;  // this wave's pieces per stage (wave-uniform)

    KOrderT<BK> ko;  // K steps are issued in order: the cursor follows the issues
    ko.init(p, PAIR);
    const int kimg = PAIR ? ko.s * ko.cin : 0;  // K offset of a stage's second tap
    auto issue = [&](int stage) {
        __bf16* st = lds + stage * STG;
        const int k0 = ko.offset();
        ko.next();
        const int kb = k0 * 2;  // bytes
#pragma unroll
        for (int q = 0; q < PMAX; ++q) {
            const int j = ldw + q * NLD;
            if (j < TPA) {
                const int pl = j / (AR / RPP), rb = j % (AR / RPP);
                const __amdgpu_buffer_rsrc_t rs = pl == 0 ? arsrc[0] : (pl == 1 ? arsrc[1 % NS] : arsrc[NS - 1]);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)(st + pl * APL + rb * RPP * BK), 16, soff[q] + kb, 0,
                    0, 0);
            } else if (j < TP) {
                const int jb = j - TPA;
                const int pi = jb / (BN / RPP), rb = jb % (BN / RPP);  // pi = plane * NB + image
                const int img = pi % NB;
                __builtin_amdgcn_global_load_lds(
                    (const void*)(Wp + soff[q] + k0 + img * kimg),
                    (__attribute__((address_space(3))) void*)(st + BOFF + pi * BPL + rb * RPP * BK), 16, 0, 0);
            }
        }
    };

    accT acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < NACC; ++r) acc[i][j][r] = 0.0f;

    const int arow = wm * TM * MF + (lane & (MF - 1));
    const int brow = wn * TN * MF + (lane & (MF - 1));
    const int hsel = MF == 32 ? lane >> 5 : lane >> 4;  // k chunk of the lane within an MFMA k-step

    // fragments of MFMA k-step ks of the stage at As / Bs (B image `img`, A rows shifted down by img)
    auto read_frags = [&](const __bf16* As, const __bf16* Bs, int ks, bf16x8 (&af)[NS][TM], bf16x8 (&bf)[NS][TN],
                          int img = 0) {
        const int lc = MF == 32 ? ks * 2 + hsel : hsel;
#pragma unroll
        for (int pl = 0; pl < NS; ++pl) {
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = arow + i * MF + img;
                const int phys = (lc ^ chunk_swz<BK, MF>(row)) * 8;
                af[pl][i] = *reinterpret_cast<const bf16x8*>(As + pl * APL + row * BK + phys);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int row = brow + j * MF;
                const int phys = (lc ^ chunk_swz<BK, MF>(row)) * 8;
                bf[pl][j] = *reinterpret_cast<const bf16x8*>(Bs + (pl * NB + img) * BPL + row * BK + phys);
            }
        }
    };

    // KG ring stages per barrier (FL_KG2 / FL_KG4): the loaders retire a group of KG stages at once and the
    // compute waves run its KG K steps back to back (their fragment reads free to overlap the previous step's
    // MFMAs); the ring keeps the next group(s) in flight, STAGES >= 2 KG
    if constexpr (LW > 0) {
        {  // compute waves (the loaders run their own loop above)
            if constexpr (LNA) ln_prologue();
            for (int kt = 0; kt < KT; kt += KG) {
                const int ng = min(KG, KT - kt);
                __builtin_amdgcn_s_barrier();
                if (FL & FL_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int q = 0; q < KG; ++q) {
                    if (q >= ng) break;
                    const __bf16* Bs = lds + ((kt + q) % STAGES) * STG + BOFF;
                    const __bf16* As = LNA ? lds + LDS_EL + (kt + q) * NS * APL : Bs - BOFF;
                    bf16x8 af[NS][TM], bf[NS][TN];
#pragma unroll
                    for (int img = 0; img < NB; ++img)
#pragma unroll
                        for (int ks = 0; ks < KSUB; ++ks) {
                            read_frags(As, Bs, ks, af, bf, img);
                            if (!(FL & FL_DIAG_NOMMA)) mma_split<NS, TM, TN, F16>(acc, af, bf);
                        }
                }
                if (FL & FL_PRIO) __builtin_amdgcn_s_setprio(0);
            }
        }
    } else {
    if (loader) {
#pragma unroll
        for (int s = 0; s < STAGES - KG; ++s)
            if (s < KT) issue(s);
    }

    for (int kt = 0; kt < KT; kt += KG) {
        const int ng = min(KG, KT - kt);  // stages in this group
        if (loader) {
            // retire this wave's pieces of the group's stages; the stages issued after them stay in flight
            const int later = min(KT, kt + STAGES - KG) - (kt + ng);
            if (PMAX == PMIN || npieces == PMAX)
                wait_stages<PMAX, STAGES - 2 * KG>(later);
            else
                wait_stages<PMIN, STAGES - 2 * KG>(later);
        }
        __builtin_amdgcn_s_barrier();
        // the group consumed before this barrier is free: refill its slots with the stages STAGES - KG ahead
        if (!(FL & FL_DIAG_NODMA) && loader) {
#pragma unroll
            for (int q = 0; q < KG; ++q)
                if (kt + STAGES - KG + q < KT) issue((kt + STAGES - KG + q) % STAGES);
        }
        if (!compute) continue;
        if (FL & FL_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int q = 0; q < KG; ++q) {
            if (q >= ng) break;
            const __bf16* Bs = lds + ((kt + q) % STAGES) * STG + BOFF;
            const __bf16* As = LNA ? lds + LDS_EL + (kt + q) * NS * APL : Bs - BOFF;
            bf16x8 af[NS][TM], bf[NS][TN];
#pragma unroll
            for (int img = 0; img < NB; ++img)
#pragma unroll
                for (int ks = 0; ks < KSUB; ++ks) {
                    read_frags(As, Bs, ks, af, bf, img);
                    if (!(FL & FL_DIAG_NOMMA)) mma_split<NS, TM, TN, F16>(acc, af, bf);
                }
        }
        if (FL & FL_PRIO) __builtin_amdgcn_s_setprio(0);
    }
    }  // LW == 0

    // ---- epilogue.  Phase 1 (MFMA layout): the epilogue math, into a wave-private fp32 tile in the (now idle)
    // LDS ring.  32x32 tiles: lane holds col lane&31, rows (r&3) + 8(r>>2) + 4(lane>>5); 16x16 tiles: col
    // lane&15, rows 4(lane>>4) + r.  Phase 2: each lane reads 8 consecutive columns of one row back and
    // stores them as 2 x 16 B fp32 and / or one 16-B bf16x8 per plane -- instead of one scattered 4-B (2-B
    // per plane) store per value.
    __syncthreads();  // every wave is done with the ring
    if (compute) {
    float* stg = reinterpret_cast<float*>(lds + PFS) + wave * (RW * LDE);
    const float* __restrict__ Rb = p.R ? p.R + c_base_of(b) : nullptr;
    const int rbase = m0 + wm * RW;
    const int cbase = n0 + wn * CW + (lane & (MF - 1));
    const float us = F16 ? p.unscale : 1.0f;  // 1 / (activation scale x weight scale): exact power of two
    const int Mb = RG ? min(M, p.m_rows[b]) : M;  // this item's valid output rows
#pragma unroll
    for (int jh = 0; jh < JH; ++jh) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = jh * TNC; j < (jh + 1) * TNC; ++j) {
            const int col = cbase + j * MF;
            float bias = 0.0f, scale = 0.0f;
            if (col < N) {
                if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU || EPI == EPI_BIAS_RES_ELU || EPI == EPI_BIAS_OUT)
                    bias = p.bias[col];
                if (EPI == EPI_SCALE_RES) scale = p.scale[col];
            }
#pragma unroll
            for (int r = 0; r < NACC; ++r) {
                const int lrow = MF == 32 ? i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel : i * 16 + 4 * hsel + r;
                const int row = rbase + lrow;
                const bool ok = row < Mb && col < N;
                float v = F16 ? acc[i][j][r] * us : acc[i][j][r];
                if (EPI == EPI_BIAS || EPI == EPI_BIAS_OUT) {
                    v = v + bias;
                } else if (EPI == EPI_BIAS_ELU) {
                    v = elu1(v + bias);
                } else if (EPI == EPI_BIAS_RES_ELU) {
                    // + R and ELU in phase 2 (vector R loads).  fp16 planes: acc * unscale + bias as one FMA -- the same
                    // value (the power-of-two unscale makes the product exact) in one instruction, as res1_stream and
                    // the fused blocks form it
                    v = F16 ? __builtin_fmaf(acc[i][j][r], us, bias) : v + bias;
                } else if (EPI == EPI_GELU) {
                    // f16x3: the branch-free erfc form (fc1 0.583 -> 0.561-0.565 ms per B = 32 step; codes bitwise
                    // equal on the bench batches, profiles/r6g1_ab_gelu.txt); the bf16 modes keep OCML's erff
                    v = F16 ? gelu_fast(v) : gelu_erf(v);
                } else if (EPI == EPI_SCALE_RES) {
                    v = scale * v;  // + R in phase 2
                } else if (EPI == EPI_ROPE) {
                    if (ok && col < p.rope_cols) {
                        // head_dim = 64: the pair (d, d + 32) sits in tiles j, j + 32/MF of the same lane
                        constexpr int PJ = 32 / MF;
                        const int d = col % 64;
                        const int pos = p.rope_pos ? p.rope_pos[row] : row;  // packed rows: the item's own position
                        const float c = p.rope_cos[(long long)pos * 32 + (d & 31)];
                        const float sn = p.rope_sin[(long long)pos * 32 + (d & 31)];
                        if (((j / PJ) & 1) == 0) {
                            const float x2 = F16 ? acc[i][j + PJ][r] * us : acc[i][j + PJ][r];
                            v = rope_lo(v, x2, c, sn);
                        } else {
                            const float x1 = F16 ? acc[i][j - PJ][r] * us : acc[i][j - PJ][r];
                            v = rope_hi(v, x1, c, sn);
                        }
                    }
                }
                stg[lrow * LDE + (j - jh * TNC) * MF + (lane & (MF - 1))] = v;
            }
        }
    }
    float* __restrict__ Cb = p.C ? p.C + c_base_of(b) : nullptr;
    static_assert(!F16 || ONS == 0 || ONS == 2, "fp16 output planes: 2");
    __bf16* __restrict__ Cpb = ONS ? reinterpret_cast<__bf16*>(p.Cp) + c_base_of(b) : nullptr;
    constexpr bool SC1 = (FL & FL_SC1OUT) != 0;
    static_assert(!SC1 || !ONS || F16, "sc1 output stores: fp32 and fp16 planes");
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    // (SC1: buffer resources over the item's output; a null base only ever meets a store that is not issued)
    const __amdgpu_buffer_rsrc_t c_rs = make_rsrc(SC1 ? (void*)Cb : nullptr, SC1 ? 0x7fffffffLL : 0);
    const __amdgpu_buffer_rsrc_t cp_rs = make_rsrc(SC1 ? (void*)Cpb : nullptr, SC1 ? 0x7fffffffLL : 0);
    constexpr int LPR = CWC / 8;  // lanes per row
    constexpr int RPS = 64 / LPR;  // rows per pass
    // (16 x 16 wave tiles: one pass of 32 lanes, the upper half idle)
    static_assert(RW % RPS == 0 || RW < RPS, "epilogue: a wave's tile holds whole passes of 64 lanes x 8 columns");
    constexpr int NPS = RW < RPS ? 1 : RW / RPS;
#pragma unroll
    for (int ps = 0; ps < NPS; ++ps) {
        const int lr = ps * RPS + lane / LPR, lc = (lane % LPR) * 8;
        if (RW < RPS && lr >= RW) continue;
        f32x4 v0 = *reinterpret_cast<const f32x4*>(stg + lr * LDE + lc);
        f32x4 v1 = *reinterpret_cast<const f32x4*>(stg + lr * LDE + lc + 4);
        const int row = m0 + wm * RW + lr, col = n0 + wn * CW + jh * CWC + lc;
        if (row >= Mb || col >= N) continue;  // N % 8 == 0: a lane's 8 columns are all in or all out
        const long long off = (long long)row * p.ldc + col;
        if (EPI == EPI_BIAS_RES_ELU || EPI == EPI_SCALE_RES) {
            const f32x4 r0 = *reinterpret_cast<const f32x4*>(Rb + off);
            const f32x4 r1 = *reinterpret_cast<const f32x4*>(Rb + off + 4);
            v0 = r0 + v0;  // R + (acc + bias) / R + scale * acc: the reference's operation order
            v1 = r1 + v1;
            if (EPI == EPI_BIAS_RES_ELU) {
                v0.x = elu1(v0.x); v0.y = elu1(v0.y); v0.z = elu1(v0.z); v0.w = elu1(v0.w);
                v1.x = elu1(v1.x); v1.y = elu1(v1.y); v1.z = elu1(v1.z); v1.w = elu1(v1.w);
            }
        }
        if (ONS) {
            // planes out (of ELU(v) when OELU: the next residual block's conv input), fp32 v beside
            float pv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
            if (OELU) {
#pragma unroll
                for (int e = 0; e < 8; ++e) pv[e] = elu1(pv[e]);
            }
            if constexpr (SC1) {  // store_act8's fp16 split, stored sc1
                uint4 ha, hb;
                split2_f16s(pv[0], pv[1], p.out_scale, ha.x, hb.x);
                split2_f16s(pv[2], pv[3], p.out_scale, ha.y, hb.y);
                split2_f16s(pv[4], pv[5], p.out_scale, ha.z, hb.z);
                split2_f16s(pv[6], pv[7], p.out_scale, ha.w, hb.w);
#pragma unroll
                for (int e = 0; e < 8; ++e) omx = fmaxf(omx, fabsf(pv[e]));
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, ha), cp_rs, (int)(off * 2), 0, 16);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hb), cp_rs,
                                                       (int)((off + p.c_pstride) * 2), 0, 16);
            } else {
                store_act8(Cpb, p.c_pstride, ONS, off, pv, F16 ? p.out_scale : 0.0f, &omx);
            }
        }
        if (Cb) {
            if constexpr (SC1) {
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v0), c_rs, (int)(off * 4), 0, 16);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v1), c_rs, (int)(off * 4 + 16), 0, 16);
            } else {
                *reinterpret_cast<f32x4*>(Cb + off) = v0;
                *reinterpret_cast<f32x4*>(Cb + off + 4) = v1;
            }
        }
    }
    asm volatile("" ::: "memory");  // this pass's staging reads precede the next pass's writes (same wave)
    }
    }  // compute waves
    if (FL & FL_PERSIST) {
        // the staging reads are done before the next tile's DMA lands in the ring; the stores keep draining
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
    }  // tiles
    if (F16 && ONS && compute) amax_commit(p.out_amax, omx);
    if (LNA && compute) amax_commit(p.ln_amax, ln_mx);
#endif
}

}  // namespace mimi
