// Prototype kept for tools/gemm_bench.hip only (not built into libmimi_hip.so): a streaming persistent form of
// gemm_planes_kernel that was measured bit-identical but not faster (profiles/r2_gemm_bench_stream.log).
#pragma once
#include "gemm_planes.h"

namespace mimi {

// ------------------------------------------------------------------------------------------------
// Streaming persistent form of gemm_planes_kernel for the fp16-plane GEMMs (F16, NS = 2, 16x16x32 MFMAs, BK = 32):
// a grid of (CUs x resident workgroups) walks its tiles (tile = blockIdx.x + i * gridDim.x, XCD map applied) as
// ONE continuous K-step stream -- the loader waves run straight from one tile's last stages into the next
// tile's first ones, so there is no per-tile ring fill; and the epilogue needs no LDS: the accumulators go
// through a 4 x 4 transpose inside each lane quad (DPP quad permutations) that gives every lane 4 consecutive
// columns of one row, stored as 16-B (fp32) / 8-B (fp16 planes) vectors straight from registers while the
// loaders already stream the next tile.  Every output element takes the SAME instruction sequence as in
// gemm_planes_kernel (MFMA order, epilogue operations), so the two kernels give identical bits.
// ------------------------------------------------------------------------------------------------
// y[e] = x of lane (quad base + e), register (this lane's index in its quad): a 4 x 4 transpose between the
// lane-in-quad index and the register index, as two butterfly stages on DPP quad permutations
__device__ __forceinline__ void quad_transpose(f32x4& x) {
    const int q = threadIdx.x & 3;
    auto xchg = [](float v, int ctrl) {
        return __int_as_float(ctrl == 0xB1 ? __builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true)
                                           : __builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));
    };
    // stage 1: lane bit 0 <-> register bit 0 (quad_perm [1, 0, 3, 2])
    {
        const bool odd = q & 1;
        const float s0 = odd ? x[0] : x[1], s1 = odd ? x[2] : x[3];
        const float r0 = xchg(s0, 0xB1), r1 = xchg(s1, 0xB1);
        x[0] = odd ? r0 : x[0];
        x[1] = odd ? x[1] : r0;
        x[2] = odd ? r1 : x[2];
        x[3] = odd ? x[3] : r1;
    }
    // stage 2: lane bit 1 <-> register bit 1 (quad_perm [2, 3, 0, 1])
    {
        const bool hi = q & 2;
        const float s0 = hi ? x[0] : x[2], s1 = hi ? x[1] : x[3];
        const float r0 = xchg(s0, 0x4E), r1 = xchg(s1, 0x4E);
        x[0] = hi ? r0 : x[0];
        x[2] = hi ? x[2] : r0;
        x[1] = hi ? r1 : x[1];
        x[3] = hi ? x[3] : r1;
    }
}

template <int BM, int BN, int WM, int WN, int STAGES, int EPI, int OUTP, int TAG, int LW, int FL>
__global__ __launch_bounds__((WM * WN + LW) * 64) void gemm_stream_kernel(GemmArgs p) {
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr int NS = 2, BK = 32, MF = 16;
    constexpr int NW = WM * WN;
    constexpr int NLD = LW > 0 ? LW : NW;
    constexpr int CPR = BK / 8;
    constexpr int RPP = 64 / CPR;
    constexpr int TM = BM / WM / MF;
    constexpr int TN = BN / WN / MF;
    constexpr bool PAIR = (FL & FL_PAIR) != 0;
    constexpr int XR = PAIR ? RPP : 0;
    constexpr int NB = PAIR ? 2 : 1;
    constexpr int AR = BM + XR;
    constexpr int APL = AR * BK, BPL = BN * BK;
    constexpr int STG = NS * (APL + NB * BPL);
    constexpr int TPA = NS * AR / RPP, TP = TPA + NS * NB * BN / RPP;
    constexpr int PMAX = (TP + NLD - 1) / NLD;
    constexpr int PMIN = TP / NLD;
    constexpr int ONS = OUTP & 7;
    constexpr bool OELU = (OUTP & 8) != 0;
    static_assert(TM >= 1 && TN >= 1, "tile");
    static_assert(NS * BM % RPP == 0 && NS * BN % RPP == 0, "whole pieces");
    static_assert(STAGES >= 2 && STAGES <= 4, "stages");
    static_assert(PMAX * (STAGES - 2) <= 63, "vmcnt range");
    static_assert(EPI != EPI_ROPE || TN % 4 == 0, "rope pairs (d, d+32) in one lane");
    static_assert(ONS == 0 || ONS == 2, "fp16 output planes: 2");
    static_assert(STAGES * STG * 2 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) __bf16 lds[STAGES * STG];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool loader = LW == 0 || wave >= NW;
    const bool compute = LW == 0 || wave < NW;
    const int ldw = LW > 0 ? (loader ? wave - NW : 0) : wave;
    const int wm = compute ? wave / WN : 0;
    const int wn = compute ? wave % WN : 0;
    const int M = p.M, N = p.N, K = p.K;
    const int MT = (M + BM - 1) / BM, NTn = (N + BN - 1) / BN;
    const int ntiles = MT * NTn * p.batch;
    const int KT = K / BK / NB;
    // this workgroup's stream: tiles blockIdx.x, + gridDim.x, ... (the host launches at most ntiles workgroups)
    const int G = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x * KT;
    auto coords = [&](int tile, int& b, int& m0, int& n0) {
        const int logical = xcd_remap(tile, ntiles);
        const int nt = logical % NTn;
        const int rest = logical / NTn;
        m0 = (rest % MT) * BM;
        n0 = nt * BN;
        b = rest / MT;
    };

    // ---- loader state: the tile being issued, its DMA sources (as gemm_planes_kernel) and K cursor
    const int prow = lane / CPR, pch = lane % CPR;
    const __bf16* __restrict__ Wp = reinterpret_cast<const __bf16*>(p.Wsplit);
    __amdgpu_buffer_rsrc_t arsrc[NS];
    int soff[PMAX];
    KOrderT<BK> ko;
    int ltile = blockIdx.x, lk = 0;
    auto setup = [&](int tile) {
        int b, m0, n0;
        coords(tile, b, m0, n0);
        const __bf16* __restrict__ Abase = reinterpret_cast<const __bf16*>(p.Ap) + (long long)b * p.a_bstride;
#pragma unroll
        for (int pl = 0; pl < NS; ++pl) arsrc[pl] = make_rsrc(Abase + (long long)pl * p.a_pstride, p.a_len * 2);
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
                soff[q] = (m < M + (PAIR ? 1 : 0)) ? (int)(e * 2) : -16;
            } else if (j < TP) {
                const int jb = j - TPA;
                const int pl = jb / (NB * BN / RPP), rb = jb % (BN / RPP);
                const int row = rb * RPP + prow;
                const int c = pch ^ chunk_swz<BK, MF>(row);
                int n = n0 + row;
                n = n < N ? n : N - 1;
                soff[q] = (int)(((long long)pl * N + n) * K + c * 8);
            }
        }
        ko.init(p, PAIR);
    };
    if (loader) setup(ltile);
    const int kimg = PAIR ? K / 2 : 0;  // K offset of a stage's second tap (k = 2s: s Cin)
    const int npieces = ldw < TP % NLD ? PMAX : PMIN;
    auto issue = [&](int stage) {
        if (lk == KT) {  // the next tile of the stream
            lk = 0;
            ltile += gridDim.x;
            setup(ltile);
        }
        ++lk;
        __bf16* st = lds + stage * STG;
        const int k0 = ko.offset();
        ko.next();
        const int kb = k0 * 2;
#pragma unroll
        for (int q = 0; q < PMAX; ++q) {
            const int j = ldw + q * NLD;
            if (j < TPA) {
                const int pl = j / (AR / RPP), rb = j % (AR / RPP);
                const __amdgpu_buffer_rsrc_t rs = pl == 0 ? arsrc[0] : arsrc[1];
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)(st + pl * APL + rb * RPP * BK), 16, soff[q] + kb, 0,
                    0, 0);
            } else if (j < TP) {
                const int jb = j - TPA;
                const int pi = jb / (BN / RPP), rb = jb % (BN / RPP);
                const int img = pi % NB;
                __builtin_amdgcn_global_load_lds(
                    (const void*)(Wp + soff[q] + k0 + img * kimg),
                    (__attribute__((address_space(3))) void*)(st + NS * APL + pi * BPL + rb * RPP * BK), 16, 0, 0);
            }
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.0f;
    const int arow = wm * TM * MF + (lane & (MF - 1));
    const int brow = wn * TN * MF + (lane & (MF - 1));
    const int hsel = lane >> 4;
    auto read_frags = [&](const __bf16* As, const __bf16* Bs, int img, bf16x8 (&af)[NS][TM], bf16x8 (&bf)[NS][TN]) {
#pragma unroll
        for (int pl = 0; pl < NS; ++pl) {
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = arow + i * MF + img;
                af[pl][i] = *reinterpret_cast<const bf16x8*>(As + pl * APL + row * BK + (hsel ^ chunk_swz<BK, MF>(row)) * 8);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int row = brow + j * MF;
                bf[pl][j] = *reinterpret_cast<const bf16x8*>(Bs + (pl * NB + img) * BPL + row * BK +
                                                              (hsel ^ chunk_swz<BK, MF>(row)) * 8);
            }
        }
    };

    // ---- epilogue, deferred: at a tile's last K step the accumulators go through the per-element epilogue
    // math of gemm_planes_kernel (MFMA layout: lane holds column lane & 15 of each 16 x 16 block, rows
    // 4 (lane >> 4) + r) and the quad transpose into ob (4 consecutive columns of one row per lane and block);
    // the blocks' stores are then spread over the NEXT tile's K steps, so the output bytes leave while the
    // matrix cores work instead of in one burst per tile.
    constexpr int NG = TM * TN;
    float omx = 0.0f;
    const float us = p.unscale;
    f32x4 ob[TM][TN];
    int ob_b = 0, ob_m0 = 0, ob_n0 = 0, ob_next = NG;  // ob_next == NG: nothing pending
    auto finish = [&](int tile) {
        int b, m0, n0;
        coords(tile, b, m0, n0);
        ob_b = b;
        ob_m0 = m0;
        ob_n0 = n0;
        ob_next = 0;
        const int rbase = m0 + wm * TM * MF;
        const int cbase = n0 + wn * TN * MF;
        float bias[TN], scl[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = cbase + j * MF + (lane & 15);
            bias[j] = 0.0f;
            scl[j] = 0.0f;
            if (col < N) {
                if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU || EPI == EPI_BIAS_RES_ELU || EPI == EPI_BIAS_OUT)
                    bias[j] = p.bias[col];
                if (EPI == EPI_SCALE_RES) scl[j] = p.scale[col];
            }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = rbase + i * MF + 4 * hsel + r;
                    const int col = cbase + j * MF + (lane & 15);
                    float x = acc[i][j][r] * us;
                    if (EPI == EPI_BIAS || EPI == EPI_BIAS_OUT) {
                        x = x + bias[j];
                    } else if (EPI == EPI_BIAS_ELU) {
                        x = elu1(x + bias[j]);
                    } else if (EPI == EPI_BIAS_RES_ELU) {
                        x = x + bias[j];
                    } else if (EPI == EPI_GELU) {
                        x = gelu_erf(x);
                    } else if (EPI == EPI_SCALE_RES) {
                        x = scl[j] * x;
                    } else if (EPI == EPI_ROPE) {
                        if (row < M && col < N && col < p.rope_cols) {
                            constexpr int PJ = 2;  // (d, d + 32) sit in tiles j, j + 2 of the same lane
                            const int d = col % 64;
                            const float c = p.rope_cos[(long long)row * 32 + (d & 31)];
                            const float sn = p.rope_sin[(long long)row * 32 + (d & 31)];
                            if (((j / PJ) & 1) == 0) {
                                const float x2 = acc[i][(j + PJ) % TN][r] * us;
                                x = x * c + (-x2) * sn;
                            } else {
                                const float x1 = acc[i][(j + TN - PJ) % TN][r] * us;
                                x = x * c + x1 * sn;
                            }
                        }
                    }
                    v[r] = x;
                }
                // lane (g, 4q + e) now holds row 4g + e, columns 4q .. 4q + 3 of the block
                quad_transpose(v);
                ob[i][j] = v;
            }
        }
    };
    // the stores of block q = i TN + j of the pending tile
    auto flush = [&](f32x4 v, int i, int j) {
        const int row = ob_m0 + wm * TM * MF + i * MF + 4 * hsel + (lane & 3);
        const int col = ob_n0 + wn * TN * MF + j * MF + (lane & 12);
        if (row >= M || col >= N) return;  // N % 8 == 0: a lane's 4 columns are all in or all out
        const long long off = (long long)row * p.ldc + col;
        if (EPI == EPI_BIAS_RES_ELU || EPI == EPI_SCALE_RES) {
            const f32x4 rr = *reinterpret_cast<const f32x4*>(p.R + (long long)ob_b * p.c_bstride + off);
            v = rr + v;  // R + (acc + bias) / R + scale * acc: the reference's operation order
            if (EPI == EPI_BIAS_RES_ELU) {
                v.x = elu1(v.x); v.y = elu1(v.y); v.z = elu1(v.z); v.w = elu1(v.w);
            }
        }
        if (ONS) {
            typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
            _Float16* __restrict__ Cpb = reinterpret_cast<_Float16*>(p.Cp) + (long long)ob_b * p.c_bstride;
            f16x4_t h0, h1;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float pv = OELU ? elu1(v[e]) : v[e];
                const float t = pv * p.out_scale;
                h0[e] = (_Float16)t;
                h1[e] = (_Float16)(t - (float)h0[e]);
                omx = fmaxf(omx, fabsf(pv));
            }
            *reinterpret_cast<f16x4_t*>(Cpb + off) = h0;
            *reinterpret_cast<f16x4_t*>(Cpb + p.c_pstride + off) = h1;
        }
        if (p.C) *reinterpret_cast<f32x4*>(p.C + (long long)ob_b * p.c_bstride + off) = v;
    };
    // blocks [ob_next, hi) of the pending tile (wave-uniform bounds)
    auto drain = [&](int hi) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                if (i * TN + j >= ob_next && i * TN + j < hi) flush(ob[i][j], i, j);
        ob_next = hi > ob_next ? hi : ob_next;
    };
    const int per = (NG + KT - 1) / KT;  // blocks stored per K step

    if (loader) {
#pragma unroll
        for (int s = 0; s < STAGES - 1; ++s)
            if (s < G) issue(s);
    }
    int kt = 0, ctile = blockIdx.x;
    for (int g = 0; g < G; ++g) {
        if (loader) {
            const int later = min(STAGES - 2, G - 1 - g);
            if (STAGES >= 4 && later >= 2) {
                if (PMAX == PMIN || npieces == PMAX)
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PMAX) : "memory");
                else
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PMIN) : "memory");
            } else if (STAGES >= 3 && later >= 1) {
                if (PMAX == PMIN || npieces == PMAX)
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PMAX) : "memory");
                else
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PMIN) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __builtin_amdgcn_s_barrier();
        const __bf16* As = lds + (g % STAGES) * STG;
        const __bf16* Bs = As + NS * APL;
        if (loader && g + STAGES - 1 < G) issue((g + STAGES - 1) % STAGES);
        if (compute) {
#pragma unroll
            for (int img = 0; img < NB; ++img) {
                bf16x8 af[NS][TM], bf[NS][TN];
                read_frags(As, Bs, img, af, bf);
                mma_split<NS, TM, TN, true>(acc, af, bf);
            }
            if (ob_next < NG) drain(min(NG, (kt + 1) * per));
        }
        if (++kt == KT) {
            kt = 0;
            if (compute) {
                finish(ctile);  // (the pending tile has been drained: KT * per >= NG)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.0f;
            }
            ctile += gridDim.x;
        }
    }
    if (compute && ob_next < NG) drain(NG);
    if (ONS && compute) amax_commit(p.out_amax, omx);
#endif
}

}  // namespace mimi
