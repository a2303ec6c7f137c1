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
#include "gemm_kernel.h"

namespace mimi {

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const long long lim = bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)lim, 0x00020000);
}
#endif

// (XCD-aware) linear workgroup index -> logical tile index; bijective for any count.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// LW > 0: warp-specialised -- LW extra loader waves issue every LDS-DMA piece and do the counted waits, the
// WM x WN compute waves only ds_read and MFMA (an LDS-DMA piece costs its issuing wave ~60-185 cycles,
// MI355X_MICROARCH.md; with LW = 0 the compute waves pay it between their MFMAs).  Both kinds meet at the one
// barrier per K step.
template <int BM, int BN, int WM, int WN, int NS, int STAGES, int EPI, int OUTP, int TAG, int LW = 0>
__global__ __launch_bounds__((WM * WN + LW) * 64) void gemm_planes_kernel(GemmArgs p) {
#if defined(__HIP_DEVICE_COMPILE__)  // buffer-resource builtins exist only in the device pass
    constexpr int NW = WM * WN;
    constexpr int NLD = LW > 0 ? LW : NW;        // waves issuing DMA
    constexpr int BK = 32;
    constexpr int TM = BM / WM / 32;
    constexpr int TN = BN / WN / 32;
    constexpr int APL = BM * BK, BPL = BN * BK;  // bf16 per plane image
    constexpr int STG = NS * (APL + BPL);        // bf16 per stage
    constexpr int APW = NS * BM / 16 / NLD;      // A pieces per loading wave per stage
    constexpr int BPW = NS * BN / 16 / NLD;      // B pieces per loading wave per stage
    constexpr int PPW = APW + BPW;
    static_assert(APW * NLD * 16 == NS * BM && BPW * NLD * 16 == NS * BN, "pieces must split evenly over waves");
    static_assert(STAGES >= 2 && STAGES <= 4, "stages");
    static_assert(PPW * (STAGES - 2) <= 63, "vmcnt range");
    static_assert(EPI != EPI_ROPE || (TN % 2 == 0), "rope pairs need even TN");
    // OUTP: 0 = fp32 C only; 2/3 = that many bf16 planes of the output (+ fp32 C when p.C is set);
    // | 8 = the planes hold ELU(output) (fp32 C keeps the raw value)
    constexpr int ONS = OUTP & 7;
    constexpr bool OELU = (OUTP & 8) != 0;

    __shared__ __attribute__((aligned(16))) __bf16 lds[STAGES * STG];

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
    const int logical = xcd_remap(blockIdx.x, gridDim.x);
    const int nt = logical % NTn;
    const int rest = logical / NTn;
    const int mt = rest % MT;
    const int b = rest / MT;
    const int m0 = mt * BM, n0 = nt * BN;

    // ---- DMA sources for this lane (16 rows x 4 chunks per piece; lane -> row lane>>2, chunk lane&3)
    const __bf16* __restrict__ Abase = reinterpret_cast<const __bf16*>(p.Ap) + (long long)b * p.a_bstride;
    __amdgpu_buffer_rsrc_t arsrc[NS];
#pragma unroll
    for (int pl = 0; pl < NS; ++pl) arsrc[pl] = make_rsrc(Abase + (long long)pl * p.a_pstride, p.a_len * 2);
    int aoff[APW];  // byte offset of this lane's chunk at k0 = 0 (may be negative: reads 0)
#pragma unroll
    for (int q = 0; q < APW; ++q) {
        const int j = ldw + q * NLD;
        const int rb = j % (BM / 16);
        const int row = rb * 16 + (lane >> 2);
        const int c = (lane & 3) ^ ((row >> 2) & 3);
        const int m = m0 + row;
        const long long e = p.a_off + (long long)m * p.a_rs + c * 8;
        aoff[q] = (m < M) ? (int)(e * 2) : -16;  // rows past M load 0 (never stored)
    }
    const __bf16* __restrict__ Wp = reinterpret_cast<const __bf16*>(p.Wsplit);
    const __bf16* bsrc[BPW];
#pragma unroll
    for (int q = 0; q < BPW; ++q) {
        const int j = ldw + q * NLD;
        const int pl = j / (BN / 16), rb = j % (BN / 16);
        const int row = rb * 16 + (lane >> 2);
        const int c = (lane & 3) ^ ((row >> 2) & 3);
        int n = n0 + row;
        n = n < N ? n : N - 1;  // rows past N only feed columns that are never stored
        bsrc[q] = Wp + ((long long)pl * N + n) * K + c * 8;
    }

    KOrder ko;  // K steps are issued in order: the cursor follows the issues
    ko.init(p);
    auto issue = [&](int stage) {
        __bf16* st = lds + stage * STG;
        const int k0 = ko.offset();
        ko.next();
        const int kb = k0 * 2;  // bytes
#pragma unroll
        for (int q = 0; q < APW; ++q) {
            const int j = ldw + q * NLD;
            const int pl = j / (BM / 16), rb = j % (BM / 16);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                arsrc[pl], (__attribute__((address_space(3))) void*)(st + pl * APL + rb * 16 * BK), 16,
                aoff[q] + kb, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < BPW; ++q) {
            const int j = ldw + q * NLD;
            const int pl = j / (BN / 16), rb = j % (BN / 16);
            __builtin_amdgcn_global_load_lds((const void*)(bsrc[q] + k0),
                                             (__attribute__((address_space(3))) void*)(st + NS * APL + pl * BPL +
                                                                                        rb * 16 * BK),
                                             16, 0, 0);
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
    const int hsel = lane >> 5;

    if (loader) {
#pragma unroll
        for (int s = 0; s < STAGES - 1; ++s)
            if (s < KT) issue(s);
    }

    for (int kt = 0; kt < KT; ++kt) {
        if (loader) {
            // retire this wave's pieces of stage kt; the later stages stay in flight
            const int later = min(STAGES - 2, KT - 1 - kt);
            if (STAGES >= 4 && later >= 2) {
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW) : "memory");
            } else if (STAGES >= 3 && later >= 1) {
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __builtin_amdgcn_s_barrier();
        // the stage consumed in step kt-1 is free: refill it with step kt + STAGES - 1
        if (loader && kt + STAGES - 1 < KT) issue((kt + STAGES - 1) % STAGES);
        if (!compute) continue;
        const __bf16* As = lds + (kt % STAGES) * STG;
        const __bf16* Bs = As + NS * APL;
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
            bf16x8 af[NS][TM], bf[NS][TN];
#pragma unroll
            for (int pl = 0; pl < NS; ++pl) {
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int row = arow + i * 32;
                    const int phys = ((kk * 2 + hsel) ^ ((row >> 2) & 3)) * 8;
                    af[pl][i] = *reinterpret_cast<const bf16x8*>(As + pl * APL + row * BK + phys);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int row = brow + j * 32;
                    const int phys = ((kk * 2 + hsel) ^ ((row >> 2) & 3)) * 8;
                    bf[pl][j] = *reinterpret_cast<const bf16x8*>(Bs + pl * BPL + row * BK + phys);
                }
            }
            mma_split<NS, TM, TN>(acc, af, bf);
        }
    }

    // ---- epilogue.  Phase 1 (MFMA layout: lane holds col lane&31, rows (r&3) + 8(r>>2) + 4h of each 32x32
    // tile): the epilogue math, into a wave-private fp32 tile in the (now idle) LDS ring.  Phase 2: each lane
    // reads 8 consecutive columns of one row back and stores them as 2 x 16 B fp32 and / or one 16-B bf16x8
    // per plane -- instead of one scattered 4-B (2-B per plane) store per value.
    constexpr int CW = TN * 32, LDE = CW + 4, RW = TM * 32;
    static_assert(NW * RW * LDE * 4 <= STAGES * STG * 2, "epilogue staging fits the ring");
    __syncthreads();  // every wave is done with the ring
    if (!compute) return;
    float* stg = reinterpret_cast<float*>(lds) + wave * (RW * LDE);
    const float* __restrict__ Rb = p.R ? p.R + (long long)b * p.c_bstride : nullptr;
    const int rbase = m0 + wm * RW + 4 * hsel;
    const int cbase = n0 + wn * CW + (lane & 31);
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
                const int lrow = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel;
                const int row = rbase + i * 32 + (r & 3) + 8 * (r >> 2);
                const bool ok = row < M && col < N;
                float v = acc[i][j][r];
                if (EPI == EPI_BIAS || EPI == EPI_BIAS_OUT) {
                    v = v + bias;
                } else if (EPI == EPI_BIAS_ELU) {
                    v = elu1(v + bias);
                } else if (EPI == EPI_BIAS_RES_ELU) {
                    v = v + bias;  // + R and ELU in phase 2 (vector R loads)
                } else if (EPI == EPI_GELU) {
                    v = gelu_erf(v);
                } else if (EPI == EPI_SCALE_RES) {
                    v = scale * v;  // + R in phase 2
                } else if (EPI == EPI_ROPE) {
                    if (ok && col < p.rope_cols) {
                        const int d = col % 64;  // head_dim = 64: pairs (d, d + 32) sit in tiles j, j + 1
                        const float c = p.rope_cos[(long long)row * 32 + (d & 31)];
                        const float sn = p.rope_sin[(long long)row * 32 + (d & 31)];
                        if ((j & 1) == 0) {
                            const float x2 = acc[i][j + 1][r];
                            v = v * c + (-x2) * sn;
                        } else {
                            const float x1 = acc[i][j - 1][r];
                            v = v * c + x1 * sn;
                        }
                    }
                }
                stg[lrow * LDE + j * 32 + (lane & 31)] = v;
            }
        }
    }
    float* __restrict__ Cb = p.C ? p.C + (long long)b * p.c_bstride : nullptr;
    __bf16* __restrict__ Cpb = ONS ? reinterpret_cast<__bf16*>(p.Cp) + (long long)b * p.c_bstride : nullptr;
    constexpr int LPR = CW / 8;  // lanes per row
    constexpr int RPP = 64 / LPR;  // rows per pass
#pragma unroll
    for (int ps = 0; ps < RW / RPP; ++ps) {
        const int lr = ps * RPP + lane / LPR, lc = (lane % LPR) * 8;
        f32x4 v0 = *reinterpret_cast<const f32x4*>(stg + lr * LDE + lc);
        f32x4 v1 = *reinterpret_cast<const f32x4*>(stg + lr * LDE + lc + 4);
        const int row = m0 + wm * RW + lr, col = n0 + wn * CW + lc;
        if (row >= M || col >= N) continue;  // N % 8 == 0: a lane's 8 columns are all in or all out
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
            float rem[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
            if (OELU) {
#pragma unroll
                for (int e = 0; e < 8; ++e) rem[e] = elu1(rem[e]);
            }
#pragma unroll
            for (int pl = 0; pl < ONS; ++pl) {
                bf16x8 hv;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    hv[e] = (__bf16)rem[e];
                    rem[e] = rem[e] - (float)hv[e];
                }
                *reinterpret_cast<bf16x8*>(Cpb + pl * p.c_pstride + off) = hv;
            }
        }
        if (Cb) {
            *reinterpret_cast<f32x4*>(Cb + off) = v0;
            *reinterpret_cast<f32x4*>(Cb + off + 4) = v1;
        }
    }
#endif
}

}  // namespace mimi
