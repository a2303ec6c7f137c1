// Stage-2 k = 1 residual conv + skip + ELU as a streaming kernel (PREC_F16X3): y = ELU(x + b1 + W1 . h), the
// second half of MimiResnetBlock (TF/modeling_mimi.py:433-447) and the ELU in front of the next down conv
// (:455-476), from the k3 conv's h planes.  The planes GEMM (gemm_planes.h, ROLE_RES1P, EPI_BIAS_RES_ELU) runs it
// as 128 x 128 tiles through an LDS-DMA ring: per tile a 4-step K loop, then the skip x is fetched in the
// epilogue -- two dependent HBM round trips per tile with nothing of the next tile in flight (4.3 TB/s, 0.54 of
// the HBM roofline at B = 32 x 10 s).  This layer moves 983 MB and does 25 GFLOP: it is HBM-bound.
//
// Here each of a workgroup's 4 waves keeps its 64 output channels' W1 planes in registers for the whole launch (4
// channel tiles x K / 32 k-steps x 2 planes of v_mfma_f32_16x16x32_f16 A fragments: 128 VGPRs at K = 128) and walks
// 16-step time tiles through a 2-deep ring of register tiles: the next tile's h fragments (straight from global;
// the 4 waves read the same bytes: L1 hits) and skip values load while the current tile's MFMAs and epilogue run.
// Transposed (W is the A operand): a lane's accumulator is 4 channels of one step, and the channel tiles of a wave
// interleave their rows (tile ct row r <-> channel c0 + 16 (r / 4) + 4 ct + r % 4), so a lane owns 16 consecutive
// channels of one step: 64-B skip reads and two 16-B stores per plane, a wave's row stores whole 128-B lines (with
// 32 channels per wave, half lines: 25 % slower).
//
// Every output element is the planes GEMM's: the same fragments (k chunk 8 (lane / 16) of each 32-wide K step, K
// steps in order), the same product order per K step (h_lo W_hi, h_hi W_lo, h_hi W_hi; the transposition swaps
// the MFMA operands, not the products -- as in stage0_fused.hip), and the same epilogue expressions (fma(acc,
// unscale, bias), then R + that, ELU, store_act8's fp16 split).  Bitwise the ROLE_RES1P output (tests/test_res1_stream.py).
#include <algorithm>

#include "gemm_planes.h"
#include "kernels.h"

namespace mimi {



// DEPTH: register tiles in the ring (DEPTH - 1 tiles of loads in flight under a tile's compute); CPW: output
// channels per wave (CT = CPW / 16 channel tiles; a lane owns CPW / 4 consecutive channels of one step)
constexpr int R1S_MAXB = 256;  // ragged batches: items the in-kernel tile table holds (more: the planes GEMM runs)

// RG: a ragged batch (p.m_rows) -- its own instantiation, so the uniform kernel's loop carries none of the tile-table
// lookups (run-time-branched into one kernel they cost the uniform batches 13 %: 0.220 -> 0.249 ms per B = 32 step)
// A workgroup is 4 waves x CPW output channels; NG = N / (4 CPW) workgroup columns (blockIdx.y) cover N.  Stage 2
// (K = 128, N = 256): one column, W1 128 VGPRs per wave.  Stage 3 (K = 256, N = 512): two columns, W1 256 registers
// per wave -- the compiler keeps them beside the ring in the accumulation registers (256 VGPRs + 236 AGPRs, no
// scratch; one wave per SIMD), and both columns of a tile run at the same time on one XCD (workgroup x and x + G
// share x mod 8), so its h rows come from that XCD's L2 the second time.
template <int K, int DEPTH, int CPW, bool RG>
__global__ __launch_bounds__(256) void res1_stream_kernel(GemmArgs p, int ntiles) {
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr int N = 2 * K, KS = K / 32, CT = CPW / 16, LC = CPW / 4, NG = N / (4 * CPW);
    static_assert(NG >= 1 && NG * 4 * CPW == N, "4 waves x CPW channels per workgroup column");
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c0 = ((NG > 1 ? (int)blockIdx.y : 0) * 4 + wave) * CPW;
    const int l16 = lane & 15, q = lane >> 4;
    // W1 fragments: [channel tile][k step][plane]; row l16 of tile ct = channel c0 + LC (l16 / 4) + 4 ct + l16 % 4
    h8 wf[CT][KS][2];
    {
        const _Float16* W = reinterpret_cast<const _Float16*>(p.Wsplit);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const int ch = c0 + LC * (l16 >> 2) + 4 * ct + (l16 & 3);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                for (int pl = 0; pl < 2; ++pl)
                    wf[ct][ks][pl] = *reinterpret_cast<const h8*>(W + ((long long)pl * N + ch) * K + ks * 32 + 8 * q);
        }
    }
    // this lane's LC channels: c0 + LC q .. + LC - 1 (rows 4 q .. 4 q + 3 of every channel tile)
    const int cl = c0 + LC * q;
    float bias[LC];
#pragma unroll
    for (int e = 0; e < LC; ++e) bias[e] = p.bias[cl + e];
    const float us = p.unscale, os = p.out_scale;
    const long long rows = (long long)p.M * p.batch;  // items back to back: row = item * M + t
    const __amdgpu_buffer_rsrc_t h0 = make_rsrc(p.Ap, rows * K * 2);
    const __amdgpu_buffer_rsrc_t h1 = make_rsrc(reinterpret_cast<const _Float16*>(p.Ap) + p.a_pstride, rows * K * 2);
    const __amdgpu_buffer_rsrc_t rr = make_rsrc(p.R, rows * N * 4);
    // ragged batches: only the items' valid 16-step tiles (item b's ceil(m_rows[b] / 16) tiles from tst[b]), so the
    // padding rows cost nothing (a walk over all batch x M rows read and skipped them: YODAS2-style batches +28 %)
    __shared__ int tst[R1S_MAXB + 1];
    if constexpr (RG) {
        if (tid == 0) {
            int acc = 0;
            for (int b = 0; b < p.batch; ++b) {
                tst[b] = acc;
                acc += (p.m_rows[b] + 15) >> 4;
            }
            tst[p.batch] = acc;
        }
        __syncthreads();
        ntiles = tst[p.batch];
    }
    // a tile's first row and (ragged) its item's valid steps from there
    auto tile_at = [&](int tile, int& lim) -> long long {
        int lo = 0, hi = p.batch - 1;  // the last item whose first tile is <= tile
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (tst[mid] <= tile) lo = mid; else hi = mid - 1;
        }
        const int tt = tile - tst[lo];
        lim = p.m_rows[lo] - 16 * tt;
        return (long long)lo * p.M + 16 * tt;
    };

    struct Tile {
        h8 b[KS][2];  // h fragments (B operand): step l16 of the tile, k chunk 8 q of each K step
        f32x4 r[CT];  // skip x: channels cl .. cl + LC - 1 of step l16
    };
    auto load = [&](int tile, Tile& t) {
        long long row;  // (past the rows: the buffer range check loads 0)
        if constexpr (RG) {
            int lim;
            row = tile_at(tile, lim) + l16;
        } else {
            row = (long long)tile * 16 + l16;
        }
        const int ho = (int)((row * K + 8 * q) * 2);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            t.b[ks][0] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(h0, ho + ks * 64, 0, 0));
            t.b[ks][1] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(h1, ho + ks * 64, 0, 0));
        }
        const int ro = (int)((row * N + cl) * 4);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
            t.r[ct] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, ro + 16 * ct, 0, 0));
    };
    float omx = 0.0f;
    // this tile's MFMAs + epilogue from t
    auto run = [&](int tile, const Tile& t) __attribute__((always_inline)) {
        f32x4 acc[CT];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {  // mma_split's order per K step: lo x hi, hi x lo, hi x hi
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[ct][ks][0], t.b[ks][1], acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[ct][ks][1], t.b[ks][0], acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[ct][ks][0], t.b[ks][0], acc[ct], 0, 0, 0);
            }
        long long row;
        bool ok;
        if constexpr (RG) {
            int lim;
            row = tile_at(tile, lim) + l16;
            ok = row < rows && l16 < lim;  // (the item's valid steps only -- its rows past them are never stored)
        } else {
            row = (long long)tile * 16 + l16;
            ok = row < rows;
            if (ok && p.m_rows) {  // (never taken: the launch sends ragged batches to RG; kept because this form of the
                                   // loop is the one hipcc schedules best -- 20 waits against 29-41 without it)
                const long long b = row / p.M;
                ok = row - b * p.M < p.m_rows[b];
            }
        }
        if (ok) {
#pragma unroll
            for (int g = 0; g < LC / 8; ++g) {
                float pv[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int c = 8 * g + e;
                    const float v = __builtin_fmaf(acc[c >> 2][c & 3], us, bias[c]);  // (the planes GEMM's phase 1)
                    const float rv = t.r[c >> 2][c & 3];
                    pv[e] = elu1(rv + v);  // phase 2: R + (acc + bias), ELU
                }
                store_act8(p.Cp, p.c_pstride, 2, row * N + cl + 8 * g, pv, os, &omx);
            }
        }
    };
    // a ring of DEPTH register tiles: tile i + DEPTH - 1 loads while tile i computes (unrolled by the depth so
    // every slot is a fixed set of registers)
    const int G = (int)gridDim.x;
    Tile ring[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH - 1; ++d)
        if ((int)blockIdx.x + d * G < ntiles) load((int)blockIdx.x + d * G, ring[d]);
    for (int tile = (int)blockIdx.x; tile < ntiles; tile += DEPTH * G) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const int tl = tile + d * G;
            if (tl >= ntiles) break;
            const int ahead = tl + (DEPTH - 1) * G;
            if (ahead < ntiles) load(ahead, ring[(d + DEPTH - 1) % DEPTH]);
            run(tl, ring[d]);
        }
    }
    amax_commit(p.out_amax, omx);
#endif
}

// the stage-2 shape (K = 128, N = 256; uniform or ragged) or the stage-3 shape (K = 256, N = 512; uniform batches)
// with the engine's layouts: h planes [rows][K], skip / planes out [rows][N], items back to back (rows = batch x M),
// no fp32 output; otherwise hipErrorInvalidValue (the engine keeps the GEMM)
bool res1_stream_ok(const GemmArgs& a) {
    return ((a.K == 128 && a.N == 256) || (a.K == 256 && a.N == 512 && !a.m_rows)) && a.Ap && a.Wsplit && a.R &&
           a.Cp && !a.C && a.bias && a.out_amax &&
           a.a_rs == a.K && a.a_cin == a.K && a.a_off == 0 && a.ldc == a.N && a.a_bstride == (long long)a.M * a.K &&
           a.c_bstride == (long long)a.M * a.N && !a.a_boff && !a.c_boff && (!a.m_rows == !a.a_rows) &&
           (!a.m_rows || a.batch <= R1S_MAXB) &&
           (long long)a.M * a.batch * a.N * 4 < 0x7fffffffLL && a.out_scale > 0.0f && a.unscale > 0.0f;
}

template <int K, int DEPTH, int CPW>
static hipError_t run_res1_stream(const GemmArgs& a, hipStream_t s, const char** kname) {
    constexpr int NT = 256, NG = 2 * K / (4 * CPW);
    static thread_local char nm[80];
    const bool rg = a.m_rows != nullptr;
    snprintf(nm, sizeof nm, "mimi::res1_stream_kernel<%d, %d, %d, %s>(mimi::GemmArgs, int)", K, DEPTH, CPW,
             rg ? "true" : "false");
    if (kname) *kname = nm;
    const long long rows = (long long)a.M * a.batch;
    const int ntiles = (int)((rows + 15) / 16);
    static const int slots = [] {  // (once per instantiation; thread-safe initialisation)
        int dev = 0, ncu = 256, occ = 1;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, res1_stream_kernel<K, DEPTH, CPW, false>, NT, 0);
        // NG columns share the resident slots; a multiple of the 8 XCDs per column keeps a tile's columns on one XCD
        return std::max(8, ncu * (occ > 0 ? occ : 1) / NG / 8 * 8);
    }();
    const int grid = ntiles < slots ? ntiles : slots;
    if constexpr (K == 128) {
        if (rg) {
            hipLaunchKernelGGL((res1_stream_kernel<K, DEPTH, CPW, true>), dim3((unsigned)grid), dim3(NT), 0, s, a,
                               ntiles);
            return hipGetLastError();
        }
    } else if (rg) {
        return hipErrorInvalidValue;  // (res1_stream_ok keeps ragged stage-3 batches on the planes GEMM)
    }
    hipLaunchKernelGGL((res1_stream_kernel<K, DEPTH, CPW, false>), dim3((unsigned)grid, (unsigned)NG), dim3(NT), 0, s,
                       a, ntiles);
    return hipGetLastError();
}


// (A/B at B = 32 x 10 s, res1_s2 per step, profiles/r5b_ab_res1_stream.txt: the planes GEMM 0.229-0.231 ms; 32 channels
// per wave with a 1- / 2- / 3-deep ring 0.288 / 0.31 / 0.31 (half-line stores); 64 per wave without a ring 0.315, with
// the 2-deep ring 0.218-0.221 (kept); W1 in LDS, 64 per wave, 2 row groups x 2- / 3-deep, 3 groups x 2-deep:
// 0.235-0.243)
#ifndef MIMI_R1S_DEPTH2
#define MIMI_R1S_DEPTH2 2  // ring depth of the stage-2 form (A/B builds: tools/build_variant.sh)
#endif
#ifndef MIMI_R1S_DEPTH3
#define MIMI_R1S_DEPTH3 2  // ring depth of the stage-3 form
#endif
hipError_t launch_res1_stream(const GemmArgs& a, hipStream_t s, const char** kname) {
    if (!res1_stream_ok(a)) return hipErrorInvalidValue;
    if (a.K == 256) return run_res1_stream<256, MIMI_R1S_DEPTH3, 64>(a, s, kname);
    return run_res1_stream<128, MIMI_R1S_DEPTH2, 64>(a, s, kname);
}

}  // namespace mimi
