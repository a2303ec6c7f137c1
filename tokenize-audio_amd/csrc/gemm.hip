// Implicit-GEMM Conv1d / Linear on fp32 MFMA (v_mfma_f32_32x32x2_f32) for gfx950.
//
// Every conv of the Mimi encoder (TF/modeling_mimi.py:210-347, causal MimiConv1d) and every dense
// projection of its transformer (:657-726, :602-615) is one GEMM over a channels-last activation:
//   out[t][co] = sum_{kk, ci} x[t*s - pad + kk][ci] * W'[co][kk*Cin + ci]
// With channels-last storage, row t of the im2col matrix is the CONTIGUOUS span
//   x_flat[(t*s - pad)*Cin, (t*s - pad + k)*Cin)
// so A is an ordinary row-major operand with row stride s*Cin (rows overlap in memory when k > s); no
// im2col buffer, no gather.  Causal left padding / right "extra" padding are bounds checks on that span.
//
// Tile: BM x BN x 32, WM x WN waves, each wave a (BM/WM) x (BN/WN) block of 32x32 MFMA tiles.
// Operands are staged global -> registers -> LDS ([row][32+4] fp32, +4 pad makes the ds_read_b128
// fragment reads conflict-free); the next K-slice's global loads are issued before the current slice's
// MFMAs so their latency hides under 64 * (BM/WM/32) * (BN/WN/32) MFMA cycles per wave.
// Fused prologue: ELU on A as it is written to LDS.  Fused epilogues: bias, ELU, residual add, GELU(erf),
// layer scale + residual, RoPE (rotate-half pairs (d, d+32) live in the same lane of tiles tn, tn+1).
#include <algorithm>
#include <cstdio>
#include <cstdlib>


#include "gemm_planes.h"

#ifndef MIMI_QKV_V
#define MIMI_QKV_V 1
#endif
#ifndef MIMI_FC1_V
#define MIMI_FC1_V 0
#endif
// the smallest small-grid tile (16 rows) at 16 x 32 with one compute wave instead of 16 x 64 with two, per role (bit 0
// o_proj, 1 final conv, 2 downsample, 3 input_proj): twice the workgroups on a batch-1 grid, the same instruction
// sequence per output element (codes and taps bitwise equal, r6f / r6g).  Per batch-1 encode (three alternations each,
// gpurun_out/r6f/ab.log, r6g/ab.log): o_proj 85-89 -> 80-82 us, final 27-29 -> 25, downsample 26-28 -> 23-25, input_proj
// equal; all four on: 10.14k -> 10.28k audio-s/s on the r6g box
#ifndef MIMI_SMALL16_32W
#define MIMI_SMALL16_32W 1  // (A/B) compute waves of the 16 x 32 small-grid tile: 1 (16 x 32 each) or 2 (16 x 16 each,
#endif                      // same bits; batch 1 equal within noise, o_proj 0.081 -> 0.084 ms: gpurun_out/r6j/ab.log)
#ifndef MIMI_SMALL16_32
#define MIMI_SMALL16_32 15
#endif


namespace mimi {

// ------------------------------------------------------------------------------------------------
// role -> instantiation
// ------------------------------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, int BK, int NBUF, bool NFAST, bool ELU_IN, int PAD, int EPI, int TAG>
static const char* kernel_symbol() {
    static thread_local char name[160];
    if (!name[0])
        snprintf(name, sizeof(name), "mimi::gemm_f32_kernel<%d, %d, %d, %d, %d, %d, %s, %s, %d, %d, %d>", BM, BN, WM,
                 WN, BK, NBUF, NFAST ? "true" : "false", ELU_IN ? "true" : "false", PAD, EPI, TAG);
    return name;
}

static thread_local const char* g_last_kernel = nullptr;

template <int BM, int BN, int WM, int WN, int BK, int NBUF, bool NFAST, bool ELU_IN, int PAD, int EPI, int TAG>
static hipError_t run(const GemmArgs& a, hipStream_t s) {
    g_last_kernel = kernel_symbol<BM, BN, WM, WN, BK, NBUF, NFAST, ELU_IN, PAD, EPI, TAG>();
    if (a.K % BK != 0) return hipErrorInvalidValue;
    dim3 grid((a.M + BM - 1) / BM, (a.N + BN - 1) / BN, a.batch);
    dim3 block(WM * WN * 64);
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, BK, NBUF, NFAST, ELU_IN, PAD, EPI, TAG>), grid, block, 0, s, a);
    return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int NS, bool ELU_IN, int PAD, int EPI, int TAG>
static hipError_t run_split(const GemmArgs& a, hipStream_t s) {
    static thread_local char name[160];
    if (!name[0])
        snprintf(name, sizeof(name), "mimi::gemm_bf16x_kernel<%d, %d, %d, %d, %d, %s, %d, %d, %d>", BM, BN, WM, WN, NS,
                 ELU_IN ? "true" : "false", PAD, EPI, TAG);
    g_last_kernel = name;
    if (a.K % 32 != 0 || !a.Wsplit) return hipErrorInvalidValue;
    dim3 grid((a.M + BM - 1) / BM, (a.N + BN - 1) / BN, a.batch);
    hipLaunchKernelGGL((gemm_bf16x_kernel<BM, BN, WM, WN, NS, ELU_IN, PAD, EPI, TAG>), grid, dim3(WM * WN * 64), 0, s,
                       a);
    return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int NS, int ST, int EPI, int OUTP, int TAG, int LW = 0, int BK = 32, int MF = 32,
          int FL = 0, bool F16 = false>
static hipError_t run_planes(const GemmArgs& a, hipStream_t s) {
    if constexpr (F16 && !(FL & (FL_RAGGED | FL_LNA))) {  // ragged batch: the same tile with per-item rows (gemm_planes.h)
        if (a.m_rows || a.a_rows) {
            if (!a.m_rows || !a.a_rows) return hipErrorInvalidValue;
            return run_planes<BM, BN, WM, WN, NS, ST, EPI, OUTP, TAG, LW, BK, MF, FL | FL_RAGGED, F16>(a, s);
        }
    }
    static thread_local char name[160];
    if (!name[0])
        snprintf(name, sizeof(name), "mimi::gemm_planes_kernel<%d, %d, %d, %d, %d, %d, %d, %d, %d, %d, %d, %d, %d, %s>", BM,
                 BN, WM, WN, NS, ST, EPI, OUTP, TAG, LW, BK, MF, FL, F16 ? "true" : "false");
    g_last_kernel = name;
    if (a.K % BK != 0 || !a.Wsplit || !a.Ap || ((OUTP & 7) && !a.Cp) || (!(OUTP & 7) && !a.C) ||
        ((OUTP & 8) && !a.C) || (EPI == EPI_BIAS_RES_ELU && !a.R))
        return hipErrorInvalidValue;
    if (a.a_len * 2 > 0x7fffffffLL) return hipErrorInvalidValue;  // buffer-resource byte offsets are 32-bit
    // the staged epilogue writes 8 consecutive outputs per lane (16-B vectors)
    if (a.N % 8 || a.ldc % 8 || a.c_bstride % 8 || a.c_pstride % 8) return hipErrorInvalidValue;
    const long long nwg = (long long)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN) * a.batch;
    if (nwg > 0x7fffffffLL) return hipErrorInvalidValue;
    if (F16 && ((OUTP & 7) ? a.out_scale <= 0.0f : false)) return hipErrorInvalidValue;
    if constexpr ((FL & FL_SC1OUT) != 0) {  // 32-bit byte offsets from an item's output base (gemm_planes.h)
        // an item's output rows are at most M (a ragged item's m_rows <= M; a batched item's base is c_base_of(b)
        // and its rows M), so M rows of ldc bound every sc1 store's offset from that base
        const long long rows = a.M;
        if ((rows * a.ldc + a.N) * 4 > 0x7fffffffLL || ((OUTP & 7) && (a.c_pstride + rows * a.ldc) * 2 > 0x7fffffffLL))
            return run_planes<BM, BN, WM, WN, NS, ST, EPI, OUTP, TAG, LW, BK, MF, FL & ~FL_SC1OUT, F16>(a, s);
    }
    auto kern = gemm_planes_kernel<BM, BN, WM, WN, NS, ST, EPI, OUTP, TAG, LW, BK, MF, FL, F16>;
    long long grid = nwg;
    if (FL & FL_PERSIST) {  // one workgroup per resident slot, a multiple of the 8 XCDs
        static const int slots = [kern] {  // (once per instantiation; thread-safe initialisation)
            int dev = 0, ncu = 256, occ = 1;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, (WM * WN + LW) * 64, 0);
            return std::max(8, ncu * std::max(1, occ) / 8 * 8);
        }();
        grid = std::min<long long>(nwg, slots);
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3((WM * WN + LW) * 64), 0, s, a);
    return hipGetLastError();
}

// Tiles of the planes kernel (tools/gemm_bench.hip; profiles/r1_gemm_bench_planes*.log, r1_gemm_bench_ws.log,
// r1_gemm_bench_f16.log):
//   big:    256x128, 8 compute waves, 2 stages (NS = 3; 3 at NS = 2), 144 KiB LDS: down convs, k3 convs, fc1
//   big_ld: 256x128, 4 compute waves of 128x64 + 4 loader waves (warp-specialised DMA): down_s3
//   small:  128x128, 8 compute waves of 32x64, 3 stages: final conv, q/k/v (M = B*250 rows)
//   small_ld: 128x128, 4 compute waves of 64x64 + 4 loader waves, 3 stages: o_proj, fc2
// fp16 planes (PREC_F16X3, 2 planes): 16x16x32 MFMAs; big = 256x128 x 3 stages (fc1, k3 convs; the down
// convs take run_planes_down_h16), small = 128x128 x 4 stages (q/k/v), small_ld = 128x128 x 4 stages with 4
// compute + 4 loader waves (o_proj, fc2, final conv).
template <int EPI, int OUTP3, int OUTP2, int TAG>
static hipError_t run_planes_big(const GemmArgs& a, hipStream_t s, int prec) {
    if (prec == PREC_F16X3) return run_planes<256, 128, 4, 2, 2, 3, EPI, OUTP2, TAG, 0, 32, 16, 0, true>(a, s);
    if (prec == PREC_BF16X6) return run_planes<256, 128, 4, 2, 3, 2, EPI, OUTP3, TAG>(a, s);
    return run_planes<256, 128, 4, 2, 2, 3, EPI, OUTP2, TAG>(a, s);
}
template <int EPI, int OUTP3, int OUTP2, int TAG>
static hipError_t run_planes_big_ld(const GemmArgs& a, hipStream_t s, int prec) {
    if (prec == PREC_F16X3) return run_planes<256, 128, 4, 2, 2, 3, EPI, OUTP2, TAG, 0, 32, 16, 0, true>(a, s);
    if (prec == PREC_BF16X6) return run_planes<256, 128, 2, 2, 3, 2, EPI, OUTP3, TAG, 4>(a, s);
    return run_planes<256, 128, 2, 2, 2, 3, EPI, OUTP2, TAG, 4>(a, s);
}
template <int EPI, int TAG>
static hipError_t run_planes_small(const GemmArgs& a, hipStream_t s, int prec) {
    if (prec == PREC_F16X3) return run_planes<128, 128, 4, 2, 2, 4, EPI, 0, TAG, 0, 32, 16, 0, true>(a, s);
    if (prec == PREC_BF16X6) return run_planes<128, 128, 4, 2, 3, 3, EPI, 0, TAG>(a, s);
    return run_planes<128, 128, 4, 2, 2, 3, EPI, 0, TAG>(a, s);
}
template <int EPI, int TAG>
static hipError_t run_planes_small_ld(const GemmArgs& a, hipStream_t s, int prec) {
    // fp16: 3 stages (o_proj / fc2 -2 %, final conv equal vs 4; profiles/r1l_ab_small_kernels.txt); 8 compute
    // waves instead of 4 (N = 512: 252 tiles, one round, so shorter per-tile chains win): o_proj -3 %, fc2 -1.4 %
    // (profiles/r2e_ab_8waves_oproj_fc2.log)
    if (prec == PREC_F16X3) {
        // (128 x 64 tiles, twice the workgroups: fc2 0.50 -> 0.61, o_proj 0.21 -> 0.23, final 0.088 -> 0.112 ms per B = 32
        // step, gpurun_out/r6h/ab.log)
        if (a.sc1) return run_planes<128, 128, 4, 2, 2, 3, EPI, 0, TAG, 4, 32, 16, FL_SC1OUT, true>(a, s);
        return run_planes<128, 128, 4, 2, 2, 3, EPI, 0, TAG, 4, 32, 16, 0, true>(a, s);
    }
    if (prec == PREC_BF16X6) return run_planes<128, 128, 2, 2, 3, 3, EPI, 0, TAG, 4>(a, s);
    return run_planes<128, 128, 2, 2, 2, 3, EPI, 0, TAG, 4>(a, s);
}

template <bool ELU_IN, int PAD, int EPI, int TAG>
static hipError_t run_prec(const GemmArgs& a, hipStream_t s, int prec);

// Tile choice by output width: N = 32 gets 256x32, N = 64 gets 256x64, wider gets 128x128; transformer-sized
// problems (M <= 1024 per item) use 64-row tiles to keep >1 workgroup per CU.
template <bool ELU_IN, int PAD, int EPI, int TAG>
static hipError_t run_auto(const GemmArgs& a, hipStream_t s) {
    if (a.N <= 32) return run<256, 32, 4, 1, 32, 1, false, ELU_IN, PAD, EPI, TAG>(a, s);
    if (a.N <= 64) return run<256, 64, 4, 1, 32, 1, false, ELU_IN, PAD, EPI, TAG>(a, s);
    if (a.M <= 1024) return run<64, 128, 1, 2, 32, 1, false, ELU_IN, PAD, EPI, TAG>(a, s);
    return run<128, 128, 2, 2, 32, 1, false, ELU_IN, PAD, EPI, TAG>(a, s);
}

static hipError_t dispatch(int role, const GemmArgs& a, hipStream_t s);

static thread_local int g_prec = PREC_F32;

template <bool ELU_IN, int PAD, int EPI, int TAG>
static hipError_t run_prec(const GemmArgs& a, hipStream_t s, int prec) {
    // fp32 activations in a split mode (downsample, or clips too long for the plane buffers): register split
    if (prec == PREC_BF16X6 || prec == PREC_F16X3) return run_split<128, 128, 2, 2, 3, ELU_IN, PAD, EPI, TAG>(a, s);
    if (prec == PREC_BF16X3) return run_split<128, 128, 2, 2, 2, ELU_IN, PAD, EPI, TAG>(a, s);
    return run_auto<ELU_IN, PAD, EPI, TAG>(a, s);
}

// Self-check of fc1's f16x3 GELU (gemm_kernel.h gelu_fast): out[i] = gelu_fast(in[i]).  Diagnostic entry
// mimi_gelu_check (tests/test_gelu.py compares it with float64 GELU and with torch's)
__global__ __launch_bounds__(256) void gelu_check_kernel(const float* __restrict__ in, long long n,
                                                         float* __restrict__ out) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) out[i] = gelu_fast(in[i]);
}
hipError_t launch_gelu_check(const float* in, long long n, float* out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const long long blocks = std::min<long long>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(gelu_check_kernel, dim3((unsigned)blocks), dim3(256), 0, st, in, n, out);
    return hipGetLastError();
}

hipError_t launch_gemm(int role, const GemmArgs& a, hipStream_t s, const char** kname, int precision) {
    if (a.K % 32 != 0 || a.a_cin % 4 != 0 || a.a_rs % 4 != 0 || a.M <= 0 || a.N <= 0 || a.batch <= 0)
        return hipErrorInvalidValue;
    if (a.Ap && (a.a_cin % 8 != 0 || a.a_rs % 8 != 0 || a.a_off % 8 != 0)) return hipErrorInvalidValue;  // 16-B chunks
    g_last_kernel = nullptr;
    g_prec = precision;
    hipError_t e = dispatch(role, a, s);
    if (kname) *kname = g_last_kernel ? g_last_kernel : "?";
    return e;
}

// A k = 2s conv in the KOrder chain layout (gemm_planes.h FL_PAIR): taps j, j + s read the same input lines
static bool pair_ok(const GemmArgs& a) {
    if (a.a_cin <= 0 || a.a_cin % 64 || a.K % a.a_cin || a.a_rs % a.a_cin) return false;
    const int k = a.K / a.a_cin, st = a.a_rs / a.a_cin;
    return st > 0 && k == 2 * st && a.K % 64 == 0;
}

// fp16 down convs: 256x128 tiles, tap-pair stages (2 x 67.6 KiB), A's LDS-DMA halved, issued by 4 loader
// waves beside the 8 compute waves: -4..-15 % against the 3-stage ring without loaders
// (profiles/r1j_gemm_bench_pair.log, r1j_gemm_bench_ld.log)
// Small grids (a batch of 1-4 utterances): when the default tile leaves fewer than kSmallGrid workgroups, the
// fp16 GEMMs switch to 64-row tiles of the SAME kernel family -- same MFMA shape (16x16x32), K step, K order,
// tap pairing and epilogue -- so every output element is produced by the identical instruction sequence and an
// utterance's codes do not depend on the batch it is encoded in (test_full_size_batch_properties compares B = 1
// against B = 32 bitwise).
constexpr long long kSmallGrid = 128;
static long long tiles(const GemmArgs& a, int bm, int bn) {
    return (long long)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn) * a.batch;
}

// ring depths of the small-grid down convs (ring depth changes only when bytes land, not the arithmetic).  Batch 1,
// one box, alternated twice (profiles/r6h1_ab_small_rings.txt): down_s3 6 vs 4 stages 0.050-0.051 vs 0.061 ms (8: 0.051),
// down_s2 3 vs 2 stages 0.034-0.036 vs 0.040 ms (down_s1 equal; 4: 0.048-0.049, slower); 10.43-10.46k -> 10.48-10.49k
#ifndef MIMI_DOWN_SMALL_ST
#define MIMI_DOWN_SMALL_ST 6  // long K (down_s3) at batch 1 (32x32 tiles), 2 pair stages per barrier
#endif
#ifndef MIMI_DOWN_SMALL2_ST
#define MIMI_DOWN_SMALL2_ST 3  // shorter K (down_s1 / s2), 1 pair stage per barrier
#endif
template <int EPI, int OUTP, int TAG>
static hipError_t run_planes_down_h16(const GemmArgs& a, hipStream_t s) {
    // small grids: long K (down_s3, K = 8192) retires 2 pair stages per barrier from a 4-deep ring (batch 1:
    // 100 -> 83 us in the engine; the same grouping made the K <= 3072 transformer GEMMs slower there although
    // faster in tools/gemm_bench.hip with warm caches, profiles/r2_gemm_bench_kg.log); shorter K: 2-stage ring
    if (pair_ok(a) && tiles(a, 256, 128) < kSmallGrid && a.K >= 4096) {
        // batch 1: 64x64 tiles leave 64 workgroups, each at its CU's LDS-DMA ceiling for 8192 / 64 pair stages;
        // 32x32 tiles spread the same stream over 256 CUs
        if (tiles(a, 64, 64) < 256)
            return run_planes<32, 32, 1, 2, 2, MIMI_DOWN_SMALL_ST, EPI, OUTP, TAG, 4, 32, 16, FL_PAIR | FL_KG2, true>(a, s);
        return run_planes<64, 64, 2, 2, 2, 4, EPI, OUTP, TAG, 4, 32, 16, FL_PAIR | FL_KG2, true>(a, s);
    }
    if (pair_ok(a) && tiles(a, 256, 128) < kSmallGrid)
        return run_planes<64, 64, 2, 2, 2, MIMI_DOWN_SMALL2_ST, EPI, OUTP, TAG, 4, 32, 16, FL_PAIR, true>(a, s);
    // fp32-only output (down_s0): the next tile's first stage loads under the epilogue (FL_PF: -2.6 %; with the
    // planes epilogues of down_s1 / s2 it costs +2..3 %, profiles/r2c_ab_pf_pair.log)
    constexpr int PF = OUTP == 0 ? FL_PF : 0;
    // (4 compute waves of 128 x 64 or 64 x 128 -- a third fewer LDS fragment reads per MFMA -- measured 5-6 % slower:
    // profiles/r5o_ab_down_4waves.txt)
    if (pair_ok(a)) return run_planes<256, 128, 4, 2, 2, 2, EPI, OUTP, TAG, 4, 32, 16, FL_PAIR | FL_PERSIST | PF, true>(a, s);
    return run_planes<256, 128, 4, 2, 2, 3, EPI, OUTP, TAG, 0, 32, 16, 0, true>(a, s);
}

// Small grids, f16x3 (fewer than kSmallGrid 128x128 tiles: 1-4 utterances): per role three tile sizes of the same
// kernel family -- 64, 32 and 16 rows -- and the largest one that still gives >= 256 workgroups (one per CU) runs,
// else the smallest.  These GEMMs are latency-bound at this size (a few K steps per microsecond per workgroup, each
// workgroup streaming its own A and W slices), so more, smaller tiles finish sooner even though they re-read more.
// Measured per role at B = 1 and B = 4 (profiles/r2d_ab_small_tiles.log): the rule picks the fastest of the three
// everywhere; B = 1: 7.3k -> 8.0k audio-s/s.
#ifndef MIMI_SMALL_ST
#define MIMI_SMALL_ST 4  // (A/B knob) ring depth of the small-grid tiles; 6 measured slower at batch 1 (q/k/v 0.109 ->
#endif                   // 0.137 ms per encode: fewer workgroups per CU fit, profiles/r6h1_ab_small_rings.txt)
#ifndef MIMI_LNA_ST
#define MIMI_LNA_ST 4  // (A/B knob) ring depth of the LayerNorm-prologue q/k/v and fc1 tiles
#endif
template <int EPI, int OUTP, int TAG, int BN0, int BM1, int BN1, int WM1, int WN1, int BN2, int WN2, int ST = MIMI_SMALL_ST,
          int FL = 0, int BM0 = 64, int WN0 = 2>
static hipError_t run_small_h16(const GemmArgs& a, hipStream_t s) {
    if (tiles(a, BM0, BN0) >= 256) return run_planes<BM0, BN0, 2, WN0, 2, ST, EPI, OUTP, TAG, 4, 32, 16, FL, true>(a, s);
    if (tiles(a, BM1, BN1) >= 256) return run_planes<BM1, BN1, WM1, WN1, 2, ST, EPI, OUTP, TAG, 4, 32, 16, FL, true>(a, s);
    return run_planes<16, BN2, 1, WN2, 2, ST, EPI, OUTP, TAG, 4, 32, 16, FL, true>(a, s);
}

// The LayerNorm prologue (FL_LNA, gemm_planes.h) replaces the LayerNorm launch in front of q/k/v and fc1 on the
// small grids: every tile recomputes its rows' LayerNorm (N / BN times per row), cheap beside a launch when the
// rows are few (batch 1-4), and its A image (BM x 2 KiB) fits beside the ring for the 16-64-row tiles.
bool gemm_ln_prologue_ok(int role, const GemmArgs& a, int precision) {
    return precision == PREC_F16X3 && (role == ROLE_QKV || role == ROLE_FC1) && a.K == 512 && a.a_rs == 512 &&
           a.a_off == 0 && !a.a_rows && !a.m_rows && !a.a_boff && tiles(a, 128, 128) < kSmallGrid;
}

static hipError_t dispatch_planes(int role, const GemmArgs& a, hipStream_t s) {
    const int prec = g_prec;
    if (prec != PREC_BF16X6 && prec != PREC_BF16X3 && prec != PREC_F16X3) return hipErrorInvalidValue;
    if (a.ln_x) {  // LayerNorm prologue: only where it is built (never silently dropped)
        if (!gemm_ln_prologue_ok(role, a, prec) || !a.ln_g || !a.ln_b || !(a.ln_scale > 0.0f)) return hipErrorInvalidValue;
        // the tile rule of run_small_h16 (q/k/v never reaches its 64-row tile on a small grid)
        if (role == ROLE_QKV) {
            if (tiles(a, 32, 128) >= 256) return run_planes<32, 128, 2, 2, 2, MIMI_LNA_ST, EPI_ROPE, 0, 5, 4, 32, 16, FL_LNA, true>(a, s);
            if (a.ln_tile == 1) return run_planes<32, 64, 2, 1, 2, MIMI_LNA_ST, EPI_ROPE, 0, 5, 4, 32, 16, FL_LNA, true>(a, s);
            if (a.ln_tile == 2) return run_planes<16, 128, 1, 2, 2, MIMI_LNA_ST, EPI_ROPE, 0, 5, 4, 32, 16, FL_LNA, true>(a, s);
            return run_planes<16, 64, 1, 1, 2, MIMI_LNA_ST, EPI_ROPE, 0, 5, 4, 32, 16, FL_LNA, true>(a, s);
        }
        if (tiles(a, 64, 64) >= 256) return run_planes<64, 64, 2, 2, 2, MIMI_LNA_ST, EPI_GELU, 2, 7, 4, 32, 16, FL_LNA, true>(a, s);
        // (16 x 64 tiles at batch 1 measured slower: fc1 0.142 -> 0.188 ms per encode, gpurun_out/r6f/ab.log)
        if (tiles(a, 32, 64) >= 256) return run_planes<32, 64, 2, 2, 2, MIMI_LNA_ST, EPI_GELU, 2, 7, 4, 32, 16, FL_LNA, true>(a, s);
        return run_planes<16, 64, 1, 2, 2, MIMI_LNA_ST, EPI_GELU, 2, 7, 4, 32, 16, FL_LNA, true>(a, s);
    }
#ifndef MIMI_SMALL_ROLES
#define MIMI_SMALL_ROLES 1
#endif
    // below one 128x128 workgroup per CU the small-grid tiles (the same MFMA sequence per output) run instead: the
    // quantizer's GEMMs (downsample, input_proj: M = B x 125 rows, N = 512) leave half the CUs idle up to B = 63 on
    // 128x128 tiles (0.079 + 0.025 -> 0.056 + 0.018 ms per B = 32 step, profiles/r4ak_ab_quantizer_tiles.txt)
    const bool qsmall = tiles(a, 128, 128) < 256 &&
                        (((MIMI_SMALL_ROLES & 1) && (role == ROLE_DOWNSAMPLE || role == ROLE_INPROJ)) ||
                         ((MIMI_SMALL_ROLES & 2) && role == ROLE_OPROJ) || ((MIMI_SMALL_ROLES & 4) && role == ROLE_FC2) ||
                         ((MIMI_SMALL_ROLES & 8) && role == ROLE_FINAL));
    if (prec == PREC_F16X3 && (tiles(a, 128, 128) < kSmallGrid || qsmall)) {
        // <EPI, OUTP, TAG, 64-row BN, 32-row BM x BN / waves, 16-row BN / waves>; 16 x 16 wave tiles are too small for
        // the staged epilogue (64 lanes x 8 columns), and RoPE needs 64 columns per wave
        switch (role) {
            case ROLE_FINAL:
                if (MIMI_SMALL16_32 & 2) return run_small_h16<EPI_BIAS_OUT, 0, 4, 64, 32, 64, 2, 2, 32, MIMI_SMALL16_32W>(a, s);
                return run_small_h16<EPI_BIAS_OUT, 0, 4, 64, 32, 64, 2, 2, 64, 2>(a, s);
            case ROLE_QKV: return run_small_h16<EPI_ROPE, 0, 5, 128, 32, 128, 2, 2, 64, 1>(a, s);
            case ROLE_OPROJ:
                if (MIMI_SMALL16_32 & 1) return run_small_h16<EPI_SCALE_RES, 0, 6, 64, 32, 64, 2, 2, 32, MIMI_SMALL16_32W>(a, s);
                return run_small_h16<EPI_SCALE_RES, 0, 6, 64, 32, 64, 2, 2, 64, 2>(a, s);
            case ROLE_FC1: return run_small_h16<EPI_GELU, 2, 7, 64, 32, 64, 2, 2, 64, 2>(a, s);
            case ROLE_FC2:  // K = 2048: 6-deep rings retired 2 stages per barrier (-14 % at batch 1, profiles/r2c_ab_b1.log)
                if (a.Cp)  // the last layer: fp32 residual stream + its planes (the downsample's input)
                    return run_small_h16<EPI_SCALE_RES, 2, 8, 32, 32, 32, 1, 2, 32, MIMI_SMALL16_32W, 6, FL_KG2>(a, s);
                return run_small_h16<EPI_SCALE_RES, 0, 8, 32, 32, 32, 1, 2, 32, MIMI_SMALL16_32W, 6, FL_KG2>(a, s);
            case ROLE_DOWNSAMPLE:  // zero-padded here; engine.cpp adds the replicate rows (launch_ds_edge_fix)
                if (MIMI_SMALL16_32 & 4) return run_small_h16<EPI_NONE, 2, 9, 64, 32, 64, 2, 2, 32, MIMI_SMALL16_32W>(a, s);
                return run_small_h16<EPI_NONE, 2, 9, 64, 32, 64, 2, 2, 64, 2>(a, s);
            case ROLE_INPROJ:
                if (MIMI_SMALL16_32 & 8) return run_small_h16<EPI_NONE, 0, 10, 64, 32, 64, 2, 2, 32, MIMI_SMALL16_32W>(a, s);
                return run_small_h16<EPI_NONE, 0, 10, 64, 32, 64, 2, 2, 64, 2>(a, s);
            case ROLE_RES3P: return run_small_h16<EPI_BIAS_ELU, 2, 12, 64, 32, 64, 2, 2, 64, 2, 3>(a, s);
            default: break;
        }
    }
    if (prec == PREC_F16X3) {
        switch (role) {
            case ROLE_FC2:
                if (a.Cp) return run_planes<128, 128, 4, 2, 2, 3, EPI_SCALE_RES, 2, 8, 4, 32, 16, 0, true>(a, s);
                break;
            case ROLE_DOWNSAMPLE: return run_planes<128, 128, 4, 2, 2, 2, EPI_NONE, 2, 9, 0, 32, 16, 0, true>(a, s);
            case ROLE_INPROJ: return run_planes<128, 128, 4, 2, 2, 2, EPI_NONE, 0, 10, 0, 32, 16, 0, true>(a, s);
            default: break;
        }
        switch (role) {
            case ROLE_DOWN: return run_planes_down_h16<EPI_BIAS, 0, 2>(a, s);
            case ROLE_DOWN_ELU: return run_planes_down_h16<EPI_BIAS_ELU, 2, 3>(a, s);
            case ROLE_DOWN_XE: return run_planes_down_h16<EPI_BIAS, 2 | 8, 11>(a, s);
            default: break;
        }
    }
    switch (role) {
        case ROLE_DOWN: return run_planes_big<EPI_BIAS, 0, 0, 2>(a, s, prec);
        case ROLE_DOWN_ELU: return run_planes_big_ld<EPI_BIAS_ELU, 3, 2, 3>(a, s, prec);  // planes out: final conv
        case ROLE_FINAL: return run_planes_small_ld<EPI_BIAS_OUT, 4>(a, s, prec);
        case ROLE_QKV:  // fp16: persistent 128x128 tiles (M = 250 rows per item: 768 tiles, 1.5 rounds of a
                        // non-persistent grid) on a 3-stage ring fed by 4 loader waves, the next tile's first stages
                        // loading under the RoPE epilogue: 0.503 -> 0.485 ms per B = 32 step vs the 2-stage
                        // non-persistent ring (profiles/r3c_ab_qkv_fc1.log; the same for fc1 measured +6 %)
            if (prec == PREC_F16X3) {
#if MIMI_QKV_V == 1
                if (a.sc1)
                    return run_planes<128, 128, 4, 2, 2, 3, EPI_ROPE, 0, 5, 4, 32, 16, FL_PERSIST | FL_PF | FL_SC1OUT, true>(a, s);
                return run_planes<128, 128, 4, 2, 2, 3, EPI_ROPE, 0, 5, 4, 32, 16, FL_PERSIST | FL_PF, true>(a, s);
#elif MIMI_QKV_V == 2
                return run_planes<128, 128, 4, 2, 2, 2, EPI_ROPE, 0, 5, 0, 32, 16, 0, true>(a, s);
#else
                return run_planes<128, 128, 4, 2, 2, 2, EPI_ROPE, 0, 5, 4, 32, 16, 0, true>(a, s);
#endif
            }
            return run_planes_small<EPI_ROPE, 5>(a, s, prec);  // (256x256: -11 % alone, 0 in the engine)
        case ROLE_OPROJ:
            return run_planes_small_ld<EPI_SCALE_RES, 6>(a, s, prec);
        case ROLE_FC1:  // planes out: fc2; fp16: 128x128 on a 2-stage ring (two workgroups per CU): -4 % vs
                        // 256x256 x 2 stages, which beat 256x128 x 3 by 8-11 % (profiles/r1j_gemm_bench_256.log,
                        // r1l_ab_small_kernels.txt)
            // (256x128 persistent tiles with FL_PF: -8 % in tools/gemm_bench.hip, +5 % in the engine with the GELU
            // planes epilogue -- profiles/r2c_gemm_bench_pf.log, r2c_ab_fc1.log)
            if (prec == PREC_F16X3) {
#if MIMI_FC1_V == 1  // (+6 % again in round 6 with the cheaper GELU epilogue, profiles/r6g3_ab_fc_rings.txt)
                return run_planes<128, 128, 4, 2, 2, 3, EPI_GELU, 2, 7, 4, 32, 16, FL_PERSIST | FL_PF, true>(a, s);
#else
                if (a.sc1) return run_planes<128, 128, 4, 2, 2, 2, EPI_GELU, 2, 7, 0, 32, 16, FL_SC1OUT, true>(a, s);
                return run_planes<128, 128, 4, 2, 2, 2, EPI_GELU, 2, 7, 0, 32, 16, 0, true>(a, s);
#endif
            }
            return run_planes_big<EPI_GELU, 3, 2, 7>(a, s, prec);
        case ROLE_FC2:
#ifdef MIMI_FC2_ST  // (A/B knob) fc2's ring depth / flags on large grids (K = 2048, one 128 x 128 tile per CU):
                    // 4 / 5 stages and 4 stages x 2 per barrier measured 2 / 3 / 10 % slower (profiles/r6g3_ab_fc_rings.txt)
            if (prec == PREC_F16X3 && !a.sc1)
                return run_planes<128, 128, 4, 2, 2, MIMI_FC2_ST, EPI_SCALE_RES, 0, 8, 4, 32, 16, MIMI_FC2_FL, true>(a, s);
#endif
            return run_planes_small_ld<EPI_SCALE_RES, 8>(a, s, prec);
        case ROLE_DOWN_XE: return run_planes_big<EPI_BIAS, 3 | 8, 2 | 8, 11>(a, s, prec);
        case ROLE_RES3P:  // fp16: 256x128 on a 3-stage ring fed by 4 loader waves: -8 / -13 % vs 128x128 x 2
            if (prec == PREC_F16X3)  // without loaders (stage 2 / 3, profiles/r2c_ab_dispatch.log)
                return run_planes<256, 128, 4, 2, 2, 3, EPI_BIAS_ELU, 2, 12, 4, 32, 16, 0, true>(a, s);
            return run_planes_big<EPI_BIAS_ELU, 3, 2, 12>(a, s, prec);
        case ROLE_RES1P:  // K = C/2 = 128 / 256: short K, output-heavy
            if (prec == PREC_F16X3) {  // fp16: 128x128 x 8 waves on a 2-stage ring (64 KiB, two workgroups per CU):
                                       // -18 % vs 128x64 x 4 waves (profiles/r2c_ab_dispatch.log); + 4 loader
                                       // waves: -4..-5 % (profiles/r2e_ab_loaders_res1.log)
                // (round 5 A/B at B = 32 x 10 s, res1_s2 / res1_s3 ms per step, profiles/r5a_ab_res1p.txt: this tile
                // 0.229 / 0.108; persistent + next-tile prefetch 0.263 / 0.119; 256x128 0.258 / 0.110; 128x256
                // 0.253 / 0.111; sc1 stores 0.227 / 0.106; 3 stages 0.300 / 0.127; 64x128 0.270 / 0.129; persistent
                // 0.264 / 0.122.  Stage 2 runs res1_stream.hip)
                return run_planes<128, 128, 4, 2, 2, 2, EPI_BIAS_RES_ELU, 2, 13, 4, 32, 16, 0, true>(a, s);
            }
            if (prec == PREC_BF16X6) return run_planes<128, 64, 2, 2, 3, 2, EPI_BIAS_RES_ELU, 3, 13>(a, s);
            return run_planes<128, 64, 2, 2, 2, 2, EPI_BIAS_RES_ELU, 2, 13>(a, s);
        default: return hipErrorInvalidValue;
    }
}

static hipError_t dispatch(int role, const GemmArgs& a, hipStream_t s) {
    if (a.Ap) return dispatch_planes(role, a, s);
    switch (role) {
        case ROLE_DOWN: return run_prec<false, PAD_ZERO, EPI_BIAS, 2>(a, s, g_prec);
        case ROLE_DOWN_ELU: return run_prec<false, PAD_ZERO, EPI_BIAS_ELU, 3>(a, s, g_prec);
        case ROLE_FINAL: return run_prec<false, PAD_ZERO, EPI_BIAS_OUT, 4>(a, s, g_prec);
        case ROLE_QKV:
            if (g_prec == PREC_BF16X6 || g_prec == PREC_F16X3) return run_split<128, 128, 2, 2, 3, false, PAD_ZERO, EPI_ROPE, 5>(a, s);
            if (g_prec == PREC_BF16X3) return run_split<128, 128, 2, 2, 2, false, PAD_ZERO, EPI_ROPE, 5>(a, s);
            return run<64, 128, 1, 2, 32, 1, false, false, PAD_ZERO, EPI_ROPE, 5>(a, s);
        case ROLE_OPROJ: return run_prec<false, PAD_ZERO, EPI_SCALE_RES, 6>(a, s, g_prec);
        case ROLE_FC1: return run_prec<false, PAD_ZERO, EPI_GELU, 7>(a, s, g_prec);
        case ROLE_FC2: return run_prec<false, PAD_ZERO, EPI_SCALE_RES, 8>(a, s, g_prec);
        case ROLE_DOWNSAMPLE:  // small grids: 64x64 tiles, same 32x32 MFMA sequence per output (see kSmallGrid)
            if ((g_prec == PREC_BF16X6 || g_prec == PREC_F16X3) && tiles(a, 128, 128) < kSmallGrid)
                return run_split<64, 64, 1, 2, 3, false, PAD_REPLICATE, EPI_NONE, 9>(a, s);
            return run_prec<false, PAD_REPLICATE, EPI_NONE, 9>(a, s, g_prec);
        case ROLE_INPROJ: return run_auto<false, PAD_ZERO, EPI_NONE, 10>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mimi
