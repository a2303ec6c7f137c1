// Stage-2 residual block (C = 256, H = 128) as ONE kernel on fp16 planes, large batches (TF/modeling_mimi.py
// MimiResnetBlock.forward :299-312: y = x + conv_k1(ELU(conv_k3(ELU(x)))), then the down conv's ELU).
//
// The unfused path is three HBM round trips: the down conv before it writes fp32 x AND the ELU(x) planes (393 MB at
// B = 32 x 10 s), the k3 GEMM reads those and writes the hidden planes h (197 MB), the k1 GEMM reads h and the fp32
// x (the skip) and writes the y planes -- 0.25 + 0.23 ms per B = 32 step.  Here a workgroup of 16 waves takes a tile
// of 128 frames of one item, wave (g, hh) owning frames 16 g .. +15 and half of the columns of each conv:
//   1. k3 conv, K = 768 (tap-major, the planes GEMM's K-step order: 64-channel block, tap, 32-channel half):
//      64 of the 128 hidden channels per wave; its A fragments are built in registers from the
//      fp32 x rows (frame + tap - 2, 8 channels per lane: ELU, then the hi / lo fp16 split at the ELU(x) planes'
//      scale -- the values the down conv would have stored), two K steps ahead; the W3 planes stream through a
//      4-deep LDS-DMA ring.  The epilogue (bias, ELU, split at the h scale) writes h into an LDS image, never HBM.
//   2. k1 conv, K = 128: A = h from LDS, the W1 planes through a 2-deep ring; the epilogue adds the fp32 x skip
//      (L2-warm: the tile just read it), applies the ELU and stores the y planes.
// Every value is formed with the planes GEMMs' instruction sequence (16x16x32 MFMAs, their K order, mma_split's
// product order, the same epilogue expressions), so h, y and the codes are bitwise the unfused path's (batch 1 keeps
// it: too few tiles), and the ELU(x) / h maxima still go to their activation slots for the scale calibration.
#include "gemm_rows.h"

#ifndef RR_DIAG
#define RR_DIAG 0  // timing diagnostics (tools builds only; results garbage): 1 no ELU / split of x (raw bits), 2 no k1 + y
#endif             // epilogue, 4 no W3 refills

namespace mimi {

template <int C, int BM, int WN>
__global__ __launch_bounds__(BM / 16 * WN * 64) void resblock_rows_h16_kernel(ResRowsArgs p) {
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr int H = C / 2, NG = BM / 16, NW = NG * WN, BK = 32;  // NG row groups x WN column parts
    constexpr int K3 = 3 * C, KT3 = K3 / BK, KT1 = H / BK;
    constexpr int TN3 = H / 16 / WN, TN1 = C / 16 / WN;             // a wave's hidden / output tiles
    constexpr int S3 = 4, S1 = 2, PA = WN == 1 ? 2 : 1;
    constexpr int B3 = H * BK, B3STG = 2 * B3;  // halves: a W3 plane image / ring stage (H rows x 32)
    constexpr int B1 = C * BK, B1STG = 2 * B1;  // W1 (C rows x 32)
    constexpr int NP3 = 2 * H / 16, NP1 = 2 * C / 16;
    constexpr int PPW3 = (NP3 + NW - 1) / NW, PPW1 = (NP1 + NW - 1) / NW;
    constexpr int HS = H + 16;                   // h image row stride (halves): 288 B for H = 128, conflict-free reads
    constexpr int HIMG = BM * HS;                // halves per h plane image
    constexpr int LDE = 64 + 4;                  // epilogue staging row (floats)
    constexpr int RING3 = S3 * B3STG, RING1 = S1 * B1STG, STG = NW * 16 * LDE * 2;
    constexpr int RING = RING3 > RING1 ? (RING3 > STG ? RING3 : STG) : (RING1 > STG ? RING1 : STG);
    static_assert(C % 64 == 0 && H % 32 == 0 && BM % 16 == 0, "shape");
    static_assert((2 * HIMG + RING + 512) * 2 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) _Float16 lds[2 * HIMG + RING + 512];
    _Float16* const himg = lds;                  // [plane][BM][HS]
    _Float16* const ring = lds + 2 * HIMG;
    _Float16* const dummy = ring + RING;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = p.T;
    const int mtiles = (T + BM - 1) / BM, ntiles = mtiles * p.batch;
    const long long xbytes = (long long)p.batch * T * C * 4;
    const __amdgpu_buffer_rsrc_t xrs = make_rsrc(p.x, xbytes);
    const __amdgpu_buffer_rsrc_t w3rs = make_rsrc(p.w3, 2LL * H * K3 * 2);
    const __amdgpu_buffer_rsrc_t w1rs = make_rsrc(p.w1, 2LL * C * H * 2);
    const int prow = lane >> 2, pch = lane & 3;
    const float us3 = p.us3, us1 = p.us1, xs = p.xscale, hs = p.hscale, ys = p.yscale;
    float xmx = 0.0f, hmx = 0.0f, ymx = 0.0f;

    // the planes GEMM's K-step order of the k3 conv (gemm_kernel.h KOrderT, k = 3, s = 1): 64-channel block, tap,
    // 32-channel half -> (tap, first channel)
    auto k3_tap = [](int s) { return (s % 6) >> 1; };
    auto k3_ch = [](int s) { return (s / 6) * 64 + (s & 1) * 32; };

    // W3 / W1 ring pieces of this wave: piece j = plane j / (rows / 16), rows 16 (j % (rows / 16)) ..
    int w3off[PPW3], w3dst[PPW3], w1off[PPW1], w1dst[PPW1];
#pragma unroll
    for (int q = 0; q < PPW3; ++q) {
        const int j0 = wave + q * NW, j = j0 < NP3 ? j0 : wave;
        const int pl = j / (H / 16), nl = (j % (H / 16)) * 16 + prow;
        w3off[q] = (int)((((long long)pl * H + nl) * K3 + (pch ^ chunk_swz<BK, 16>(nl)) * 8) * 2);
        w3dst[q] = j0 < NP3 ? pl * B3 + (j % (H / 16)) * 16 * BK : -1;
    }
#pragma unroll
    for (int q = 0; q < PPW1; ++q) {
        const int j0 = wave + q * NW, j = j0 < NP1 ? j0 : wave;
        const int pl = j / (C / 16), nl = (j % (C / 16)) * 16 + prow;
        w1off[q] = (int)((((long long)pl * C + nl) * H + (pch ^ chunk_swz<BK, 16>(nl)) * 8) * 2);
        w1dst[q] = j0 < NP1 ? pl * B1 + (j % (C / 16)) * 16 * BK : -1;
    }
    // (the K-step byte offsets go in the scalar offset: a per-step VGPR sum was hoisted out of the tile loop for all
    // 24 steps and spilled)
    auto issue3 = [&](int s, int slot) {
        _Float16* st = ring + slot * B3STG;
        const int kb = (k3_tap(s) * C + k3_ch(s)) * 2;
#pragma unroll
        for (int q = 0; q < PPW3; ++q)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                w3rs, (__attribute__((address_space(3))) void*)(w3dst[q] >= 0 ? st + w3dst[q] : dummy), 16,
                w3off[q], kb, 0, 0);
    };
    auto issue1 = [&](int s, int slot) {
        _Float16* st = ring + slot * B1STG;
#pragma unroll
        for (int q = 0; q < PPW1; ++q)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                w1rs, (__attribute__((address_space(3))) void*)(w1dst[q] >= 0 ? st + w1dst[q] : dummy), 16,
                w1off[q], s * BK * 2, 0, 0);
    };

    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int b = tile / mtiles, m0 = (tile % mtiles) * BM;
        const int len = p.tlen ? p.tlen[b] : T;
        if (m0 >= len) continue;  // (ragged: past this item's frames; wave-uniform for the whole workgroup)
        const long long ibase = (long long)b * T;  // the item's first row
        // lane-derived values through an opaque copy per tile: otherwise every lane-only address / bias below is
        // hoisted out of the tile loop and held (spilled) across it
        int lanev = lane;
        asm volatile("" : "+v"(lanev));
        const int hsel = lanev >> 4, l16 = lanev & 15;
        const int g = wave % NG, hh = wave / NG;     // this wave's 16 frames and column part
        const int frow = m0 + g * 16 + l16;          // this lane's frame (A / k3 rows)
        // x fragment of K step s for this lane: 8 fp32 of row frow + tap - 2, channels ch + 8 hsel (the channel offset
        // in the scalar offset); rows before the item's start are the causal zero padding (of the ELU(x) planes): an
        // out-of-range offset loads 0
        int xo[3];
#pragma unroll
        for (int tap = 0; tap < 3; ++tap)
            xo[tap] = frow + tap - 2 >= 0 ? (int)(((ibase + frow + tap - 2) * C + hsel * 8) * 4) : (int)0x80000000;
        const bool rowok = frow < len;
        auto loadx = [&](int s, f32x4 (&v)[2]) {
            const int tap = k3_tap(s), cb = k3_ch(s) * 4;
            v[0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, xo[tap], cb, 0));
            v[1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, xo[tap], cb + 16, 0));
        };
        // ELU(x) planes of a fragment (the down conv epilogue's store_act8 split at the ELU(x) scale); the ELU(x)
        // maximum over this tile's own frames from the tap-2 steps (they cover every channel of every frame)
        auto xplanes = [&](int s, const f32x4 (&v)[2], bf16x8 (&a)[2]) {
            const bool own = k3_tap(s) == 2 && rowok;
            typedef _Float16 h8 __attribute__((ext_vector_type(8)));
            h8 hi, lo;
            if (RR_DIAG & 1) {
                a[0] = __builtin_bit_cast(bf16x8, v[0]);
                a[1] = __builtin_bit_cast(bf16x8, v[1]);
                return;
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float ev = elu1(v[e >> 2][e & 3]);
                if (own) xmx = fmaxf(xmx, fabsf(ev));
                const float tv = ev * xs;
                hi[e] = (_Float16)tv;
                lo[e] = (_Float16)(tv - (float)hi[e]);
            }
            a[0] = __builtin_bit_cast(bf16x8, hi);
            a[1] = __builtin_bit_cast(bf16x8, lo);
        };

        // ---- 1. k3 conv: acc3[j] = h tile j (hidden 16 j ..) of this wave's 16 frames
        f32x4 acc3[TN3];
#pragma unroll
        for (int j = 0; j < TN3; ++j) acc3[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        f32x4 xr[PA + 1][2];
#pragma unroll
        for (int i = -(S3 - 1); i < 0; ++i) {
            if (i + PA >= 0) loadx(i + PA, xr[i + PA]);
            if (i + S3 - 1 >= 0) issue3(i + S3 - 1, i + S3 - 1);
        }
        auto step3 = [&](int s, int sw, int sa, int san, int nwait, bool refA, bool refW) __attribute__((always_inline)) {
            vm_wait(nwait);
            __builtin_amdgcn_s_barrier();
            if (refA) loadx(s + PA, xr[san]);
            if (refW && !(RR_DIAG & 4)) issue3(s + S3 - 1, sw == 0 ? S3 - 1 : sw - 1);
            bf16x8 a[2];
            xplanes(s, xr[sa], a);
            const __bf16* Bs = reinterpret_cast<const __bf16*>(ring + sw * B3STG);
#pragma unroll
            for (int j = 0; j < TN3; ++j) {
                const int nl = hh * (H / WN) + j * 16 + l16;
                const int off = nl * BK + (hsel ^ chunk_swz<BK, 16>(nl)) * 8;
                const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(Bs + off);
                const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(Bs + B3 + off);
                acc3[j] = mfma16<true>(a[1], b0, acc3[j]);
                acc3[j] = mfma16<true>(a[0], b1, acc3[j]);
                acc3[j] = mfma16<true>(a[0], b0, acc3[j]);
            }
        };
        {
            constexpr int TAIL = S3 - 1, U = rows_lcm(S3, PA + 1);
            constexpr int NSTEADY = KT3 > TAIL ? (KT3 - TAIL) / U * U : 0;
            constexpr int NSS = rows_dma_after<S3, 1 << 20, PPW3>(0);
            for (int base = 0; base < NSTEADY; base += U) {
#pragma unroll
                for (int u = 0; u < U; ++u) step3(base + u, u % S3, u % (PA + 1), (u + PA) % (PA + 1), NSS, true, true);
            }
#pragma unroll
            for (int s = NSTEADY; s < KT3; ++s)
                step3(s, s % S3, s % (PA + 1), (s + PA) % (PA + 1), rows_dma_after<S3, KT3, PPW3>(s), s + PA < KT3,
                      s + S3 - 1 < KT3);
        }
        __syncthreads();  // the W3 ring is free (and every wave is past the previous tile's h reads)
        issue1(0, 0);     // W1 stage 0 loads under the h epilogue
        // ---- h epilogue (the k3 GEMM's EPI_BIAS_ELU + fp16 planes at the h scale), into the LDS image
#pragma unroll
        for (int j = 0; j < TN3; ++j) {
            const int col = hh * (H / WN) + j * 16 + l16;
            const float bias = p.b3[col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = g * 16 + 4 * hsel + r;
                const float v = elu1(acc3[j][r] * us3 + bias);
                if (m0 + row < len) hmx = fmaxf(hmx, fabsf(v));
                const float tv = v * hs;
                const _Float16 h0 = (_Float16)tv;
                const int pos = row * HS + col;
                himg[pos] = h0;
                himg[HIMG + pos] = (_Float16)(tv - (float)h0);
            }
        }
        if (RR_DIAG & 2) {
            if (hmx == 1234.5f) p.yamax[0] = 0u;
            __syncthreads();
            continue;
        }
        // ---- 2. k1 conv: acc1[j] = y tile j (channels 16 j ..) of this wave's frames
        f32x4 acc1[TN1];
#pragma unroll
        for (int j = 0; j < TN1; ++j) acc1[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KT1; ++s) {
            vm_wait(0);
            __syncthreads();  // (s = 0: the h image is complete) W1 stage s landed; stage s - 1 is free
            if (s + 1 < KT1) issue1(s + 1, (s + 1) % S1);
            const int apos = (g * 16 + l16) * HS + s * BK + hsel * 8;
            const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(himg + apos);
            const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(himg + HIMG + apos);
            const __bf16* Bs = reinterpret_cast<const __bf16*>(ring + (s % S1) * B1STG);
#pragma unroll
            for (int j = 0; j < TN1; ++j) {
                const int nl = hh * (C / WN) + j * 16 + l16;
                const int off = nl * BK + (hsel ^ chunk_swz<BK, 16>(nl)) * 8;
                const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(Bs + off);
                const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(Bs + B1 + off);
                acc1[j] = mfma16<true>(a1, b0, acc1[j]);
                acc1[j] = mfma16<true>(a0, b1, acc1[j]);
                acc1[j] = mfma16<true>(a0, b0, acc1[j]);
            }
        }
        __syncthreads();  // the W1 ring is free: epilogue staging
        // ---- y epilogue (the k1 GEMM's EPI_BIAS_RES_ELU + planes): phase 1 bias in the MFMA layout -> a wave-private
        // [16][LDE] fp32 tile per 64 channels; phase 2 lane -> frame lane / 8 (+ 8), channels 8 (lane % 8) ..: + x,
        // ELU, the y planes split, 16-B stores
        float* stg = reinterpret_cast<float*>(ring) + wave * 16 * LDE;
#pragma unroll
        for (int jp = 0; jp < C / WN / 64; ++jp) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int j = jp * 4 + jj;
                const float bias = p.b1[hh * (C / WN) + j * 16 + l16];
#pragma unroll
                for (int r = 0; r < 4; ++r) stg[(4 * hsel + r) * LDE + jj * 16 + l16] = acc1[j][r] * us1 + bias;
            }
            asm volatile("" ::: "memory");
#pragma unroll
            for (int hr = 0; hr < 2; ++hr) {
                const int lr = (lane >> 3) + 8 * hr, lc = (lane & 7) * 8;
                const int t = m0 + g * 16 + lr, col = hh * (C / WN) + jp * 64 + lc;
                if (t >= len) continue;
                const long long off = (ibase + t) * C + col;
                f32x4 v0 = *reinterpret_cast<const f32x4*>(stg + lr * LDE + lc);
                f32x4 v1 = *reinterpret_cast<const f32x4*>(stg + lr * LDE + lc + 4);
                const f32x4 r0 = *reinterpret_cast<const f32x4*>(p.x + off);
                const f32x4 r1 = *reinterpret_cast<const f32x4*>(p.x + off + 4);
                v0 = r0 + v0;  // R + (acc + bias): the reference's operation order
                v1 = r1 + v1;
                const float pv[8] = {elu1(v0.x), elu1(v0.y), elu1(v0.z), elu1(v0.w),
                                     elu1(v1.x), elu1(v1.y), elu1(v1.z), elu1(v1.w)};
                store_act8(p.yp, p.y_pstride, 2, off, pv, ys, &ymx);
            }
            asm volatile("" ::: "memory");
        }
        __syncthreads();  // staging reads done before the next tile's W3 stages land in the ring
    }
    amax_commit(p.xamax, xmx);
    amax_commit(p.hamax, hmx);
    amax_commit(p.yamax, ymx);
#endif
}

hipError_t launch_resblock_rows(int C, const ResRowsArgs& a, hipStream_t s, const char** kname) {
    if (C != 256 || a.batch <= 0 || a.T <= 0 || !a.x || !a.w3 || !a.w1 || !a.b3 || !a.b1 || !a.yp ||
        !(a.xscale > 0.0f) || !(a.hscale > 0.0f) || !(a.yscale > 0.0f))
        return hipErrorInvalidValue;
    if ((long long)a.batch * a.T * C * 4 > 0x7fffffffLL) return hipErrorInvalidValue;  // 32-bit buffer offsets
    constexpr int BM = 128, WN = 1;
    auto kern = resblock_rows_h16_kernel<256, BM, WN>;
    static int slots = 0;
    if (!slots) {
        int dev = 0, ncu = 256, occ = 1;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, BM / 16 * WN * 64, 0);
        slots = ncu * (occ > 0 ? occ : 1);
    }
    const long long ntiles = (long long)a.batch * ((a.T + BM - 1) / BM);
    hipLaunchKernelGGL(kern, dim3((unsigned)std::min<long long>(ntiles, slots)), dim3(BM / 16 * WN * 64), 0, s, a);
    if (kname) *kname = "mimi::resblock_rows_h16_kernel<256, 128, 1>";
    return hipGetLastError();
}

}  // namespace mimi
