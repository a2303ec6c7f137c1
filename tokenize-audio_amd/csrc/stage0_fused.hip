// Stage 0 fused with down conv 0 (PREC_F16X3).  A file of its own: built with -fno-slp-vectorize (Makefile), since
// packed f32 VALU issues slowly beside the conv waves' MFMAs (MI355X_MICROARCH.md, per-instruction constants).
#include <type_traits>

#include "resblock_h16.h"

namespace mimi {

// ------------------------------------------------------------------------------------------------
// Stage 0 with its down conv fused (PREC_F16X3): conv0 + residual block + ELU (resblock0_h16_kernel's per-block
// arithmetic, unchanged) and down conv 0 (64 -> 128, k = 8, s = 4, TF/modeling_mimi.py:269-279 padding) in one
// persistent kernel, so y -- the block's output, 2 fp16 planes, 4 B per channel-step -- never leaves the CU.
// The codes are bit-identical to the unfused pair: every y plane value is resblock0_h16_kernel's, and every
// down-conv MFMA (operand fragments, K-step order, product order) is the planes GEMM's (gemm_planes.h, FL_PAIR
// K order: tap j, then j + 4, per 32-channel half; products lo.hi, hi.lo, hi.hi).
//
// One workgroup of 12 waves per CU (3 per SIMD, <= 168 VGPRs each), two roles meeting at one barrier per round:
//   4 block waves (one per SIMD) -- each walks its own contiguous range of 32-step blocks, one per round: the
//      block (conv0 -> slab -> GEMM1 -> h -> GEMM2 -> y) with y, zeroed past the item's end, written to section
//      w of y buffer n % 2 (rows 4..35; rows 0..3 = the 4 causal halo steps: the same section's rows 32..35 of
//      buffer (n-1) % 2, zeros at t = 0) + a descriptor (item, first 6 kHz step, rows to store)
//   8 conv waves -- the down conv of round n-1's 4 sections (32 output steps, 8 per section) for 16 output
//      channels each: 16 K steps x 2 tiles x 3 products of v_mfma_f32_16x16x32_f16, y fragments from buffer
//      (n-1) % 2, the weights (16 channels x 512 k x 2 planes = 128 VGPRs) resident in registers.  Transposed (W
//      is the A operand): a lane's accumulator is 4 consecutive channels of one step -> one 16-B fp32 store
// so a SIMD runs one block wave (VALU-heavy: ELU, plane splits) beside two conv waves (MFMA + LDS only).  A block
// wave whose range starts inside an item first recomputes the preceding block (round 0: its y only feeds the
// halo; nothing is stored for it).
// y buffer [plane][section 4][36 rows][72 halves] + 32 B between sections, 16-B chunk c of row r at c ^ 2 (r & 1):
// the block waves' row writes (ds_write_b64) and the conv waves' fragment reads (ds_read_b128) are conflict-free.
// LDS: block weights 36 KB + biases + 4 x 9.75 KB slabs + 2 x 40.75 KB y buffers = 157.3 KB.
// ------------------------------------------------------------------------------------------------
#ifndef S0F_HELP
#define S0F_HELP 1  // the conv waves (idle ~2.9k of the 10.7k-cycle round) split the next round's audio window into
#endif              // planes and copy each section's y halo, off the block waves' chain (0: the block waves do both;
                    // same bits, stage 0 1.29 / 1.29 / 1.30 -> 1.28 / 1.27 / 1.29 ms alternated, gpurun_out/r6o/ab.log)
#ifndef S0F_DIAG
#define S0F_DIAG 0  // tuning diagnostics (results are garbage): 1 = conv waves skip their MFMAs, 2 = block waves skip
#endif              // their blocks, 3 = block waves without the explicit LDS drains (s_waitcnt lgkmcnt(0))
#if S0F_DIAG == 3
#define S0F_DRAIN() asm volatile("" ::: "memory")
#else
#define S0F_DRAIN() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#endif
namespace s0f {
constexpr int NA = 4, NC = 8, NW = NA + NC;  // block waves, conv waves
constexpr int YLD = 72, YSR = 36, YSS = YSR * YLD + 16, YPS = 4 * YSS, YBS = 2 * YPS;  // halves
constexpr int OFF_SLAB = r0h::NFRAG * 1024 + r0h::BIAS * 4;
constexpr int OFF_Y = OFF_SLAB + NA * r0h::WAVE_BYTES;
constexpr int OFF_D = OFF_Y + 2 * YBS * 2;
constexpr int OFF_A2 = OFF_D + 2 * NA * 16 + 16;  // (S0F_HELP) audio plane images [block wave][round parity 2][2][AUD]
constexpr int LDS_BYTES = OFF_A2 + (S0F_HELP ? NA * 2 * 2 * r0h::AUD * 2 : 0);
static_assert(OFF_SLAB % 16 == 0 && OFF_Y % 16 == 0 && (YSS * 2) % 16 == 0, "16-B alignment");
static_assert(LDS_BYTES <= 160 * 1024, "LDS");
static_assert(NC * 16 == 128, "conv waves x 16 channels = down conv 0's output channels");
}  // namespace s0f

#if S0F_STAMP  // in-kernel phase stamps (tuning): per-wave cycle sums printed by workgroup 0 of large launches
#define S0F_T0() unsigned long long st_last = __builtin_readcyclecounter(), st_acc[6] = {0, 0, 0, 0, 0, 0}
#define S0F_T(i)                                                  \
    do {                                                          \
        const unsigned long long now_ = __builtin_readcyclecounter(); \
        st_acc[i] += now_ - st_last;                              \
        st_last = now_;                                           \
    } while (0)
#define S0F_TPRINT(tag)                                                                                         \
    if (blockIdx.x == 0 && lane == 0 && R > 64)                                                                 \
    printf("s0f %s wave %d rounds %d: %llu %llu %llu %llu %llu %llu\n", tag, wave, R, st_acc[0], st_acc[1],     \
           st_acc[2], st_acc[3], st_acc[4], st_acc[5])
#else
#define S0F_T0()
#define S0F_T(i)
#define S0F_TPRINT(tag)
#endif
__global__ __launch_bounds__(768) void stage0_fused_h16_kernel(ResArgs p) {
    using namespace r0h;
    constexpr int YLD = s0f::YLD, YSS = s0f::YSS, YPS = s0f::YPS, YBS = s0f::YBS, NA = s0f::NA;
    __shared__ __attribute__((aligned(16))) char lds[s0f::LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    {
        const uint4* src = reinterpret_cast<const uint4*>(p.wh16);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (int i = tid; i < NFRAG * 64; i += s0f::NW * 64) dst[i] = src[i];
        float* bw = reinterpret_cast<float*>(lds + NFRAG * 1024);
        if (tid < 64) {
            bw[tid] = p.b0[tid];
            bw[96 + tid] = p.b1[tid];
        }
        if (tid < 32) bw[64 + tid] = p.b3[tid];
    }
    _Float16* ybase = reinterpret_cast<_Float16*>(lds + s0f::OFF_Y);
    int4* desc = reinterpret_cast<int4*>(lds + s0f::OFF_D);  // [buffer 2][section 4]: item, first step, rows
    int* rcount = reinterpret_cast<int*>(lds + s0f::OFF_D + 2 * NA * 16);

    const long long T = p.T;
    const unsigned tpi = (unsigned)((T + 31) >> 5);
    const unsigned long long NT = p.istart ? p.istart[p.batch] : (unsigned long long)tpi * p.batch;
    const unsigned long long NWT = (unsigned long long)gridDim.x * NA;
    // block wave w's range of blocks [g0, g1) (the conv waves compute it too, for the round count)
    auto range = [&](int w, unsigned& g0, unsigned& g1) {
        const unsigned long long wid = (unsigned long long)blockIdx.x * NA + w;
        g0 = (unsigned)(wid * NT / NWT);
        g1 = (unsigned)((wid + 1) * NT / NWT);
    };
    if (wave < NA) {
        unsigned g0, g1;
        range(wave, g0, g1);
        TileWalk tw(p, tpi, g0);
        if (lane == 0) {
            rcount[wave] = (int)(g1 - g0) + ((g0 < g1 && tw.t0 > 0) ? 1 : 0);
            desc[NA + wave] = make_int4(0, 0, 0, 0);  // round 0's conv (buffer 1) stores nothing
        }
    }
    __syncthreads();
    int R = 0;
#pragma unroll
    for (int w = 0; w < NA; ++w) R = max(R, rcount[w]);
    // global (not flat) loads: a flat load in flight also holds lgkmcnt, so every LDS drain would wait for HBM
    const __attribute__((address_space(1))) float* __restrict__ audio =
        (const __attribute__((address_space(1))) float*)io_pointer(p.audio_ref, p.audio);
    [[maybe_unused]] _Float16* aud2 = reinterpret_cast<_Float16*>(lds + s0f::OFF_A2);  // (S0F_HELP) [wave][parity][hi | lo]

    if (wave >= NA) {
        // ---------------- conv waves: output channels co0 .. co0 + 15 ----------------
        const int co0 = 16 * (wave - NA);
        const int c16 = lane & 15, kq = lane >> 4;
        // wr[K step s][plane] = the planes GEMM's B fragment (channel lane & 15, k chunk lane >> 4) of K step
        // s = 4 j + 2 lo + img: tap j + 4 img, input channels 32 lo .. 32 lo + 31
        f16x8 wr[16][2];
        {
            const _Float16* wd = reinterpret_cast<const _Float16*>(p.wdown);
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                const int tap = (s >> 2) + 4 * (s & 1), lo = (s >> 1) & 1;
#pragma unroll
                for (int pl = 0; pl < 2; ++pl)
                    wr[s][pl] = *reinterpret_cast<const f16x8*>(wd + (long long)(pl * 128 + co0 + c16) * 512 + tap * 64 +
                                                                32 * lo + 8 * kq);
            }
        }
        const f32x4 bd = *reinterpret_cast<const f32x4*>(p.bdown + co0 + 4 * kq);
        const float ud = p.unscale_d;
        // output tile i: channels co0 + 4 kq + r (acc row) x 6 kHz step 16 i + (lane & 15) of the round = section
        // 2 i + sec_l, step rho of that section (acc column)
        const int sec_l = (lane >> 3) & 1, rho = lane & 7;
#if S0F_HELP
        // helper work for block wave hw = (wave - NA) / 2, walking its blocks: the even conv wave splits the audio
        // window of its next round's block into aud2 (planes as the block wave's conv0 reads them), the odd one
        // copies the section's y halo (rows 0..3 = rows 32..35 of the previous round's y, zeros at t = 0)
        const int hw = (wave - NA) >> 1, hrole = (wave - NA) & 1;
        unsigned hg0, hg1;
        range(hw, hg0, hg1);
        TileWalk htw(p, tpi, hg0);
        const int hhs = (hg0 < hg1 && htw.t0 > 0) ? 1 : 0;
        htw.t0 -= 32 * hhs;
        const int hRw = (int)(hg1 - hg0) + hhs;
        float mxa = 0.0f;
        auto haload = [&]() {
            const long long pos = htw.t0 - 8 + lane;
            const bool ok = lane < AUD && pos >= 0 && pos < htw.Tb;
            const float v = audio[ok ? (long long)htw.b * T + pos : 0];
            return ok ? v : 0.0f;
        };
        auto hsplit = [&](int n, float av) {  // the block wave's conv0 operand image for its round-n block
            if (lane < AUD) {
                mxa = fmaxf(mxa, fabsf(av));
                unsigned hw_, lw_;
                split2_f16s(av, 0.0f, p.ascale, hw_, lw_);
                _Float16* im = aud2 + (hw * 2 + (n & 1)) * (2 * AUD);
                im[lane] = __builtin_bit_cast(f16x2, hw_)[0];
                im[AUD + lane] = __builtin_bit_cast(f16x2, lw_)[0];
            }
        };
        const int hrow_ = (lane >> 3) & 3;
        const int hoff_ = (lane >> 5) * YPS + hw * YSS + hrow_ * YLD + 8 * ((lane & 7) ^ ((hrow_ & 1) * 2));
        float hnext = 0.0f;
        if (hrole == 0 && hRw > 0) {
            hsplit(0, haload());
            htw.next();
            if (hRw > 1) hnext = haload();
        }
        __syncthreads();  // round 0's audio images
#endif
        S0F_T0();
        for (int n = 0; n <= R; ++n) {
#if S0F_HELP
            if (hrole == 1 && n < hRw) {  // y halo of this round's section hw (the block wave writes rows 4..35)
                uint4 v = make_uint4(0u, 0u, 0u, 0u);
                if (htw.t0 > 0) v = *reinterpret_cast<const uint4*>(ybase + ((n + 1) & 1) * YBS + hoff_ + 32 * YLD);
                *reinterpret_cast<uint4*>(ybase + (n & 1) * YBS + hoff_) = v;
                htw.next();
            }
#endif
            if (n > 0) {
                const _Float16* yb = ybase + ((n + 1) & 1) * YBS;
                const int4* dsc = desc + ((n + 1) & 1) * NA;
                f32x4 acc[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) acc[i] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int s = 0; s < 16; ++s) {
                    const int tap = (s >> 2) + 4 * (s & 1), lo = (s >> 1) & 1;
                    const int row = 4 * rho + tap, ch = 4 * lo + kq;  // y step 4 (t1_0 + rho) - 4 + tap
                    const int o = row * YLD + 8 * (ch ^ ((row & 1) * 2));
                    f16x8 yf[2][2];
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int pl = 0; pl < 2; ++pl)
                            yf[pl][i] = *reinterpret_cast<const f16x8*>(yb + pl * YPS + (2 * i + sec_l) * YSS + o);
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        if (S0F_DIAG == 1) continue;
                        acc[i] = mfma_h16(wr[s][0], yf[1][i], acc[i]);  // y_lo w_hi
                        acc[i] = mfma_h16(wr[s][1], yf[0][i], acc[i]);  // y_hi w_lo
                        acc[i] = mfma_h16(wr[s][0], yf[0][i], acc[i]);  // y_hi w_hi
                    }
                }
                S0F_T(0);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int4 d = dsc[2 * i + sec_l];
                    if (rho < d.z) {
                        f32x4 v;
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] = acc[i][r] * ud + bd[r];  // the planes GEMM's EPI_BIAS
                        *reinterpret_cast<f32x4*>(p.xout + ((long long)d.x * p.T1 + d.y + rho) * 128 + co0 + 4 * kq) = v;
                    }
                }
                S0F_T(1);
            }
#if S0F_HELP
            if (hrole == 0 && n + 1 < hRw) {  // the next round's audio image (loaded a round ahead)
                hsplit(n + 1, hnext);
                htw.next();
                if (n + 2 < hRw) hnext = haload();
            }
#endif
            __syncthreads();
            S0F_T(2);
        }
        S0F_TPRINT("conv");
#if S0F_HELP
        amax_commit(p.aamax, mxa);
#endif
        return;
    }

    // ---------------- block waves ----------------
#ifdef S0F_PRIO
    __builtin_amdgcn_s_setprio(S0F_PRIO);  // the block waves' dependent chain is the critical path
#endif
    const f16x8* wf = reinterpret_cast<const f16x8*>(lds);
    const float* bl = reinterpret_cast<const float*>(lds + NFRAG * 1024);
    _Float16* slab = reinterpret_cast<_Float16*>(lds + s0f::OFF_SLAB + wave * WAVE_BYTES);
    _Float16* hb = slab + 2 * SLD;
    float* aud = reinterpret_cast<float*>(slab + 2 * SPL);
    unsigned g0, g1;
    range(wave, g0, g1);
    TileWalk tw(p, tpi, g0);
    const int hstart = (g0 < g1 && tw.t0 > 0) ? 1 : 0;  // range starts inside an item: recompute the block before
    tw.t0 -= 32 * hstart;
    const int Rw = (int)(g1 - g0) + hstart;  // this wave's rounds with a block
    const int j = lane & 31, hh = lane >> 5;
    const float sa = p.ascale, sx = p.xscale, sh = p.hscale, sy = p.yscale;
    const float u0 = p.unscale0, u1 = p.unscale1, u2 = p.unscale2;
    float mxa = 0.0f, mxx = 0.0f, mxh = 0.0f, mxy = 0.0f;
    auto aload = [&](unsigned bb, long long t0) {
        const long long pos = t0 - 8 + lane;
        // (bb == tw.b) an unconditional load at a clamped address: issued here, not sunk by the compiler to its use
        // in the next tile (which exposed the whole HBM latency once per tile)
        const bool ok = lane < AUD && pos >= 0 && pos < tw.Tb;
        const float v = audio[ok ? (long long)bb * T + pos : 0];
        return ok ? v : 0.0f;
    };
    // the audio window as its two fp16 planes: each lane splits its own sample once (kernels.h split2_f16s) and
    // stores hi / lo halves; a lane then reads its 8 taps' halves of the plane it feeds (hh) -- 8 d16 LDS reads
    // instead of 8 float reads and 4 pair splits per lane on the block wave's chain (the same values)
    _Float16* audh = reinterpret_cast<_Float16*>(aud);  // [AUD] hi plane, then [AUD] lo plane (the AUD floats' bytes)
    // conv0 from an audio plane image (this wave's own, or the one a conv wave split for this round: S0F_HELP)
    auto conv0_img = [&](const _Float16* img, f32x16 (&x0)[2]) {
        f16x8 bq;
        const _Float16* ap = img + (hh ? AUD : 0) + j + 2;
#pragma unroll
        for (int k = 0; k < 8; ++k) bq[k] = ap[k];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            f32x16 acc;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
            acc = mfma_h(wf[(FR_W0 + 2 * mt + 1) * 64 + lane], bq, acc);
            acc = mfma_h(wf[(FR_W0 + 2 * mt) * 64 + lane], bq, acc);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + 32 * mt + 8 * g + 4 * hh);
#pragma unroll
                for (int q = 0; q < 4; ++q) x0[mt][4 * g + q] = __builtin_fmaf(acc[4 * g + q], u0, bb[q]);
            }
        }
    };
    auto conv0 = [&](float av, f32x16 (&x0)[2]) {
        if (lane < AUD) {
            mxa = fmaxf(mxa, fabsf(av));
            unsigned hw, lw;
            split2_f16s(av, 0.0f, sa, hw, lw);
            audh[lane] = __builtin_bit_cast(f16x2, hw)[0];
            audh[AUD + lane] = __builtin_bit_cast(f16x2, lw)[0];
        }
        S0F_DRAIN();
        conv0_img(audh, x0);
    };
    auto slab_put = [&](const f32x16 (&x0)[2], int rowoff) {
        const int row = j + rowoff;
        if (row < 0 || row >= SROWS) return;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float z[4] = {x0[mt][4 * g], x0[mt][4 * g + 1], x0[mt][4 * g + 2], x0[mt][4 * g + 3]};
                float t[4];
                elu_s4<true>(z, sx, t, mxx);
                uint2 hi, lo;
                split4_t(t, hi, lo);
                const int o = row * SLD + 32 * mt + 8 * g + 4 * hh;
                *reinterpret_cast<uint2*>(slab + o) = hi;
                *reinterpret_cast<uint2*>(slab + SPL + o) = lo;
            }
    };
    const int cpl = lane >> 5, crow = (lane >> 4) & 1, cc = (lane & 15) * 4;
    // y halo copy lanes: plane, row 0..3, 16-B chunk (rows r and 32 + r have the same chunk order)
    const int hrow = (lane >> 3) & 3;
    const int hoff = (lane >> 5) * YPS + wave * YSS + hrow * YLD + 8 * ((lane & 7) ^ ((hrow & 1) * 2));
    const int yrow = 4 + j, ysw = (yrow & 1) * 2;

    if (S0F_DIAG == 2) {  // (the skipped blocks leave zeros: finite x1, no overflow fallback)
        for (int i = lane; i < YSS / 8; i += 64)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<uint4*>(ybase + q * YPS + wave * YSS + 8 * i) = make_uint4(0u, 0u, 0u, 0u);
    }
#if S0F_HELP
    __syncthreads();  // round 0's audio images (the conv waves' prologue)
#else
    float anext = Rw > 0 ? aload(tw.b, tw.t0) : 0.0f;
#endif
    S0F_T0();
    for (int n = 0; n <= R; ++n) {
        _Float16* ycur = ybase + (n & 1) * YBS;
        const _Float16* yprev = ybase + ((n + 1) & 1) * YBS;
        int4* dcur = desc + (n & 1) * NA;
        if (n < Rw && S0F_DIAG == 2) {
            if (lane == 0) dcur[wave] = make_int4((int)tw.b, (int)(tw.t0 >> 2), n < hstart ? 0 : 1, 0);
            tw.next();
        } else if (n < Rw) {
            const unsigned b = tw.b;
            const long long t0 = tw.t0;
            const long long Tb = tw.Tb;
            if (!S0F_HELP) {
                uint4 v = make_uint4(0u, 0u, 0u, 0u);
                if (t0 > 0) v = *reinterpret_cast<const uint4*>(yprev + hoff + 32 * YLD);
                *reinterpret_cast<uint4*>(ycur + hoff) = v;
            }
            if (lane == 0) {
                const long long T1b = (Tb + 3) >> 2;  // ceil(T0 / 4): down conv 0's output steps
                const long long t10 = t0 >> 2;
                dcur[wave] = make_int4((int)b, (int)t10, n < hstart ? 0 : (int)min(8LL, T1b - t10), 0);
            }
            if (t0 == 0) {
                *reinterpret_cast<uint2*>(slab + cpl * SPL + crow * SLD + cc) = make_uint2(0u, 0u);
            } else if (n == 0) {
                f32x16 xp[2];
                conv0(aload(b, t0 - 32), xp);
                slab_put(xp, -30);
            }
            S0F_T(0);
            f32x16 x0[2];
#if S0F_HELP
            tw.next();
            conv0_img(aud2 + (wave * 2 + (n & 1)) * (2 * AUD), x0);
#else
            const float acur = anext;
            tw.next();
            anext = aload(tw.b, tw.t0);  // (past the range: a valid address, never used)
            conv0(acur, x0);
#endif
            S0F_T(1);
            slab_put(x0, 2);
            S0F_DRAIN();
            S0F_T(2);

            f32x16 acc1;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc1[r] = 0.0f;
            // fragments one K step ahead of their MFMAs (one wave per SIMD: nothing else hides the LDS latency)
            f16x8 fr[2][4];
            auto g1load = [&](int ks, f16x8 (&f)[4]) {
                const int o = (j + (ks >> 2)) * SLD + (ks & 3) * 16 + 8 * hh;
                f[0] = *reinterpret_cast<const f16x8*>(slab + o);
                f[1] = *reinterpret_cast<const f16x8*>(slab + SPL + o);
                f[2] = wf[(FR_W3 + 2 * ks) * 64 + lane];
                f[3] = wf[(FR_W3 + 2 * ks + 1) * 64 + lane];
            };
            g1load(0, fr[0]);
#pragma unroll
            for (int ks = 0; ks < 12; ++ks) {
                if (ks + 1 < 12) g1load(ks + 1, fr[(ks + 1) & 1]);
                const f16x8(&f)[4] = fr[ks & 1];
                acc1 = mfma_h(f[3], f[0], acc1);
                acc1 = mfma_h(f[2], f[1], acc1);
                acc1 = mfma_h(f[2], f[0], acc1);
            }
            {
                _Float16* sp = slab + cpl * SPL;
                const uint2 v = *reinterpret_cast<const uint2*>(sp + (32 + crow) * SLD + cc);
                *reinterpret_cast<uint2*>(sp + crow * SLD + cc) = v;
            }
            asm volatile("" ::: "memory");
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + 64 + 8 * gq + 4 * hh);
                float z[4], t[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) z[q] = __builtin_fmaf(acc1[4 * gq + q], u1, bb[q]);
                elu_s4<true>(z, sh, t, mxh);
                uint2 hi, lo;
                split4_t(t, hi, lo);
                const int o = j * SLD + 8 * gq + 4 * hh;
                *reinterpret_cast<uint2*>(hb + o) = hi;
                *reinterpret_cast<uint2*>(hb + SPL + o) = lo;
            }
            S0F_DRAIN();
            S0F_T(3);

            // GEMM2 + y per 32-channel half: the second half's MFMAs are independent of the first half's epilogue
            f16x8 bh[2][2];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int o = j * SLD + ks * 16 + 8 * hh;
                bh[ks][0] = *reinterpret_cast<const f16x8*>(hb + o);
                bh[ks][1] = *reinterpret_cast<const f16x8*>(hb + SPL + o);
            }
            // y = ELU(x0 + (acc + b1)) -> planes of y * yscale, section row 4 + j (zeros past the item's end)
            float tmy = 0.0f;
            const bool yin = t0 + j < Tb;
            _Float16* ys = ycur + wave * YSS + yrow * YLD + 4 * hh;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                f32x16 acc2;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc2[r] = 0.0f;
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    const f16x8 aw0 = wf[(FR_W1 + (mt * 2 + ks) * 2) * 64 + lane];
                    const f16x8 aw1 = wf[(FR_W1 + (mt * 2 + ks) * 2 + 1) * 64 + lane];
                    acc2 = mfma_h(aw1, bh[ks][0], acc2);
                    acc2 = mfma_h(aw0, bh[ks][1], acc2);
                    acc2 = mfma_h(aw0, bh[ks][0], acc2);
                }
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    const f32x4 bb = *reinterpret_cast<const f32x4*>(bl + 96 + 32 * mt + 8 * gq + 4 * hh);
                    float z[4], t[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) z[q] = x0[mt][4 * gq + q] + __builtin_fmaf(acc2[4 * gq + q], u2, bb[q]);
                    elu_s4<true>(z, sy, t, tmy);
                    uint2 hi, lo;
                    split4_t(t, hi, lo);
                    if (!yin) hi = lo = make_uint2(0u, 0u);
                    const int o = 8 * ((4 * mt + gq) ^ ysw);
                    *reinterpret_cast<uint2*>(ys + o) = hi;
                    *reinterpret_cast<uint2*>(ys + YPS + o) = lo;
                    if (p.yp && yin) {  // taps only: the y planes in resblock0_h16_kernel's HBM layout too
                        _Float16* g = reinterpret_cast<_Float16*>(p.yp) + ((long long)b * T + t0 + j) * 64 + 32 * mt +
                                      8 * gq + 4 * hh;
                        *reinterpret_cast<uint2*>(g) = hi;
                        *reinterpret_cast<uint2*>(g + p.y_pstride) = lo;
                    }
                }
            }
            if (yin) mxy = fmaxf(mxy, tmy);
            S0F_T(4);  // (slots: 0 halo + descriptor, 1 conv0, 2 slab, 3 GEMM1 + h, 4 GEMM2 + y, 5 barrier)
        } else if (lane == 0) {
            dcur[wave] = make_int4(0, 0, 0, 0);
        }
        __syncthreads();
        S0F_T(5);
    }
    S0F_TPRINT("block");
    amax_commit(p.aamax, mxa);
    amax_commit(p.xamax, mxx * (1.0f / sx));
    amax_commit(p.hamax, mxh * (1.0f / sh));
    amax_commit(p.yamax, mxy * (1.0f / sy));
}

hipError_t launch_stage0_fused(const ResArgs& a, hipStream_t s, const char** kname) {
    if (a.T <= 0 || a.batch <= 0 || !a.audio || !a.wh16 || !a.wdown || !a.bdown || !a.xout ||
        a.T1 != (a.T + 3) / 4)
        return hipErrorInvalidValue;
    static const char* nm = "mimi::stage0_fused_h16_kernel(mimi::ResArgs)";
    if (kname) *kname = nm;
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    hipLaunchKernelGGL(stage0_fused_h16_kernel, dim3((unsigned)ncu), dim3(64 * s0f::NW), 0, s, a);
    return hipGetLastError();
}

}  // namespace mimi
