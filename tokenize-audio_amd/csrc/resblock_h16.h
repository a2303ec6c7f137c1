// fp16-plane helpers shared by the fused residual-block kernels (resblock.hip) and the fused stage-0 kernel
// (stage0_fused.hip): the stage-0 block's LDS plan, the plane split, the scaled ELU and the persistent tile walk.
#pragma once
#include "gemm_kernel.h"

namespace mimi {

typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace r0h {
constexpr int SLD = 72, SROWS = 34, SPL = SROWS * SLD;  // slab [2 planes][34][72 halves]: 144-B rows, 36 dwords
                                                        // (an odd multiple of 16 B: conflict-free ds_read_b128
                                                        // column reads); h [2][32][32] reuses rows 2..33
constexpr int AUD = 48;                                 // audio window floats
constexpr int WAVE_BYTES = 2 * SPL * 2 + AUD * 4;
constexpr int NW = 12;
constexpr int FR_W0 = 0, FR_W3 = 4, FR_W1 = 28, NFRAG = 36;  // 1-KB A fragments [64 lanes][8 halves]
constexpr int BIAS = 64 + 32 + 64;                           // b0 | b3 | b1
constexpr int LDS_BYTES = NFRAG * 1024 + BIAS * 4 + NW * WAVE_BYTES;
static_assert(NFRAG == RES0_H16_FRAGS, "fragment count");
static_assert(LDS_BYTES <= 160 * 1024, "LDS");
}  // namespace r0h

__device__ __forceinline__ f32x16 mfma_h(f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// fp16 planes of 4 already-scaled values t: hi = fp16(t) (packed converts), lo = fp16(t - hi), the difference
// taken exactly in fp32 and rounded once by v_fma_mix{lo,hi}_f16 (the same bits as fp16(t - (float)hi), 2
// instructions instead of 4 per pair)
__device__ __forceinline__ void split4_t(const float (&t)[4], uint2& hi, uint2& lo) {
    unsigned hu[2], lu[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const f16x2 h = __builtin_convertvector((f32x2){t[2 * q], t[2 * q + 1]}, f16x2);
        hu[q] = __builtin_bit_cast(unsigned, h);
        asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
            : "=&v"(lu[q])
            : "v"(hu[q]), "v"(t[2 * q]), "v"(t[2 * q + 1]));
    }
    hi = make_uint2(hu[0], hu[1]);
    lo = make_uint2(lu[0], lu[1]);
}

// ELU(z) * s for a power-of-two s, two values at a time: med3(z s, fma(exp(z), s, -s), 0).  For z > 0 the
// median is z s (exp(z) - 1 > z); for z <= 0 it is (exp(z) - 1) s (z <= exp(z) - 1 <= 0).  That is elu_fast's
// select (exp as v_exp_f32 of z log2(e)) followed by an exact scaling, bit for bit, with no compare.
// SC: per-element scalar ops (the same bits) instead of packed f32 -- packed VALU issues slowly beside another
// wave's MFMAs on the SIMD (stage0_fused.hip); the resblock kernels keep the packed form (fewer issues, faster there)
template <bool SC = false>
__device__ __forceinline__ f32x2 elu_s2(f32x2 z, float s) {
    if constexpr (SC) {
        float r[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const float e = __builtin_amdgcn_exp2f(z[q] * 1.44269504f);
            r[q] = __builtin_amdgcn_fmed3f(z[q] * s, __builtin_fmaf(e, s, -s), 0.0f);
        }
        return (f32x2){r[0], r[1]};
    } else {
        const f32x2 l = z * 1.44269504f;
        const f32x2 e = {__builtin_amdgcn_exp2f(l[0]), __builtin_amdgcn_exp2f(l[1])};
        const f32x2 n = __builtin_elementwise_fma(e, (f32x2){s, s}, (f32x2){-s, -s});
        const f32x2 zs = z * s;
        return (f32x2){__builtin_amdgcn_fmed3f(zs[0], n[0], 0.0f), __builtin_amdgcn_fmed3f(zs[1], n[1], 0.0f)};
    }
}

// 4 values z -> t = ELU(z) * s, max |t| into mx
template <bool SC = false>
__device__ __forceinline__ void elu_s4(const float (&z)[4], float s, float (&t)[4], float& mx) {
#pragma unroll
    for (int q = 0; q < 4; q += 2) {
        const f32x2 r = elu_s2<SC>((f32x2){z[q], z[q + 1]}, s);
        t[q] = r[0];
        t[q + 1] = r[1];
        asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(mx) : "v"(mx), "v"(r[0]), "v"(r[1]));
    }
}

// The persistent fp16 blocks' walk over 32-step tiles: the items' tiles concatenated (uniform: tpi per item;
// ragged: item b's ceil(ilen[b] / 32) tiles from istart[b]), a wave / workgroup taking a contiguous range of them.
struct TileWalk {
    const ResArgs& p;
    unsigned tpi;
    unsigned b = 0;
    long long t0 = 0;
    long long Tb = 0;  // item b's length (ragged: read once per item, not per load)
    __device__ TileWalk(const ResArgs& pa, unsigned tiles_per_item, unsigned g) : p(pa), tpi(tiles_per_item) {
        if (p.istart) {
            while (b + 1 < (unsigned)p.batch && p.istart[b + 1] <= g) ++b;
            t0 = (long long)(g - p.istart[b]) * 32;
        } else {
            b = g / tpi;
            t0 = (long long)(g - b * tpi) * 32;
        }
        Tb = len(b);
    }
    __device__ long long len(unsigned bb) const { return p.ilen ? (long long)p.ilen[bb] : p.T; }
    __device__ void next() {
        t0 += 32;
        if (t0 >= Tb) {
            ++b;
            t0 = 0;
            Tb = b < (unsigned)p.batch ? len(b) : 0;
        }
    }
};

__device__ __forceinline__ f32x4 mfma_h16(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

}  // namespace mimi
