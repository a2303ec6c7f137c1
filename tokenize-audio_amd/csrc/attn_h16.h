// fp16-plane attention helpers shared by attention_t256_h16_kernel / attention_band_h16_kernel (ops.hip) and the
// fused q/k/v + attention kernel (qkv_attn.hip): plane scales, the 32-key chunk step (two 3-product MFMA passes
// around an fp32 online softmax), the row-major V image and the T <= 256 task table.  See ops.hip for the
// kernels' description.
#pragma once
#include "kernels.h"

namespace mimi {

#ifndef MIMI_ATTN_TYPES
#define MIMI_ATTN_TYPES
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
#endif

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ float pow2_scale(float mx) {
    return mx > 0.0f && mx < INFINITY ? ldexpf(1.0f, 13 - ilogbf(mx)) : 1.0f;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
// hi / lo fp16 planes of 8 scaled values
__device__ __forceinline__ void split8_h(const float (&v)[8], float sc, f16x8& hi, f16x8& lo) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float t = v[e] * sc;
        hi[e] = (_Float16)t;
        lo[e] = (_Float16)(t - (float)hi[e]);
    }
}

// One 32-key chunk of the fp16-plane attention for the wave's 32 queries: S^T = K . Q^T and O^T += V^T . P^T as
// 3 fp16 plane products each, fp32 online softmax (as attn_chunk).  Kc: the chunk's 32 K rows (plane stride KPL,
// row stride KLD); Vc: column 0 of the chunk's keys in the V^T planes (plane stride VPL, row stride VLD, keys
// permuted inside each 16 as the S^T accumulator holds them); us = 1 / (K scale x Q scale).
// TRV (the T <= 256 kernel): V as row-major planes [256 keys][64 dims] (16-B chunks XOR-swizzled by key, see
// attn_vrow_off), the V^T fragments read with ds_read_b64_tr_b16 -- two 4-key reads per fragment, the same 8 values in
// the same order as the V^T image's b128 read; vlb[t]: this lane's offset for dim tile t (attn_vlane_base).
template <int KLD, int KPL, int VLD, int VPL, bool TRV = false>
__device__ __forceinline__ void attn_chunk_h16(f32x16 (&o)[2], float& m, float& l, const f16x8 (&qf)[4][2],
                                               const _Float16* Kc, const _Float16* Vc, int c0, int qw, int qi,
                                               int kend, int window, int hf, int col, float us,
                                               float ofac = 1.0f, float pscale = 16384.0f, int vlb0 = 0,
                                               int vlb1 = 0) {
    // S^T[key][query] = K . Q^T
    f32x16 st;
#pragma unroll
    for (int r = 0; r < 16; ++r) st[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        const int ko = col * KLD + 16 * ks + 8 * hf;
        const f16x8 k0 = *reinterpret_cast<const f16x8*>(Kc + ko);
        const f16x8 k1 = *reinterpret_cast<const f16x8*>(Kc + KPL + ko);
        st = __builtin_amdgcn_mfma_f32_32x32x16_f16(k1, qf[ks][0], st, 0, 0, 0);
        st = __builtin_amdgcn_mfma_f32_32x32x16_f16(k0, qf[ks][1], st, 0, 0, 0);
        st = __builtin_amdgcn_mfma_f32_32x32x16_f16(k0, qf[ks][0], st, 0, 0, 0);
    }
    // mask + online softmax for this lane's query (fp32, as attn_chunk)
    float cmax = -INFINITY;
    const bool full = c0 + 31 <= qw && c0 > qw + 31 - window && c0 + 31 <= kend;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        float v = st[r] * us;
        if (!full) {
            const int key = c0 + (r & 3) + 8 * (r >> 2) + 4 * hf;
            const bool ok = key <= qi && key > qi - window && key <= kend;
            v = ok ? v : -INFINITY;
        }
        st[r] = v;
        cmax = fmaxf(cmax, v);
    }
    cmax = fmaxf(cmax, __shfl_xor(cmax, 32));
    const float mnew = fmaxf(m, cmax);
    const float corr = (m == -INFINITY) ? 0.f : __expf(m - mnew);
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float pv = (st[r] == -INFINITY) ? 0.f : __expf(st[r] - mnew);
        st[r] = pv;
        psum += pv;
    }
    psum += __shfl_xor(psum, 32);
    l = l * corr + psum;
    m = mnew;
    const float oc = corr * ofac;  // ofac: a power of two (a change of the V scale), so o * oc rounds as o * corr
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] *= oc;
    // O^T[d][query] += V^T . P^T: k-step ks = keys 16 ks .. +15 of the chunk, lane half hf element e =
    // st[8 ks + e] (key (e & 3) + 8 (e >> 2) + 4 hf)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        float pe[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) pe[e] = st[8 * ks + e];
        f16x8 p0, p1;
        split8_h(pe, pscale, p0, p1);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            f16x8 v0, v1;
            if constexpr (TRV) {
                typedef short v4s __attribute__((vector_size(8)));
                typedef __attribute__((address_space(3))) v4s lv4s;
                const _Float16* vb = Vc + (c0 + 16 * ks) * 64 + (t ? vlb1 : vlb0);  // keys +0..3 / +8..11 of the half
                const v4s a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lv4s*)(vb));
                const v4s a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lv4s*)(vb + 8 * 64));
                const v4s b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lv4s*)(vb + VPL));
                const v4s b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lv4s*)(vb + VPL + 8 * 64));
                typedef _Float16 h4 __attribute__((ext_vector_type(4)));
                v0 = __builtin_shufflevector(__builtin_bit_cast(h4, a0), __builtin_bit_cast(h4, a1), 0, 1, 2, 3, 4, 5, 6, 7);
                v1 = __builtin_shufflevector(__builtin_bit_cast(h4, b0), __builtin_bit_cast(h4, b1), 0, 1, 2, 3, 4, 5, 6, 7);
            } else {
                const int vo = (32 * t + col) * VLD + 16 * ks + 8 * hf;
                v0 = *reinterpret_cast<const f16x8*>(Vc + vo);
                v1 = *reinterpret_cast<const f16x8*>(Vc + VPL + vo);
            }
            o[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(v1, p0, o[t], 0, 0, 0);
            o[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(v0, p1, o[t], 0, 0, 0);
            o[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(v0, p0, o[t], 0, 0, 0);
        }
    }
}
// position of key r inside the V^T image: keys permuted inside each 16 as the S^T accumulator holds them
__device__ __forceinline__ int vt_key_pos(int r) {
    const int k = r & 15;
    return (r & ~15) + 8 * ((k >> 2) & 1) + (k & 3) + 4 * ((k >> 3) & 1);
}
// row-major V planes of the T <= 256 kernel: dim d of key r at 16-B chunk (d >> 3) ^ 4 ((r >> 1) & 1) of the 128-B
// row -- the 16-lane row writes (ds_write_b64) and the transposed reads (4 keys x 32 dims per 32-lane half) are
// both conflict-free (MI355X_MICROARCH.md LDS banking)
__device__ __forceinline__ int attn_vrow_off(int r, int d) { return r * 64 + 8 * ((d >> 3) ^ (((r >> 1) & 1) << 2)) + (d & 7); }
// this lane's ds_read_b64_tr_b16 address inside a 16-key step of dim tile t, relative to that step's first row: lane
// 4 q + p of its 16-lane group supplies row (key) 4 hf + q, dims 32 t + 16 ((lane >> 4) & 1) + 4 p .. +3, and
// receives dim 32 t + (lane & 31) of the 4 keys -- the A-operand order of the S^T accumulator (keys 4 hf + 0..3,
// then + 8)
__device__ __forceinline__ int attn_vlane_base(int lane, int t) {
    const int q = (lane >> 2) & 3, p = lane & 3, hf = lane >> 5;
    return attn_vrow_off(4 * hf + q, 32 * t + 16 * ((lane >> 4) & 1) + 4 * p);
}

__device__ __forceinline__ int attn_task(int qg, int z, int wave) {
    unsigned long long tbl;
    if (qg == 1) {
        tbl = 0x31207456AB89DCFEull;  // wave w -> nibble w = 2 tile + half
    } else if (qg == 2) {
        if (wave >= 8) return -1;
        tbl = z == 0 ? 0x670198FEull : 0x4523BADCull;
    } else {
        if (wave >= 4) return -1;
        return 2 * (wave < 2 ? 7 - z : z) + (wave & 1);
    }
    return (int)((tbl >> (4 * wave)) & 15);
}

// tile t's output is stored by the workgroup that holds its tasks
__device__ __forceinline__ bool attn_tile_in_wg(int qg, int z, int t) {
    return qg == 1 || (qg == 2 ? ((t & 3) == z || (t & 3) == 3 - z) : (t == z || t == 7 - z));
}

}  // namespace mimi
