// Internal launcher interface between the engine (engine.cpp) and the HIP kernels (gemm.hip, ops.hip).
// Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace mimi {

// sets the thread-local mimi_last_error() text (engine.cpp); returns code
int set_error_message(int code, const char* msg);

// ELU(x) = x (x > 0), expm1(x) (x <= 0), branchless, as exp(x) - 1 on the exp unit (v_exp_f32 of x*log2(e)):
// 4 VALU.  exp(x) - 1 cancels for small |x|, but the error stays ABSOLUTE ~1e-7 (an ulp of 1.0), the size of
// the fp32 rounding of any O(1) activation, so the block outputs are unchanged at the 1e-6 level (the
// per-stage parity tests bound it).  The SEANet applies ELU to every conv input and output: it is the
// dominant VALU cost of the fused residual blocks.
__device__ __forceinline__ float elu_fast(float x) {
    const float e = __expf(x) - 1.0f;
    return x > 0.0f ? x : e;
}

// Activation store in the consumer's format: fp32 (ns == 0), ns bf16 planes x = x0 + x1 [+ x2] with
// x_p = bf16(x - x0 - ... - x_{p-1}) (the split of gemm_kernel.h), or -- hscale > 0, PREC_F16X3 -- 2 fp16 planes
// of x * hscale (h0 = fp16(x * hscale), h1 = fp16(x * hscale - h0): 22-bit significand; hscale a power of two
// chosen by the engine so that max|x| * hscale sits inside fp16's range, see engine.cpp "activation scales").
// Plane p at planes + p * pstride.  The planes feed gemm_planes_kernel, which then only moves bytes
// (gemm_planes.h).  In fp16 mode *mx accumulates max|x| for the engine's range check (amax_commit).
__device__ __forceinline__ void store_act(float* f32, void* planes, long long pstride, int ns, long long idx,
                                          float v, float hscale = 0.0f, float* mx = nullptr) {
    if (ns == 0) {
        f32[idx] = v;
        return;
    }
    if (hscale > 0.0f) {
        _Float16* hp = reinterpret_cast<_Float16*>(planes) + idx;
        const float t = v * hscale;
        const _Float16 h0 = (_Float16)t;
        hp[0] = h0;
        hp[pstride] = (_Float16)(t - (float)h0);
        *mx = fmaxf(*mx, fabsf(v));
        return;
    }
    __bf16* pp = reinterpret_cast<__bf16*>(planes) + idx;
    const __bf16 h0 = (__bf16)v;
    pp[0] = h0;
    const float r1 = v - (float)h0;
    const __bf16 h1 = (__bf16)r1;
    pp[pstride] = h1;
    if (ns == 3) pp[2 * pstride] = (__bf16)(r1 - (float)h1);
}

// 8 consecutive values as planes (16-B stores per plane): bf16 (ns = 2/3) or scaled fp16 (hscale > 0)
// The 2 fp16 planes of (v0, v1) * s (s a power of two) as exact arithmetic defines them: hi = RN16(v s),
// lo = RN16(v s - hi), two values per dword.  lo is one FMA (v s - hi exact, then one rounding), which hipcc emits as
// v_fma_mix_f32 (hi read straight from its fp16 half) + one v_cvt_pk per pair: 6 instructions a pair instead of 8
// for mul, cvt, cvt back, sub, cvt.  The same bits as that form wherever v s is exact in fp32 (a power-of-two
// scale); where v s underflows fp32 both give a zero lo plane, this form with the sign of the exact product
// (tests/test_split_planes.py checks it against float64 arithmetic).
__device__ __forceinline__ void split2_f16s(float v0, float v1, float s, unsigned& hi, unsigned& lo) {
    typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
    typedef float f2_t __attribute__((ext_vector_type(2)));
    const f2_t t = {v0 * s, v1 * s};
    const h2_t h = __builtin_convertvector(t, h2_t);
    h2_t l;
    l[0] = (_Float16)__builtin_fmaf(v0, s, -(float)h[0]);
    l[1] = (_Float16)__builtin_fmaf(v1, s, -(float)h[1]);
    hi = __builtin_bit_cast(unsigned, h);
    lo = __builtin_bit_cast(unsigned, l);
}

__device__ __forceinline__ void store_act8(void* planes, long long pstride, int ns, long long idx, const float (&v)[8],
                                           float hscale, float* mx) {
    typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
    if (hscale > 0.0f) {
        uint4 a, b;
        split2_f16s(v[0], v[1], hscale, a.x, b.x);
        split2_f16s(v[2], v[3], hscale, a.y, b.y);
        split2_f16s(v[4], v[5], hscale, a.z, b.z);
        split2_f16s(v[6], v[7], hscale, a.w, b.w);
#pragma unroll
        for (int e = 0; e < 8; ++e) *mx = fmaxf(*mx, fabsf(v[e]));
        _Float16* hp = reinterpret_cast<_Float16*>(planes) + idx;
        *reinterpret_cast<uint4*>(hp) = a;
        *reinterpret_cast<uint4*>(hp + pstride) = b;
        return;
    }
    float rem[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) rem[e] = v[e];
    __bf16* dst = reinterpret_cast<__bf16*>(planes) + idx;
    for (int pl = 0; pl < ns; ++pl) {
        bf16x8_t hv;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            hv[e] = (__bf16)rem[e];
            rem[e] = rem[e] - (float)hv[e];
        }
        *reinterpret_cast<bf16x8_t*>(dst + pl * pstride) = hv;
    }
}

// max over the wave of the lanes' running max|x|, max-ed by one atomic per wave into one of AMAX_SUB sub-slots
// of the tensor's slot (picked by workgroup, AMAX_STRIDE words apart), so the thousands of waves of a launch do
// not serialise on one address.  No cached pre-read of the sub-slot: an earlier version skipped the atomic when
// a plain read showed a larger value, and in hipGraph replays such reads (and the fold's plain reads) could see
// another XCD's stale line -- spurious maxima, one spurious overflow fallback.  Non-negative floats order as
// their bit patterns.  Every lane of the wave must call it; amax == null: no-op.  amax_reduce_kernel folds (and
// resets) the sub-slots.
constexpr int AMAX_SUB = 64, AMAX_STRIDE = 16, AMAX_SLOT_WORDS = AMAX_SUB * AMAX_STRIDE;
__device__ __forceinline__ void amax_commit(unsigned* amax, float mx) {
    if (!amax) return;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if ((threadIdx.x & 63) == 0 && mx > 0.0f) {
        unsigned* a = amax + ((blockIdx.x + 7 * blockIdx.y + 13 * blockIdx.z) & (AMAX_SUB - 1)) * AMAX_STRIDE;
        atomicMax(a, __float_as_uint(mx));  // device scope, at the memory side (no cached pre-read: see amax_reduce)
    }
}

// LayerNorm row arithmetic (TF/modeling_mimi.py:737-738), shared by layernorm_kernel (ops.hip) and the LayerNorm
// prologue of the small-batch q/k/v and fc1 GEMMs (gemm_planes.h FL_LNA), so both give the same bits: one wave
// per row of C, lane l holding columns q*256 + 4l + e; two-pass mean / variance in fp32, then
// y = (x * rstd + (-mean * rstd)) * gamma + beta as the torch CPU kernel forms it.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
template <int C>
__device__ __forceinline__ void ln_row_coeffs(const float (&v)[C / 64], float eps, float& sc, float& bi) {
    constexpr int PER = C / 64;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) s += v[i];
    const float mean = wave_sum(s) / (float)C;
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const float d = v[i] - mean;
        s2 += d * d;
    }
    const float var = wave_sum(s2) / (float)C;
    const float rstd = 1.0f / sqrtf(var + eps);
    sc = rstd;
    bi = -rstd * mean;
}
__device__ __forceinline__ float ln_affine(float v, float sc, float bi, float g, float b) { return (v * sc + bi) * g + b; }
// fp16 planes of 4 LayerNorm outputs o * yscale (PREC_F16X3): hi / lo as 4 halves each
__device__ __forceinline__ void ln_split4_f16(const float (&o)[4], float yscale, uint2& hi, uint2& lo) {
    split2_f16s(o[0], o[1], yscale, hi.x, lo.x);
    split2_f16s(o[2], o[3], yscale, hi.y, lo.y);
}

// A pointer a captured hipGraph reads at run time: the engine's io block, written by set_io_kernel in front of
// every replay (a vector load that bypasses the scalar cache, made wave-uniform).  ref == null: direct.
template <typename T>
__device__ __forceinline__ T* io_pointer(T* const* ref, T* direct) {
    if (!ref) return direct;
    const unsigned long long v = *reinterpret_cast<const volatile unsigned long long*>(ref);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return reinterpret_cast<T*>(((unsigned long long)hi << 32) | lo);
}
// io[0] = audio, io[1] = codes (the pointers of one graph replay)
hipError_t launch_split_check(const float* in, long long npairs, float s, unsigned* out, hipStream_t st);
hipError_t launch_gelu_check(const float* in, long long n, float* out, hipStream_t st);
hipError_t launch_set_io(void** io, const float* audio, int32_t* codes, hipStream_t s, unsigned* hamax = nullptr,
                         unsigned* hflag = nullptr, void* zero = nullptr, size_t zero_bytes = 0);

// out[i] = max over the AMAX_SUB sub-slots of slot i (one wave per slot); the sub-slots are left at 0
// (+ an encode ticket's pinned host words: hamax[slot] = the folded maximum, *hflag = *flag when both are given; io:
// take hamax / hflag from io[2] / io[3] (set_io) at run time -- the form a captured graph holds)
hipError_t launch_amax_reduce(unsigned* amax, int nslots, unsigned* out, hipStream_t s, unsigned* hamax = nullptr,
                              const unsigned* flag = nullptr, unsigned* hflag = nullptr, void* const* io = nullptr);

// Epilogues of the implicit-GEMM conv / linear kernel.
enum Epi : int {
    EPI_NONE = 0,          // C = acc                                  (input_proj, downsample)
    EPI_BIAS = 1,          // C = acc + bias                           (down convs 0-2)
    EPI_BIAS_ELU = 2,      // C = ELU(acc + bias)                      (res conv k3, down conv 3)
    EPI_BIAS_RES_ELU = 3,  // C = ELU(R + (acc + bias))                (res conv k1 + identity skip)
    EPI_GELU = 4,          // C = GELU_erf(acc)                        (fc1)
    EPI_SCALE_RES = 5,     // C = R + scale * acc                      (o_proj, fc2 with layer scale)
    EPI_ROPE = 6,          // C = RoPE(acc) on columns < rope_cols      (fused q/k/v projection)
    EPI_BIAS_OUT = 7,      // C = acc + bias  (final conv, channel-last output = transformer input)
};

enum Pad : int { PAD_ZERO = 0, PAD_REPLICATE = 1 };

// C[b][m][n] = epi( sum_k A(b, m, k) * W[n][k] ) with the im2col view of a channels-last activation:
//   A(b, m, k) = Aptr[b*a_bstride + a_off + m*a_rs + k]      (k in [0, K), K = ksize*Cin)
// Elements outside [0, a_len) of a batch item read as 0 (causal / extra zero padding) or, for
// PAD_REPLICATE, as the nearest valid time step (torch 'replicate' pad).  Cin % 4 == 0 is required.
struct GemmArgs {
    const float* A;
    long long a_bstride;
    long long a_off;
    int a_rs;
    int a_cin;
    long long a_len;
    const float* W;       // fp32 [N][K]
    const void* Wsplit;   // bf16 planes [3][N][K] of W (x = x0 + x1 + x2), for the split-bf16 modes
    const void* Ap;       // bf16 planes of A (gemm_planes_kernel): plane p at Ap + p*a_pstride, same indexing as A
    long long a_pstride;
    int M, N, K;
    int batch;
    const float* bias;
    const float* R;
    const float* scale;
    const float* rope_cos;  // [T][head_dim/2]
    const float* rope_sin;
    int rope_cols;
    float* C;
    long long c_bstride;
    int ldc;
    void* Cp;             // optional bf16 planes of the output (planes-out epilogues), plane stride c_pstride
    long long c_pstride;
    // fp16-plane mode (PREC_F16X3, gemm_planes_kernel<..., F16 = true>): 1 / (activation scale x weight scale)
    // applied to the accumulator before the epilogue (exact: powers of two); fp16 output planes hold
    // out * out_scale and max|out| goes to *out_amax
    float unscale;
    float out_scale;
    unsigned* out_amax;
    // ragged batches (mimi_encode_ragged): per-item valid rows of the A input (rows past a_rows[b] read as 0, the
    // item's own extra padding: a_len = a_rows[b] * a_cin) and of the output (tiles from m_rows[b] on are skipped,
    // rows past it are neither stored nor in max|out|); null = every item has M rows / a_len elements
    const int* a_rows;
    const int* m_rows;
    // ragged batches whose items' rows are PACKED (the transformer section: item b's rows start at row a_boff[b] /
    // c_boff[b] of one [sum of rows][...] tensor instead of at b x a_bstride / c_bstride; FL_RAGGED kernels only)
    const int* a_boff;  // A: item b starts at element a_boff[b] * a_cin
    const int* c_boff;  // C / Cp / R: item b starts at row c_boff[b] (element c_boff[b] * ldc)
    // EPI_ROPE over packed rows: the RoPE position of output row m (null: m itself)
    const int* rope_pos;
    // LayerNorm prologue (small-batch q/k/v and fc1 in f16x3, gemm_planes.h FL_LNA): A = LayerNorm(ln_x) (fp32, the
    // same [rows][K] indexing as the A planes, which are then not read), computed per tile as layernorm_kernel
    // computes it; its fp16 planes (of A * ln_scale) go straight to LDS, max|A| to ln_amax.  ln_x == null: off.
    const float* ln_x;
    const float* ln_g;
    const float* ln_b;
    float ln_eps;
    float ln_scale;
    unsigned* ln_amax;
    // host-side dispatch hint (not read by the kernels): 1 = take the FL_SC1OUT instantiation where the role has one
    // (engine option sc1_out; the same bits either way)
    int sc1;
    int ln_tile;  // host-side hint: the q/k/v LayerNorm-prologue tile on small grids (0 16x64, 1 32x64, 2 16x128)
    int ncg;  // planes kernels: XCD column groups of the tile order (0 / 1 none; must divide the N tiles, else none;
              // engine option fc1_cg; which workgroup computes a tile only, the same bits either way)
};
// Stage-2 k = 1 residual conv + skip + ELU -> y planes as a streaming kernel (res1_stream.hip): W1 register-resident
// per wave, 16-step time tiles with the next tile's h and skip in flight; bitwise the ROLE_RES1P planes GEMM.
// res1_stream_ok: the shapes / layouts it takes (else launch_res1_stream returns hipErrorInvalidValue).
bool res1_stream_ok(const GemmArgs& a);
hipError_t launch_res1_stream(const GemmArgs& a, hipStream_t s, const char** kname);
// true when launch_gemm(role, a, precision) runs a tile with the LayerNorm prologue (a.ln_* then feed A)
bool gemm_ln_prologue_ok(int role, const GemmArgs& a, int precision);

// Launch the GEMM for a given conv/linear role (the role picks tile shape and template flags).
enum GemmRole : int {
    ROLE_RES3 = 0,   // ELU-on-load, bias + ELU epilogue
    ROLE_RES1,       // bias + residual + ELU
    ROLE_DOWN,       // bias (raw output; next res block needs it for the skip)
    ROLE_DOWN_ELU,   // bias + ELU (last down conv: only the final conv reads it, through ELU)
    ROLE_FINAL,      // bias
    ROLE_QKV,        // RoPE
    ROLE_OPROJ,      // scale + residual
    ROLE_FC1,        // GELU
    ROLE_FC2,        // scale + residual
    ROLE_DOWNSAMPLE, // replicate pad, no bias
    ROLE_INPROJ,     // plain
    ROLE_DOWN_XE,    // planes path: bias, fp32 out (the residual skip) + ELU(out) planes (the next conv3 input)
    ROLE_RES3P,      // planes path, unfused residual block: k3 conv, bias + ELU -> h planes
    ROLE_RES1P,      // planes path, unfused residual block: k1 conv, bias + skip + ELU -> y planes
    ROLE_COUNT
};
// Arithmetic of the GEMMs: fp32 MFMA, or fp32 emulated on the bf16 matrix cores with 3 (6 products) or
// 2 (3 products) bf16 planes per operand (gemm_kernel.h).
// PREC_F16X3: 2 fp16 planes per operand (3 products) with power-of-two scales: 22-bit operands.
enum Precision : int { PREC_F32 = 0, PREC_BF16X6 = 1, PREC_BF16X3 = 2, PREC_F16X3 = 3 };

// *kname (optional) receives the kernel symbol as rocprofv3 prints it, for per-kernel profile aggregation.
hipError_t launch_gemm(int role, const GemmArgs& a, hipStream_t s, const char** kname = nullptr,
                       int precision = PREC_F32);

// Fused residual block + trailing ELU: y = ELU(x + b1 + W1 . ELU(b3 + W3 (*) ELU(x))), [B][T][C].
struct ResArgs {
    const float* x;       // [B][T][C] raw input (unused when audio != null)
    const float* audio;   // stage 0 only: [B][T] waveform; x = conv0(audio) is recomputed in-kernel
    const float* const* audio_ref;  // non-null (a captured hipGraph): the waveform pointer is read from here
    const float* w0;      // conv0 weight [64][7]
    const float* b0;      // conv0 bias [64]
    long long T;
    int batch;
    const float* w3;  // [C/2][3*C]  (W'[n][kk*C + ci])
    const float* b3;
    const float* w1;  // [C][C/2]
    const float* b1;
    float* y;
    void* yp;             // when yns > 0: y is written as yns bf16 planes (plane stride y_pstride) instead of fp32
    long long y_pstride;
    int yns;
    float yscale;         // > 0: 2 fp16 planes of y * yscale (PREC_F16X3), max|y| into *yamax
    unsigned* yamax;
    const float* w3frag;  // optional: W3 / W1 in MFMA-fragment order [ntile][kquad][64 lanes][4] (stage 0)
    const float* w1frag;
    // PREC_F16X3 fused block (stage 0: resblock0_h16_kernel): weights as 2 scaled fp16 planes in 32x32x16-MFMA
    // A-fragment order (layout in resblock.hip, built by engine.cpp make_res_h16).  The block's inputs and
    // internal operands are split in-kernel at power-of-two scales chosen by the engine; each one's max|v| is
    // max-reduced into its activation slot for the range check.  unscale* = 1 / (operand scale x weight scale).
    const void* wh16;
    float ascale, xscale, hscale;     // audio (conv0 input), ELU(x) (conv3 input), ELU(h) (conv1 input)
    float unscale0, unscale1, unscale2;
    unsigned *aamax, *xamax, *hamax;
    // ragged batches (fp16 blocks): item b has ilen[b] steps (T is then the row stride); istart[b] = the item's first
    // 32-step tile in the concatenation of every item's tiles (istart[batch] = their count); null = uniform T
    const int* ilen;
    const unsigned* istart;
    // stage 0 fused with down conv 0 (stage0_fused_h16_kernel): the down conv's 2 fp16 weight planes [2][128][512]
    // (K = tap-major 8 x 64, the planes GEMM's layout), bias, unscale_d = 1 / (yscale x weight scale), and its
    // fp32 output [B][T1][128] (T1 = ceil(T / 4): the row stride; ragged: item b has ceil(ilen[b] / 4) rows)
    const void* wdown;
    const float* bdown;
    float unscale_d;
    float* xout;
    long long T1;
    // stage 1 fp16 block (resblock128_h16_kernel): 0 = one 8-wave workgroup per CU, 1 = two 4-wave workgroups per CU
    // (engine option res1_form; which wave computes a tile only, the same bits)
    int form;
};
hipError_t launch_resblock(int C, const ResArgs& a, hipStream_t s, const char** kname);
// stage 0 + down conv 0 in one kernel (PREC_F16X3)
hipError_t launch_stage0_fused(const ResArgs& a, hipStream_t s, const char** kname);

// fp16-plane fused stage-0 block: fragment buffer size in halves ([frag][64 lanes][8])
constexpr int RES0_H16_FRAGS = 36;
// fp16-plane fused stage-1 block (C = 128): W3 [4][12][2] + W1 [8][2][2] 16x16x32 A fragments
constexpr int RES1_H16_FRAGS = 128;

// conv0: Cin = 1, k = 7 causal conv, channels-last output [B][T][64].
hipError_t launch_conv0(const float* x, long long L, int batch, const float* w /*[64][7]*/,
                        const float* b, float* y, int cout, int ksize, hipStream_t s);

// LayerNorm over the last dim (C = 512) of rows; output fp32 (yns == 0) or yns bf16 planes.
// row_len (ragged batches): row r belongs to item r / row_T at step r % row_T and is skipped past row_len[item]
hipError_t launch_layernorm(const float* x, const float* g, const float* b, float* y, long long rows,
                            int C, float eps, hipStream_t s, void* yp = nullptr, long long y_pstride = 0,
                            int yns = 0, float yscale = 0.0f, unsigned* yamax = nullptr, const int* row_len = nullptr,
                            int row_T = 0, int rpw = 0);

// Sliding-window causal attention on the fused qkv tensor [B][T][3*H*D] (q, k already rotated);
// output [B][T][H*D].  h16: the fp16-plane kernels (PREC_F16X3; T <= 256 needs fp16-plane output), else fp32.
// tlen (ragged batches, h16 only): item b has tlen[b] frames (T is the row stride); each item runs the kernel it
// would run alone (tlen[b] <= 256: attention_t256_h16_kernel, else the banded one)
hipError_t launch_attention(const float* qkv, float* out, int batch, int T, int H, int D, int window,
                            float scale, hipStream_t s, void* outp, long long out_pstride, int outns, float oscale,
                            unsigned* oamax, bool h16, const int* tlen = nullptr, int max_tlen = 0, int min_tlen = 0,
                            const int* toff = nullptr, const char** kname = nullptr, int band_split_mode = 1);

// Replicate-padding fix of the downsample conv (k = 4, s = 2) run as a zero-padded planes GEMM: per item,
// out[0] += (W_0 + W_1) . x[0] (the 2 left pad rows replicate x[0]) and, when T is odd (one right "extra" pad
// row), out[F-1] += W_3 . x[T-1]; the fixed rows are re-written as fp32 and as fp16 planes of out * oscale.
// wfix: fp32 [2][C][N] (W_0 + W_1, W_3, input channel major); x: fp32 [B][T][C]; out: fp32 [B][F][N].
// tlen / flen (ragged batches): per-item T and F (T, F are then the row strides)
hipError_t launch_ds_edge_fix(const float* x, const float* wfix, float* out, void* outp, long long out_pstride,
                              float oscale, unsigned* oamax, int B, int T, int F, int C, int N, hipStream_t s,
                              const int* tlen = nullptr, const int* flen = nullptr, const int* toff = nullptr);

// ragged batches with packed transformer rows: rpos[toff[b] + t] = t for t < tlen[b]
hipError_t launch_ragged_rows(const int* tlen, const int* toff, int B, int* rpos, hipStream_t s);

// the banded fp16-plane attention at any T (tools/attn_check.hip compares it with the T <= 256 kernel); split: its
// decomposition (0 = 128-query workgroups, 1 = by grid size, 2 = one 32-query tile per workgroup; same values)
hipError_t launch_attention_band(const float* qkv, int batch, int T, int H, int window, float scale,
                                 hipStream_t s, void* outp, long long out_pstride, float oscale, unsigned* oamax,
                                 int split = 1);

// Fused q/k/v projection + RoPE + attention for items of at most 256 frames (qkv_attn.hip): one workgroup per
// (item, head) computes the head's 192 q/k/v columns of the item's rows on the fp16 planes (the q/k/v GEMM's
// instruction sequence per output element) and runs attention_t256_h16_kernel's arithmetic on them in LDS -- the
// fp32 q/k/v tensor never goes to HBM.  Bitwise the same attention output as launch_gemm(ROLE_QKV) +
// launch_attention.
struct QkvAttnArgs {
    const void* Ap;            // LayerNorm output, 2 fp16 planes [rows][K] (plane 1 at + a_pstride elements)
    long long a_pstride;
    long long a_rows;          // rows in the planes buffer (range of the A loads)
    const void* Wp;            // q/k/v weights, 2 fp16 planes [3 H 64][K]
    float unscale;             // 1 / (activation scale x weight scale)
    const float* rope_cos;     // [pos][32]
    const float* rope_sin;
    int K;                     // hidden size (multiple of 32)
    int Ts;                    // uniform batches: frames per item (row stride)
    int H;                     // heads (head_dim 64)
    int window;
    float scale;               // 1 / sqrt(64)
    void* outp;                // attention output planes [rows][H 64], plane stride out_pstride
    long long out_pstride;
    float oscale;
    unsigned* oamax;
    const int* tlen;           // ragged batches: frames per item and first packed row (else null)
    const int* toff;
    float* qkv;                // optional: the fp32 q/k/v rows as the GEMM would store them (taps)
    int xcd;                   // 1: an item's heads on one XCD (workgroup order; speed only)
};
hipError_t launch_qkv_attention(const QkvAttnArgs& a, int items, hipStream_t s);

// planes -> fp32 (x0 + x1 [+ x2], or (h0 + h1) / hscale for fp16 planes); used only to materialise per-stage
// taps of plane-format activations.
hipError_t launch_planes_to_f32(const void* planes, long long pstride, int ns, float* out, long long n,
                                hipStream_t s, float hscale = 0.0f);

// Split RVQ: proj [F][2*Dq] (semantic | acoustic projections), codebooks in fragment layout, codes
// out[level][F] int32 (or [b][level][t] when frames_per_item > 0).
struct RvqArgs {
    const float* proj;      // [F][2*D]
    long long frames;
    int D;                  // codebook dim (256)
    int ncodes;             // 2048
    int levels;             // K
    int nsem;               // semantic levels (1)
    const float* cb_frag;   // [level][ncodes/32][D/8][64 lanes][4]
    const float* cb_rows;   // [level][ncodes][D]
    const float* cb_norm;   // [level][ncodes]
    // approximate-then-exact distances (rvq_level_h16_kernel): fp16 planes of embed * cb_scale[level] in
    // 32x32x16 B-fragment order [level][ncodes/32][D/16][2 planes][64 lanes][8 halves], 1 / cb_scale and
    // max_j |embed_j| per level; null -> the all-fp32-MFMA kernel
    const void* cb_h16;
    const float* cb_unscale;
    const float* cb_emax;
    int32_t* codes;
    int32_t* const* codes_ref;  // non-null (a captured hipGraph): the codes pointer is read from here
    int frames_per_item;    // T (for [b][level][t] output); 0 -> [level][frame]
    void* work;             // rvq_work_bytes(frames): residual ping-pong + per-slice partial argmins
    int sem_split;          // (set by launch_rvq) semantic + first acoustic level in one launch
    const int* flen;        // ragged batches: item b's valid frames (frame f of item f / frames_per_item); the
                            // others read a zero projection and their codes are unspecified.  null: all valid
    int form;               // level-kernel form (engine option rvq_form; same codes): 0 default (2), 1 three-product
                            // approximation (round 3), 2..6 one-product variants (launch_rvq)
    int chain;              // small grids: all levels in one persistent launch (rvq_chain_h16_kernel; engine option
                            // rvq_chain; same codes)
    int xcd_group_ok;       // large grids: the slices of a frame tile on one XCD (engine option rvq_xcd; speed only)
    int xcd_group;          // (set by launch_rvq)
    int chain_fault;        // fault injection for the chain's give-up path (engine option rvq_chain_fault, tests only):
                            // 0 off, 1 a zero spin budget, 2 every sweep gives up at once
};
size_t rvq_work_bytes(long long frames);
// kname: the level kernel's symbol.  chain_flag (may be null): set to the device word the persistent chain raises when a
// sweep gave up (the launch's codes are then invalid and the caller re-runs without the chain), or to null when this
// launch did not take the chain
// clear_bytes (with chain_flag): the persistent chain's flag + granules are NOT zeroed here; *clear_bytes = how many
// bytes from *chain_flag the caller zeroes before every launch (a captured graph's replays: set_io_kernel)
hipError_t launch_rvq(const RvqArgs& a, hipStream_t s, const char** kname = nullptr, unsigned** chain_flag = nullptr,
                      size_t* clear_bytes = nullptr);

// polyphase resampler (resample.hip): clips packed at in_off / out_off (device int64 arrays), one launch
hipError_t launch_resample_poly(const float* x, const long long* in_off, const long long* in_len, int nclips,
                                float* y, const long long* out_off, const long long* out_len, long long max_out,
                                const float* h, int lh, int up, int down, long long pre_remove, hipStream_t s);

}  // namespace mimi
