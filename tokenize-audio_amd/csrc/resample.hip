// Host-ingest resampler on the GPU: the polyphase (upfirdn) resampling of librosa's res_type='polyphase'
// (= scipy.signal.resample_poly, Kaiser(5.0) low-pass of 2*10*max(up,down)+1 taps), bit-exact with scipy on
// float32 input.  Ref call sites: librosa.load(path, sr=24000) in librispeech-mimi/utils.py:84-87,
// emilia-mimi/process_shard.py:479-482, yodas2-mimi/process_shard.py:389 (their default soxr_hq mode is
// libsoxr, absent here: unpinned).
//
// Output m of a clip sits at up-sampled position p = (m + pre_remove) * down and is the sum over input
// samples j in [ceil((p - (lh-1)) / up), min(p / up, n_in - 1)] of x[j] * h[p - j*up], added in ASCENDING j
// to a 0-initialised fp32 accumulator with one rounding per product and per add -- the inner-loop order of
// scipy's upfirdn (_upfirdn_apply.pyx), which is what makes the result bitwise equal.
//
// HBM-bound byte work: 4 B read per input sample, 4 B written per output (x re-reads of neighbouring outputs
// are served from LDS: each pass stages its input window once, coalesced); the filter sits in LDS too.  One
// thread per output sample, consecutive outputs on consecutive lanes (coalesced stores); blockIdx.y = clip, so
// a batch of ragged clips is one launch.
#include "kernels.h"

namespace mimi {

constexpr int RS_BLOCK = 256;  // outputs per workgroup pass (one per thread)

// input samples one pass's 256 consecutive outputs touch: ((256-1) * down + lh - 1) / up + 2
__host__ __device__ inline long long resample_window(int lh, int up, int down) {
    return ((long long)(RS_BLOCK - 1) * down + lh - 1) / up + 2;
}

// window start of the pass beginning at output m0: jlo of m0 (jlo is non-decreasing in m)
__device__ __forceinline__ long long pass_w0(long long m0, long long pre_remove, int lh, int up, int down, int kc,
                                             long long* q0o, int* r0o) {
    const long long p0 = (m0 + pre_remove) * down;
    const long long q0 = p0 / up;
    const int r0 = (int)(p0 - q0 * up);
    *q0o = q0;
    *r0o = r0;
    return max(q0 + (r0 - (lh - 1) + kc * up + up - 1) / up - kc, 0LL);
}

// WPT > 0: the next pass's window (<= WPT * 256 samples) is loaded into registers while this pass computes, then
// stored into the other half of a double-buffered LDS window (one barrier per pass, HBM latency hidden);
// WPT == 0: load-then-compute (windows over 1024 samples: extreme ratios only)
// UPC > 0: the up-sampling factor as a compile-time constant (1: 48/72/96 -> 24 kHz, 3: 8/16 -> 24 kHz), so the
// unrolled tap loop's LDS addresses are immediate offsets from two bases (2 ds_read + mul + add per tap); 0:
// any factor, read at run time
// HG: the filter stays in global memory (L2 / L1-cached reads) instead of LDS -- the long linear-phase filters of the
// soxr_hq-spec mode for 44.1 / 22.05 kHz sources (~28-30k taps, ~350 per output phase) do not fit beside the window
template <int WPT, int UPC, bool HG = false>
__global__ __launch_bounds__(RS_BLOCK) void resample_poly_kernel(const float* __restrict__ x,
                                                                 const long long* __restrict__ in_off,
                                                                 const long long* __restrict__ in_len,
                                                                 float* __restrict__ y,
                                                                 const long long* __restrict__ out_off,
                                                                 const long long* __restrict__ out_len,
                                                                 const float* __restrict__ h, int lh, int up_rt,
                                                                 int down, long long pre_remove) {
    const int up = UPC > 0 ? UPC : up_rt;
    extern __shared__ float lds[];
    const int W = (int)resample_window(lh, up, down);
    const float* hs = HG ? h : lds;  // the filter, lh taps
    float* xsb = lds + (HG ? 0 : lh);   // input window(s): [2][W] (WPT > 0) or [W]
    const int tid = threadIdx.x;
    if (!HG)
        for (int i = tid; i < lh; i += RS_BLOCK) lds[i] = h[i];
    const int c = blockIdx.y;
    const long long n_in = in_len[c], n_out = out_len[c];
    const float* __restrict__ xc = x + in_off[c];
    float* __restrict__ yc = y + out_off[c];
    // jlo(p) = max(ceil((p - (lh-1)) / up), 0), jhi(p) = min(floor(p / up), n_in - 1).  64-bit divisions only
    // once per pass (wave-uniform); per output, p = q0*up + pr with pr = r0 + tid*down < 2^31, so the rest is
    // 32-bit: ceil((pr - (lh-1)) / up) = (pr - (lh-1) + kc*up + up-1) / up - kc with kc*up >= lh-1
    const int kc = (lh - 1 + up - 1) / up;
    const long long mstep = (long long)gridDim.x * RS_BLOCK;
    long long m0 = (long long)blockIdx.x * RS_BLOCK;
    if (m0 >= n_out) return;  // whole workgroup: uniform
    long long q0;
    int r0;
    long long w0 = pass_w0(m0, pre_remove, lh, up, down, kc, &q0, &r0);
    float pf[WPT > 0 ? WPT : 1];
    if (WPT > 0) {
#pragma unroll
        for (int u = 0; u < WPT; ++u) {
            const int i = tid + u * RS_BLOCK;
            const long long j = w0 + i;
            if (i < W) xsb[i] = j < n_in ? xc[j] : 0.0f;
        }
    }
    for (int pass = 0; m0 < n_out; ++pass, m0 += mstep) {
        float* xs = xsb + (WPT > 0 ? (pass & 1) * W : 0);
        const long long mn = m0 + mstep;
        long long qn = 0, wn = 0;
        int rn = 0;
        if (WPT > 0) {
            // issue the next pass's window loads now; they land while this pass computes
            if (mn < n_out) wn = pass_w0(mn, pre_remove, lh, up, down, kc, &qn, &rn);
#pragma unroll
            for (int u = 0; u < WPT; ++u) {
                const int i = tid + u * RS_BLOCK;
                const long long j = wn + i;
                pf[u] = (mn < n_out && i < W && j < n_in) ? xc[j] : 0.0f;
            }
        } else {
            __syncthreads();  // previous pass done with xs
            for (int i = tid; i < W; i += RS_BLOCK) {
                const long long j = w0 + i;
                xs[i] = j < n_in ? xc[j] : 0.0f;
            }
        }
        __syncthreads();  // this pass's window (and, first pass, the filter) visible
        const long long m = m0 + tid;
        if (m < n_out) {
            const int pr = r0 + tid * down;
            const long long jhi = min(q0 + pr / up, n_in - 1);
            const long long jlo = max(q0 + (pr - (lh - 1) + kc * up + up - 1) / up - kc, 0LL);
            float acc = 0.0f;
            const int k = pr - (int)(jlo - q0) * up;  // filter index of the first term (< lh)
            const float* xp = xs + (int)(jlo - w0);
            const float* hp = hs + k;
            const int cnt = (int)(jhi - jlo + 1);
#pragma unroll 8
            for (int t = 0; t < cnt; ++t) acc = __fadd_rn(acc, __fmul_rn(xp[t], hp[-t * up]));
            yc[m] = acc;
        }
        if (WPT > 0) {
            // the other buffer was last read in the previous pass, which every thread finished before this
            // pass's barrier: safe to fill without another barrier
            float* xn = xsb + ((pass + 1) & 1) * W;
#pragma unroll
            for (int u = 0; u < WPT; ++u) {
                const int i = tid + u * RS_BLOCK;
                if (i < W) xn[i] = pf[u];
            }
            q0 = qn;
            r0 = rn;
            w0 = wn;
        }
    }
}

// ---- specialised register FIR for the common up-sampling pairs (16 / 8 kHz -> 24 kHz: up 3)
// With (up, down) fixed, resample_poly's filter length and n_pre_remove are constants, and for a pass that starts
// at an output m0 = 0 (mod up) every output's tap phase, tap count and input offset relative to the pass are
// compile-time functions of its position.  Each thread computes R consecutive outputs (R a multiple of up): it
// loads its NX-sample input window from LDS into registers once and keeps the up phases' taps in registers, so a
// tap is one fmul + one fadd (same order and roundings as the generic kernel: ascending input index).  Passes
// touching a clip edge (left zero region, right end) take the generic per-output path.
__host__ __device__ constexpr int rs_cdiv(int a, int b) { return a >= 0 ? (a + b - 1) / b : -((-a) / b); }
__host__ __device__ constexpr int rs_fdiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

template <int UP, int DOWN, int R>
struct RsFir {
    static constexpr int MR = UP > DOWN ? UP : DOWN;
    static constexpr int HALF = 10 * MR;
    static constexpr int PREPAD = DOWN - HALF % DOWN;
    static constexpr int LH = 2 * HALF + 1 + PREPAD;     // filter taps incl. the zero pre-padding
    static constexpr int PRE = (HALF + PREPAD) / DOWN;   // n_pre_remove
    static constexpr int C0 = (PRE * DOWN) % UP;         // p(m0) mod up for m0 = 0 (mod up)
    // output r of a thread's group (its first output at m = 0 mod up):
    static constexpr int jlo(int r) { return rs_cdiv(C0 + r * DOWN - (LH - 1), UP); }  // relative to floor(p0/up)
    static constexpr int jhi(int r) { return rs_fdiv(C0 + r * DOWN, UP); }
    static constexpr int off(int r) { return jlo(r) - jlo(0); }                          // input offset of output r
    static constexpr int cnt(int r) { return jhi(r) - jlo(r) + 1; }                      // its taps
    static constexpr int kfirst(int r) { return C0 + r * DOWN - UP * jlo(r); }           // its first filter index
    static constexpr int NT = cnt(0) > cnt(UP - 1) ? cnt(0) : cnt(UP - 1);               // (bounds every phase)
    static constexpr int NX = off(R - 1) + cnt(R - 1);                                   // window per thread
    static constexpr int TSTEP = R / UP * DOWN;                                           // window shift per thread
    static constexpr int W = TSTEP * (RS_BLOCK - 1) + NX;                                // window per pass
    static_assert(R % UP == 0, "R");
};

template <int UP, int DOWN, int R>
__global__ __launch_bounds__(RS_BLOCK) void resample_fir_kernel(const float* __restrict__ x,
                                                                const long long* __restrict__ in_off,
                                                                const long long* __restrict__ in_len,
                                                                float* __restrict__ y,
                                                                const long long* __restrict__ out_off,
                                                                const long long* __restrict__ out_len,
                                                                const float* __restrict__ h) {
    using F = RsFir<UP, DOWN, R>;
    constexpr int LH = F::LH, PRE = F::PRE, NT = F::NT, NX = F::NX, W = F::W;
    __shared__ float hs[LH];
    __shared__ float xs[W];
    const int tid = threadIdx.x;
    for (int i = tid; i < LH; i += RS_BLOCK) hs[i] = h[i];
    __syncthreads();
    // the up phases' taps, in the order each output adds them (wave-uniform loads from the kernel argument:
    // they can stay in scalar registers)
    float hr[UP][NT];
#pragma unroll
    for (int r = 0; r < UP; ++r)
#pragma unroll
        for (int i = 0; i < NT; ++i) hr[r][i] = i < F::cnt(r) ? h[F::kfirst(r) - i * UP] : 0.0f;
    const int c = blockIdx.y;
    const long long n_in = in_len[c], n_out = out_len[c];
    const float* __restrict__ xc = x + in_off[c];
    float* __restrict__ yc = y + out_off[c];
    constexpr int PASS = RS_BLOCK * R;
    for (long long m0 = (long long)blockIdx.x * PASS; m0 < n_out; m0 += (long long)gridDim.x * PASS) {
        const long long p0 = (m0 + PRE) * DOWN;
        const long long q0 = (p0 - F::C0) / UP;            // exact: p0 = C0 (mod up)
        const long long w0 = q0 + F::jlo(0);                // first input of the pass (unclamped)
        const long long mlast = m0 + PASS - 1;
        const bool interior = w0 >= 0 && mlast < n_out && (mlast + PRE) * DOWN / UP <= n_in - 1;
        __syncthreads();  // previous pass done with xs
        if (interior) {
            for (int i = tid; i < W; i += RS_BLOCK) xs[i] = xc[w0 + i];
            __syncthreads();
            float xr[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) xr[i] = xs[tid * F::TSTEP + i];
            const long long mt = m0 + (long long)tid * R;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                float acc = 0.0f;
#pragma unroll
                for (int i = 0; i < NT; ++i)
                    if (i < F::cnt(r % UP)) acc = __fadd_rn(acc, __fmul_rn(xr[F::off(r) + i], hr[r % UP][i]));
                yc[mt + r] = acc;
            }
        } else {
            // edge pass: each output on its own (clamped j range, taps from LDS, inputs from global)
            const int kc = (LH - 1 + UP - 1) / UP;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const long long m = m0 + (long long)tid * R + r;
                if (m >= n_out) continue;
                const long long p = (m + PRE) * DOWN;
                const long long jhi = min(p / UP, n_in - 1);
                const long long jlo = max((p - (LH - 1) + (long long)kc * UP + UP - 1) / UP - kc, 0LL);  // ceil
                float acc = 0.0f;
                for (long long j = jlo; j <= jhi; ++j) acc = __fadd_rn(acc, __fmul_rn(xc[j], hs[p - j * UP]));
                yc[m] = acc;
            }
        }
    }
}

hipError_t launch_resample_poly(const float* x, const long long* in_off, const long long* in_len, int nclips,
                                float* y, const long long* out_off, const long long* out_len, long long max_out,
                                const float* h, int lh, int up, int down, long long pre_remove, hipStream_t s) {
    if (nclips <= 0 || max_out <= 0) return hipSuccess;
    {
        // specialised register FIR (the filter and pre-removal are what resample_poly builds for that pair)
        long long bx = (max_out + RS_BLOCK * 3 - 1) / (RS_BLOCK * 3);
        const long long cap = (4096 + nclips - 1) / nclips;
        if (bx > cap) bx = cap;
#define RS_FIR(U, D, R)                                                                                        \
    if (up == U && down == D && lh == RsFir<U, D, R>::LH && pre_remove == RsFir<U, D, R>::PRE) {               \
        long long b = (max_out + RS_BLOCK * R - 1) / (RS_BLOCK * R);                                            \
        if (b > cap) b = cap;                                                                                  \
        hipLaunchKernelGGL((resample_fir_kernel<U, D, R>), dim3((unsigned)b, (unsigned)nclips), dim3(RS_BLOCK), 0, \
                           s, x, in_off, in_len, y, out_off, out_len, h);                                      \
        return hipGetLastError();                                                                              \
    }
        (void)bx;
        RS_FIR(3, 2, 3)  // 16 kHz -> 24 kHz
        RS_FIR(3, 1, 3)  // 8 kHz -> 24 kHz
        // (1, 2) -- 48 kHz -> 24 kHz -- measured slower as a register FIR (43 taps x 4 outputs: 115 VGPRs, half
        // the occupancy): 0.70 vs 0.52 ms per 256 x 10 s; it stays on the generic kernel
#undef RS_FIR
    }
    const long long W = resample_window(lh, up, down);
    const int wpt = W <= RS_BLOCK ? 1 : W <= 2 * RS_BLOCK ? 2 : W <= 4 * RS_BLOCK ? 4 : 0;
    long long lds_bytes = (lh + (wpt > 0 ? 2 : 1) * W) * 4;
    const bool hg = lds_bytes > 64 * 1024;  // default dynamic-LDS limit: the filter is read from global memory
    if (hg) lds_bytes -= (long long)lh * 4;
    if (lds_bytes > 64 * 1024) return hipErrorInvalidValue;
    // ~4096 workgroups in all (16 per CU), each sweeping many 256-output passes of one clip: a workgroup per
    // pass would spend more time being dispatched and loading the filter than resampling
    long long bx = (max_out + RS_BLOCK - 1) / RS_BLOCK;
    const long long cap = (4096 + nclips - 1) / nclips;
    if (bx > cap) bx = cap;
    const dim3 grid((unsigned)bx, (unsigned)nclips);
#define RS_LAUNCH(N, U)                                                                                          \
    if (hg)                                                                                                      \
        hipLaunchKernelGGL((resample_poly_kernel<N, 0, true>), grid, dim3(RS_BLOCK), (size_t)lds_bytes, s, x,   \
                           in_off, in_len, y, out_off, out_len, h, lh, up, down, pre_remove);                    \
    else                                                                                                         \
        hipLaunchKernelGGL((resample_poly_kernel<N, U>), grid, dim3(RS_BLOCK), (size_t)lds_bytes, s, x, in_off,  \
                           in_len, y, out_off, out_len, h, lh, up, down, pre_remove)
#define RS_LAUNCH_W(U)              \
    switch (wpt) {                  \
        case 1: RS_LAUNCH(1, U); break; \
        case 2: RS_LAUNCH(2, U); break; \
        case 4: RS_LAUNCH(4, U); break; \
        default: RS_LAUNCH(0, U); break; \
    }
    if (up == 3) {
        RS_LAUNCH_W(3);
    } else if (up == 1) {
        RS_LAUNCH_W(1);
    } else {
        RS_LAUNCH_W(0);
    }
#undef RS_LAUNCH_W
#undef RS_LAUNCH
    return hipGetLastError();
}

}  // namespace mimi
