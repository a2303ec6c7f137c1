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
template <int WPT, int UPC>
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
    float* hs = lds;           // the filter, lh taps
    float* xsb = lds + lh;     // input window(s): [2][W] (WPT > 0) or [W]
    const int tid = threadIdx.x;
    for (int i = tid; i < lh; i += RS_BLOCK) hs[i] = h[i];
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

hipError_t launch_resample_poly(const float* x, const long long* in_off, const long long* in_len, int nclips,
                                float* y, const long long* out_off, const long long* out_len, long long max_out,
                                const float* h, int lh, int up, int down, long long pre_remove, hipStream_t s) {
    if (nclips <= 0 || max_out <= 0) return hipSuccess;
    const long long W = resample_window(lh, up, down);
    const int wpt = W <= RS_BLOCK ? 1 : W <= 2 * RS_BLOCK ? 2 : W <= 4 * RS_BLOCK ? 4 : 0;
    const long long lds_bytes = (lh + (wpt > 0 ? 2 : 1) * W) * 4;
    if (lds_bytes > 64 * 1024) return hipErrorInvalidValue;  // default dynamic-LDS limit
    // ~4096 workgroups in all (16 per CU), each sweeping many 256-output passes of one clip: a workgroup per
    // pass would spend more time being dispatched and loading the filter than resampling
    long long bx = (max_out + RS_BLOCK - 1) / RS_BLOCK;
    const long long cap = (4096 + nclips - 1) / nclips;
    if (bx > cap) bx = cap;
    const dim3 grid((unsigned)bx, (unsigned)nclips);
#define RS_LAUNCH(N, U)                                                                                      \
    hipLaunchKernelGGL((resample_poly_kernel<N, U>), grid, dim3(RS_BLOCK), (size_t)lds_bytes, s, x, in_off, in_len, \
                       y, out_off, out_len, h, lh, up, down, pre_remove)
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
