// Mimi encode engine: weights, workspace, stage sequencing and the C ABI of include/mimi_hip.h.
//
// Data layout in HBM (all fp32, channels-last so that every conv is a plain GEMM, see gemm.hip):
//   audio            [B][L]
//   SEANet stage s   x_s [B][T_s][C_s]  (C_s = 64 << s, T_0 = L, T_{s+1} = ceil(T_s / ratio_s))
//   transformer      [B][T][512]  (T = T_4 frames at 25 Hz), fused qkv [B][T][1536], mlp [B][T][2048]
//   quantizer input  [B*T'][512]  (T' = ceil(T/2) frames at 12.5 Hz), projections [B*T'][512]
//   codes            int32 [B][K][T']
// Weights are re-laid out once at finalize: conv W[co][ci][k] -> W'[co][k*Cin + ci]; q/k/v fused into
// one [1536][512]; the two input_proj stacked into one [512][512]; codebooks materialised as
// embed = embed_sum / clamp(cluster_usage, eps) (TF/modeling_mimi.py:979-983) in row layout (for the
// residual update) and in MFMA-fragment layout (for the distance GEMM), with |e|^2 in torch's order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "../../include/mimi_hip.h"
#include "host_io.h"
#include "kernels.h"

using namespace mimi;

// ------------------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------------------
static thread_local std::string g_last_error;

static int set_err(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                                \
    do {                                                                                             \
        hipError_t _e = (expr);                                                                      \
        if (_e != hipSuccess) {                                                                      \
            return set_err(_e == hipErrorOutOfMemory ? MIMI_ERR_OUT_OF_MEMORY : MIMI_ERR_HIP,        \
                           "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
        }                                                                                            \
    } while (0)

extern "C" const char* mimi_last_error(void) { return g_last_error.c_str(); }

namespace mimi {
// for the host-side C ABI files (flac.cpp): one thread-local last error behind mimi_last_error
int set_last_error(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}
}  // namespace mimi

int mimi::set_error_message(int code, const char* msg) {
    g_last_error = msg;
    return code;
}

// ------------------------------------------------------------------------------------------------
// config / length math
// ------------------------------------------------------------------------------------------------
// mimi_config_default and mimi_config_from_json: config_json.cpp (host-only)

// MimiConv1d output length, reproducing the reference's float32 tensor arithmetic
// (TF/modeling_mimi.py:269-279): n_frames = ceil(float32(L - s) / float32(s) + 1) - 1; out = n_frames + 1.
static int64_t conv_out_len(int64_t length, int kernel, int stride) {
    const int64_t pt = kernel - stride;
    volatile float num = (float)(length - kernel + pt);
    volatile float q = num / (float)stride;
    volatile float nf = q + 1.0f;
    const int64_t n_frames = (int64_t)std::ceil((float)nf) - 1;
    return n_frames + 1;
}

struct StagePlan {
    int64_t T[5];  // T[0] = conv0 out; T[s+1] = down conv s out
    int64_t frames25, frames12;
};

static StagePlan plan_lengths(const mimi_config& c, int64_t L) {
    StagePlan p{};
    int64_t t = conv_out_len(L, c.kernel_size, 1);
    p.T[0] = t;
    for (int s = 0; s < c.num_ratios; ++s) {
        const int ratio = c.upsampling_ratios[c.num_ratios - 1 - s];
        t = conv_out_len(t, c.residual_kernel_size, 1);
        t = conv_out_len(t, 1, 1);
        t = conv_out_len(t, 2 * ratio, ratio);
        p.T[s + 1] = t;
    }
    t = conv_out_len(t, c.last_kernel_size, 1);
    p.frames25 = t;
    p.frames12 = conv_out_len(t, c.downsample_kernel, c.downsample_stride);
    return p;
}

extern "C" int64_t mimi_encoded_length_cfg(const mimi_config* cfg, int64_t length) {
    mimi_config d;
    if (!cfg) {
        mimi_config_default(&d);
        cfg = &d;
    }
    if (length < 0) return -1;
    return plan_lengths(*cfg, length).frames12;
}

extern "C" int64_t mimi_encoded_length(int64_t length) { return mimi_encoded_length_cfg(nullptr, length); }

// ------------------------------------------------------------------------------------------------
// host-ingest resampler (no engine handle: pure function of its device buffers)
// ------------------------------------------------------------------------------------------------
extern "C" int mimi_resample_poly(const float* dev_in, const int64_t* dev_in_off, const int64_t* dev_in_len,
                                  int32_t nclips, float* dev_out, const int64_t* dev_out_off,
                                  const int64_t* dev_out_len, int64_t max_out, const float* dev_filter,
                                  int32_t filter_len, int32_t up, int32_t down, int64_t pre_remove, void* stream) {
    if (nclips < 0 || up < 1 || down < 1 || pre_remove < 0 || max_out < 0)
        return set_err(MIMI_ERR_INVALID_ARGUMENT, "mimi_resample_poly: bad sizes (nclips %d, up %d, down %d)",
                       nclips, up, down);
    if (filter_len < 1 || filter_len > MIMI_RESAMPLE_MAX_TAPS)
        return set_err(MIMI_ERR_UNSUPPORTED, "mimi_resample_poly: filter of %d taps (max %d)", filter_len,
                       MIMI_RESAMPLE_MAX_TAPS);
    if (nclips == 0 || max_out == 0) return MIMI_OK;
    if (!dev_in || !dev_in_off || !dev_in_len || !dev_out || !dev_out_off || !dev_out_len || !dev_filter)
        return set_err(MIMI_ERR_INVALID_ARGUMENT, "mimi_resample_poly: null buffer");
    const hipError_t e = launch_resample_poly(dev_in, reinterpret_cast<const long long*>(dev_in_off),
                                              reinterpret_cast<const long long*>(dev_in_len), nclips, dev_out,
                                              reinterpret_cast<const long long*>(dev_out_off),
                                              reinterpret_cast<const long long*>(dev_out_len), max_out, dev_filter,
                                              filter_len, up, down, pre_remove, (hipStream_t)stream);
    if (e != hipSuccess) return set_err(MIMI_ERR_HIP, "resample_poly launch: %s", hipGetErrorString(e));
    return MIMI_OK;
}

extern "C" int mimi_split_check(const float* dev_in, int64_t npairs, float scale, uint32_t* dev_out, void* stream) {
    if (npairs < 0 || (npairs > 0 && (!dev_in || !dev_out)) || !(scale > 0.0f))
        return set_err(MIMI_ERR_INVALID_ARGUMENT, "mimi_split_check: bad arguments");
    const hipError_t e = launch_split_check(dev_in, npairs, scale, dev_out, (hipStream_t)stream);
    if (e != hipSuccess) return set_err(MIMI_ERR_HIP, "split_check launch: %s", hipGetErrorString(e));
    return MIMI_OK;
}

extern "C" int mimi_gelu_check(const float* dev_in, int64_t n, float* dev_out, void* stream) {
    if (n < 0 || (n > 0 && (!dev_in || !dev_out))) return set_err(MIMI_ERR_INVALID_ARGUMENT, "mimi_gelu_check: bad arguments");
    const hipError_t e = launch_gelu_check(dev_in, n, dev_out, (hipStream_t)stream);
    if (e != hipSuccess) return set_err(MIMI_ERR_HIP, "gelu_check launch: %s", hipGetErrorString(e));
    return MIMI_OK;
}

// ------------------------------------------------------------------------------------------------
// engine
// ------------------------------------------------------------------------------------------------
struct DevConv {
    int cin = 0, cout = 0, k = 0, stride = 1;
    float* w = nullptr;      // [cout][k*cin]
    void* wsplit = nullptr;  // bf16 planes [3][cout][k*cin] of w (split-bf16 precision modes)
    void* wh = nullptr;      // fp16 planes [2][cout][k*cin] of w * wscale (PREC_F16X3)
    float wscale = 1.0f;
    float* wfrag = nullptr;  // w in 32x32x2-MFMA fragment order [cout/32][k*cin/8][64][4] (stage-0 block)
    float* b = nullptr;      // [cout] or null
};

#ifndef MIMI_LN_CHECK_SKIP
#define MIMI_LN_CHECK_SKIP 1  // (A/B) 0: every LayerNorm output keeps its range-check atomics
#endif
struct DevXfmr {
    float *ln1_w, *ln1_b, *wqkv, *wo, *ls1, *ln2_w, *ln2_b, *w1, *w2, *ls2;
    void *wqkv_s, *wo_s, *w1_s, *w2_s;  // bf16 planes
    void *wqkv_h, *wo_h, *w1_h, *w2_h;  // fp16 planes (x scale)
    float wqkv_hs, wo_hs, w1_hs, w2_hs;
    // max |LayerNorm output| any input can give: max_c |gamma_c| sqrt(D - 1) + |beta_c| (a normalised value is at most
    // sqrt(D - 1) in magnitude; x 1.001 for rounding).  Below the fp16 plane limit at the tensor's scale, the
    // output's range check cannot fire and its max |x| atomics are skipped.
    float ln1_bound = INFINITY, ln2_bound = INFINITY;
};

struct ProfEvent {
    std::string name;  // "stage|kernel symbol"

    hipEvent_t ev;
    double flops;
    double bytes;
};

struct ProfStat {
    double ms = 0, flops = 0, bytes = 0;
    int64_t launches = 0;
};

constexpr int kMaxActSlots = 256;  // plane-format tensors per encode (~41 for kyutai/mimi)

struct mimi_engine {
    mimi_config cfg;
    int device = 0;
    std::mutex mu;
    bool finalized = false;
    int levels_available = 0;
    int precision = PREC_F16X3;
    // planes path: residual blocks of stages >= kUnfuseFrom run as two plane GEMMs (k3 -> h planes, k1 + skip);
    // stages 0 and 1 run the fused fp16 blocks (resblock.hip)
    static constexpr int kUnfuseFrom = 2;

    std::unordered_map<std::string, std::vector<float>> host_w;
    std::unordered_map<std::string, std::vector<int64_t>> expected;  // name -> shape
    std::vector<void*> allocations;

    DevConv conv0;
    std::vector<DevConv> res3, res1, down;
    // PREC_F16X3 fused stage-0 block: conv0 / W3 / W1 fp16-plane A fragments (resblock.hip r0h) and their scales
    void* res0_h16 = nullptr;
    float res0_wsc[3] = {1.0f, 1.0f, 1.0f};
    // ... and the stage-1 (C = 128) block: W3 / W1 16x16x32 fragments and scales
    void* res1_h16 = nullptr;
    float res1_wsc[2] = {1.0f, 1.0f};
    DevConv final_conv;
    std::vector<DevXfmr> xf;
    DevConv ds;
    float* inproj = nullptr;  // [2*vq][hidden]
    void* inproj_h = nullptr;   // its fp16 planes (PREC_F16X3)
    float inproj_hs = 1.0f;
    float* ds_fix = nullptr;    // [2][hidden in][hidden out]: W_0 + W_1 and W_3 of the downsample (replicate edges)
    float* cb_rows = nullptr;
    float* cb_frag = nullptr;
    float* cb_norm = nullptr;
    void* cb_h16 = nullptr;       // fp16 planes for the approximate distances (ops.hip rvq_level_h16_kernel)
    float* cb_unscale = nullptr;  // [level]
    float* cb_emax = nullptr;     // [level]

    float* rope_cos = nullptr;
    float* rope_sin = nullptr;
    int64_t rope_T = 0;

    void* ws = nullptr;
    size_t ws_bytes = 0;

    hipEvent_t ws_free = nullptr;  // recorded at the end of every encode: the next one (any stream) waits on it

    // PREC_F16X3 activation scales (see "activation scales" above calibrate_scales): plane-format tensor `name`
    // is stored as fp16 planes of x * act_scale[slot_of[name]], a power of two fixed at mimi_finalize from a
    // calibration encode -- never from the caller's audio, so codes are a pure function of each item's input.
    // Its producer max-reduces |x| into amax_dev[slot] for the overflow check.
    std::map<std::string, int> slot_of;
    std::vector<float> act_scale;
    bool calibrating = false;
    bool calibrated = false;         // calibrate_scales has run (lazily, before the first f16x3 encode)
    bool uncalibrated_slot = false;  // the current encode named a tensor the calibration did not see (reset per encode)
    unsigned* amax_dev = nullptr;   // [kMaxActSlots][AMAX_SLOT_WORDS] sub-slots, then [kMaxActSlots] reduced
    unsigned* amax_red = nullptr;
    unsigned* amax_host = nullptr;  // pinned
    int32_t* item_codes = nullptr;  // one item's codes (per-item overflow fallback)
    // encodes enqueued by mimi_encode_async and not yet waited (see encode_async_locked)
    struct Pending {
        int64_t id = 0;  // ticket; 0 = free
        bool claimed = false;  // a mimi_encode_wait is synchronising on it (outside the engine lock)
        hipEvent_t done = nullptr;
        unsigned* amax = nullptr;  // pinned [kMaxActSlots]: this encode's per-tensor maxima (f16x3)
        int nslots = 0;
        bool h16 = false;
        const float* audio = nullptr;
        int B = 0, K = 0;
        int64_t L = 0;
        int32_t* codes = nullptr;
        hipStream_t s = nullptr;
        bool ragged = false;          // a ragged batch (lens: the items' lengths, for the overflow fallback)
        std::vector<int64_t> lens;
        int* rg_pinned = nullptr;     // pinned image of its RaggedTable (read by the encode's async upload)
        size_t rg_cap = 0;
        bool chain = false;           // the encode ran the persistent RVQ chain: chain_word holds its give-up flag
        unsigned* chain_word = nullptr;  // pinned, copied from the chain's flag behind the encode
    };
    static constexpr int kMaxPending = 16;
    Pending pend[kMaxPending];
    // mimi_encode_host's buffers: one set per concurrent caller, claimed under mu, grown on demand
    struct HostIo {
        bool busy = false;
        float* d_audio = nullptr;
        float* h_audio = nullptr;    // pinned staging of the caller's samples (the H2D then runs under the launches)
        size_t audio_cap = 0;        // bytes (both audio buffers)
        int32_t* d_codes = nullptr;
        int32_t* h_codes = nullptr;  // pinned
        size_t codes_cap = 0;        // bytes (both code buffers)
        hipEvent_t done = nullptr;   // the codes' D2H
    };
    HostIo hostio[kMaxPending];
    int64_t next_ticket = 1;
    size_t item_codes_cap = 0;
    int f16_reruns = 0;             // encodes that took the overflow fallback (diagnostic)
    std::vector<float> last_amax;   // per-slot max|x| of the last waited f16x3 encode (diagnostic)
    int profiling = 0;  // 1: every stage between events; 2: the first stage of each pass only (two events)
    std::vector<ProfEvent> pending;  // recorded since last read; first event of each encode named ""
    std::vector<hipEvent_t> event_pool;
    std::map<std::string, ProfStat> prof;
    std::vector<std::string> prof_order;
    std::vector<std::string> last_seq;  // "stage|kernel" of the last profiled encode, in launch order

    // hipGraph replay of the f16x3 encode (see graph_encode): one captured graph per (batch, length, K), the
    // audio / codes pointers passed through io_dev
    struct Graph {
        int B = 0, K = 0;
        int64_t L = 0;
        int ws_gen = 0, rope_gen = 0;
        hipGraph_t g = nullptr;
        hipGraphExec_t x = nullptr;
        uint64_t used = 0;
        unsigned* chain_flag = nullptr;  // the captured RVQ chain's give-up flag (null: no chain in the graph)
        size_t chain_clear = 0;          // bytes from chain_flag zeroed before each replay (set_io_kernel)
    };
    static constexpr int kMaxGraphs = 8;
    std::vector<Graph> graphs;
    std::map<std::tuple<int, int64_t, int>, int> graph_seen;  // eager encodes per shape (capture on the 2nd)
    bool graphs_enabled = true;
    bool capturing = false;
    void** io_dev = nullptr;  // [audio, codes, pinned maxima, pinned give-up word] of the replay
    size_t cap_chain_clear = 0;  // (capture) the captured chain's flag + granule bytes
    hipStream_t cap_stream = nullptr;
    int ws_gen = 0, rope_gen = 0;
    uint64_t graph_clock = 0;
    int64_t graph_replays = 0;

    bool taps = false;
    int stage0_fused = 1;  // 0: stage-0 block + down conv 0 as two kernels; 1: one fused kernel
    // LayerNorm prologue on small grids (gemm_planes.h FL_LNA): 0 off, 1 fc1 (default), 2 fc1 and q/k/v.  Batch 1
    // (rocprofv3, profiles/r3j_*): fc1 15.0 us with it vs 10.1 + 5.2 us (+ a launch gap) for fc1 + LayerNorm; q/k/v
    // 20.8 vs 10.4 + 5.2 us -- its one compute wave and 16-row tiles leave the prologue's chain exposed
    int ln_fused = 1;
    int rvq_form = 0;  // RVQ level-kernel form (mimi_set_option "rvq_form"; RvqArgs::form)
    int ln_rpw = 1;  // LayerNorm rows per wave (mimi_set_option "ln_rpw": 1 (A/B r4h: 0.186 vs 0.200 ms per B = 32 step for 2), 2, 4, 8; the same bits)
    int rvq_xcd = 1;  // large grids: a frame tile's RVQ slices on one XCD (mimi_set_option "rvq_xcd"; same bits)
    int rvq_chain = 1;  // small grids: the persistent all-levels RVQ (mimi_set_option "rvq_chain"; RvqArgs::chain)
    // The chain is taken only where its give-up flag is read back (chain_ok: the main encode path, whose ticket carries
    // the flag to mimi_encode_wait, and mimi_rvq_encode, which checks it itself); every fallback and internal pass runs
    // the per-level kernels.  chain_flag: the flag word of the chain launched by the last run_rvq (null: none)
    bool chain_ok = false;
    unsigned* chain_flag = nullptr;
    int rvq_chain_fault = 0;    // tests only (mimi_set_option "rvq_chain_fault"; RvqArgs::chain_fault)
    int64_t chain_reruns = 0;   // encodes re-run without the chain after a sweep gave up (diagnostic)
    // q/k/v + attention as one kernel (qkv_attn.hip) for items of <= 256 frames: 0 off, 1 when the batch has at least
    // 256 (item, head) pairs (one workgroup per CU), 2 whenever the items fit (mimi_set_option "qkv_attn"; same bits)
    int qkv_attn = 1;
    int qkv_attn_xcd = 1;  // its workgroups: an item's heads on one XCD (mimi_set_option "qkv_attn_xcd"; same bits)
    int attn_band_split = 1;  // items over 256 frames: the banded attention's decomposition (0 / 1 auto / 2; same bits)
    // transformer GEMMs with sc1 output stores (gemm_planes.h FL_SC1OUT; mimi_set_option "sc1_out"): bit 0 q/k/v,
    // bit 1 fc1, bit 2 o_proj and fc2 (large batches; the same bits either way)
    int sc1_out = 2;  // (A/B, round 4: fc1 0.594 -> 0.576 ms per B = 32 step; q/k/v, o_proj and fc2 slower with it)
    // fc1's tile order in XCD column groups (GemmArgs::ncg, gemm_planes.h; mimi_set_option "fc1_cg": 0 / 1 none, 2, 4;
    // same bits): each XCD re-serves 1 / fc1_cg of W1 from its L2.  (A/B r4y: 2 groups cut fc1's fetch 85 -> 54 MB per
    // launch but not its time, 0.59-0.60 vs 0.61-0.62 ms per step; profiles/r4y_ab_fc1_cg.txt)
    int fc1_cg = 1;
    // stage-1 fp16 block form (resblock.hip resblock128_h16_kernel; mimi_set_option "res1_form"; same bits): 0 one
    // 8-wave workgroup per CU, 1 two 4-wave workgroups per CU (each wave both 16-step tiles of its M tile; their block
    // chains interleave on the SIMDs: 0.59 -> 0.555 ms per B = 32 step, profiles/r4aa_ab_res1_form.txt)
    int res1_form = 1;
    // the k1 conv + skip + ELU as the streaming kernel (res1_stream.hip) instead of the planes GEMM (mimi_set_option
    // "res1_stream": 1 stage 2 (default), 2 stages 2 and 3, 0 off; same bits): res1_s2 0.229-0.231 -> 0.218-0.221 ms
    // per B = 32 step (round 5); stage 3 measured slower on it, 0.116-0.117 vs 0.109-0.113 (round 6, r6d / r6e)
    int res1_stream = 1;
    struct Tap {
        float* d = nullptr;
        size_t cap = 0;
        int64_t dims[3] = {0, 0, 0};
    };
    std::map<std::string, Tap> tapmap;
};

static int dev_alloc(mimi_engine* e, void** p, size_t bytes) {
    hipError_t err = hipMalloc(p, bytes);
    if (err != hipSuccess) {
        (void)hipGetLastError();
        return set_err(err == hipErrorOutOfMemory ? MIMI_ERR_OUT_OF_MEMORY : MIMI_ERR_HIP, "hipMalloc(%zu): %s",
                       bytes, hipGetErrorString(err));
    }
    e->allocations.push_back(*p);
    return MIMI_OK;
}

static int upload(mimi_engine* e, float** dst, const std::vector<float>& host) {
    int rc = dev_alloc(e, reinterpret_cast<void**>(dst), host.size() * sizeof(float));
    if (rc) return rc;
    HIP_TRY(hipMemcpy(*dst, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice));
    return MIMI_OK;
}

// x = x0 + x1 + x2 with x_p = bf16_rne(x - x0 - ... - x_{p-1}) (each subtraction exact in fp32)
static uint16_t f2bf_rne(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    u += 0x7FFF + ((u >> 16) & 1);
    return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t h) {
    const uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

static int upload_split(mimi_engine* e, void** dst, const std::vector<float>& host) {
    const size_t n = host.size();
    std::vector<uint16_t> planes(3 * n);
    for (size_t i = 0; i < n; ++i) {
        float r = host[i];
        for (int p = 0; p < 3; ++p) {
            const uint16_t h = f2bf_rne(r);
            planes[p * n + i] = h;
            r = r - bf2f(h);
        }
    }
    int rc = dev_alloc(e, dst, planes.size() * sizeof(uint16_t));
    if (rc) return rc;
    HIP_TRY(hipMemcpy(*dst, planes.data(), planes.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    return MIMI_OK;
}

// fp16 planes of w * scale: h0 = fp16(w s), h1 = fp16(w s - h0) (22-bit significand), scale a power of two
// putting max|w| s in [2^13, 2^14): every weight >= 2^-17 max|w| keeps its full 22 bits, and no product of a
// plane with an activation plane (|x s_x| < 2^15) can overflow the fp32 accumulator
static int upload_f16(mimi_engine* e, void** dst, const std::vector<float>& host, float* scale) {
    const size_t n = host.size();
    float wmax = 0.0f;
    for (float v : host) wmax = std::max(wmax, std::fabs(v));
    const float sc = wmax > 0.0f && std::isfinite(wmax) ? std::ldexp(1.0f, 13 - std::ilogb(wmax)) : 1.0f;
    std::vector<_Float16> planes(2 * n);
    for (size_t i = 0; i < n; ++i) {
        const float t = host[i] * sc;
        const _Float16 h0 = (_Float16)t;
        planes[i] = h0;
        planes[n + i] = (_Float16)(t - (float)h0);
    }
    int rc = dev_alloc(e, dst, planes.size() * sizeof(_Float16));
    if (rc) return rc;
    HIP_TRY(hipMemcpy(*dst, planes.data(), planes.size() * sizeof(_Float16), hipMemcpyHostToDevice));
    *scale = sc;
    return MIMI_OK;
}

// power of two putting max|w| s in [2^13, 2^14) (see upload_f16)
static float f16_weight_scale(const std::vector<float>& w) {
    float wmax = 0.0f;
    for (float v : w) wmax = std::max(wmax, std::fabs(v));
    return wmax > 0.0f && std::isfinite(wmax) ? std::ldexp(1.0f, 13 - std::ilogb(wmax)) : 1.0f;
}

// Appends W [M][K] (row-major) * sc as fp16 planes in 32x32x16-MFMA A-fragment order, [mt][ks][plane] 1-KB
// fragments of [64 lanes][8 halves]: lane (i, h) holds W[32 mt + i][16 ks + 8 h + e].
static void append_afrags_h16(std::vector<_Float16>& out, const std::vector<float>& w, int M, int K, float sc) {
    for (int mt = 0; mt < M / 32; ++mt)
        for (int ks = 0; ks < K / 16; ++ks)
            for (int pl = 0; pl < 2; ++pl)
                for (int lane = 0; lane < 64; ++lane)
                    for (int e = 0; e < 8; ++e) {
                        const float t = w[(size_t)(32 * mt + (lane & 31)) * K + 16 * ks + 8 * (lane >> 5) + e] * sc;
                        const _Float16 h0 = (_Float16)t;
                        out.push_back(pl == 0 ? h0 : (_Float16)(t - (float)h0));
                    }
}

// W [N][K] -> Wf[nt][kq][lane][s] = W[32*nt + (lane & 31)][8*kq + 4*(lane >> 5) + s]: a wave's B fragment
// for one 8-wide K quad of one 32-column tile is one contiguous 1 KB load.
static std::vector<float> frag_layout(const std::vector<float>& w, int N, int K) {
    std::vector<float> f((size_t)N * K);
    for (int nt = 0; nt < N / 32; ++nt)
        for (int kq = 0; kq < K / 8; ++kq)
            for (int lane = 0; lane < 64; ++lane)
                for (int s = 0; s < 4; ++s)
                    f[(((size_t)nt * (K / 8) + kq) * 64 + lane) * 4 + s] =
                        w[(size_t)(32 * nt + (lane & 31)) * K + 8 * kq + 4 * (lane >> 5) + s];
    return f;
}

static std::string conv_name_first() { return "encoder.layers.0.conv"; }

static void build_expected(mimi_engine* e) {
    const mimi_config& c = e->cfg;
    auto& ex = e->expected;
    ex.clear();
    ex[conv_name_first() + ".weight"] = {c.num_filters, c.audio_channels, c.kernel_size};
    ex[conv_name_first() + ".bias"] = {c.num_filters};
    int idx = 1;
    int C = c.num_filters;
    for (int s = 0; s < c.num_ratios; ++s) {
        const int ratio = c.upsampling_ratios[c.num_ratios - 1 - s];
        const std::string p = "encoder.layers." + std::to_string(idx) + ".block.";
        ex[p + "1.conv.weight"] = {C / c.compress, C, c.residual_kernel_size};
        ex[p + "1.conv.bias"] = {C / c.compress};
        ex[p + "3.conv.weight"] = {C, C / c.compress, 1};
        ex[p + "3.conv.bias"] = {C};
        idx += 2;
        const std::string d = "encoder.layers." + std::to_string(idx) + ".conv.";
        ex[d + "weight"] = {2 * C, C, 2 * ratio};
        ex[d + "bias"] = {2 * C};
        idx += 1;
        C *= 2;
    }
    idx += 1;
    const std::string f = "encoder.layers." + std::to_string(idx) + ".conv.";
    ex[f + "weight"] = {c.hidden_size, C, c.last_kernel_size};
    ex[f + "bias"] = {c.hidden_size};
    const int h = c.hidden_size;
    for (int l = 0; l < c.num_hidden_layers; ++l) {
        const std::string p = "encoder_transformer.layers." + std::to_string(l) + ".";
        for (const char* n : {"q_proj", "k_proj", "v_proj"})
            ex[p + "self_attn." + n + ".weight"] = {c.num_attention_heads * c.head_dim, h};
        ex[p + "self_attn.o_proj.weight"] = {h, c.num_attention_heads * c.head_dim};
        ex[p + "mlp.fc1.weight"] = {c.intermediate_size, h};
        ex[p + "mlp.fc2.weight"] = {h, c.intermediate_size};
        for (const char* n : {"input_layernorm", "post_attention_layernorm"}) {
            ex[p + n + ".weight"] = {h};
            ex[p + n + ".bias"] = {h};
        }
        ex[p + "self_attn_layer_scale.scale"] = {h};
        ex[p + "mlp_layer_scale.scale"] = {h};
    }
    ex["downsample.conv.weight"] = {h, h, c.downsample_kernel};
    for (const char* q : {"semantic", "acoustic"})
        ex[std::string("quantizer.") + q + "_residual_vector_quantizer.input_proj.weight"] = {c.vq_hidden_dim, h, 1};
}

static std::string codebook_prefix(const mimi_config& c, int level) {
    if (level < c.num_semantic_quantizers)
        return "quantizer.semantic_residual_vector_quantizer.layers." + std::to_string(level) + ".codebook.";
    return "quantizer.acoustic_residual_vector_quantizer.layers." + std::to_string(level - c.num_semantic_quantizers) +
           ".codebook.";
}

static int check_supported(const mimi_config& c) {
    if (c.audio_channels != 1) return set_err(MIMI_ERR_UNSUPPORTED, "audio_channels must be 1");
    if (c.num_filters != 64 || c.kernel_size != 7)
        return set_err(MIMI_ERR_UNSUPPORTED, "first conv must be 1->64, k=7");
    if (c.hidden_size != 512 || c.head_dim != 64 || c.num_attention_heads * c.head_dim != c.hidden_size)
        return set_err(MIMI_ERR_UNSUPPORTED, "transformer must be 512 wide with 64-dim heads");
    if (c.codebook_dim != 256 || c.vq_hidden_dim != 256 || c.codebook_size % 256 != 0)
        return set_err(MIMI_ERR_UNSUPPORTED, "codebooks must be [n*256][256]");
    if (c.num_ratios < 1 || c.num_ratios > 8) return set_err(MIMI_ERR_UNSUPPORTED, "num_ratios out of range");
    if (c.residual_kernel_size * c.num_filters / c.compress % 32 != 0 && c.compress != 2)
        return set_err(MIMI_ERR_UNSUPPORTED, "compress must be 2");
    if (c.num_semantic_quantizers < 1 || c.num_semantic_quantizers >= c.num_quantizers)
        return set_err(MIMI_ERR_UNSUPPORTED, "num_semantic_quantizers out of range");
    return MIMI_OK;
}

extern "C" int mimi_create(const mimi_config* cfg, int device, mimi_engine** out) {
    if (!out) return set_err(MIMI_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = nullptr;
    std::unique_ptr<mimi_engine> e(new mimi_engine());
    if (cfg)
        e->cfg = *cfg;
    else
        mimi_config_default(&e->cfg);
    int rc = check_supported(e->cfg);
    if (rc) return rc;
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return set_err(MIMI_ERR_INVALID_ARGUMENT, "device %d of %d", device, ndev);
    e->device = device;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipEventCreateWithFlags(&e->ws_free, hipEventDisableTiming));
    HIP_TRY(hipMalloc(&e->amax_dev, ((size_t)kMaxActSlots * AMAX_SLOT_WORDS + kMaxActSlots) * sizeof(unsigned)));
    e->amax_red = e->amax_dev + (size_t)kMaxActSlots * AMAX_SLOT_WORDS;
    HIP_TRY(hipMemset(e->amax_dev, 0, ((size_t)kMaxActSlots * AMAX_SLOT_WORDS + kMaxActSlots) * sizeof(unsigned)));
    HIP_TRY(hipHostMalloc(&e->amax_host, kMaxActSlots * sizeof(unsigned), hipHostMallocDefault));
    build_expected(e.get());
    *out = e.release();
    return MIMI_OK;
}

// The one-call constructor: a checkpoint directory in the HF layout (config.json + *.safetensors,
// what MimiModel.from_pretrained("kyutai/mimi") reads: emilia-mimi/process_shard.py:57-60) or a lone .safetensors
// file (default config) -> a finalized engine.  config_json.cpp parses the config and picks the file; on any failure
// the half-built engine is released and the first error is the one mimi_last_error reports.
extern "C" int mimi_create_from_dir(const char* weights_dir, int device, mimi_engine** out) {
    if (!out) return set_err(MIMI_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = nullptr;
    if (!weights_dir) return set_err(MIMI_ERR_INVALID_ARGUMENT, "weights_dir is NULL");
    std::string cfg_path, st_path;
    int rc = mimi::find_checkpoint(weights_dir, cfg_path, st_path);
    if (rc) return rc;
    mimi_config cfg;
    mimi_config_default(&cfg);
    if (!cfg_path.empty() && (rc = mimi_config_from_json(cfg_path.c_str(), &cfg))) return rc;
    mimi_engine* e = nullptr;
    if ((rc = mimi_create(&cfg, device, &e))) return rc;
    if ((rc = mimi_load_safetensors(e, st_path.c_str())) || (rc = mimi_finalize(e))) {
        const std::string msg = g_last_error;
        mimi_destroy(e);
        g_last_error = msg;
        return rc;
    }
    *out = e;
    return MIMI_OK;
}

extern "C" int mimi_set_weight(mimi_engine* e, const char* name, const float* data, int64_t numel) {
    if (!e || !name || (!data && numel > 0)) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null argument");
    if (e->finalized) return set_err(MIMI_ERR_STATE, "weights are frozen after mimi_finalize");
    std::lock_guard<std::mutex> lk(e->mu);
    e->host_w[name].assign(data, data + numel);
    return MIMI_OK;
}

// Checkpoint files: safetensors.cpp (host-only, bounds-checked; built under ASan/UBSan by tools/asan).  A tensor
// is read when the encode path needs it (the names build_expected lists, the quantizer's codebooks, weight-norm
// factors of a conv); the decoder / upsample tensors of a full checkpoint are skipped unread.
extern "C" int mimi_load_safetensors(mimi_engine* e, const char* path) {
    if (!e || !path) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null argument");
    if (e->finalized) return set_err(MIMI_ERR_STATE, "weights are frozen after mimi_finalize");
    std::lock_guard<std::mutex> lk(e->mu);
    auto wanted = [&](const std::string& name) {
        if (name.rfind("decoder", 0) == 0 || name.rfind("upsample", 0) == 0) return false;
        const bool quant = name.rfind("quantizer.", 0) == 0 &&  // input_proj + codebooks (not output_proj)
                           (name.find(".codebook.") != std::string::npos || name.find("input_proj") != std::string::npos);
        return e->expected.count(name) > 0 || quant ||
               name.find("weight_g") != std::string::npos || name.find("weight_v") != std::string::npos ||
               name.find("original0") != std::string::npos || name.find("original1") != std::string::npos;
    };
    std::map<std::string, std::vector<float>> got;
    std::string err;
    const int rc = st_load(path, wanted, got, err);
    if (rc) return set_err(rc, "%s", err.c_str());
    for (auto& kv : got) e->host_w[kv.first] = std::move(kv.second);
    return MIMI_OK;
}

// weight-norm checkpoints store weight_g [cout,1,1] and weight_v [cout,cin,k]: w = g * v / ||v|| per cout
static bool resolve_weight_norm(mimi_engine* e, const std::string& wname, const std::vector<int64_t>& shape) {
    const std::string base = wname.substr(0, wname.size() - std::string("weight").size());
    const std::string gk[] = {base + "weight_g", base + "parametrizations.weight.original0"};
    const std::string vk[] = {base + "weight_v", base + "parametrizations.weight.original1"};
    for (int i = 0; i < 2; ++i) {
        auto g = e->host_w.find(gk[i]);
        auto v = e->host_w.find(vk[i]);
        if (g == e->host_w.end() || v == e->host_w.end()) continue;
        const int64_t cout = shape[0];
        const int64_t per = (int64_t)v->second.size() / cout;
        std::vector<float> w(v->second.size());
        for (int64_t o = 0; o < cout; ++o) {
            double n2 = 0;
            for (int64_t j = 0; j < per; ++j) n2 += (double)v->second[o * per + j] * v->second[o * per + j];
            const float s = (float)(g->second[o] / std::sqrt(n2));
            for (int64_t j = 0; j < per; ++j) w[o * per + j] = v->second[o * per + j] * s;
        }
        e->host_w[wname] = std::move(w);
        return true;
    }
    return false;
}

static int get_w(mimi_engine* e, const std::string& name, std::vector<float>** out) {
    auto it = e->host_w.find(name);
    auto ex = e->expected.find(name);
    if (it == e->host_w.end() && ex != e->expected.end() && resolve_weight_norm(e, name, ex->second))
        it = e->host_w.find(name);
    if (it == e->host_w.end()) return set_err(MIMI_ERR_WEIGHTS, "missing parameter %s", name.c_str());
    if (ex != e->expected.end()) {
        int64_t n = 1;
        for (int64_t d : ex->second) n *= d;
        if ((int64_t)it->second.size() != n)
            return set_err(MIMI_ERR_WEIGHTS, "parameter %s has %zu elements, expected %lld", name.c_str(),
                           it->second.size(), (long long)n);
    }
    *out = &it->second;
    return MIMI_OK;
}

// W[co][ci][k] -> W'[co][k*cin + ci]
static std::vector<float> relayout_conv(const std::vector<float>& w, int cout, int cin, int k) {
    std::vector<float> o((size_t)cout * cin * k);
    for (int co = 0; co < cout; ++co)
        for (int ci = 0; ci < cin; ++ci)
            for (int kk = 0; kk < k; ++kk) o[((size_t)co * k + kk) * cin + ci] = w[((size_t)co * cin + ci) * k + kk];
    return o;
}

// As append_afrags_h16 for the 16x16x32 MFMA: fragments [mt][ks][plane], lane (i, q) holding
// W[16 mt + i][32 ks + 8 q + e] (i = lane & 15, q = lane >> 4).
static void append_afrags16_h16(std::vector<_Float16>& out, const std::vector<float>& w, int M, int K, float sc) {
    for (int mt = 0; mt < M / 16; ++mt)
        for (int ks = 0; ks < K / 32; ++ks)
            for (int pl = 0; pl < 2; ++pl)
                for (int lane = 0; lane < 64; ++lane)
                    for (int e = 0; e < 8; ++e) {
                        const float t = w[(size_t)(16 * mt + (lane & 15)) * K + 32 * ks + 8 * (lane >> 4) + e] * sc;
                        const _Float16 h0 = (_Float16)t;
                        out.push_back(pl == 0 ? h0 : (_Float16)(t - (float)h0));
                    }
}

// The stage-1 (C = 128) fp16 block's weight image (resblock.hip resblock128_h16_kernel): W3 [64][384] then
// W1 [128][64] as 16x16x32 A fragments.
static int make_res1_h16(mimi_engine* e) {
    const mimi_config& c = e->cfg;
    if (c.num_filters != 64 || c.residual_kernel_size != 3 || c.compress != 2 || c.num_ratios < 2) return MIMI_OK;
    std::vector<float>*w3, *w1;
    int rc;
    if ((rc = get_w(e, "encoder.layers.4.block.1.conv.weight", &w3)) ||
        (rc = get_w(e, "encoder.layers.4.block.3.conv.weight", &w1)))
        return rc;
    const std::vector<float> w3l = relayout_conv(*w3, 64, 128, 3);  // [64][3*128], tap-major
    const std::vector<float>& w1l = *w1;                             // [128][64][1]
    const float s3 = f16_weight_scale(w3l), s1 = f16_weight_scale(w1l);
    std::vector<_Float16> img;
    img.reserve((size_t)RES1_H16_FRAGS * 512);
    append_afrags16_h16(img, w3l, 64, 384, s3);
    append_afrags16_h16(img, w1l, 128, 64, s1);
    if (img.size() != (size_t)RES1_H16_FRAGS * 512) return set_err(MIMI_ERR_WEIGHTS, "res1 fp16 image size");
    if ((rc = dev_alloc(e, &e->res1_h16, img.size() * sizeof(_Float16)))) return rc;
    HIP_TRY(hipMemcpy(e->res1_h16, img.data(), img.size() * sizeof(_Float16), hipMemcpyHostToDevice));
    e->res1_wsc[0] = s3;
    e->res1_wsc[1] = s1;
    return MIMI_OK;
}

// The stage-0 fp16 block's weight image (resblock.hip resblock0_h16_kernel): 4 conv0 fragments
// [mt][variant] -- variant 0: every lane (i, h) holds w_hi[32 mt + i][0..6], 0; variant 1: lanes h = 0 hold
// w_lo, lanes h = 1 zeros (against the audio taps' hi | lo planes: w_hi a_hi + w_hi a_lo, then w_lo a_hi) --
// then W3 [32][192] and W1 [64][32] as append_afrags_h16.
static int make_res0_h16(mimi_engine* e) {
    const mimi_config& c = e->cfg;
    if (c.num_filters != 64 || c.kernel_size != 7 || c.residual_kernel_size != 3 || c.compress != 2) return MIMI_OK;
    std::vector<float>*w0, *w3, *w1;
    int rc;
    if ((rc = get_w(e, "encoder.layers.0.conv.weight", &w0)) || (rc = get_w(e, "encoder.layers.1.block.1.conv.weight", &w3)) ||
        (rc = get_w(e, "encoder.layers.1.block.3.conv.weight", &w1)))
        return rc;
    const std::vector<float> w3l = relayout_conv(*w3, 32, 64, 3);  // [32][3*64], tap-major
    const std::vector<float>& w1l = *w1;                            // [64][32][1]
    const float s0 = f16_weight_scale(*w0), s3 = f16_weight_scale(w3l), s1 = f16_weight_scale(w1l);
    std::vector<_Float16> img;
    img.reserve((size_t)RES0_H16_FRAGS * 512);
    for (int mt = 0; mt < 2; ++mt)
        for (int var = 0; var < 2; ++var)
            for (int lane = 0; lane < 64; ++lane)
                for (int k = 0; k < 8; ++k) {
                    _Float16 v = (_Float16)0.0f;
                    if (k < 7) {
                        const float t = (*w0)[(size_t)(32 * mt + (lane & 31)) * 7 + k] * s0;
                        const _Float16 h0 = (_Float16)t;
                        if (var == 0) v = h0;
                        else if ((lane >> 5) == 0) v = (_Float16)(t - (float)h0);
                    }
                    img.push_back(v);
                }
    append_afrags_h16(img, w3l, 32, 192, s3);
    append_afrags_h16(img, w1l, 64, 32, s1);
    if (img.size() != (size_t)RES0_H16_FRAGS * 512) return set_err(MIMI_ERR_WEIGHTS, "res0 fp16 image size");
    if ((rc = dev_alloc(e, &e->res0_h16, img.size() * sizeof(_Float16)))) return rc;
    HIP_TRY(hipMemcpy(e->res0_h16, img.data(), img.size() * sizeof(_Float16), hipMemcpyHostToDevice));
    e->res0_wsc[0] = s0;
    e->res0_wsc[1] = s3;
    e->res0_wsc[2] = s1;
    return MIMI_OK;
}

static int make_conv(mimi_engine* e, DevConv& dc, const std::string& prefix, int cin, int cout, int k, int stride,
                     bool bias) {
    std::vector<float>* w;
    int rc = get_w(e, prefix + "weight", &w);
    if (rc) return rc;
    if ((int64_t)w->size() != (int64_t)cin * cout * k)
        return set_err(MIMI_ERR_WEIGHTS, "%sweight: bad size", prefix.c_str());
    dc.cin = cin;
    dc.cout = cout;
    dc.k = k;
    dc.stride = stride;
    const std::vector<float> wl = cin == 1 ? *w : relayout_conv(*w, cout, cin, k);
    rc = upload(e, &dc.w, wl);
    if (rc) return rc;
    if (cin % 4 == 0 && (k * cin) % 32 == 0 &&
        ((rc = upload_split(e, &dc.wsplit, wl)) || (rc = upload_f16(e, &dc.wh, wl, &dc.wscale))))
        return rc;
    if (cout % 32 == 0 && (k * cin) % 8 == 0 && (rc = upload(e, &dc.wfrag, frag_layout(wl, cout, k * cin)))) return rc;
    if (bias) {
        std::vector<float>* b;
        rc = get_w(e, prefix + "bias", &b);
        if (rc) return rc;
        rc = upload(e, &dc.b, *b);
        if (rc) return rc;
    }
    return MIMI_OK;
}

// sum of squares in torch's x.pow(2).sum(-1) order for rows of 8*m floats (see ops.hip)
static float torch_sqsum_host(const float* r, int D) {
    float lanes[8];
    for (int l = 0; l < 8; ++l) {
        float a[4] = {0.f, 0.f, 0.f, 0.f};
        for (int blk = 0; blk < D / 8; ++blk) {
            volatile float sq = r[blk * 8 + l] * r[blk * 8 + l];
            a[blk & 3] = a[blk & 3] + sq;
        }
        volatile float t = a[0] + a[1];
        t = t + a[2];
        t = t + a[3];
        lanes[l] = t;
    }
    volatile float tot = lanes[0];
    for (int l = 1; l < 8; ++l) tot = tot + lanes[l];
    return tot;
}

static int calibrate_scales(mimi_engine* e);

extern "C" int mimi_finalize(mimi_engine* e) {
    if (!e) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    if (e->finalized) return MIMI_OK;
    HIP_TRY(hipSetDevice(e->device));
    const mimi_config& c = e->cfg;
    int rc = make_conv(e, e->conv0, "encoder.layers.0.conv.", 1, c.num_filters, c.kernel_size, 1, true);
    if (rc) return rc;
    int idx = 1, C = c.num_filters;
    e->res3.resize(c.num_ratios);
    e->res1.resize(c.num_ratios);
    e->down.resize(c.num_ratios);
    for (int s = 0; s < c.num_ratios; ++s) {
        const int ratio = c.upsampling_ratios[c.num_ratios - 1 - s];
        const std::string p = "encoder.layers." + std::to_string(idx) + ".block.";
        if ((rc = make_conv(e, e->res3[s], p + "1.conv.", C, C / c.compress, c.residual_kernel_size, 1, true))) return rc;
        if ((rc = make_conv(e, e->res1[s], p + "3.conv.", C / c.compress, C, 1, 1, true))) return rc;
        idx += 2;
        if ((rc = make_conv(e, e->down[s], "encoder.layers." + std::to_string(idx) + ".conv.", C, 2 * C, 2 * ratio,
                            ratio, true)))
            return rc;
        idx += 1;
        C *= 2;
    }
    if ((rc = make_res0_h16(e)) || (rc = make_res1_h16(e))) return rc;
    idx += 1;
    if ((rc = make_conv(e, e->final_conv, "encoder.layers." + std::to_string(idx) + ".conv.", C, c.hidden_size,
                        c.last_kernel_size, 1, true)))
        return rc;
    const int h = c.hidden_size;
    e->xf.resize(c.num_hidden_layers);
    for (int l = 0; l < c.num_hidden_layers; ++l) {
        const std::string p = "encoder_transformer.layers." + std::to_string(l) + ".";
        DevXfmr& x = e->xf[l];
        std::vector<float>*q, *k, *v, *t;
        if ((rc = get_w(e, p + "self_attn.q_proj.weight", &q)) || (rc = get_w(e, p + "self_attn.k_proj.weight", &k)) ||
            (rc = get_w(e, p + "self_attn.v_proj.weight", &v)))
            return rc;
        std::vector<float> qkv;
        qkv.reserve(q->size() * 3);
        qkv.insert(qkv.end(), q->begin(), q->end());
        qkv.insert(qkv.end(), k->begin(), k->end());
        qkv.insert(qkv.end(), v->begin(), v->end());
        if ((rc = upload(e, &x.wqkv, qkv)) || (rc = upload_split(e, &x.wqkv_s, qkv)) ||
            (rc = upload_f16(e, &x.wqkv_h, qkv, &x.wqkv_hs)))
            return rc;
        struct {
            const char* n;
            float** d;
        } simple[] = {{"self_attn.o_proj.weight", &x.wo},
                      {"mlp.fc1.weight", &x.w1},
                      {"mlp.fc2.weight", &x.w2},
                      {"input_layernorm.weight", &x.ln1_w},
                      {"input_layernorm.bias", &x.ln1_b},
                      {"post_attention_layernorm.weight", &x.ln2_w},
                      {"post_attention_layernorm.bias", &x.ln2_b},
                      {"self_attn_layer_scale.scale", &x.ls1},
                      {"mlp_layer_scale.scale", &x.ls2}};
        for (auto& sp : simple) {
            if ((rc = get_w(e, p + sp.n, &t))) return rc;
            if ((rc = upload(e, sp.d, *t))) return rc;
            void** sd = sp.d == &x.wo ? &x.wo_s : sp.d == &x.w1 ? &x.w1_s : sp.d == &x.w2 ? &x.w2_s : nullptr;
            void** hd = sp.d == &x.wo ? &x.wo_h : sp.d == &x.w1 ? &x.w1_h : sp.d == &x.w2 ? &x.w2_h : nullptr;
            float* hs = sp.d == &x.wo ? &x.wo_hs : sp.d == &x.w1 ? &x.w1_hs : sp.d == &x.w2 ? &x.w2_hs : nullptr;
            if (sd && ((rc = upload_split(e, sd, *t)) || (rc = upload_f16(e, hd, *t, hs)))) return rc;
        }
        for (int k = 0; k < 2; ++k) {
            std::vector<float>*g, *bb;
            const std::string n = k ? "post_attention_layernorm." : "input_layernorm.";
            if ((rc = get_w(e, p + n + "weight", &g)) || (rc = get_w(e, p + n + "bias", &bb))) return rc;
            double bound = 0.0;
            const double r = std::sqrt((double)h - 1.0) * 1.001;
            for (size_t i = 0; i < g->size() && i < bb->size(); ++i) {
                const double v = std::fabs((double)(*g)[i]) * r + std::fabs((double)(*bb)[i]);
                bound = std::isfinite(v) ? std::max(bound, v) : INFINITY;
            }
            (k ? x.ln2_bound : x.ln1_bound) = (float)bound;
        }
    }
    if ((rc = make_conv(e, e->ds, "downsample.conv.", h, h, c.downsample_kernel, c.downsample_stride, false))) return rc;
    if (c.downsample_kernel == 4 && c.downsample_stride == 2) {  // replicate-edge terms of the planes downsample
        std::vector<float>* w;
        if ((rc = get_w(e, "downsample.conv.weight", &w))) return rc;
        const std::vector<float> wl = relayout_conv(*w, h, h, 4);  // [co][kk*h + ci]
        std::vector<float> fix((size_t)2 * h * h);
        for (int co = 0; co < h; ++co)
            for (int ci = 0; ci < h; ++ci) {
                const size_t r = (size_t)co * 4 * h;
                fix[(size_t)ci * h + co] = wl[r + ci] + wl[r + h + ci];  // [edge][ci][co]
                fix[(size_t)h * h + (size_t)ci * h + co] = wl[r + 3 * h + ci];
            }
        if ((rc = upload(e, &e->ds_fix, fix))) return rc;
    }
    {
        std::vector<float>*ps, *pa;
        if ((rc = get_w(e, "quantizer.semantic_residual_vector_quantizer.input_proj.weight", &ps)) ||
            (rc = get_w(e, "quantizer.acoustic_residual_vector_quantizer.input_proj.weight", &pa)))
            return rc;
        std::vector<float> both(*ps);
        both.insert(both.end(), pa->begin(), pa->end());
        if ((rc = upload(e, &e->inproj, both)) || (rc = upload_f16(e, &e->inproj_h, both, &e->inproj_hs))) return rc;
    }
    // codebooks: as many consecutive levels as the checkpoint provides (32 for kyutai/mimi)
    const int n = c.codebook_size, D = c.codebook_dim;
    int L = 0;
    while (L < c.num_quantizers && e->host_w.count(codebook_prefix(c, L) + "embed_sum")) ++L;
    if (L <= c.num_semantic_quantizers) return set_err(MIMI_ERR_WEIGHTS, "no acoustic codebooks found");
    std::vector<float> rows((size_t)L * n * D), frag((size_t)L * n * D), norms((size_t)L * n);
    for (int lv = 0; lv < L; ++lv) {
        std::vector<float>*es, *us;
        const std::string p = codebook_prefix(c, lv);
        if ((rc = get_w(e, p + "embed_sum", &es)) || (rc = get_w(e, p + "cluster_usage", &us))) return rc;
        if ((int64_t)es->size() != (int64_t)n * D || (int64_t)us->size() != n)
            return set_err(MIMI_ERR_WEIGHTS, "%s: bad codebook shape", p.c_str());
        float* R = rows.data() + (size_t)lv * n * D;
        for (int j = 0; j < n; ++j) {
            const float u = std::max((*us)[j], c.codebook_eps);
            for (int d = 0; d < D; ++d) {
                volatile float q = (*es)[(size_t)j * D + d] / u;
                R[(size_t)j * D + d] = q;
            }
            norms[(size_t)lv * n + j] = torch_sqsum_host(R + (size_t)j * D, D);
        }
        // fragment layout: [jt][u][lane][s] = embed[32*jt + (lane&31)][8u + 2s + (lane>>5)]
        float* F = frag.data() + (size_t)lv * n * D;
        for (int jt = 0; jt < n / 32; ++jt)
            for (int u = 0; u < D / 8; ++u)
                for (int lane = 0; lane < 64; ++lane)
                    for (int s = 0; s < 4; ++s)
                        F[(((size_t)jt * (D / 8) + u) * 64 + lane) * 4 + s] =
                            R[(size_t)(32 * jt + (lane & 31)) * D + 8 * u + 2 * s + (lane >> 5)];
    }
    if ((rc = upload(e, &e->cb_rows, rows)) || (rc = upload(e, &e->cb_frag, frag)) || (rc = upload(e, &e->cb_norm, norms)))
        return rc;
    {
        // fp16 planes of embed * cs (cs: power of two putting max|embed| in [2^13, 2^14)) in 32x32x16 B-fragment
        // order [level][code tile][k step][plane][lane (j, h)][8]: embed[32 ct + j][16 ks + 8 h + q]
        std::vector<_Float16> h16((size_t)L * n * D * 2);
        std::vector<float> unsc(L), emax(L);
        for (int lv = 0; lv < L; ++lv) {
            const float* R = rows.data() + (size_t)lv * n * D;
            float amax = 0.0f, nmax = 0.0f;
            for (size_t i = 0; i < (size_t)n * D; ++i) amax = std::max(amax, std::fabs(R[i]));
            for (int j = 0; j < n; ++j) nmax = std::max(nmax, norms[(size_t)lv * n + j]);
            const float cs = amax > 0.0f && std::isfinite(amax) ? std::ldexp(1.0f, 13 - std::ilogb(amax)) : 1.0f;
            unsc[lv] = 1.0f / cs;
            emax[lv] = std::sqrt(nmax) * (1.0f + 1e-6f);
            _Float16* H = h16.data() + (size_t)lv * n * D * 2;
            size_t o = 0;
            for (int ct = 0; ct < n / 32; ++ct)
                for (int ks = 0; ks < D / 16; ++ks)
                    for (int pl = 0; pl < 2; ++pl)
                        for (int lane = 0; lane < 64; ++lane)
                            for (int q = 0; q < 8; ++q) {
                                const float t = R[(size_t)(32 * ct + (lane & 31)) * D + 16 * ks + 8 * (lane >> 5) + q] * cs;
                                const _Float16 hi = (_Float16)t;
                                H[o++] = pl == 0 ? hi : (_Float16)(t - (float)hi);
                            }
        }
        if ((rc = dev_alloc(e, &e->cb_h16, h16.size() * sizeof(_Float16)))) return rc;
        HIP_TRY(hipMemcpy(e->cb_h16, h16.data(), h16.size() * sizeof(_Float16), hipMemcpyHostToDevice));
        if ((rc = upload(e, &e->cb_unscale, unsc)) || (rc = upload(e, &e->cb_emax, emax))) return rc;
    }
    e->levels_available = L;
    e->host_w.clear();
    e->finalized = true;  // (the f16x3 activation scales are calibrated before the first f16x3 encode)
    return MIMI_OK;
}

// ------------------------------------------------------------------------------------------------
// encode
// ------------------------------------------------------------------------------------------------
struct Workspace {
    float *x, *y;                  // SEANet ping-pong (the residual blocks keep their hidden tile on chip)
    float *t0, *t1, *qkv, *att, *ff;  // transformer
    float *dsout, *proj;
    float* rvq;  // rvq_work_bytes(frames)
    float *xe, *h;  // planes path, unfused residual blocks: ELU(x) planes, hidden planes
    int* rg;        // ragged batches: the per-item length table (RaggedTable)
};

// Ragged batches (mimi_encode_ragged): item b is encoded exactly as it would be alone at its own length L_b --
// every kernel reads only its item's valid rows (the rest read as zero: the item's own extra padding) and
// computes / stores / max-reduces only its valid rows.  The per-item lengths of every stage live in one small
// device table, stage-major: T[0..4][B] (conv0 / down-conv outputs), T25[B], F[B] (12.5 Hz frames), then the
// fused blocks' tile prefixes st0[B + 1], st1[B + 1] (32-step tiles over T[0] / T[1]), then the transformer
// section's PACKED row layout: toff[B] (item b's first row: the items' 25 Hz frames back to back, R rows in all).
// Behind the table, in the workspace only, rpos[R]: the position of each packed row inside its item (RoPE), written
// on the device from toff (launch_ragged_rows) -- the host table stays a few hundred bytes.
struct RaggedTable {
    enum { NST = 7 };
    int B = 0;
    int64_t R = 0;                // packed transformer rows: sum of the items' 25 Hz frames
    std::vector<StagePlan> plan;  // per item
    std::vector<int64_t> len;     // samples per item
    int minT25 = 0, maxT25 = 0;
    static size_t ints(int B) { return (size_t)NST * B + 2 * ((size_t)B + 1) + (size_t)B; }  // the host table
    static size_t toff_at(int B) { return (size_t)NST * B + 2 * ((size_t)B + 1); }
    void fill(int* h) const {  // the device image (host side)
        int* toff = h + toff_at(B);
        int64_t r = 0;
        for (int b = 0; b < B; ++b) {
            toff[b] = (int)r;
            r += plan[b].frames25;
        }
        for (int b = 0; b < B; ++b) {
            for (int st = 0; st < 5; ++st) h[st * B + b] = (int)plan[b].T[st];
            h[5 * B + b] = (int)plan[b].frames25;
            h[6 * B + b] = (int)plan[b].frames12;
        }
        unsigned* s0 = reinterpret_cast<unsigned*>(h + NST * B);
        unsigned* s1 = s0 + B + 1;
        s0[0] = s1[0] = 0;
        for (int b = 0; b < B; ++b) {
            s0[b + 1] = s0[b] + (unsigned)((plan[b].T[0] + 31) / 32);
            s1[b + 1] = s1[b] + (unsigned)((plan[b].T[1] + 31) / 32);
        }
    }
    double rows(int st) const {  // valid rows of stage st (0..4: T, 5: T25, 6: F) summed over the items
        double r = 0;
        for (const auto& p : plan) r += st < 5 ? (double)p.T[st] : st == 5 ? (double)p.frames25 : (double)p.frames12;
        return r;
    }
};

// Planes of the split-bf16 path: activations consumed only by GEMMs (resblock outputs, the last down conv's
// output, LayerNorm / attention / GELU outputs) are stored as NS bf16 planes instead of fp32 so the GEMMs
// only move bytes (gemm_planes.h).  0 = fp32 activations (f32 mode, or a clip so long that a batch item's
// plane exceeds the 2 GiB buffer-resource range).
static int act_planes(const mimi_engine* e, const StagePlan& p, int prec) {
    const int ns = prec == PREC_BF16X6 ? 3 : (prec == PREC_BF16X3 || prec == PREC_F16X3) ? 2 : 0;
    if (ns == 0) return 0;
    const mimi_config& c = e->cfg;
    int C = c.num_filters;
    for (int si = 0; si <= c.num_ratios; ++si) {
        if ((double)p.T[si] * C * 2 * 2 >= 2147483647.0) return 0;  // k*Cin span of the last row included
        C *= 2;
    }
    if ((double)p.frames25 * c.intermediate_size * 2 >= 2147483647.0) return 0;
    return ns;
}

static size_t ws_layout(const mimi_engine* e, int B, const StagePlan& p, Workspace* w, int prec, bool ragged = false) {
    const mimi_config& c = e->cfg;
    const int ns = act_planes(e, p, prec);
    // a plane-format buffer of n values takes ns * n bf16 = ns * n / 2 floats
    auto act = [&](size_t n) { return ns ? (n * ns + 1) / 2 : n; };
    size_t xmax = 0, ymax = 0, xemax = 0;
    int C = c.num_filters;
    for (int s = 0; s < c.num_ratios; ++s) {
        // x at stage 0 only holds the conv0 tap (the stage-0 block recomputes conv0 from the audio)
        if (s > 0 || e->taps) xmax = std::max(xmax, (size_t)p.T[s] * C);
        ymax = std::max(ymax, (size_t)p.T[s] * C);
        if (ns && s >= mimi_engine::kUnfuseFrom && s > 0) xemax = std::max(xemax, (size_t)p.T[s] * C);
        C *= 2;
    }
    xmax = std::max(xmax, act((size_t)p.T[c.num_ratios] * C));  // last down conv's (planes) output
    const size_t T = (size_t)p.frames25, Hd = (size_t)c.hidden_size;
    const size_t sizes[] = {xmax * B,
                            act(ymax * B),
                            T * Hd * B,
                            act(T * Hd * B),
                            T * 3 * Hd * B,
                            act(T * Hd * B),
                            act(T * (size_t)c.intermediate_size * B),
                            (size_t)p.frames12 * Hd * B,
                            (size_t)p.frames12 * 2 * c.vq_hidden_dim * B,
                            rvq_work_bytes((long long)p.frames12 * B) / sizeof(float),
                            act(xemax * B),
                            act(xemax / 2 * B),
                            ragged ? RaggedTable::ints(B) + (size_t)B * p.frames25 : 0};  // (+ rpos)
    size_t off = 0;
    float* rgp = nullptr;
    float** ptrs[] = {&w->x, &w->y, &w->t0, &w->t1, &w->qkv, &w->att, &w->ff, &w->dsout, &w->proj, &w->rvq,
                      &w->xe, &w->h, &rgp};
    char* base = reinterpret_cast<char*>(e->ws);
    for (size_t i = 0; i < sizeof(sizes) / sizeof(sizes[0]); ++i) {
        if (w) *ptrs[i] = reinterpret_cast<float*>(base + off);
        off += ((sizes[i] * sizeof(float) + 255) / 256) * 256;
    }
    if (w) w->rg = reinterpret_cast<int*>(rgp);
    return off;
}

extern "C" int64_t mimi_workspace_bytes(const mimi_engine* e, int32_t batch, int64_t length) {
    if (!e || batch <= 0 || length <= 0) return -1;
    return (int64_t)ws_layout(e, batch, plan_lengths(e->cfg, length), nullptr, e->precision);
}

static int ensure_ws(mimi_engine* e, size_t bytes, hipStream_t s) {
    if (bytes <= e->ws_bytes) return MIMI_OK;
    HIP_TRY(hipStreamSynchronize(s));
    if (e->ws) {
        HIP_TRY(hipFree(e->ws));
        e->ws = nullptr;
        e->ws_bytes = 0;
    }
    hipError_t err = hipMalloc(&e->ws, bytes);
    if (err != hipSuccess) {
        (void)hipGetLastError();  // clear it: the launch checks (hipGetLastError) must not see this failure
        e->ws = nullptr;
        return set_err(err == hipErrorOutOfMemory ? MIMI_ERR_OUT_OF_MEMORY : MIMI_ERR_HIP,
                       "workspace hipMalloc(%zu bytes): %s", bytes, hipGetErrorString(err));
    }
    e->ws_bytes = bytes;
    ++e->ws_gen;  // captured graphs address the old workspace
    return MIMI_OK;
}

static int ensure_rope(mimi_engine* e, int64_t T) {
    if (T <= e->rope_T) return MIMI_OK;
    const int half = e->cfg.head_dim / 2;
    const int64_t Tn = std::max<int64_t>(T, 256);
    std::vector<float> cs((size_t)Tn * half), sn((size_t)Tn * half);
    for (int d = 0; d < half; ++d) {
        // inv_freq = 1 / theta^(2d / dim) in float32 (TF/modeling_mimi.py:546), freq = inv_freq * pos in float32
        const float expo = (float)(2 * d) / (float)e->cfg.head_dim;
        const float pw = (float)std::pow((double)e->cfg.rope_theta, (double)expo);
        const float inv = 1.0f / pw;
        for (int64_t t = 0; t < Tn; ++t) {
            volatile float fr = inv * (float)t;
            cs[(size_t)t * half + d] = (float)std::cos((double)fr);
            sn[(size_t)t * half + d] = (float)std::sin((double)fr);
        }
    }
    if (e->rope_cos) {
        HIP_TRY(hipFree(e->rope_cos));
        HIP_TRY(hipFree(e->rope_sin));
    }
    HIP_TRY(hipMalloc(&e->rope_cos, cs.size() * 4));
    HIP_TRY(hipMalloc(&e->rope_sin, sn.size() * 4));
    HIP_TRY(hipMemcpy(e->rope_cos, cs.data(), cs.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(e->rope_sin, sn.data(), sn.size() * 4, hipMemcpyHostToDevice));
    e->rope_T = Tn;
    ++e->rope_gen;
    return MIMI_OK;
}

static hipEvent_t pool_event(mimi_engine* e) {
    if (!e->event_pool.empty()) {
        hipEvent_t ev = e->event_pool.back();
        e->event_pool.pop_back();
        return ev;
    }
    hipEvent_t ev = nullptr;
    (void)hipEventCreate(&ev);
    return ev;
}

struct Recorder {
    mimi_engine* e;
    hipStream_t s;
    int marks = 0;
    void begin() {
        if (!e->profiling) return;
        ProfEvent pe{"", pool_event(e), 0, 0};
        (void)hipEventRecord(pe.ev, s);
        e->pending.push_back(pe);
    }
    void mark(const std::string& name, double flops, double bytes, const char* kernel) {
        if (!e->profiling) return;
        if (e->profiling == 2 && marks++ >= 1) return;  // level 2: the pass's first stage only
        ProfEvent pe{name + "|" + kernel, pool_event(e), flops, bytes};
        (void)hipEventRecord(pe.ev, s);
        e->pending.push_back(pe);
    }
};

static int save_tap(mimi_engine* e, const char* name, const float* src, int64_t b, int64_t t, int64_t ch,
                    hipStream_t s) {
    if (!e->taps) return MIMI_OK;
    auto& tp = e->tapmap[name];
    const size_t n = (size_t)(b * t * ch);
    if (tp.cap < n) {
        if (tp.d) HIP_TRY(hipFree(tp.d));
        HIP_TRY(hipMalloc(&tp.d, n * 4));
        tp.cap = n;
    }
    HIP_TRY(hipMemcpyAsync(tp.d, src, n * 4, hipMemcpyDeviceToDevice, s));
    tp.dims[0] = b;
    tp.dims[1] = t;
    tp.dims[2] = ch;
    return MIMI_OK;
}

// tap of a plane-format activation (materialised as fp32 only when taps are on)
static int save_tap_planes(mimi_engine* e, const char* name, const void* planes, int ns, int64_t b, int64_t t,
                           int64_t ch, hipStream_t s, float hscale = 0.0f) {
    if (!e->taps) return MIMI_OK;
    if (ns == 0) return save_tap(e, name, reinterpret_cast<const float*>(planes), b, t, ch, s);
    auto& tp = e->tapmap[name];
    const size_t n = (size_t)(b * t * ch);
    if (tp.cap < n) {
        if (tp.d) HIP_TRY(hipFree(tp.d));
        HIP_TRY(hipMalloc(&tp.d, n * 4));
        tp.cap = n;
    }
    HIP_TRY(launch_planes_to_f32(planes, (long long)n, ns, tp.d, (long long)n, s, hscale));
    tp.dims[0] = b;
    tp.dims[1] = t;
    tp.dims[2] = ch;
    return MIMI_OK;
}

// A operand of a GEMM read from plane-format activations (plane stride = the activation's element count)
static void planes_in(GemmArgs& a, const void* planes, long long n) {
    a.Ap = planes;
    a.a_pstride = n;
}

static GemmArgs conv_args(const DevConv& cv, const float* in, int64_t Tin, float* out, int64_t Tout, int B) {
    GemmArgs a{};
    a.A = in;
    a.a_bstride = Tin * cv.cin;
    a.a_off = -(int64_t)(cv.k - cv.stride) * cv.cin;  // causal left pad
    a.a_rs = cv.stride * cv.cin;
    a.a_cin = cv.cin;
    a.a_len = Tin * cv.cin;
    a.W = cv.w;
    a.Wsplit = cv.wsplit;
    a.M = (int)Tout;
    a.N = cv.cout;
    a.K = cv.k * cv.cin;
    a.batch = B;
    a.bias = cv.b;
    a.C = out;
    a.c_bstride = Tout * cv.cout;
    a.ldc = cv.cout;
    return a;
}

static GemmArgs linear_args(const float* in, int64_t rows, int K, const float* W, int N, float* out) {
    GemmArgs a{};
    a.A = in;
    a.a_bstride = 0;
    a.a_off = 0;
    a.a_rs = K;
    a.a_cin = K;
    a.a_len = rows * K;
    a.W = W;
    a.M = (int)rows;
    a.N = N;
    a.K = K;
    a.batch = 1;
    a.C = out;
    a.c_bstride = 0;
    a.ldc = N;
    return a;
}

#define LAUNCH_TRY(expr, what)                                                                           \
    do {                                                                                                 \
        hipError_t _e = (expr);                                                                          \
        if (_e != hipSuccess) return set_err(MIMI_ERR_HIP, "launch %s: %s", what, hipGetErrorString(_e)); \
    } while (0)

static const char* ln_kname(int rpw) {
    switch (rpw) {
        case 1: return "mimi::layernorm_kernel<512, 1>";
        case 4: return "mimi::layernorm_kernel<512, 4>";
        case 8: return "mimi::layernorm_kernel<512, 8>";
        default: return "mimi::layernorm_kernel<512, 2>";
    }
}

static int run_rvq(mimi_engine* e, const float* proj, int64_t frames, int K, int32_t* codes, int frames_per_item,
                   void* work, hipStream_t s, Recorder& rec, const int* flen = nullptr, double valid_share = 1.0) {
    RvqArgs r{};
    r.flen = flen;
    r.work = work;
    r.proj = proj;
    r.frames = frames;
    r.D = e->cfg.codebook_dim;
    r.ncodes = e->cfg.codebook_size;
    r.levels = K;
    r.nsem = e->cfg.num_semantic_quantizers;
    r.cb_frag = e->cb_frag;
    r.cb_rows = e->cb_rows;
    r.cb_norm = e->cb_norm;
    r.cb_h16 = e->cb_h16;
    r.cb_unscale = e->cb_unscale;
    r.cb_emax = e->cb_emax;
    r.codes = codes;
    r.codes_ref = e->capturing ? reinterpret_cast<int32_t* const*>(e->io_dev + 1) : nullptr;
    r.frames_per_item = frames_per_item;
    r.form = e->rvq_form;
    r.chain = e->rvq_chain;
    r.chain_fault = e->rvq_chain_fault;
    r.xcd_group_ok = e->rvq_xcd;
    const char* kname = "?";
    unsigned* cflag = nullptr;
    e->chain_flag = nullptr;
    size_t clear = 0;  // (capturing: the replay's set_io_kernel zeroes the chain's words instead of a memset node)
    LAUNCH_TRY(launch_rvq(r, s, &kname, e->chain_ok ? &cflag : nullptr, e->capturing ? &clear : nullptr), "rvq");
    e->chain_flag = cflag;
    if (e->capturing) e->cap_chain_clear = cflag ? clear : 0;
    rec.mark("rvq", 2.0 * frames * valid_share * r.D * r.ncodes * K,
             (double)frames * (2 * r.D) * 4 + (double)frames * K * 4, kname);
    return MIMI_OK;
}

// One pass of the whole encode at precision prec.
static int encode_pass(mimi_engine* e, const float* audio, int B, int64_t L, int K, int32_t* codes, hipStream_t s,
                       int prec, const RaggedTable* rg = nullptr, const int* rg_pinned = nullptr) {
    const mimi_config& c = e->cfg;
    const StagePlan p = plan_lengths(c, L);
    Workspace w{};
    int rc = ensure_ws(e, ws_layout(e, B, p, nullptr, prec, rg != nullptr), s);
    if (rc) return rc;
    ws_layout(e, B, p, &w, prec, rg != nullptr);
    if ((rc = ensure_rope(e, p.frames25))) return rc;
    const int ns = act_planes(e, p, prec);  // 0: fp32 activations; 2/3: plane-format GEMM inputs
    // fp16 planes: each plane-format tensor takes the next activation-scale slot (launch order)
    const bool h16 = prec == PREC_F16X3 && ns == 2;
    struct Act {
        float scale = 0.0f;  // > 0: fp16 planes of x * scale
        unsigned* amax = nullptr;
    };
    // the activation-scale slot of plane tensor `name` (fixed names, so a tensor keeps its scale whatever the
    // batch, length or code path); new names only while calibrating
    auto new_act = [&](const std::string& name) {
        Act a;
        if (!h16) return a;
        auto it = e->slot_of.find(name);
        int slot;
        if (it != e->slot_of.end()) {
            slot = it->second;
        } else {
            if (!e->calibrating) e->uncalibrated_slot = true;
            if ((int)e->slot_of.size() >= kMaxActSlots) return a;
            slot = (int)e->slot_of.size();
            e->slot_of[name] = slot;
            e->act_scale.resize(slot + 1, 1.0f);
        }
        a.scale = e->act_scale[slot];
        a.amax = e->amax_dev + (size_t)slot * AMAX_SLOT_WORDS;
        return a;
    };
    // a LayerNorm output whose bound (DevXfmr::ln*_bound) times its scale stays under half the fp16 plane limit
    // (2^15) needs no range check (calibration still records its maximum: it sets the scale)
    auto ln_check_free = [&](const Act& a, float bound) {
        return MIMI_LN_CHECK_SKIP && !e->calibrating && a.amax && a.scale > 0.0f && bound * a.scale < 16384.0f;
    };
    // fp16 weight planes + 1 / (activation scale x weight scale) for a GEMM reading plane tensor `in`
    auto use_h = [&](GemmArgs& a, const void* wh, float wscale, const Act& in) {
        if (!h16) return;
        a.Wsplit = wh;
        a.unscale = 1.0f / (in.scale * wscale);
    };
    auto out_act = [&](GemmArgs& a, const Act& o) {
        a.out_scale = o.scale;
        a.out_amax = o.amax;
    };
    Recorder rec{e, s};
    const char* kname = "?";
    if (!e->capturing) HIP_TRY(hipStreamWaitEvent(s, e->ws_free, 0));  // (a replay waits outside the graph)
    // ragged batches: the length table (pinned host image, alive until the encode is waited) -> workspace
    const int* dT[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    const int *dT25 = nullptr, *dF = nullptr;
    const unsigned *dst0 = nullptr, *dst1 = nullptr;
    const int *dToff = nullptr, *dRpos = nullptr;  // the transformer section's packed rows (RaggedTable)
    if (rg) {
        if (!rg_pinned || rg->B != B || !w.rg) return set_err(MIMI_ERR_STATE, "ragged encode without its length table");
        HIP_TRY(hipMemcpyAsync(w.rg, rg_pinned, RaggedTable::ints(B) * sizeof(int), hipMemcpyHostToDevice, s));
        for (int st = 0; st < 5; ++st) dT[st] = w.rg + st * B;
        dT25 = w.rg + 5 * B;
        dF = w.rg + 6 * B;
        dst0 = reinterpret_cast<const unsigned*>(w.rg + RaggedTable::NST * B);
        dst1 = dst0 + B + 1;
        dToff = w.rg + RaggedTable::toff_at(B);
        dRpos = w.rg + RaggedTable::ints(B);
        LAUNCH_TRY(launch_ragged_rows(w.rg + 5 * B, dToff, B, w.rg + RaggedTable::ints(B), s), "ragged rows");
    }
    // (profile bookkeeping) a GEMM's algorithmic FLOPs over the items' valid rows
    auto rows_of = [&](int st, double uniform) { return rg ? rg->rows(st) : uniform; };
    rec.begin();
    auto gemm_flops = [](const GemmArgs& a) { return 2.0 * a.batch * (double)a.M * a.N * a.K; };
    auto gemm_bytes = [](const GemmArgs& a, bool res) {
        // algorithmic: activation span read once, output written once (+ residual read), weights once
        const double in = (double)a.batch * a.a_len * 4, out = (double)a.batch * a.M * a.N * 4;
        return in + out * (res ? 2 : 1) + (double)a.N * a.K * 4;
    };

    // ---- SEANet encoder ----
    // conv0 is fused into the stage-0 residual block (x0 is recomputed per tile from the audio); the standalone
    // conv0 kernel only runs to materialise the "conv0" tap for per-stage parity tests.
    if (e->taps) {
        LAUNCH_TRY(launch_conv0(audio, L, B, e->conv0.w, e->conv0.b, w.x, c.num_filters, c.kernel_size, s), "conv0");
        if ((rc = save_tap(e, "conv0", w.x, B, p.T[0], c.num_filters, s))) return rc;
    }
    int C = c.num_filters;
    char nm[64];
    Act yact, xact, xeact, hact;  // the tensors currently held by y, x (last down conv), xe, h
    const auto nmf = [](const char* fmt, int i) {
        char b[48];
        snprintf(b, sizeof b, fmt, i);
        return std::string(b);
    };
    for (int si = 0; si < c.num_ratios; ++si) {
        const int64_t T = p.T[si];
        const bool unf = ns && si > 0 && si >= mimi_engine::kUnfuseFrom;
        if (!unf) {
            ResArgs ra{};
            ra.x = w.x;
            if (si == 0) {
                ra.audio = audio;
                ra.audio_ref = e->capturing ? const_cast<const float* const*>(reinterpret_cast<float**>(e->io_dev)) : nullptr;
                ra.w0 = e->conv0.w;
                ra.b0 = e->conv0.b;
                ra.w3frag = e->res3[0].wfrag;
                ra.w1frag = e->res1[0].wfrag;
            }
            ra.T = T;
            ra.batch = B;
            if (rg) {
                ra.ilen = dT[si];
                ra.istart = si == 0 ? dst0 : dst1;
            }
            ra.w3 = e->res3[si].w;
            ra.b3 = e->res3[si].b;
            ra.w1 = e->res1[si].w;
            ra.b1 = e->res1[si].b;
            ra.y = w.y;
            ra.yp = w.y;
            ra.y_pstride = (long long)B * T * C;
            ra.yns = ns;
            yact = new_act(nmf("y%d", si));
            ra.yscale = yact.scale;
            ra.yamax = yact.amax;
            if (h16 && (si > 1 || (si == 0 && !e->res0_h16) || (si == 1 && !(C == 128 && e->res1_h16))))
                return set_err(MIMI_ERR_UNSUPPORTED, "f16x3: no fp16 fused block for stage %d", si);
            if (h16 && (unsigned long long)B * (unsigned long long)((T + 31) / 32) >= (1ull << 32))
                return set_err(MIMI_ERR_UNSUPPORTED, "f16x3: %d x %lld steps exceed the block index range", B,
                               (long long)T);
            if (si == 0 && h16) {
                // fp16-plane stage-0 block: audio, ELU(x0) and ELU(h) are split in-kernel, each at its own scale
                const Act aa = new_act("s0.audio"), xa = new_act("s0.x"), ha = new_act("s0.h");
                ra.wh16 = e->res0_h16;
                ra.ascale = aa.scale;
                ra.xscale = xa.scale;
                ra.hscale = ha.scale;
                ra.unscale0 = 1.0f / (aa.scale * e->res0_wsc[0]);
                ra.unscale1 = 1.0f / (xa.scale * e->res0_wsc[1]);
                ra.unscale2 = 1.0f / (ha.scale * e->res0_wsc[2]);
                ra.aamax = aa.amax;
                ra.xamax = xa.amax;
                ra.hamax = ha.amax;
            }
            if (si == 1 && h16) {
                // fp16-plane stage-1 block: ELU(x) and ELU(h) split in-kernel at their own scales
                const Act xa = new_act("s1.x"), ha = new_act("s1.h");
                ra.wh16 = e->res1_h16;
                ra.xscale = xa.scale;
                ra.hscale = ha.scale;
                ra.unscale1 = 1.0f / (xa.scale * e->res1_wsc[0]);
                ra.unscale2 = 1.0f / (ha.scale * e->res1_wsc[1]);
                ra.xamax = xa.amax;
                ra.hamax = ha.amax;
                ra.form = e->res1_form;
            }
            if (rg && !(h16 && (si == 0 || si == 1))) return set_err(MIMI_ERR_UNSUPPORTED, "ragged: fp16 blocks only");
            const double H = C / c.compress;
            const double BT = rows_of(si, (double)B * T);
            const double fl = 2.0 * BT * (3.0 * C * H + H * C) + (si == 0 ? 2.0 * BT * C * c.kernel_size : 0.0);
            const DevConv& dc0 = e->down[0];
            bool t1_ceil = p.T[1] == (T + 3) / 4;  // the kernel's output steps: ceil(T0 / 4) per item
            if (rg)
                for (int b = 0; b < B; ++b) t1_ceil = t1_ceil && rg->plan[b].T[1] == (rg->plan[b].T[0] + 3) / 4;
            if (si == 0 && h16 && e->stage0_fused && C == 64 && dc0.cin == 64 && dc0.cout == 128 &&
                dc0.k == 8 && dc0.stride == 4 && dc0.wh && dc0.b && t1_ceil) {
                // y stays on chip: the block's output feeds down conv 0 in the same kernel (x1 = its fp32 output)
                ra.wdown = dc0.wh;
                ra.bdown = dc0.b;
                ra.unscale_d = 1.0f / (yact.scale * dc0.wscale);
                ra.xout = w.x;
                ra.T1 = p.T[1];
                ra.yp = e->taps ? w.y : nullptr;  // taps only: y planes to HBM as well
                LAUNCH_TRY(launch_stage0_fused(ra, s, &kname), "stage 0 + down conv 0");
                const double BT1 = rows_of(1, (double)B * p.T[1]);
                const double fld = 2.0 * BT1 * 128.0 * 512.0;
                // HBM: audio in, x1 out, both weight sets (y never leaves the CU)
                const double by = BT * 4 + BT1 * 128 * 4 + (3.0 * C * H + H * C) * 4 + 128.0 * 512 * 4;
                rec.mark("res_down_s0", fl + fld, by, kname);
                if ((rc = save_tap_planes(e, "res0_elu", w.y, ns, B, T, C, s, yact.scale))) return rc;
                if ((rc = save_tap_planes(e, "down0", w.x, 0, B, p.T[1], 2 * C, s, 0.0f))) return rc;
                C *= 2;
                continue;
            }
            LAUNCH_TRY(launch_resblock(C, ra, s, &kname), "resblock");
            snprintf(nm, sizeof nm, "res_s%d", si);
            const double by = BT * 4 * (si == 0 ? 1 + C : 2 * C) + (3.0 * C * H + H * C) * 4;
            rec.mark(nm, fl, by, kname);
        } else {
            // two plane GEMMs: h = ELU(b3 + W3 (*) ELU(x)) from the ELU(x) planes the down conv wrote, then
            // y = ELU(x + b1 + W1 . h) with the fp32 x as the skip
            const int Hh = C / c.compress;
            GemmArgs a3 = conv_args(e->res3[si], nullptr, T, nullptr, T, B);
            planes_in(a3, w.xe, (long long)B * T * C);
            use_h(a3, e->res3[si].wh, e->res3[si].wscale, xeact);
            a3.Cp = w.h;
            a3.c_pstride = (long long)B * T * Hh;
            if (rg) a3.a_rows = a3.m_rows = dT[si];
            hact = new_act(nmf("h%d", si));
            out_act(a3, hact);
            LAUNCH_TRY(launch_gemm(ROLE_RES3P, a3, s, &kname, prec), "res3");
            snprintf(nm, sizeof nm, "res3_s%d", si);
            rec.mark(nm, gemm_flops(a3) * rows_of(si, (double)B * T) / ((double)B * T), gemm_bytes(a3, false), kname);
            GemmArgs a1 = conv_args(e->res1[si], nullptr, T, nullptr, T, B);
            planes_in(a1, w.h, (long long)B * T * Hh);
            use_h(a1, e->res1[si].wh, e->res1[si].wscale, hact);
            a1.R = w.x;
            a1.Cp = w.y;
            a1.c_pstride = (long long)B * T * C;
            if (rg) a1.a_rows = a1.m_rows = dT[si];
            yact = new_act(nmf("y%d", si));
            out_act(a1, yact);
            if (h16 && e->res1_stream && res1_stream_ok(a1) && (e->res1_stream == 2 || a1.K == 128))
                LAUNCH_TRY(launch_res1_stream(a1, s, &kname), "res1 stream");
            else
                LAUNCH_TRY(launch_gemm(ROLE_RES1P, a1, s, &kname, prec), "res1");
            snprintf(nm, sizeof nm, "res1_s%d", si);
            rec.mark(nm, gemm_flops(a1) * rows_of(si, (double)B * T) / ((double)B * T), gemm_bytes(a1, true), kname);
        }
        snprintf(nm, sizeof nm, "res%d_elu", si);
        if ((rc = save_tap_planes(e, nm, w.y, ns, B, T, C, s, yact.scale))) return rc;
        const bool last = si == c.num_ratios - 1;
        const bool next_unf = ns && !last && si + 1 >= mimi_engine::kUnfuseFrom;
        GemmArgs ad = conv_args(e->down[si], w.y, T, w.x, p.T[si + 1], B);
        int role = last ? ROLE_DOWN_ELU : ROLE_DOWN;
        if (ns) {
            planes_in(ad, w.y, (long long)B * T * C);
            use_h(ad, e->down[si].wh, e->down[si].wscale, yact);
            if (last) {  // only the final conv reads it: planes out
                ad.Cp = w.x;
                ad.c_pstride = (long long)B * p.T[si + 1] * 2 * C;
                ad.C = nullptr;
                xact = new_act("x_last");
                out_act(ad, xact);
            } else if (next_unf) {  // fp32 x (the skip) + ELU(x) planes (the next k3 conv's input)
                ad.Cp = w.xe;
                ad.c_pstride = (long long)B * p.T[si + 1] * 2 * C;
                role = ROLE_DOWN_XE;
                xeact = new_act(nmf("xe%d", si + 1));
                out_act(ad, xeact);
            }
        }
        if (rg) {
            ad.a_rows = dT[si];
            ad.m_rows = dT[si + 1];
        }
        LAUNCH_TRY(launch_gemm(role, ad, s, &kname, prec), "down");
        snprintf(nm, sizeof nm, "down_s%d", si);
        rec.mark(nm, gemm_flops(ad) * rows_of(si + 1, (double)B * p.T[si + 1]) / ((double)B * p.T[si + 1]),
                 gemm_bytes(ad, false), kname);
        snprintf(nm, sizeof nm, last ? "down%d_elu" : "down%d", si);
        if ((rc = save_tap_planes(e, nm, w.x, last ? ns : 0, B, p.T[si + 1], 2 * C, s, last ? xact.scale : 0.0f)))
            return rc;
        C *= 2;
    }
    const int64_t T = p.frames25;
    const int Hd = c.hidden_size;
    GemmArgs af = conv_args(e->final_conv, w.x, p.T[c.num_ratios], w.t0, T, B);
    if (ns) planes_in(af, w.x, (long long)B * p.T[c.num_ratios] * C);
    use_h(af, e->final_conv.wh, e->final_conv.wscale, xact);
    if (rg) {  // ragged: the output rows packed (item b's frames from row toff[b] on) for the transformer section
        af.a_rows = dT[c.num_ratios];
        af.m_rows = dT25;
        af.c_boff = dToff;
    }
    LAUNCH_TRY(launch_gemm(ROLE_FINAL, af, s, &kname, prec), "final");
    const double rT25 = rows_of(5, (double)B * p.frames25) / ((double)B * p.frames25);  // ragged share of the rows
    rec.mark("final", gemm_flops(af) * rT25, gemm_bytes(af, false), kname);
    // ---- transformer (x in t0) ----
    // rows: B x T, or for a ragged batch the items' frames PACKED back to back (R rows): every row-local stage
    // (LayerNorm, q/k/v, o_proj, fc1, fc2) then runs the uniform kernels over exactly the valid rows -- no per-item
    // tiles half empty -- and computes each row with the same instruction sequence as the per-item form; attention
    // and the downsample address the items through toff, RoPE takes each row's position from rpos
    const int64_t rows = rg ? rg->R : (int64_t)B * T;
    const int64_t tapB = rg ? 1 : B, tapT = rg ? rg->R : T;  // (ragged taps of the transformer section: packed)
    if ((rc = save_tap(e, "encoder", w.t0, tapB, tapT, Hd, s))) return rc;
    const int H = c.num_attention_heads, Dh = c.head_dim;
    // f16x3: downsample + input projections on fp16 planes too (zero-padded GEMM + replicate-edge fix)
    const bool ds_planes = h16 && e->ds_fix && e->inproj_h && c.downsample_kernel == 4 && c.downsample_stride == 2;
    Act dsin, dsouta;
    double att_flops = 0;
    auto att_fl = [&](int64_t Tn) {
        double f = 0;
        for (int64_t i = 0; i < Tn; ++i) f += 4.0 * Dh * std::min<int64_t>(i + 1, c.sliding_window);
        return f * H;
    };
    if (rg) {
        for (const auto& pb : rg->plan) att_flops += att_fl(pb.frames25);
    } else {
        att_flops = att_fl(T) * B;
    }
    for (int l = 0; l < c.num_hidden_layers; ++l) {
        const DevXfmr& x = e->xf[l];
        const long long nact = rows * Hd;
        Act t1a = new_act(nmf("xf%d.ln1", l));
        if (ln_check_free(t1a, x.ln1_bound)) t1a.amax = nullptr;
        // LayerNorm + fc1 (ln_fused >= 1) / q/k/v (ln_fused 2): on small grids one launch whose tiles compute their
        // rows' LayerNorm (the same bits as the LayerNorm kernel's planes, gemm_planes.h FL_LNA)
        auto ln_into = [&](GemmArgs& g, int role, const float* lw, const float* lb, const Act& act) {
            if (!h16 || e->ln_fused < (role == ROLE_QKV ? 2 : 1) || !gemm_ln_prologue_ok(role, g, prec)) return false;
            if (role == ROLE_QKV) g.ln_tile = e->ln_fused - 2;  // (2: 16x64, 3: 32x64, 4: 16x128 tiles)
            g.ln_x = w.t0;
            g.ln_g = lw;
            g.ln_b = lb;
            g.ln_eps = c.norm_eps;
            g.ln_scale = act.scale;
            g.ln_amax = act.amax;
            return true;
        };
        GemmArgs aq = linear_args(w.t1, T, Hd, x.wqkv, 3 * H * Dh, w.qkv);
        aq.Wsplit = x.wqkv_s;
        aq.batch = B;
        aq.a_bstride = T * Hd;
        aq.c_bstride = T * 3 * H * Dh;
        aq.rope_cos = e->rope_cos;
        aq.rope_sin = e->rope_sin;
        aq.rope_cols = 2 * H * Dh;
        if (rg) {  // packed rows: one flat GEMM, RoPE positions from rpos
            aq = linear_args(w.t1, rows, Hd, x.wqkv, 3 * H * Dh, w.qkv);
            aq.Wsplit = x.wqkv_s;
            aq.rope_cos = e->rope_cos;
            aq.rope_sin = e->rope_sin;
            aq.rope_cols = 2 * H * Dh;
            aq.rope_pos = dRpos;
        }
        if (ns) planes_in(aq, w.t1, nact);
        use_h(aq, x.wqkv_h, x.wqkv_hs, t1a);
        // q/k/v + attention in one kernel (qkv_attn.hip): large batches of items <= 256 frames, fp16 planes
        const bool fuse_qa = h16 && ns && e->qkv_attn && Dh == 64 && (rg ? rg->maxT25 <= 256 : T <= 256) &&
                             (e->qkv_attn == 2 || (long long)B * H >= 256);
        if (fuse_qa || !ln_into(aq, ROLE_QKV, x.ln1_w, x.ln1_b, t1a)) {
            LAUNCH_TRY(launch_layernorm(w.t0, x.ln1_w, x.ln1_b, w.t1, rows, Hd, c.norm_eps, s, w.t1, nact, ns, t1a.scale,
                                        t1a.amax, nullptr, 0, e->ln_rpw),
                       "ln1");
            rec.mark("layernorm", 0, 2.0 * rows * Hd * 4, ln_kname(e->ln_rpw));
        }
        const Act atta = new_act(nmf("xf%d.att", l));
        if (fuse_qa) {
            QkvAttnArgs qa{};
            qa.Ap = aq.Ap;
            qa.a_pstride = aq.a_pstride;
            qa.a_rows = rows;
            qa.Wp = aq.Wsplit;
            qa.unscale = aq.unscale;
            qa.rope_cos = e->rope_cos;
            qa.rope_sin = e->rope_sin;
            qa.K = Hd;
            qa.Ts = (int)T;
            qa.H = H;
            qa.window = c.sliding_window;
            qa.scale = 1.0f / std::sqrt((float)Dh);
            qa.outp = w.att;
            qa.out_pstride = nact;
            qa.oscale = atta.scale;
            qa.oamax = atta.amax;
            qa.tlen = rg ? dT25 : nullptr;
            qa.toff = rg ? dToff : nullptr;
            qa.qkv = e->taps ? w.qkv : nullptr;  // (the q/k/v tap, as the GEMM would have stored it)
            qa.xcd = e->qkv_attn_xcd;
            LAUNCH_TRY(launch_qkv_attention(qa, B, s), "qkv_attention");
            rec.mark("qkv_attention", gemm_flops(aq) + att_flops, (double)rows * Hd * 4 * 2 + 3.0 * H * Dh * Hd * 4,
                     "mimi::qkv_attention_h16_kernel<512>");
            if ((rc = save_tap(e, nmf("qkv%d", l).c_str(), w.qkv, tapB, tapT, 3 * H * Dh, s))) return rc;
        } else {
            aq.sc1 = (e->sc1_out & 1) != 0;
            LAUNCH_TRY(launch_gemm(ROLE_QKV, aq, s, &kname, prec), "qkv");
            rec.mark("qkv", gemm_flops(aq), gemm_bytes(aq, false), kname);
            if ((rc = save_tap(e, nmf("qkv%d", l).c_str(), w.qkv, tapB, tapT, 3 * H * Dh, s))) return rc;
            // fp16-plane attention in f16x3 mode (also for the no-plane long clips: the same arithmetic as their
            // prefixes); true fp32 in f32 mode and the bf16 modes
            const bool ah16 = prec == PREC_F16X3;
            const char* akn = ah16 ? (T <= 256 ? "mimi::attention_t256_h16_kernel" : "mimi::attention_band_h16_kernel")
                                   : (T <= 256 ? "mimi::attention_t256_kernel" : "mimi::attention_kernel");
            LAUNCH_TRY(launch_attention(w.qkv, w.att, B, (int)T, H, Dh, c.sliding_window, 1.0f / std::sqrt((float)Dh),
                                        s, w.att, nact, ns, atta.scale, atta.amax, ah16, rg ? dT25 : nullptr,
                                        rg ? rg->maxT25 : 0, rg ? rg->minT25 : 0, dToff, &akn, e->attn_band_split),
                       "attention");
            rec.mark("attention", att_flops, (double)rows * 4 * Hd * 4, akn);
        }
        if ((rc = save_tap_planes(e, nmf("att%d", l).c_str(), w.att, ns, tapB, tapT, H * Dh, s, atta.scale))) return rc;
        GemmArgs ao = linear_args(w.att, rows, H * Dh, x.wo, Hd, w.t0);
        ao.Wsplit = x.wo_s;
        ao.R = w.t0;
        ao.scale = x.ls1;
        if (ns) planes_in(ao, w.att, nact);
        use_h(ao, x.wo_h, x.wo_hs, atta);
        ao.sc1 = (e->sc1_out & 4) != 0;
        Act t1b = new_act(nmf("xf%d.ln2", l));
        if (ln_check_free(t1b, x.ln2_bound)) t1b.amax = nullptr;
        LAUNCH_TRY(launch_gemm(ROLE_OPROJ, ao, s, &kname, prec), "o_proj");
        rec.mark("o_proj", gemm_flops(ao), gemm_bytes(ao, true), kname);
        if ((rc = save_tap(e, nmf("oproj%d", l).c_str(), w.t0, tapB, tapT, Hd, s))) return rc;
        GemmArgs a1 = linear_args(w.t1, rows, Hd, x.w1, c.intermediate_size, w.ff);
        a1.Wsplit = x.w1_s;
        Act ffa;
        if (ns) {
            planes_in(a1, w.t1, nact);
            use_h(a1, x.w1_h, x.w1_hs, t1b);
            a1.Cp = w.ff;  // only fc2 reads it: planes out
            a1.c_pstride = rows * c.intermediate_size;
            a1.C = nullptr;
            ffa = new_act(nmf("xf%d.ff", l));
            out_act(a1, ffa);
        }
        if (!ln_into(a1, ROLE_FC1, x.ln2_w, x.ln2_b, t1b)) {
            LAUNCH_TRY(launch_layernorm(w.t0, x.ln2_w, x.ln2_b, w.t1, rows, Hd, c.norm_eps, s, w.t1, nact, ns, t1b.scale,
                                        t1b.amax, nullptr, 0, e->ln_rpw),
                       "ln2");
            rec.mark("layernorm", 0, 2.0 * rows * Hd * 4, ln_kname(e->ln_rpw));
        }
        a1.sc1 = (e->sc1_out & 2) != 0;
        a1.ncg = e->fc1_cg;
        LAUNCH_TRY(launch_gemm(ROLE_FC1, a1, s, &kname, prec), "fc1");
        rec.mark("fc1", gemm_flops(a1), gemm_bytes(a1, false), kname);
        if ((rc = save_tap_planes(e, nmf("ff%d", l).c_str(), w.ff, ns, tapB, tapT, c.intermediate_size, s, ffa.scale)))
            return rc;
        GemmArgs a2 = linear_args(w.ff, rows, c.intermediate_size, x.w2, Hd, w.t0);
        a2.Wsplit = x.w2_s;
        a2.R = w.t0;
        a2.scale = x.ls2;
        if (ns) planes_in(a2, w.ff, rows * (long long)c.intermediate_size);
        use_h(a2, x.w2_h, x.w2_hs, ffa);
        if (ds_planes && l == c.num_hidden_layers - 1) {  // + planes of the encoder output: the downsample's A
            a2.Cp = w.t1;
            a2.c_pstride = nact;
            dsin = new_act("ds.in");
            out_act(a2, dsin);
        }
        a2.sc1 = (e->sc1_out & 4) != 0;
        LAUNCH_TRY(launch_gemm(ROLE_FC2, a2, s, &kname, prec), "fc2");
        rec.mark("fc2", gemm_flops(a2), gemm_bytes(a2, true), kname);
        snprintf(nm, sizeof nm, "xfmr%d", l);
        if ((rc = save_tap(e, nm, w.t0, tapB, tapT, Hd, s))) return rc;
    }

    // ---- downsample (replicate pad) + input projections + RVQ ----
    const int64_t T2 = p.frames12;
    GemmArgs ad = conv_args(e->ds, w.t0, T, w.dsout, T2, B);
    if (ds_planes) {
        planes_in(ad, w.t1, rows * Hd);
        use_h(ad, e->ds.wh, e->ds.wscale, dsin);
        ad.Cp = w.att;  // planes of the downsample output (the input projection's A); fp32 C beside
        ad.c_pstride = (long long)B * T2 * Hd;
        dsouta = new_act("ds.out");
        out_act(ad, dsouta);
    }
    if (rg) {  // the packed encoder output in, per-item frames out
        if (!ds_planes) return set_err(MIMI_ERR_UNSUPPORTED, "ragged: planes downsample only");
        ad.a_rows = dT25;
        ad.m_rows = dF;
        ad.a_boff = dToff;
    }
    LAUNCH_TRY(launch_gemm(ROLE_DOWNSAMPLE, ad, s, &kname, prec), "downsample");
    if ((rc = save_tap(e, "ds_gemm", w.dsout, B, T2, Hd, s))) return rc;  // (before the replicate-pad rows)
    if (ds_planes)
        LAUNCH_TRY(launch_ds_edge_fix(w.t0, e->ds_fix, w.dsout, w.att, ad.c_pstride, dsouta.scale, dsouta.amax, B,
                                      (int)T, (int)T2, Hd, Hd, s, rg ? dT25 : nullptr, rg ? dF : nullptr, dToff),
                   "downsample edges");
    const double rF = rows_of(6, (double)B * T2) / ((double)B * T2);
    rec.mark("downsample", gemm_flops(ad) * rF, gemm_bytes(ad, false), kname);
    if ((rc = save_tap(e, "downsample", w.dsout, B, T2, Hd, s))) return rc;
    const int Dq = c.vq_hidden_dim;
    GemmArgs ap = linear_args(w.dsout, (int64_t)B * T2, Hd, e->inproj, 2 * Dq, w.proj);
    if (ds_planes) {
        planes_in(ap, w.att, (long long)B * T2 * Hd);
        use_h(ap, e->inproj_h, e->inproj_hs, dsouta);
    }
    if (rg) {  // ragged: per item (batch B, M = T2 frames each, the valid ones per item) -- the same instruction
               // sequence per output as the flattened [B x T2] form
        ap.batch = B;
        ap.M = (int)T2;
        ap.a_bstride = T2 * Hd;
        ap.c_bstride = T2 * 2 * Dq;
        ap.a_len = T2 * Hd;
        ap.a_rows = ap.m_rows = dF;
    }
    LAUNCH_TRY(launch_gemm(ROLE_INPROJ, ap, s, &kname, ds_planes ? PREC_F16X3 : PREC_F32), "input_proj");
    rec.mark("input_proj", gemm_flops(ap) * rF, gemm_bytes(ap, false), kname);
    if ((rc = save_tap(e, "proj", w.proj, B, T2, 2 * Dq, s))) return rc;
    if ((rc = run_rvq(e, w.proj, (int64_t)B * T2, K, codes, (int)T2, w.rvq, s, rec, rg ? dF : nullptr, rF))) return rc;
    if (!e->capturing) HIP_TRY(hipEventRecord(e->ws_free, s));
    return MIMI_OK;
}

// Activation scales (PREC_F16X3).  A plane tensor with max|x| = a stored at scale s keeps every element's full
// 22-bit significand down to 2^-3 / s (h1 = fp16(x s - h0) normal) and an absolute error <= 2^-25 / s below;
// a s < 2^15 keeps x s (and h0) finite.  The scales are FIXED per tensor name: mimi_finalize runs a calibration
// encode on three full-scale 10 s signals (calibrate_scales) and puts every tensor's calibration maximum at
// a s in [2^7, 2^8).  They never follow the caller's audio, so an item's codes are a pure function of its own
// samples and the padded length -- not of its batch-mates or of what the engine encoded before (the reference
// is a pure function of the batch too, TF/modeling_mimi.py:1297-1386).  A tensor 2^7 x louder than the
// calibration's loudest would overflow: every encode reads the per-tensor maxima back, and on an overflow each
// item is re-encoded alone (at the same padded length) and, if it overflows alone, in the scale-free bf16x6
// arithmetic -- so the fallback too depends on the item alone.  Quieter tensors need no action: their
// absolute error stays <= 2^-25 / s = 2^-32..2^-33 of the calibration maximum.
constexpr float kF16Overflow = 32768.0f;  // a s >= 2^15: x s may round to an fp16 infinity

// folds and reads back the per-slot maxima of the last pass (synchronises s)
static int read_amax(mimi_engine* e, hipStream_t s, int* n) {
    const int ns = (int)e->slot_of.size();
    *n = ns;
    if (ns == 0) return MIMI_OK;
    LAUNCH_TRY(launch_amax_reduce(e->amax_dev, ns, e->amax_red, s), "amax_reduce");
    HIP_TRY(hipMemcpyAsync(e->amax_host, e->amax_red, ns * sizeof(unsigned), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return MIMI_OK;
}

static float slot_amax(const mimi_engine* e, int i) {
    float a;
    std::memcpy(&a, &e->amax_host[i], 4);
    return a;
}

// one f16x3 pass and its overflow check.  Non-finite maxima are not overflows of the scale: they come from a
// non-finite input, which the reference propagates too.
static int f16_pass(mimi_engine* e, const float* audio, int B, int64_t L, int K, int32_t* codes, hipStream_t s,
                    bool* overflow) {
    *overflow = false;
    HIP_TRY(hipStreamWaitEvent(s, e->ws_free, 0));  // encodes enqueued on other streams use amax_dev too
    HIP_TRY(hipMemsetAsync(e->amax_dev, 0, (size_t)kMaxActSlots * AMAX_SLOT_WORDS * sizeof(unsigned), s));
    e->uncalibrated_slot = false;
    int rc = encode_pass(e, audio, B, L, K, codes, s, PREC_F16X3);
    if (rc) return rc;
    if (e->uncalibrated_slot) {
        e->uncalibrated_slot = false;
        return set_err(MIMI_ERR_STATE, "f16x3: an activation has no calibrated scale");
    }
    int n = 0;
    if ((rc = read_amax(e, s, &n))) return rc;
    for (int i = 0; i < n; ++i) {
        const float a = slot_amax(e, i);
        if (std::isfinite(a) && a * e->act_scale[i] >= kF16Overflow) *overflow = true;
    }
    return MIMI_OK;
}

static int calibrate_scales(mimi_engine* e) {
    const int B = 3;
    const int64_t L = 240000;
    std::vector<float> h((size_t)B * L);
    uint64_t st = 0x243F6A8885A308D3ull;  // splitmix64
    auto uni = [&]() {
        uint64_t z = (st += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        return (double)(z >> 11) * (1.0 / 9007199254740992.0);
    };
    const double fs = 24000.0, pi = 3.14159265358979323846;
    float pk = 0.0f;
    for (int64_t i = 0; i < L; ++i) {
        const double t = i / fs;
        h[i] = (float)(2.0 * uni() - 1.0);  // white noise, U[-1, 1]
        // harmonic mix of a gliding 90..250 Hz fundamental under a 4 Hz syllable envelope
        const double f0 = 170.0 + 80.0 * std::sin(2 * pi * 0.3 * t);
        double v = 0.0;
        for (int k = 1; k <= 12; ++k) v += std::sin(2 * pi * f0 * k * t + 0.7 * k) / k;
        v *= 0.55 + 0.45 * std::sin(2 * pi * 4.0 * t);
        h[L + i] = (float)v;
        pk = std::max(pk, std::fabs(h[L + i]));
        // logarithmic sine sweep 50 Hz -> 11 kHz over the clip, amplitude 1
        const double T = L / fs, k = std::log(11000.0 / 50.0);
        h[2 * L + i] = (float)std::sin(2 * pi * 50.0 * T / k * (std::exp(t / T * k) - 1.0));
    }
    for (int64_t i = 0; i < L; ++i) h[L + i] /= pk;
    const int K = e->cfg.num_semantic_quantizers;
    const int64_t T2 = plan_lengths(e->cfg, L).frames12;
    float* d_audio = nullptr;
    int32_t* d_codes = nullptr;
    hipStream_t s = nullptr;
    int rc = MIMI_OK;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    if (hipMalloc(&d_audio, h.size() * 4) != hipSuccess || hipMalloc(&d_codes, (size_t)B * K * T2 * 4) != hipSuccess) {
        rc = set_err(MIMI_ERR_OUT_OF_MEMORY, "calibration buffers");
    } else if (hipMemcpy(d_audio, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
        rc = set_err(MIMI_ERR_HIP, "calibration upload");
    }
    e->calibrating = true;
    for (int it = 0; rc == MIMI_OK && it < 8; ++it) {
        if (hipMemsetAsync(e->amax_dev, 0, (size_t)kMaxActSlots * AMAX_SLOT_WORDS * sizeof(unsigned), s) != hipSuccess) {
            rc = set_err(MIMI_ERR_HIP, "calibration memset");
            break;
        }
        int n = 0;
        if ((rc = encode_pass(e, d_audio, B, L, K, d_codes, s, PREC_F16X3)) || (rc = read_amax(e, s, &n))) break;
        bool changed = false;
        for (int i = 0; i < n; ++i) {
            const float a = slot_amax(e, i);
            if (!(a > 0.0f) || !std::isfinite(a)) continue;
            const float as = a * e->act_scale[i];
            if (as < 64.0f || as >= 512.0f) {  // hysteresis band around the [2^7, 2^8) target
                e->act_scale[i] = std::ldexp(1.0f, 7 - std::ilogb(a));
                changed = true;
            }
        }
        if (!changed) break;
    }
    e->calibrating = false;
    e->uncalibrated_slot = false;
    if (rc == MIMI_OK) e->calibrated = true;
    (void)hipStreamSynchronize(s);
    if (d_audio) (void)hipFree(d_audio);
    if (d_codes) (void)hipFree(d_codes);
    (void)hipStreamDestroy(s);
    return rc;
}

// Per-item overflow fallback of one f16x3 encode (see "activation scales"): every item re-encoded alone at the
// same padded length, in bf16x6 where it overflows alone.  Synchronises s.
static int overflow_fallback(mimi_engine* e, const float* audio, int B, int64_t L, int K, int32_t* codes,
                             hipStream_t s) {
    ++e->f16_reruns;
    const StagePlan p = plan_lengths(e->cfg, L);
    int rc;
    if (B == 1) {
        if ((rc = encode_pass(e, audio, 1, L, K, codes, s, PREC_BF16X6))) return rc;
        HIP_TRY(hipStreamSynchronize(s));
        return MIMI_OK;
    }
    const size_t per = (size_t)K * p.frames12;
    if (e->item_codes_cap < per) {
        HIP_TRY(hipStreamSynchronize(s));
        if (e->item_codes) HIP_TRY(hipFree(e->item_codes));
        e->item_codes = nullptr;
        e->item_codes_cap = 0;
        HIP_TRY(hipMalloc(&e->item_codes, per * sizeof(int32_t)));
        e->item_codes_cap = per;
    }
    bool ovf = false;
    for (int b = 0; b < B; ++b) {
        const float* ab = audio + (int64_t)b * L;
        if ((rc = f16_pass(e, ab, 1, L, K, e->item_codes, s, &ovf))) return rc;
        if (ovf && (rc = encode_pass(e, ab, 1, L, K, e->item_codes, s, PREC_BF16X6))) return rc;
        HIP_TRY(hipMemcpyAsync(codes + b * per, e->item_codes, per * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    return MIMI_OK;
}

// Ragged batch, item by item (each alone at its own length: the definition of the ragged result): the f16x3
// overflow fallback of a ragged encode, and the whole ragged encode where the batched form does not apply
// (precision modes other than f16x3, clips too long for the plane buffers).  Item b's codes go to
// codes[b][k][0 .. F_b) of the [B][K][Fmax] output.  Synchronises s.
static int ragged_item_by_item(mimi_engine* e, const float* audio, int B, int64_t L, const int64_t* lens, int K,
                               int32_t* codes, hipStream_t s, int prec) {
    const int64_t Fmax = plan_lengths(e->cfg, L).frames12;
    const size_t per = (size_t)K * Fmax;
    if (e->item_codes_cap < per) {
        HIP_TRY(hipStreamSynchronize(s));
        if (e->item_codes) HIP_TRY(hipFree(e->item_codes));
        e->item_codes = nullptr;
        e->item_codes_cap = 0;
        HIP_TRY(hipMalloc(&e->item_codes, per * sizeof(int32_t)));
        e->item_codes_cap = per;
    }
    int rc;
    for (int b = 0; b < B; ++b) {
        const float* ab = audio + (int64_t)b * L;
        const int64_t Fb = plan_lengths(e->cfg, lens[b]).frames12;
        if (prec == PREC_F16X3 && act_planes(e, plan_lengths(e->cfg, lens[b]), prec) == 2) {
            bool ovf = false;
            if ((rc = f16_pass(e, ab, 1, lens[b], K, e->item_codes, s, &ovf))) return rc;
            if (ovf) {
                ++e->f16_reruns;
                if ((rc = encode_pass(e, ab, 1, lens[b], K, e->item_codes, s, PREC_BF16X6))) return rc;
            }
        } else if ((rc = encode_pass(e, ab, 1, lens[b], K, e->item_codes, s, prec))) {
            return rc;
        }
        HIP_TRY(hipMemcpy2DAsync(codes + (int64_t)b * K * Fmax, Fmax * sizeof(int32_t), e->item_codes,
                                 Fb * sizeof(int32_t), Fb * sizeof(int32_t), K, hipMemcpyDeviceToDevice, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    return MIMI_OK;
}

// ---- hipGraph replay (f16x3).  A small batch is launch-bound: ~80 kernels per encode, each a few
// microseconds of GPU time.  The second encode of a (batch, length, K) shape captures the whole pass -- the
// maxima reset, every kernel, the maxima fold -- into a graph on a private stream; later encodes of that shape
// replay it on the caller's stream behind one set_io_kernel that writes this call's audio / codes pointers
// into io_dev (the stage-0 block and the RVQ kernels read them from there; every other operand lives in the
// engine: weights, workspace, rope tables).  A graph is dropped when the workspace or the rope tables it
// addresses are reallocated.  The replay is the same kernels with the same arguments: bit-identical codes.
static void destroy_graph(mimi_engine::Graph& g) {
    if (g.x) (void)hipGraphExecDestroy(g.x);
    if (g.g) (void)hipGraphDestroy(g.g);
    g.x = nullptr;
    g.g = nullptr;
}

static void drop_graphs(mimi_engine* e) {
    for (auto& g : e->graphs) destroy_graph(g);
    e->graphs.clear();
}

// Captures the f16x3 pass of (B, L, K) into a new graph.  On any failure the capture is abandoned and the
// caller runs the eager pass (the error is cleared: a graph is an optimisation, never a requirement).
static mimi_engine::Graph* capture_graph(mimi_engine* e, const float* audio, int B, int64_t L, int K,
                                          int32_t* codes) {
    if (!e->io_dev && hipMalloc(&e->io_dev, 4 * sizeof(void*)) != hipSuccess) {
        (void)hipGetLastError();
        e->io_dev = nullptr;
        return nullptr;
    }
    if (!e->cap_stream && hipStreamCreateWithFlags(&e->cap_stream, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        e->cap_stream = nullptr;
        return nullptr;
    }
    hipStream_t cs = e->cap_stream;
    if (hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    e->capturing = true;
    e->cap_chain_clear = 0;
    e->uncalibrated_slot = false;
    int rc = MIMI_OK;
    // (no maxima reset node: amax_reduce_kernel leaves every sub-slot at 0 as it reads it, so a replay starts
    // from the zeros the previous encode's fold left behind)
    rc = encode_pass(e, audio, B, L, K, codes, cs, PREC_F16X3);
    // (+ the ticket's host words from inside the graph: destinations through io_dev, set before each replay)
    if (!rc && launch_amax_reduce(e->amax_dev, (int)e->slot_of.size(), e->amax_red, cs, nullptr, e->chain_flag, nullptr,
                                  e->io_dev) != hipSuccess)
        rc = MIMI_ERR_HIP;
    e->capturing = false;
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(cs, &g);
    hipGraphExec_t x = nullptr;
    if (rc || ec != hipSuccess || !g || e->uncalibrated_slot || hipGraphInstantiate(&x, g, nullptr, nullptr, 0) != hipSuccess) {
        (void)hipGetLastError();
        e->uncalibrated_slot = false;
        if (g) (void)hipGraphDestroy(g);
        return nullptr;
    }
    if ((int)e->graphs.size() >= mimi_engine::kMaxGraphs) {  // evict the least recently used
        size_t lru = 0;
        for (size_t i = 1; i < e->graphs.size(); ++i)
            if (e->graphs[i].used < e->graphs[lru].used) lru = i;
        destroy_graph(e->graphs[lru]);
        e->graphs.erase(e->graphs.begin() + (long)lru);
    }
    mimi_engine::Graph ng;
    ng.B = B;
    ng.L = L;
    ng.K = K;
    ng.ws_gen = e->ws_gen;
    ng.rope_gen = e->rope_gen;
    ng.g = g;
    ng.x = x;
    ng.chain_flag = e->chain_flag;
    ng.chain_clear = e->chain_flag ? e->cap_chain_clear : 0;
    e->graphs.push_back(ng);
    return &e->graphs.back();
}

// Runs the f16x3 pass of (B, L, K) as a graph replay on s when it can (*replayed = true); otherwise leaves
// everything to the eager path.
static int graph_encode(mimi_engine* e, const float* audio, int B, int64_t L, int K, int32_t* codes, hipStream_t s,
                        bool* replayed, unsigned** chain_flag, unsigned* host_amax, unsigned* host_flag) {
    *replayed = false;
    *chain_flag = nullptr;
    if (!e->graphs_enabled || e->profiling || e->taps || e->calibrating) return MIMI_OK;
    // sizes first: nothing may be allocated inside a capture, and a reallocation retires the graphs
    const StagePlan p = plan_lengths(e->cfg, L);
    int rc = ensure_ws(e, ws_layout(e, B, p, nullptr, PREC_F16X3), s);
    if (rc) return rc;
    if ((rc = ensure_rope(e, p.frames25))) return rc;
    mimi_engine::Graph* gr = nullptr;
    for (auto it = e->graphs.begin(); it != e->graphs.end();) {
        if (it->ws_gen != e->ws_gen || it->rope_gen != e->rope_gen) {
            destroy_graph(*it);
            it = e->graphs.erase(it);
            continue;
        }
        if (it->B == B && it->L == L && it->K == K) gr = &*it;
        ++it;
    }
    if (!gr) {
        const auto key = std::make_tuple(B, L, K);
        if (e->graph_seen.size() > 256) e->graph_seen.clear();
        if (++e->graph_seen[key] < 2) return MIMI_OK;  // a shape seen once runs eagerly
        gr = capture_graph(e, audio, B, L, K, codes);
        if (!gr) {
            e->graphs_enabled = false;  // capture unsupported here: stay eager from now on
            return MIMI_OK;
        }
    }
    gr->used = ++e->graph_clock;
    HIP_TRY(hipStreamWaitEvent(s, e->ws_free, 0));
    LAUNCH_TRY(launch_set_io(e->io_dev, audio, codes, s, host_amax, host_flag, gr->chain_flag, gr->chain_clear),
               "set_io");
    HIP_TRY(hipGraphLaunch(gr->x, s));
    ++e->graph_replays;
    *replayed = true;
    *chain_flag = gr->chain_flag;
    return MIMI_OK;
}

// Enqueues one encode on s and returns its ticket without waiting.  In f16x3 the per-tensor maxima are folded
// and copied to this ticket's pinned slot behind the encode; mimi_encode_wait checks them.
static int encode_async_locked(mimi_engine* e, const float* audio, int B, int64_t L, int K, int32_t* codes,
                               hipStream_t s, int64_t* ticket, const int64_t* lengths = nullptr) {
    mimi_engine::Pending* P = nullptr;
    for (auto& q : e->pend)
        if (q.id == 0) {
            P = &q;
            break;
        }
    if (!P)
        return set_err(MIMI_ERR_STATE, "%d encodes in flight: call mimi_encode_wait first", mimi_engine::kMaxPending);
    if (!P->done) HIP_TRY(hipEventCreateWithFlags(&P->done, hipEventDisableTiming));
    if (!P->amax) HIP_TRY(hipHostMalloc(&P->amax, kMaxActSlots * sizeof(unsigned), hipHostMallocDefault));
    if (!P->chain_word) HIP_TRY(hipHostMalloc(&P->chain_word, 16, hipHostMallocDefault));
    // the slot's last ticket was waited, so nothing in flight writes this word: clear it here rather than trust that
    // a kernel of this encode writes it (amax_reduce skips its launch when there is nothing to reduce)
    P->chain_word[0] = 0u;
    P->chain = false;
    const int prec = e->precision;
    const bool h16 = prec == PREC_F16X3 && act_planes(e, plan_lengths(e->cfg, L), prec) == 2;
    int rc;
    int n = 0;
    // Calibrate whenever f16x3 is on, not only when this batch's longest item gets planes: a ragged batch whose
    // longest item is past the plane limit runs its short items through the planes path item by item.
    if (prec == PREC_F16X3 && !e->calibrated && (rc = calibrate_scales(e))) return rc;
    RaggedTable rt;
    if (lengths) {
        const mimi_config& c = e->cfg;
        const bool batched = h16 && e->res0_h16 && e->res1_h16 && e->ds_fix && e->inproj_h &&
                             c.downsample_kernel == 4 && c.downsample_stride == 2 && c.num_ratios >= 2;
        if (!batched) {  // item by item, synchronously (the ticket's event is then already complete)
            if ((rc = ragged_item_by_item(e, audio, B, L, lengths, K, codes, s, prec))) return rc;
            HIP_TRY(hipEventRecord(P->done, s));
            P->nslots = 0;
            P->h16 = false;
            P->ragged = false;
            P->audio = audio;
            P->B = B;
            P->L = L;
            P->K = K;
            P->codes = codes;
            P->s = s;
            P->claimed = false;
            P->id = e->next_ticket++;
            *ticket = P->id;
            return MIMI_OK;
        }
        rt.B = B;
        rt.len.assign(lengths, lengths + B);
        rt.plan.resize(B);
        for (int b = 0; b < B; ++b) rt.plan[b] = plan_lengths(c, lengths[b]);
        rt.minT25 = rt.maxT25 = (int)rt.plan[0].frames25;
        for (const auto& pb : rt.plan) {
            rt.minT25 = std::min<int>(rt.minT25, (int)pb.frames25);
            rt.maxT25 = std::max<int>(rt.maxT25, (int)pb.frames25);
            rt.R += pb.frames25;
        }
        const size_t need = RaggedTable::ints(B) * sizeof(int);
        if (P->rg_cap < need) {
            if (P->rg_pinned) HIP_TRY(hipHostFree(P->rg_pinned));
            P->rg_pinned = nullptr;
            P->rg_cap = 0;
            HIP_TRY(hipHostMalloc(&P->rg_pinned, need, hipHostMallocDefault));
            P->rg_cap = need;
        }
        rt.fill(P->rg_pinned);
    }
    if (h16) {
        bool replayed = false;
        unsigned* cflag = nullptr;
        struct ChainScope {  // the chain is allowed inside this pass only (its flag is read back below)
            mimi_engine* e;
            explicit ChainScope(mimi_engine* x) : e(x) { e->chain_ok = true; }
            ~ChainScope() { e->chain_ok = false; }
        } chain_scope(e);
        if (!lengths &&
            (rc = graph_encode(e, audio, B, L, K, codes, s, &replayed, &cflag, P->amax, P->chain_word)))
            return rc;
        n = (int)e->slot_of.size();
        if (!replayed) {
            HIP_TRY(hipStreamWaitEvent(s, e->ws_free, 0));  // the maxima buffers are part of the workspace
            HIP_TRY(hipMemsetAsync(e->amax_dev, 0, (size_t)kMaxActSlots * AMAX_SLOT_WORDS * sizeof(unsigned), s));
            e->uncalibrated_slot = false;
            if ((rc = encode_pass(e, audio, B, L, K, codes, s, PREC_F16X3, lengths ? &rt : nullptr, P->rg_pinned)))
                return rc;
            if (e->uncalibrated_slot) {  // this encode only: the next one starts clean
                e->uncalibrated_slot = false;
                return set_err(MIMI_ERR_STATE, "f16x3: an activation has no calibrated scale");
            }
            cflag = e->chain_flag;
            // the maxima and (chain) the give-up flag also into the ticket's pinned words, before ws_free (the next
            // encode's memset node zeroes the flag); a replay's graph ends with the same kernel (capture_graph)
            LAUNCH_TRY(launch_amax_reduce(e->amax_dev, n, e->amax_red, s, P->amax, cflag, cflag ? P->chain_word : nullptr),
                       "amax_reduce");
        }
        P->chain = cflag != nullptr;
        HIP_TRY(hipEventRecord(e->ws_free, s));
    } else if ((rc = encode_pass(e, audio, B, L, K, codes, s, prec))) {
        return rc;
    }
    HIP_TRY(hipEventRecord(P->done, s));
    P->nslots = n;
    P->h16 = h16;
    P->audio = audio;
    P->B = B;
    P->L = L;
    P->K = K;
    P->codes = codes;
    P->s = s;
    P->ragged = lengths != nullptr;
    if (lengths) P->lens.assign(lengths, lengths + B);
    P->claimed = false;
    P->id = e->next_ticket++;
    *ticket = P->id;
    return MIMI_OK;
}

// Waits for ticket's encode and runs its f16x3 overflow check.  The engine lock is NOT held while the host
// synchronises on the encode's event (other threads keep enqueueing on the engine meanwhile): the slot is claimed
// under the lock -- so it is neither reused nor waited twice -- and released, with the overflow check and any
// fallback, under the lock again.
static int encode_wait(mimi_engine* e, int64_t ticket) {
    mimi_engine::Pending q;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        mimi_engine::Pending* P = nullptr;
        for (auto& x : e->pend)
            if (ticket > 0 && x.id == ticket && !x.claimed) P = &x;
        if (!P) return set_err(MIMI_ERR_INVALID_ARGUMENT, "ticket %lld is not an encode in flight", (long long)ticket);
        P->claimed = true;
        q = *P;
    }
    HIP_TRY(hipSetDevice(e->device));
    const hipError_t se = hipEventSynchronize(q.done);
    std::lock_guard<std::mutex> lk(e->mu);
    mimi_engine::Pending* P = nullptr;
    for (auto& x : e->pend)
        if (x.id == ticket) P = &x;
    bool ovf = false;
    const bool chain_gave_up = q.chain && se == hipSuccess && P->chain_word[0] != 0u;
    if (q.h16 && se == hipSuccess) {
        e->last_amax.assign(q.nslots, 0.0f);
        for (int i = 0; i < q.nslots; ++i) {
            float a;
            std::memcpy(&a, &P->amax[i], 4);
            e->last_amax[i] = a;
            if (std::isfinite(a) && a * e->act_scale[i] >= kF16Overflow) ovf = true;
        }
    }
    P->claimed = false;
    P->id = 0;
    if (se != hipSuccess)
        return set_err(se == hipErrorOutOfMemory ? MIMI_ERR_OUT_OF_MEMORY : MIMI_ERR_HIP, "hipEventSynchronize: %s",
                       hipGetErrorString(se));
    if (chain_gave_up) {  // the persistent RVQ gave up (its codes are not kept): the whole encode again, without it
        ++e->chain_reruns;
        HIP_TRY(hipSetDevice(e->device));
        if (q.ragged) return ragged_item_by_item(e, q.audio, q.B, q.L, q.lens.data(), q.K, q.codes, q.s, PREC_F16X3);
        bool ovf2 = false;
        int rc = f16_pass(e, q.audio, q.B, q.L, q.K, q.codes, q.s, &ovf2);
        if (rc) return rc;
        if (!ovf2) return MIMI_OK;
        return overflow_fallback(e, q.audio, q.B, q.L, q.K, q.codes, q.s);
    }
    if (!ovf) return MIMI_OK;
    HIP_TRY(hipSetDevice(e->device));
    if (q.ragged) {  // each item alone at its own length (the ragged result's definition), bf16x6 if it overflows
        ++e->f16_reruns;
        return ragged_item_by_item(e, q.audio, q.B, q.L, q.lens.data(), q.K, q.codes, q.s, PREC_F16X3);
    }
    return overflow_fallback(e, q.audio, q.B, q.L, q.K, q.codes, q.s);
}

static int check_encode_args(mimi_engine* e, const float* audio, int32_t batch, int64_t length, int32_t* K,
                             int32_t* codes) {
    if (!e) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine");
    if (!e->finalized) return set_err(MIMI_ERR_STATE, "mimi_finalize has not been called");
    if (*K <= 0) *K = e->cfg.num_quantizers;
    if (*K > e->cfg.num_quantizers)
        return set_err(MIMI_ERR_INVALID_ARGUMENT,
                       "The number of quantizers (i.e codebooks) asked should be lower than the total number of "
                       "quantizers %d, but is currently %d.",
                       e->cfg.num_quantizers, *K);
    if (*K < e->cfg.num_semantic_quantizers)
        return set_err(MIMI_ERR_INVALID_ARGUMENT, "num_quantizers %d below the semantic quantizers %d", *K,
                       e->cfg.num_semantic_quantizers);
    if (*K > e->levels_available)
        return set_err(MIMI_ERR_WEIGHTS, "num_quantizers %d but the checkpoint has %d codebooks", *K, e->levels_available);
    if (batch <= 0 || length <= 0 || !audio || !codes)
        return set_err(MIMI_ERR_INVALID_ARGUMENT, "batch=%d length=%lld", batch, (long long)length);
    if (length > (int64_t)1 << 31) return set_err(MIMI_ERR_INVALID_ARGUMENT, "length %lld too large", (long long)length);
    return MIMI_OK;
}

extern "C" int mimi_encode_async(mimi_engine* e, const float* audio, int32_t batch, int64_t length, int32_t K,
                                 int32_t* codes, void* stream, int64_t* ticket) {
    int rc = check_encode_args(e, audio, batch, length, &K, codes);
    if (rc) return rc;
    if (!ticket) return set_err(MIMI_ERR_INVALID_ARGUMENT, "ticket is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    (void)hipGetLastError();  // a failure left by an unrelated earlier call must not fail this encode's launches
    return encode_async_locked(e, audio, batch, length, K, codes, reinterpret_cast<hipStream_t>(stream), ticket);
}

static int check_ragged(mimi_engine* e, const int64_t* lengths, int32_t batch, int64_t max_length) {
    if (!lengths) return set_err(MIMI_ERR_INVALID_ARGUMENT, "lengths is NULL");
    for (int b = 0; b < batch; ++b)
        if (lengths[b] < 1 || lengths[b] > max_length)
            return set_err(MIMI_ERR_INVALID_ARGUMENT, "lengths[%d] = %lld outside [1, %lld]", b, (long long)lengths[b],
                           (long long)max_length);
    (void)e;
    return MIMI_OK;
}

extern "C" int mimi_encode_ragged_async(mimi_engine* e, const float* audio, const int64_t* lengths, int32_t batch,
                                        int64_t max_length, int32_t K, int32_t* codes, void* stream, int64_t* ticket) {
    int rc = check_encode_args(e, audio, batch, max_length, &K, codes);
    if (rc || (rc = check_ragged(e, lengths, batch, max_length))) return rc;
    if (!ticket) return set_err(MIMI_ERR_INVALID_ARGUMENT, "ticket is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    (void)hipGetLastError();
    return encode_async_locked(e, audio, batch, max_length, K, codes, reinterpret_cast<hipStream_t>(stream), ticket,
                               lengths);
}

extern "C" int mimi_encode_ragged(mimi_engine* e, const float* audio, const int64_t* lengths, int32_t batch,
                                  int64_t max_length, int32_t K, int32_t* codes, void* stream) {
    int64_t ticket = 0;
    const int rc = mimi_encode_ragged_async(e, audio, lengths, batch, max_length, K, codes, stream, &ticket);
    if (rc) return rc;
    return encode_wait(e, ticket);
}

extern "C" int mimi_encode_wait(mimi_engine* e, int64_t ticket) {
    if (!e) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine");
    return encode_wait(e, ticket);
}

extern "C" int mimi_encode(mimi_engine* e, const float* audio, int32_t batch, int64_t length, int32_t K,
                           int32_t* codes, void* stream) {
    int rc = check_encode_args(e, audio, batch, length, &K, codes);
    if (rc) return rc;
    int64_t ticket = 0;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        HIP_TRY(hipSetDevice(e->device));
        (void)hipGetLastError();  // a failure left by an unrelated earlier call must not fail this encode's launches
        // NULL stream = the HIP null stream, as in every HIP API
        if ((rc = encode_async_locked(e, audio, batch, length, K, codes, reinterpret_cast<hipStream_t>(stream),
                                      &ticket)))
            return rc;
    }
    return encode_wait(e, ticket);
}

// Host audio in, host codes out (the per-utterance callers' path: MimiEncoder.encode_audio_chunk once per utterance,
// `librispeech-mimi/process_librispeech_dev-test.py:136-141`, `mls-en-mimi-pretrain/process_shard.py:302-307`).  The
// same encode as mimi_encode on a device copy of the audio, with no framework tensors around it: the H2D copy, the
// encode and the codes' D2H into pinned memory are enqueued on `stream` in one call and the host synchronises once
// (twice when the encode had to be re-run: a chain give-up or an f16x3 overflow re-encodes on the stream inside
// mimi_encode_wait, after which the codes are copied again).
static int host_io_grow(mimi_engine::HostIo* io, size_t ab, size_t cb) {
    if (!io->done) HIP_TRY(hipEventCreateWithFlags(&io->done, hipEventDisableTiming));
    if (io->audio_cap < ab) {
        if (io->d_audio) HIP_TRY(hipFree(io->d_audio));  // (hipFree waits for the device)
        if (io->h_audio) HIP_TRY(hipHostFree(io->h_audio));
        io->d_audio = nullptr;
        io->h_audio = nullptr;
        io->audio_cap = 0;
        const size_t cap = std::max(ab, (size_t)1 << 22);
        HIP_TRY(hipMalloc(&io->d_audio, cap));
        HIP_TRY(hipHostMalloc(&io->h_audio, cap, hipHostMallocDefault));
        io->audio_cap = cap;
    }
    if (io->codes_cap < cb) {
        if (io->d_codes) HIP_TRY(hipFree(io->d_codes));
        if (io->h_codes) HIP_TRY(hipHostFree(io->h_codes));
        io->d_codes = nullptr;
        io->h_codes = nullptr;
        io->codes_cap = 0;
        const size_t cap = std::max(cb, (size_t)1 << 16);
        HIP_TRY(hipMalloc(&io->d_codes, cap));
        HIP_TRY(hipHostMalloc(&io->h_codes, cap, hipHostMallocDefault));
        io->codes_cap = cap;
    }
    return MIMI_OK;
}

extern "C" int mimi_encode_host(mimi_engine* e, const float* host_audio, int32_t batch, int64_t length, int32_t K,
                                int32_t* host_codes, void* stream) {
    int rc = check_encode_args(e, host_audio, batch, length, &K, host_codes);
    if (rc) return rc;
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const size_t ab = (size_t)batch * (size_t)length * sizeof(float);
    const size_t cb = (size_t)batch * K * (size_t)mimi_encoded_length_cfg(&e->cfg, length) * sizeof(int32_t);
    mimi_engine::HostIo* io = nullptr;
    int64_t ticket = 0, reruns = 0;
    {  // claim a staging slot and size it under the engine lock (a re-allocation's hipFree must not land inside
       // another thread's graph capture on this engine) ...
        std::lock_guard<std::mutex> lk(e->mu);
        HIP_TRY(hipSetDevice(e->device));
        for (auto& h : e->hostio)
            if (!h.busy) {
                io = &h;
                break;
            }
        if (!io)
            return set_err(MIMI_ERR_STATE, "%d host encodes in flight", mimi_engine::kMaxPending);
        if ((rc = host_io_grow(io, ab, cb))) return rc;
        io->busy = true;  // (from here on every exit path releases it)
    }
    // ... then copy the caller's samples into its pinned buffer without the lock: other threads' encodes on this
    // engine are not held up behind a host memcpy of up to several MB (the slot's previous H2D finished before its
    // last call returned)
    if (const hipError_t de = hipSetDevice(e->device); de != hipSuccess) {
        std::lock_guard<std::mutex> lk(e->mu);
        io->busy = false;
        return set_err(MIMI_ERR_HIP, "mimi_encode_host: hipSetDevice: %s", hipGetErrorString(de));
    }
    std::memcpy(io->h_audio, host_audio, ab);
    {
        std::lock_guard<std::mutex> lk(e->mu);
        (void)hipGetLastError();
        const hipError_t ce = hipMemcpyAsync(io->d_audio, io->h_audio, ab, hipMemcpyHostToDevice, s);
        if (ce != hipSuccess) rc = set_err(MIMI_ERR_HIP, "mimi_encode_host: H2D copy: %s", hipGetErrorString(ce));
        if (!rc) rc = encode_async_locked(e, io->d_audio, batch, length, K, io->d_codes, s, &ticket);
        if (rc) {
            (void)hipStreamSynchronize(s);  // (the slot is released: nothing of this call is left in flight)
            io->busy = false;
            return rc;
        }
        reruns = e->chain_reruns + e->f16_reruns;
        hipError_t de = hipMemcpyAsync(io->h_codes, io->d_codes, cb, hipMemcpyDeviceToHost, s);
        if (de == hipSuccess) de = hipEventRecord(io->done, s);
        if (de != hipSuccess) rc = set_err(MIMI_ERR_HIP, "mimi_encode_host: D2H copy: %s", hipGetErrorString(de));
    }
    const int wrc = encode_wait(e, ticket);  // (always: it frees the ticket)
    if (!rc) rc = wrc;
    if (!rc) {
        bool again;
        {
            std::lock_guard<std::mutex> lk(e->mu);
            again = e->chain_reruns + e->f16_reruns != reruns;  // (another thread's re-run only costs a copy)
        }
        hipError_t he = hipSuccess;
        if (again) he = hipMemcpyAsync(io->h_codes, io->d_codes, cb, hipMemcpyDeviceToHost, s);
        if (again && he == hipSuccess) he = hipEventRecord(io->done, s);
        if (he == hipSuccess) he = hipEventSynchronize(io->done);
        if (he != hipSuccess)
            rc = set_err(he == hipErrorOutOfMemory ? MIMI_ERR_OUT_OF_MEMORY : MIMI_ERR_HIP, "mimi_encode_host: %s",
                         hipGetErrorString(he));
        else
            std::memcpy(host_codes, io->h_codes, cb);
    } else {
        (void)hipStreamSynchronize(s);  // the buffers are reused: nothing of this call may still be in flight
    }
    std::lock_guard<std::mutex> lk(e->mu);
    io->busy = false;
    return rc;
}

extern "C" int mimi_rvq_encode(mimi_engine* e, const float* emb, int64_t frames, int32_t K, int32_t* codes,
                               void* stream) {
    if (!e) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine");
    if (!e->finalized) return set_err(MIMI_ERR_STATE, "mimi_finalize has not been called");
    if (K <= 0) K = e->cfg.num_quantizers;
    if (K > e->levels_available || K < e->cfg.num_semantic_quantizers)
        return set_err(MIMI_ERR_INVALID_ARGUMENT, "num_quantizers %d out of range", K);
    if (frames <= 0 || !emb || !codes) return set_err(MIMI_ERR_INVALID_ARGUMENT, "frames=%lld", (long long)frames);
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);  // NULL = the HIP null stream, as in every HIP API
    const int Hd = e->cfg.hidden_size, Dq = e->cfg.vq_hidden_dim;
    const size_t projb = ((size_t)frames * 2 * Dq * sizeof(float) + 255) / 256 * 256;
    const size_t need = projb + rvq_work_bytes(frames);
    int rc = ensure_ws(e, std::max(need, e->ws_bytes), s);
    if (rc) return rc;
    float* proj = reinterpret_cast<float*>(e->ws);
    HIP_TRY(hipStreamWaitEvent(s, e->ws_free, 0));
    Recorder rec{e, s};
    rec.begin();
    GemmArgs ap = linear_args(emb, frames, Hd, e->inproj, 2 * Dq, proj);
    const char* kname = "?";
    LAUNCH_TRY(launch_gemm(ROLE_INPROJ, ap, s, &kname), "input_proj");
    rec.mark("input_proj", 2.0 * frames * Hd * 2 * Dq, 0, kname);
    e->chain_ok = true;  // (checked right here: a give-up re-runs the levels on the per-level kernels)
    rc = run_rvq(e, proj, frames, K, codes, 0, reinterpret_cast<char*>(e->ws) + projb, s, rec);
    e->chain_ok = false;
    if (rc) return rc;
    if (e->chain_flag) {
        unsigned flag = 0;
        HIP_TRY(hipMemcpyAsync(&flag, e->chain_flag, sizeof flag, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        e->chain_flag = nullptr;
        if (flag) {
            ++e->chain_reruns;
            if ((rc = run_rvq(e, proj, frames, K, codes, 0, reinterpret_cast<char*>(e->ws) + projb, s, rec))) return rc;
        }
    }
    HIP_TRY(hipEventRecord(e->ws_free, s));
    return MIMI_OK;
}

extern "C" void mimi_destroy(mimi_engine* e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    // this engine's work only (every encode ends with ws_free on its stream; a device-wide sync would wait for
    // other engines and is refused while one of them captures a graph)
    if (e->ws_free) (void)hipEventSynchronize(e->ws_free);
    for (auto& q : e->pend)
        if (q.id && q.done) (void)hipEventSynchronize(q.done);
    for (void* p : e->allocations) (void)hipFree(p);
    if (e->ws) (void)hipFree(e->ws);
    if (e->rope_cos) (void)hipFree(e->rope_cos);
    if (e->rope_sin) (void)hipFree(e->rope_sin);
    for (auto& kv : e->tapmap)
        if (kv.second.d) (void)hipFree(kv.second.d);
    for (auto& pe : e->pending) (void)hipEventDestroy(pe.ev);
    for (auto ev : e->event_pool) (void)hipEventDestroy(ev);
    if (e->ws_free) (void)hipEventDestroy(e->ws_free);
    if (e->amax_dev) (void)hipFree(e->amax_dev);
    if (e->amax_host) (void)hipHostFree(e->amax_host);
    if (e->item_codes) (void)hipFree(e->item_codes);
    for (auto& q : e->pend) {
        if (q.done) (void)hipEventDestroy(q.done);
        if (q.amax) (void)hipHostFree(q.amax);
        if (q.rg_pinned) (void)hipHostFree(q.rg_pinned);
        if (q.chain_word) (void)hipHostFree(q.chain_word);
    }
    for (auto& h : e->hostio) {
        if (h.done) (void)hipEventDestroy(h.done);
        if (h.h_audio) (void)hipHostFree(h.h_audio);
        if (h.d_audio) (void)hipFree(h.d_audio);
        if (h.d_codes) (void)hipFree(h.d_codes);
        if (h.h_codes) (void)hipHostFree(h.h_codes);
    }
    drop_graphs(e);
    if (e->io_dev) (void)hipFree(e->io_dev);
    if (e->cap_stream) (void)hipStreamDestroy(e->cap_stream);
    delete e;
}

// ------------------------------------------------------------------------------------------------
// instrumentation
// ------------------------------------------------------------------------------------------------
extern "C" int mimi_set_precision(mimi_engine* e, int32_t mode) {
    if (!e) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine");
    if (mode < MIMI_PRECISION_F32 || mode > MIMI_PRECISION_F16X3)
        return set_err(MIMI_ERR_INVALID_ARGUMENT, "precision mode %d", mode);
    std::lock_guard<std::mutex> lk(e->mu);
    e->precision = mode;
    return MIMI_OK;
}

extern "C" int mimi_set_graphs(mimi_engine* e, int32_t enable) {
    if (!e) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    e->graphs_enabled = enable != 0;
    if (!enable) {
        drop_graphs(e);
        e->graph_seen.clear();
    }
    return MIMI_OK;
}

extern "C" int64_t mimi_graph_replays(const mimi_engine* e) { return e ? e->graph_replays : -1; }

// mimi_set_option keys: engine field, allowed values (bit v of `allowed` set: value v accepted), what they select.
// Every key changes the kernel sequence (never the bits an encode produces), so a change drops captured graphs.
struct EngineOption {
    const char* key;
    int mimi_engine::*field;
    unsigned allowed;
    const char* values;
};
static const EngineOption kEngineOptions[] = {
    {"stage0_fused", &mimi_engine::stage0_fused, 0x3u, "0 or 1"},
    {"rvq_form", &mimi_engine::rvq_form, 0x7fu, "0..6"},
    {"ln_rpw", &mimi_engine::ln_rpw, 0x117u, "0, 1, 2, 4 or 8"},
    {"rvq_xcd", &mimi_engine::rvq_xcd, 0x3u, "0 or 1"},
    {"rvq_chain", &mimi_engine::rvq_chain, 0x3u, "0 or 1"},
    {"rvq_chain_fault", &mimi_engine::rvq_chain_fault, 0x7u, "0, 1 or 2"},
    {"sc1_out", &mimi_engine::sc1_out, 0xffu, "0..7"},
    {"ln_fused", &mimi_engine::ln_fused, 0x1fu, "0 .. 4"},
    {"qkv_attn", &mimi_engine::qkv_attn, 0x7u, "0, 1 or 2"},
    {"qkv_attn_xcd", &mimi_engine::qkv_attn_xcd, 0x3u, "0 or 1"},
    {"attn_band_split", &mimi_engine::attn_band_split, 0x7u, "0, 1 or 2"},
    {"fc1_cg", &mimi_engine::fc1_cg, 0x17u, "0, 1, 2 or 4"},
    {"res1_form", &mimi_engine::res1_form, 0x3u, "0 or 1"},
    {"res1_stream", &mimi_engine::res1_stream, 0x7u, "0, 1 or 2"},
};

extern "C" int mimi_set_option(mimi_engine* e, const char* key, int64_t value) {
    if (!e || !key) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine or key");
    std::lock_guard<std::mutex> lk(e->mu);
    for (const EngineOption& o : kEngineOptions) {
        if (strcmp(key, o.key)) continue;
        if (value < 0 || value > 31 || !((o.allowed >> value) & 1u))
            return set_err(MIMI_ERR_INVALID_ARGUMENT, "%s %lld (%s)", key, (long long)value, o.values);
        HIP_TRY(hipSetDevice(e->device));
        if (e->*o.field != (int)value) {  // captured graphs hold the other kernel sequence
            drop_graphs(e);
            e->graph_seen.clear();
        }
        e->*o.field = (int)value;
        return MIMI_OK;
    }
    return set_err(MIMI_ERR_INVALID_ARGUMENT, "unknown option '%s'", key);
}

extern "C" int mimi_act_scales(mimi_engine* e, int32_t max_n, char* names, float* scales, float* last_max,
                               int32_t* n) {
    if (!e) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    int i = 0;
    for (const auto& kv : e->slot_of) {
        const int slot = kv.second;
        if (i >= max_n) break;
        if (names) {
            std::strncpy(names + 64 * i, kv.first.c_str(), 63);
            names[64 * i + 63] = 0;
        }
        if (scales) scales[i] = slot < (int)e->act_scale.size() ? e->act_scale[slot] : 0.0f;
        if (last_max) last_max[i] = slot < (int)e->last_amax.size() ? e->last_amax[slot] : -1.0f;
        ++i;
    }
    if (n) *n = i;
    return MIMI_OK;
}

extern "C" int mimi_get_precision(const mimi_engine* e) { return e ? e->precision : -1; }

extern "C" int mimi_calibrate(mimi_engine* e) {
    if (!e) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine");
    if (!e->finalized) return set_err(MIMI_ERR_STATE, "mimi_finalize has not been called");
    std::lock_guard<std::mutex> lk(e->mu);
    if (e->calibrated) return MIMI_OK;
    HIP_TRY(hipSetDevice(e->device));
    (void)hipGetLastError();
    return calibrate_scales(e);
}

extern "C" int64_t mimi_f16_reruns(const mimi_engine* e) { return e ? e->f16_reruns : -1; }

extern "C" int64_t mimi_rvq_chain_reruns(const mimi_engine* e) { return e ? e->chain_reruns : -1; }

extern "C" int mimi_set_profiling(mimi_engine* e, int enable) {
    if (!e) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine");
    if (enable < 0 || enable > 2) return set_err(MIMI_ERR_INVALID_ARGUMENT, "profiling level %d (0, 1 or 2)", enable);
    std::lock_guard<std::mutex> lk(e->mu);
    e->profiling = enable;
    return MIMI_OK;
}

static int resolve_pending(mimi_engine* e) {
    HIP_TRY(hipSetDevice(e->device));
    hipEvent_t prev = nullptr;
    std::vector<std::string> seq;
    for (auto& pe : e->pending) {
        HIP_TRY(hipEventSynchronize(pe.ev));
        if (pe.name.empty()) {
            prev = pe.ev;
            if (!seq.empty()) e->last_seq = std::move(seq);
            seq.clear();
            continue;
        }
        seq.push_back(pe.name);
        float ms = 0;
        if (prev) HIP_TRY(hipEventElapsedTime(&ms, prev, pe.ev));
        if (!e->prof.count(pe.name)) e->prof_order.push_back(pe.name);
        ProfStat& st = e->prof[pe.name];
        st.ms += ms;
        st.flops += pe.flops;
        st.bytes += pe.bytes;
        st.launches += 1;
        prev = pe.ev;
    }
    if (!seq.empty()) e->last_seq = std::move(seq);
    for (auto& pe : e->pending) e->event_pool.push_back(pe.ev);
    e->pending.clear();
    return MIMI_OK;
}

extern "C" int mimi_profile_sequence(mimi_engine* e, int32_t max_stages, char* names, int32_t* n_stages) {
    if (!e) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    int rc = resolve_pending(e);
    if (rc) return rc;
    int i = 0;
    for (const auto& n : e->last_seq) {
        if (i >= max_stages) break;
        if (names) {
            std::strncpy(names + 128 * i, n.c_str(), 127);
            names[128 * i + 127] = 0;
        }
        ++i;
    }
    if (n_stages) *n_stages = i;
    return MIMI_OK;
}

extern "C" int mimi_profile_read(mimi_engine* e, int32_t max_stages, char* names, double* total_ms, int64_t* launches,
                                 double* flops, int32_t* n_stages) {
    if (!e) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    int rc = resolve_pending(e);
    if (rc) return rc;
    int i = 0;
    for (const auto& n : e->prof_order) {
        if (i >= max_stages) break;
        const ProfStat& st = e->prof[n];
        if (names) {
            std::strncpy(names + 128 * i, n.c_str(), 127);
            names[128 * i + 127] = 0;
        }
        if (total_ms) total_ms[i] = st.ms;
        if (launches) launches[i] = st.launches;
        if (flops) flops[2 * i] = st.flops, flops[2 * i + 1] = st.bytes;
        ++i;
    }
    if (n_stages) *n_stages = i;
    return MIMI_OK;
}

extern "C" int mimi_profile_reset(mimi_engine* e) {
    if (!e) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    int rc = resolve_pending(e);
    e->prof.clear();
    e->prof_order.clear();
    return rc;
}

extern "C" int mimi_set_taps(mimi_engine* e, int enable) {
    if (!e) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    e->taps = enable != 0;
    return MIMI_OK;
}

extern "C" int mimi_get_tap(mimi_engine* e, const char* name, float* dst, int64_t cap, int64_t* numel, int64_t dims[3]) {
    if (!e || !name) return set_err(MIMI_ERR_INVALID_ARGUMENT, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    auto it = e->tapmap.find(name);
    if (it == e->tapmap.end()) return set_err(MIMI_ERR_INVALID_ARGUMENT, "no tap named %s", name);
    const auto& tp = it->second;
    const int64_t n = tp.dims[0] * tp.dims[1] * tp.dims[2];
    if (numel) *numel = n;
    if (dims) std::memcpy(dims, tp.dims, sizeof(tp.dims));
    if (dst) {
        if (cap < n) return set_err(MIMI_ERR_INVALID_ARGUMENT, "tap %s needs %lld floats", name, (long long)n);
        HIP_TRY(hipSetDevice(e->device));
        // the taps were copied inside the last encode: wait for it alone (a device-wide sync is refused while any
        // other engine in the process captures a graph)
        HIP_TRY(hipEventSynchronize(e->ws_free));
        if (!e->cap_stream) HIP_TRY(hipStreamCreateWithFlags(&e->cap_stream, hipStreamNonBlocking));
        HIP_TRY(hipMemcpyWithStream(dst, tp.d, n * 4, hipMemcpyDeviceToHost, e->cap_stream));
    }
    return MIMI_OK;
}
