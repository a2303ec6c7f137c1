/*
 * mimi_hip.h — C ABI of the MI355X-native Mimi encode engine (libmimi_hip.so).
 *
 * Drop-in boundary.  The reference's encode path is Python over third-party
 * ``transformers.MimiModel`` (no native FFI of its own); the entry points below are what a binding of that
 * path binds, one for one:
 *
 *   mimi_create_from_dir (one call), or mimi_config_from_json + mimi_create / mimi_load_safetensors /
 *   mimi_set_weight / mimi_finalize
 *       replace ``MimiModel.from_pretrained(model_id).to(device).eval()``
 *       (/root/reference/emilia-mimi/process_shard.py:57-60; TF/modeling_mimi.py:1186-1228)
 *   mimi_encode
 *       replaces ``MimiModel.encode(input_values, padding_mask, num_quantizers)``
 *       (/root/reference/emilia-mimi/process_shard.py:82-85, :124-127; TF/modeling_mimi.py:1297-1386)
 *   mimi_rvq_encode
 *       replaces ``MimiSplitResidualVectorQuantizer.encode`` (TF/modeling_mimi.py:1099-1126) on a given
 *       pre-quantizer embedding (used by the bit-exact quantizer parity test)
 *   mimi_encoded_length
 *       replaces ``MimiModel.get_encoded_length`` (TF/modeling_mimi.py:1265-1278)
 *
 * Conventions: plain pointers and sizes, no exceptions, no torch types.  Every function returns a
 * mimi_status; on failure ``mimi_last_error()`` (thread-local) describes it.  Device pointers are HIP
 * device memory on the engine's device; ``stream`` is a hipStream_t (NULL = the HIP null stream);
 * work is enqueued asynchronously on it, ordered after earlier work on that stream.
 * One engine may be shared by several host threads (calls are serialised by a per-engine mutex).
 */
#ifndef MIMI_HIP_H
#define MIMI_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mimi_engine mimi_engine;

typedef enum mimi_status {
    MIMI_OK = 0,
    MIMI_ERR_INVALID_ARGUMENT = 1, /* ValueError in the reference (e.g. K > 32, channels not in {1,2}) */
    MIMI_ERR_HIP = 2,              /* a HIP runtime call failed */
    MIMI_ERR_OUT_OF_MEMORY = 3,    /* workspace allocation failed (reference: torch OOM) */
    MIMI_ERR_WEIGHTS = 4,          /* missing / mis-shaped parameter */
    MIMI_ERR_UNSUPPORTED = 5,      /* config outside the implemented architecture family */
    MIMI_ERR_IO = 6,               /* checkpoint file unreadable / malformed */
    MIMI_ERR_STATE = 7             /* call order violated (e.g. encode before finalize) */
} mimi_status;

/* Encode-path fields of MimiConfig (TF/configuration_mimi.py:86-123). */
typedef struct mimi_config {
    int32_t sampling_rate;          /* 24000 */
    int32_t audio_channels;         /* 1 */
    int32_t hidden_size;            /* 512 */
    int32_t num_filters;            /* 64 */
    int32_t num_ratios;             /* 4 */
    int32_t upsampling_ratios[8];   /* {8, 6, 5, 4}; the encoder uses them reversed */
    int32_t kernel_size;            /* 7 */
    int32_t last_kernel_size;       /* 3 */
    int32_t residual_kernel_size;   /* 3 */
    int32_t compress;               /* 2 */
    int32_t codebook_size;          /* 2048 */
    int32_t codebook_dim;           /* 256 */
    int32_t num_quantizers;         /* 32 */
    int32_t num_semantic_quantizers;/* 1 */
    int32_t vq_hidden_dim;          /* 256 */
    int32_t num_hidden_layers;      /* 8 */
    int32_t intermediate_size;      /* 2048 */
    int32_t num_attention_heads;    /* 8 */
    int32_t head_dim;               /* 64 */
    int32_t sliding_window;         /* 250 */
    int32_t downsample_kernel;      /* 4 = 2 * encodec_frame_rate / frame_rate */
    int32_t downsample_stride;      /* 2 */
    float norm_eps;                 /* 1e-5 */
    float rope_theta;               /* 10000 */
    float codebook_eps;             /* 1e-5 (MimiEuclideanCodebook epsilon) */
} mimi_config;

/* Fill *cfg with the kyutai/mimi defaults. */
void mimi_config_default(mimi_config* cfg);

/*
 * Read a checkpoint's HF config.json (path = the file, or a directory holding it) into *cfg: the encode-path
 * fields of MimiConfig (TF/configuration_mimi.py:86-175; unknown keys ignored, absent keys keep the defaults,
 * rope_theta at the top level or in rope_parameters, head_dim null -> hidden_size / num_attention_heads, the
 * downsample kernel from frame_rate).  MIMI_ERR_IO: unreadable file, malformed JSON or a field of the wrong type;
 * MIMI_ERR_UNSUPPORTED: an architecture outside the kyutai/mimi family (stereo, non-causal convs, GQA, ...).
 * Host-only: no device is touched.
 */
int mimi_config_from_json(const char* path, mimi_config* cfg);

/*
 * The one-call constructor: weights_dir is a checkpoint directory in the HF layout (config.json, optional, and
 * *.safetensors -- the first in byte order, as the Python host's sorted glob picks it) or a lone .safetensors file
 * (default config).  Reads the config, creates the engine on `device`, loads the safetensors file and finalizes:
 * = mimi_config_from_json + mimi_create + mimi_load_safetensors + mimi_finalize, with the engine released again on
 * any failure (*out stays NULL; mimi_last_error names the first failure).
 */
int mimi_create_from_dir(const char* weights_dir, int device, mimi_engine** out);

/* Create an engine on HIP device `device` (cfg NULL = defaults).  Weights are supplied next. */
int mimi_create(const mimi_config* cfg, int device, mimi_engine** out);

/* Supply one parameter by its HF name, fp32, host memory, copied. */
int mimi_set_weight(mimi_engine* e, const char* name, const float* host_data, int64_t numel);

/* Read every encode-path parameter from a safetensors file (F32 tensors, HF names). */
int mimi_load_safetensors(mimi_engine* e, const char* path);

/* Check all parameters are present, re-lay them out for the kernels and upload them. */
int mimi_finalize(mimi_engine* e);

/*
 * Encode `batch` mono waveforms of `length` samples (device f32, [batch][length], already padded to a
 * common length by the caller as EncodecFeatureExtractor does) into `num_quantizers` codebooks.
 * dev_codes: device int32 [batch][num_quantizers][mimi_encoded_length(length)].
 * num_quantizers <= 0 means config.num_quantizers (the reference default, TF/modeling_mimi.py:1335).
 */
int mimi_encode(mimi_engine* e, const float* dev_audio, int32_t batch, int64_t length,
                int32_t num_quantizers, int32_t* dev_codes, void* stream);

/*
 * mimi_encode in two halves, for callers that overlap host work (ingest, H2D of the next batch, writing
 * codes) with the encode: mimi_encode_async enqueues the encode on `stream` and returns a ticket without
 * waiting; mimi_encode_wait(ticket) waits for it on the host and, in f16x3, applies the overflow check (and the
 * per-item fallback when a fixed activation scale overflowed) before returning.  dev_codes is valid once the
 * wait returns; dev_audio and dev_codes must stay allocated, and dev_audio unmodified, until then (the wait may
 * re-encode from dev_audio: a fixed f16x3 scale overflowed, or the persistent RVQ chain gave up).  At most 16 encodes per engine may be
 * in flight; each ticket is waited exactly once.  mimi_encode = mimi_encode_async + mimi_encode_wait.
 */
int mimi_encode_async(mimi_engine* e, const float* dev_audio, int32_t batch, int64_t length, int32_t num_quantizers,
                      int32_t* dev_codes, void* stream, int64_t* ticket);
int mimi_encode_wait(mimi_engine* e, int64_t ticket);

/*
 * mimi_encode from and to HOST memory in one call: host_audio f32 [batch][length] (any host memory), host_codes
 * int32 [batch][num_quantizers][mimi_encoded_length(length)].  The engine copies the audio to its own device buffer,
 * encodes and copies the codes back on `stream`, synchronising the host once -- the per-utterance caller's path
 * (MimiEncoder.encode_audio_chunk once per utterance: librispeech-mimi/process_librispeech_dev-test.py:136-141,
 * mls-en-mimi-pretrain/process_shard.py:302-307) without a framework tensor per step.  Same codes as mimi_encode.
 */
int mimi_encode_host(mimi_engine* e, const float* host_audio, int32_t batch, int64_t length, int32_t num_quantizers,
                     int32_t* host_codes, void* stream);

/*
 * Ragged batch: item b's samples are dev_audio[b][0 .. lengths[b]) (rows max_length apart; samples past lengths[b]
 * are never read), lengths a HOST int64 array, 1 <= lengths[b] <= max_length.  Each item is encoded exactly as
 * mimi_encode(dev_audio[b], 1, lengths[b], ...) would encode it alone -- its codes, frames [0,
 * mimi_encoded_length(lengths[b])) of dev_codes[b], are bit for bit those -- while the batch runs as one pass
 * whose kernels skip every item's rows past its own length.  Frames past an item's own are unspecified.
 * dev_codes: device int32 [batch][num_quantizers][mimi_encoded_length(max_length)].
 *   - per-utterance callers (batch-1 semantics: mls-en-mimi-pretrain/process_shard.py:302-307,
 *     librispeech-mimi/process_librispeech_dev-test.py:136-141) pass each utterance's length;
 *   - pad-to-longest callers (EncodecFeatureExtractor padding, emilia-mimi/process_shard.py:113-139) pass
 *     min(max_length, 1920 ceil(L_b / 1920)) over the zero-padded batch: every frame the caller keeps,
 *     ceil(L_b / 1920), depends only on samples below that length (all convs causal, no extra padding at a
 *     multiple of 1920), so the kept frames are the padded batch's -- without the padding's compute.
 * In f16x3 the overflow check applies per batch; a fallback re-encodes each item alone at its length.
 */
int mimi_encode_ragged(mimi_engine* e, const float* dev_audio, const int64_t* lengths, int32_t batch,
                       int64_t max_length, int32_t num_quantizers, int32_t* dev_codes, void* stream);
int mimi_encode_ragged_async(mimi_engine* e, const float* dev_audio, const int64_t* lengths, int32_t batch,
                             int64_t max_length, int32_t num_quantizers, int32_t* dev_codes, void* stream,
                             int64_t* ticket);

/*
 * The quantizer alone: dev_embedding is the pre-quantizer embedding, device f32 [frames][hidden_size]
 * (frame-major, i.e. the reference's [B, 512, T] transposed to [B*T, 512]).  dev_codes: int32
 * [num_quantizers][frames].
 */
int mimi_rvq_encode(mimi_engine* e, const float* dev_embedding, int64_t frames, int32_t num_quantizers,
                    int32_t* dev_codes, void* stream);

/*
 * Arithmetic of the conv / linear GEMMs (the residual VQ distances are always exact fp32):
 *   MIMI_PRECISION_F32     v_mfma_f32_32x32x2_f32 (fp32 MFMA)
 *   MIMI_PRECISION_BF16X6  fp32 emulated on the bf16 matrix cores: both operands split into 3 bf16 planes,
 *                          6 plane products accumulated in fp32 (~fp32 accuracy, 2.7x MFMA rate)
 *   MIMI_PRECISION_BF16X3  2 planes, 3 products (~1e-5 relative, 5.3x MFMA rate)
 *   MIMI_PRECISION_F16X3   (default) fp32 emulated on the fp16 matrix cores: both operands split into 2 fp16
 *                          planes (22-bit significand) at power-of-two scales, 3 products.  Activation scales
 *                          are fixed per tensor by a calibration encode on built-in signals, run once before
 *                          the engine's first f16x3 encode or by mimi_calibrate (never from the caller's audio:
 *                          an item's codes depend on its own samples and the padded length only).  mimi_encode reads the activations' maxima back after the encode (it
 *                          synchronises its stream in this mode); on an overflow of a fixed scale each item is
 *                          re-encoded alone, and in bf16x6 if it overflows alone.
 */
enum { MIMI_PRECISION_F32 = 0, MIMI_PRECISION_BF16X6 = 1, MIMI_PRECISION_BF16X3 = 2, MIMI_PRECISION_F16X3 = 3 };
/* default: MIMI_PRECISION_F16X3 */
int mimi_set_precision(mimi_engine* e, int32_t mode);
int mimi_get_precision(const mimi_engine* e);
/* MIMI_PRECISION_F16X3: run the activation-scale calibration now (idempotent; otherwise it runs inside the first
 * f16x3 encode).  Synchronises the device. */
int mimi_calibrate(mimi_engine* e);
/* MIMI_PRECISION_F16X3: encodes that took the overflow fallback so far (diagnostic). */
int64_t mimi_f16_reruns(const mimi_engine* e);
/* Encodes (and mimi_rvq_encode calls) re-run on the per-level RVQ kernels because a sweep of the persistent RVQ
 * chain gave up waiting for a peer workgroup (its codes are never returned; diagnostic). */
int64_t mimi_rvq_chain_reruns(const mimi_engine* e);
/* hipGraph replay of MIMI_PRECISION_F16X3 encodes (default on): the second encode of a (batch, length, K) shape
 * captures the whole pass into a graph, later ones replay it (same kernels and arguments: identical codes).
 * Never used while profiling or taps are on.  enable = 0 drops the captured graphs.  Replays so far: */
int mimi_set_graphs(mimi_engine* e, int32_t enable);
int64_t mimi_graph_replays(const mimi_engine* e);
/* Kernel-variant options (tuning / A-B checks; every setting gives identical codes).  key "stage0_fused":
 * 0 = stage-0 residual block and down conv 0 as two kernels (y through HBM), 1 = one fused kernel (y stays on
 * chip; default).  key "ln_fused": on small grids (batch 1-4) 0 = LayerNorm launches before q/k/v and fc1, 1 = fc1
 * computes the LayerNorm of its own rows (default), 2-4 = fc1 and q/k/v do (q/k/v tile variants).  key "qkv_attn":
 * q/k/v projection + RoPE + attention as one kernel for items of <= 256 frames, 0 = off, 1 = when the batch has
 * >= 256 (item, head) pairs (default), 2 = whenever the items fit; "qkv_attn_xcd" 0/1 its workgroup placement.
 * RVQ: "rvq_form" 0-6 (level-kernel form, 0 = default), "rvq_chain" 0/1 (one persistent launch for all levels on
 * small grids, default 1; taken only where its give-up flag is read back: mimi_encode_wait re-runs an encode whose
 * chain gave up), "rvq_chain_fault" 0/1/2 (tests only: 1 = zero spin budget, 2 = every sweep gives up), "rvq_xcd"
 * 0/1.  "sc1_out" 0-7 (sc1 output stores: bit 0 q/k/v, 1 fc1 (default 2), 2 o_proj + fc2), "ln_rpw" 0/1/2/4/8
 * (LayerNorm rows per wave), "fc1_cg" 0/1/2/4 (fc1's tile order in XCD column groups, default 1 = none), "res1_form"
 * 0/1 (stage-1 block as one 8-wave or two 4-wave workgroups per CU, default 1), "res1_stream" 0/1/2 (the k = 1
 * residual conv as the streaming kernel with register-resident weights: 1 stage 2 (default), 2 stages 2 and 3 (stage 3
 * uniform batches; measured slower there), 0 off), "attn_band_split" 0/1/2 (items
 * over 256 frames: the banded attention as 128-query workgroups, by grid size (default), or one 32-query tile per
 * workgroup).  Unknown keys and values:
 * MIMI_ERR_INVALID_ARGUMENT.  A change drops the captured graphs. */
int mimi_set_option(mimi_engine* e, const char* key, int64_t value);
/* MIMI_PRECISION_F16X3 diagnostics: per plane tensor (64-char names), its fixed activation scale and the max|x|
 * of the last waited encode (-1: not produced by it); an overflow is max * scale >= 2^15. */
int mimi_act_scales(mimi_engine* e, int32_t max_n, char* names, float* scales, float* last_max, int32_t* n);

/* Frames produced for `length` samples with the default config (reference float32 length math). */
int64_t mimi_encoded_length(int64_t length);
int64_t mimi_encoded_length_cfg(const mimi_config* cfg, int64_t length);

/*
 * Host-ingest resampler (replaces the resampling inside librosa.load(path, sr=24000):
 * librispeech-mimi/utils.py:84-87, emilia-mimi/process_shard.py:479-482, yodas2-mimi/process_shard.py:389),
 * bit-exact with librosa's res_type='polyphase' = scipy.signal.resample_poly on float32 input, and the engine of
 * the soxr_hq-spec mode (mimi_hip.ingest: a linear-phase Kaiser FIR designed to libsoxr's published HQ quality
 * spec, same polyphase arithmetic; parity with libsoxr itself unpinned).  nclips clips
 * packed in dev_in at dev_in_off[i] (dev_in_len[i] samples) -> dev_out at dev_out_off[i] (dev_out_len[i]
 * samples, max_out = their maximum), all int64 arrays on the device.  dev_filter: the up-scaled Kaiser(5.0)
 * low-pass with its zero pre-padding, or any other FIR (filter_len taps, <= MIMI_RESAMPLE_MAX_TAPS); pre_remove: leading
 * outputs of the full upfirdn skipped (resample_poly's n_pre_remove).  No engine handle needed.
 */
#define MIMI_RESAMPLE_MAX_TAPS 65536
int mimi_resample_poly(const float* dev_in, const int64_t* dev_in_off, const int64_t* dev_in_len, int32_t nclips,
                       float* dev_out, const int64_t* dev_out_off, const int64_t* dev_out_len, int64_t max_out,
                       const float* dev_filter, int32_t filter_len, int32_t up, int32_t down, int64_t pre_remove,
                       void* stream);

/*
 * FLAC decode for host ingest (replaces libFLAC behind librosa.load -> soundfile -> libsndfile on the LibriSpeech
 * path: librispeech-mimi/process_librispeech_dev-test.py:136, utils.py:84-87).  `data` holds a whole .flac file
 * (an ID3v2 tag in front is skipped).  mimi_flac_info reads STREAMINFO.  mimi_flac_decode decodes every frame
 * into `out`, planar int32 [channels][cap_per_channel] at the stream's bit depth (out = NULL: count only), and
 * sets *n_samples (per channel); CRC-8 / CRC-16 mismatches, malformed frames and a sample count that differs
 * from STREAMINFO's return MIMI_ERR_IO.  Host-only, re-entrant (no engine handle).
 */
int mimi_flac_info(const uint8_t* data, int64_t nbytes, int32_t* sample_rate, int32_t* channels,
                   int32_t* bits_per_sample, int64_t* total_samples);
int mimi_flac_decode(const uint8_t* data, int64_t nbytes, int32_t* out, int64_t cap_per_channel, int64_t* n_samples);

/*
 * Codec-BPE training over code strings (replaces the BpeTrainer run of codec-bpe/bpe_trainer.py:147-156; driven
 * by mimi_hip/bpe.py).  The corpus: words of symbol ids (0 .. n_initial_tokens-1 = special tokens, then the
 * alphabet), concatenated in `symbols`, word w = symbols[word_offsets[w] .. word_offsets[w+1]), occurring
 * word_counts[w] times; all host memory, copied.  max_token_length <= 0: unlimited; else a pair formed by a
 * merge is counted only when its merged length is below it.  Then, per step: mimi_bpe_best gives the pair of
 * highest count (ties: smallest (left, right); count 0 when none is left), the caller decides the new token's
 * id (a new one, or the id of an existing token with the same spelling) and length, and mimi_bpe_merge applies
 * it to every word.  Ids up to 131071.
 */
typedef struct mimi_bpe mimi_bpe;
int mimi_bpe_create(int device, const int32_t* symbols, int64_t n_symbols, const int64_t* word_offsets,
                    const int64_t* word_counts, int64_t n_words, int32_t n_initial_tokens, int32_t vocab_size,
                    int32_t max_token_length, mimi_bpe** out);
int mimi_bpe_best(mimi_bpe* h, int32_t* left, int32_t* right, int64_t* count);
int mimi_bpe_merge(mimi_bpe* h, int32_t left, int32_t right, int32_t new_id, int32_t new_len);
void mimi_bpe_destroy(mimi_bpe* h);

/*
 * Diagnostic: the fp16 plane split the kernels use (two v_fma_mix per value: hi = fp16(v s), lo = fp16(v s - hi))
 * against the conversion form it replaces, on npairs value pairs of dev_in (device f32 [2 npairs], s a power of two):
 * dev_out (device u32 [npairs][4]) = the kernels' (hi, lo) words and the conversion form's (hi, lo) words.  Tests
 * require them equal on edge values (zeros of both signs, fp32 / fp16 subnormals, rounding ties, fp16 overflow).
 */
int mimi_split_check(const float* dev_in, int64_t npairs, float scale, uint32_t* dev_out, void* stream);

/*
 * Diagnostic: fc1's f16x3 GELU epilogue (the branch-free erfc form, gemm_kernel.h gelu_fast) on n values:
 * dev_out[i] = GELU(dev_in[i]) (device f32 [n] each).  Replaces torch's GELU(approximate='none') at
 * TF/modeling_mimi.py:602-615 (MimiMLP fc1 -> activation); tests bound it against float64 and torch.
 */
int mimi_gelu_check(const float* dev_in, int64_t n, float* dev_out, void* stream);

/* Device bytes the workspace needs for (batch, length); the engine grows it on demand. */
int64_t mimi_workspace_bytes(const mimi_engine* e, int32_t batch, int64_t length);

/* Release everything. */
void mimi_destroy(mimi_engine* e);

/* Thread-local description of the last failure in this thread. */
const char* mimi_last_error(void);

/* ---- instrumentation (bench / tests) ---- */

/* enable = 1: every encode records HIP events between its stages on the stream it runs on (one per stage);
 * 2: only around its first stage (two events per encode: the light form a timed region can carry); 0: off. */
int mimi_set_profiling(mimi_engine* e, int enable);
/* Per-stage totals accumulated over all profiled encodes since the last reset: names (128 chars
 * each, "stage|kernel symbol"), device ms (event pairs on the launch stream), launch counts, and algorithmic work as
 * (flops, bytes) pairs in flops_bytes[2*i], flops_bytes[2*i+1].  Synchronises the recorded events. */
int mimi_profile_read(mimi_engine* e, int32_t max_stages, char* names /* max_stages*128 */,
                      double* total_ms, int64_t* launches, double* flops_bytes, int32_t* n_stages);
int mimi_profile_reset(mimi_engine* e);
/* The "stage|kernel symbol" names of the last profiled encode, in launch order (one entry per stage event; a
 * stage's first dispatch is its named kernel).  Lets a rocprofv3 counter pass key its dispatches by stage. */
int mimi_profile_sequence(mimi_engine* e, int32_t max_stages, char* names /* max_stages*128 */, int32_t* n_stages);

/* When enabled, mimi_encode keeps a copy of each stage's output (for per-stage parity tests). */
int mimi_set_taps(mimi_engine* e, int enable);
/* Copy tap `name` to host: dst holds cap floats; *numel receives the element count; dims[0..2] the
 * [batch][time][channels] shape.  Synchronises. */
int mimi_get_tap(mimi_engine* e, const char* name, float* host_dst, int64_t cap, int64_t* numel,
                 int64_t dims[3]);

#ifdef __cplusplus
}
#endif
#endif /* MIMI_HIP_H */
