// Codec-BPE training on the GPU (mimi_hip/bpe.py drives it).
//
// The reference trains with HF tokenizers' BpeTrainer (codec-bpe/bpe_trainer.py:147-156).  Its rules, restated
// in oracle/bpe_ref.py and pinned against tokenizers 0.22.2: pair counts weighted by word count; each step
// merges the pair of highest count (ties: smallest (left id, right id)); a word is rewritten left to right
// (a run "a a a" of a pair (a, a) merges its 1st+2nd, not its 2nd+3rd); a pair formed by a merge is counted only
// if its merged length is below max_token_length.
//
// Layout: every word's symbols in one array, doubly linked (nxt / prv, -1 at the word ends), dead symbols -1;
// wc[p] = the count of p's word.  Pair counts live in an open-addressing hash table (key = left << 32 | right,
// 64-bit counts, linear probing, keys never removed until a rehash).  One merge step:
//   mark    full scan: p starts an occurrence if sym[p] = a, sym[nxt[p]] = b and (a != b or an even number of
//           a's precede p in its run) -> a compact list of starts
//   deltas  per start p (partner q = nxt[p], L = prv[p], R = nxt[q]): the pairs the rewrite destroys
//           ((sym L, a), (b, sym R) unless R starts another occurrence, whose own left side covers it) and the
//           pairs it forms ((L' , new), (new, sym R)) with L' = new when L is the partner of the previous
//           occurrence -- the net of tokenizers' sequential change list
//   relink  sym[p] = new, p -> R, q dead
// and the best pair is the max count, then the smallest (left, right) among the pairs holding it (two sweeps).
// HBM-bound integer work: one 4-B read per symbol per step for the mark scan, one table sweep for the max.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/mimi_hip.h"
#include "kernels.h"

namespace {

constexpr unsigned long long kEmpty = ~0ull;
constexpr int kIdBits = 17;
constexpr unsigned kMaxId = (1u << kIdBits) - 1;

__device__ __forceinline__ unsigned long long pair_key(int a, int b) {
    return ((unsigned long long)(unsigned)a << 32) | (unsigned)b;
}

__device__ __forceinline__ unsigned long long mix(unsigned long long k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

struct Table {
    unsigned long long* keys;
    unsigned long long* vals;  // int64 counts, two's complement
    unsigned long long mask;
    unsigned long long* nkeys;
};

// add delta to key's count; insert the key first when `insert` (a pair being formed), else skip an absent key
// (a pair that was never counted: formed past max_token_length)
__device__ void table_add(const Table& t, unsigned long long key, long long delta, bool insert) {
    unsigned long long h = mix(key) & t.mask;
    for (unsigned long long probe = 0; probe <= t.mask; ++probe) {
        const unsigned long long k = __hip_atomic_load(&t.keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == key) {
            atomicAdd(&t.vals[h], (unsigned long long)delta);
            return;
        }
        if (k == kEmpty) {
            if (!insert) return;
            const unsigned long long prev = atomicCAS(&t.keys[h], kEmpty, key);
            if (prev == kEmpty || prev == key) {
                atomicAdd(&t.vals[h], (unsigned long long)delta);
                if (prev == kEmpty) atomicAdd(t.nkeys, 1ull);
                return;
            }
        }
        h = (h + 1) & t.mask;
    }
}

__global__ void count_pairs_kernel(const int* __restrict__ sym, const int* __restrict__ nxt, const int* __restrict__ wc,
                                   long long n, Table t) {
    for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < n; p += (long long)gridDim.x * blockDim.x) {
        const int q = nxt[p];
        if (sym[p] >= 0 && q >= 0) table_add(t, pair_key(sym[p], sym[q]), wc[p], true);
    }
}

__global__ void rehash_kernel(Table from, Table to) {
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i <= from.mask;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const unsigned long long k = from.keys[i];
        const long long v = (long long)from.vals[i];
        if (k != kEmpty && v > 0) table_add(to, k, v, true);
    }
}

// The best pair in two sweeps of the table, so counts are full int64 (no packing limit): best_count_kernel takes
// the max count into best[0]; best_pair_kernel then takes, among the pairs holding that count, the max of
// (kMaxId - a) << 17 | (kMaxId - b) = the smallest (a, b), into best[1] (the BpeTrainer order).
template <bool PAIR>
__global__ __launch_bounds__(256) void best_kernel(Table t, unsigned long long* best) {
    unsigned long long m = 0;
    const unsigned long long want = PAIR ? best[0] : 0;
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i <= t.mask;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const unsigned long long k = t.keys[i];
        const long long v = (long long)t.vals[i];
        if (k != kEmpty && v > 0) {
            unsigned long long x;
            if (PAIR) {
                const unsigned a = (unsigned)(k >> 32), b = (unsigned)k;
                x = (unsigned long long)v == want ? ((unsigned long long)(kMaxId - a) << kIdBits) | (kMaxId - b) : 0;
            } else {
                x = (unsigned long long)v;
            }
            m = x > m ? x : m;
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const unsigned long long x = __shfl_xor(m, o);
        m = x > m ? x : m;
    }
    __shared__ unsigned long long red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) m = red[w] > m ? red[w] : m;
        if (m) atomicMax(best + (PAIR ? 1 : 0), m);
    }
}

__global__ void mark_kernel(const int* __restrict__ sym, const int* __restrict__ nxt, const int* __restrict__ prv,
                            long long n, int a, int b, unsigned char* __restrict__ flag, int* __restrict__ starts,
                            unsigned* __restrict__ nstarts) {
    for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < n; p += (long long)gridDim.x * blockDim.x) {
        if (sym[p] != a) continue;
        const int q = nxt[p];
        if (q < 0 || sym[q] != b) continue;
        if (a == b) {  // left-to-right rewrite of a run of a's: the occurrences start at even offsets
            int k = 0;
            for (int r = prv[p]; r >= 0 && sym[r] == a; r = prv[r]) ++k;
            if (k & 1) continue;
        }
        flag[p] = 1;
        starts[atomicAdd(nstarts, 1u)] = (int)p;
    }
}

struct MergeArgs {
    int a, b, nid, nlen, maxlen;
    const int* len;  // token lengths (characters)
};

__device__ __forceinline__ int tok_len(const MergeArgs& m, int x) { return x == m.nid ? m.nlen : m.len[x]; }

__device__ __forceinline__ bool eligible(const MergeArgs& m, int x, int y) {
    const int lx = tok_len(m, x), ly = tok_len(m, y);
    return m.maxlen <= 0 || (lx == 1 && ly == 1) || lx + ly < m.maxlen;
}

__global__ void delta_kernel(const int* __restrict__ sym, const int* __restrict__ nxt, const int* __restrict__ prv,
                             const int* __restrict__ wc, const unsigned char* __restrict__ flag,
                             const int* __restrict__ starts, const unsigned* __restrict__ nstarts, MergeArgs m,
                             Table t) {
    const unsigned ns = *nstarts;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += gridDim.x * blockDim.x) {
        const int p = starts[i];
        const int q = nxt[p], L = prv[p], R = nxt[q];
        const long long c = wc[p];
        if (L >= 0) {
            table_add(t, pair_key(sym[L], m.a), -c, false);
            const bool lpartner = prv[L] >= 0 && flag[prv[L]];
            const int ls = lpartner ? m.nid : sym[L];
            if (eligible(m, ls, m.nid)) table_add(t, pair_key(ls, m.nid), c, true);
        }
        if (R >= 0 && !flag[R]) {
            table_add(t, pair_key(m.b, sym[R]), -c, false);
            if (eligible(m, m.nid, sym[R])) table_add(t, pair_key(m.nid, sym[R]), c, true);
        }
    }
}

__global__ void relink_kernel(int* __restrict__ sym, int* __restrict__ nxt, int* __restrict__ prv,
                              unsigned char* __restrict__ flag, const int* __restrict__ starts,
                              const unsigned* __restrict__ nstarts, int nid, int nlen, int* __restrict__ len) {
    const unsigned ns = *nstarts;
    if (blockIdx.x == 0 && threadIdx.x == 0) len[nid] = nlen;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += gridDim.x * blockDim.x) {
        const int p = starts[i];
        const int q = nxt[p], R = nxt[q];
        sym[p] = nid;
        nxt[p] = R;
        if (R >= 0) prv[R] = p;
        sym[q] = -1;
        nxt[q] = -1;
        prv[q] = -1;
        flag[p] = 0;
    }
}

__global__ void zero_pair_kernel(Table t, unsigned long long key) {
    unsigned long long h = mix(key) & t.mask;
    for (unsigned long long probe = 0; probe <= t.mask; ++probe) {
        const unsigned long long k = t.keys[h];
        if (k == key) {
            t.vals[h] = 0;
            return;
        }
        if (k == kEmpty) return;
        h = (h + 1) & t.mask;
    }
}

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return mimi::set_error_message(code, buf);  // mimi_last_error(), as every entry point
}

}  // namespace

struct mimi_bpe {
    int device = 0;
    hipStream_t s = nullptr;
    long long n = 0;
    int vocab = 0, maxlen = 0;
    int *sym = nullptr, *nxt = nullptr, *prv = nullptr, *wc = nullptr, *len = nullptr, *starts = nullptr;
    unsigned char* flag = nullptr;
    unsigned* nstarts = nullptr;
    unsigned long long* best = nullptr;
    Table t{};
    unsigned long long* host = nullptr;  // pinned: best count, best pair, nkeys
    int grid = 1024;
};

#define BPE_TRY(expr)                                                                                       \
    do {                                                                                                    \
        hipError_t _e = (expr);                                                                             \
        if (_e != hipSuccess) {                                                                             \
            (void)hipGetLastError();                                                                        \
            return fail(_e == hipErrorOutOfMemory ? MIMI_ERR_OUT_OF_MEMORY : MIMI_ERR_HIP, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(_e), __FILE__, __LINE__);                                  \
        }                                                                                                   \
    } while (0)

// (the fills are ordered on s: the kernels that use the table run on s, a non-blocking stream that does not
// wait for the null stream)
static int table_alloc(Table& t, unsigned long long cap, hipStream_t s) {
    t.mask = cap - 1;
    BPE_TRY(hipMalloc(&t.keys, cap * 8));
    BPE_TRY(hipMalloc(&t.vals, cap * 8));
    BPE_TRY(hipMalloc(&t.nkeys, 8));
    BPE_TRY(hipMemsetAsync(t.keys, 0xff, cap * 8, s));
    BPE_TRY(hipMemsetAsync(t.vals, 0, cap * 8, s));
    BPE_TRY(hipMemsetAsync(t.nkeys, 0, 8, s));
    return MIMI_OK;
}

static void table_free(Table& t) {
    if (t.keys) (void)hipFree(t.keys);
    if (t.vals) (void)hipFree(t.vals);
    if (t.nkeys) (void)hipFree(t.nkeys);
    t = Table{};
}

static unsigned long long pow2_at_least(unsigned long long x) {
    unsigned long long c = 1024;
    while (c < x) c <<= 1;
    return c;
}

// rebuild the table at capacity cap, dropping keys whose count reached 0 (merged pairs never come back)
static int rehash(mimi_bpe* h, unsigned long long cap) {
    Table nt{};
    int rc = table_alloc(nt, cap, h->s);
    if (rc) {
        table_free(nt);
        return rc;
    }
    hipLaunchKernelGGL(rehash_kernel, dim3(h->grid), dim3(256), 0, h->s, h->t, nt);
    BPE_TRY(hipGetLastError());
    BPE_TRY(hipStreamSynchronize(h->s));
    table_free(h->t);
    h->t = nt;
    return MIMI_OK;
}

extern "C" void mimi_bpe_destroy(mimi_bpe* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->s) (void)hipStreamSynchronize(h->s);
    for (void* p : {(void*)h->sym, (void*)h->nxt, (void*)h->prv, (void*)h->wc, (void*)h->len, (void*)h->starts,
                    (void*)h->flag, (void*)h->nstarts, (void*)h->best})
        if (p) (void)hipFree(p);
    table_free(h->t);
    if (h->host) (void)hipHostFree(h->host);
    if (h->s) (void)hipStreamDestroy(h->s);
    delete h;
}

extern "C" int mimi_bpe_create(int device, const int32_t* symbols, int64_t n_symbols, const int64_t* word_offsets,
                               const int64_t* word_counts, int64_t n_words, int32_t n_initial_tokens,
                               int32_t vocab_size, int32_t max_token_length, mimi_bpe** out) {
    if (!out) return fail(MIMI_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = nullptr;
    if (n_symbols < 0 || n_words < 0 || (n_symbols > 0 && (!symbols || !word_offsets || !word_counts)))
        return fail(MIMI_ERR_INVALID_ARGUMENT, "bad corpus arguments");
    if (n_initial_tokens < 1 || vocab_size < n_initial_tokens || (unsigned)vocab_size > kMaxId)
        return fail(MIMI_ERR_INVALID_ARGUMENT, "vocab_size %d must be in [%d, %u]", vocab_size, n_initial_tokens,
                    kMaxId);
    if (n_symbols >= (1ll << 31)) return fail(MIMI_ERR_UNSUPPORTED, "more than 2^31 symbols");
    // host: links and per-symbol word counts (pair counts are int64 on the device: no corpus-size limit)
    std::vector<int> nxt(n_symbols), prv(n_symbols), wc(n_symbols);
    if (n_words > 0 && (word_offsets[0] != 0 || word_offsets[n_words] != n_symbols))
        return fail(MIMI_ERR_INVALID_ARGUMENT, "word offsets must run from 0 to n_symbols");
    for (int64_t w = 0; w < n_words; ++w) {
        const int64_t b0 = word_offsets[w], b1 = word_offsets[w + 1];
        if (b1 < b0) return fail(MIMI_ERR_INVALID_ARGUMENT, "word offsets must be non-decreasing");
        if (word_counts[w] < 0 || word_counts[w] > 0x7fffffffll)
            return fail(MIMI_ERR_UNSUPPORTED, "word count %lld", (long long)word_counts[w]);
        for (int64_t p = b0; p < b1; ++p) {
            if (symbols[p] < 0 || symbols[p] >= n_initial_tokens)
                return fail(MIMI_ERR_INVALID_ARGUMENT, "symbol %d outside the initial tokens", symbols[p]);
            prv[p] = p > b0 ? (int)(p - 1) : -1;
            nxt[p] = p + 1 < b1 ? (int)(p + 1) : -1;
            wc[p] = (int)word_counts[w];
        }
    }
    std::unique_ptr<mimi_bpe> h(new mimi_bpe());
    mimi_bpe* H = h.get();
    H->device = device;
    H->n = n_symbols;
    H->vocab = vocab_size;
    H->maxlen = max_token_length;
    BPE_TRY(hipSetDevice(device));
    BPE_TRY(hipStreamCreateWithFlags(&H->s, hipStreamNonBlocking));
    const size_t nb = (size_t)std::max<int64_t>(n_symbols, 1);
    BPE_TRY(hipMalloc(&H->sym, nb * 4));
    BPE_TRY(hipMalloc(&H->nxt, nb * 4));
    BPE_TRY(hipMalloc(&H->prv, nb * 4));
    BPE_TRY(hipMalloc(&H->wc, nb * 4));
    BPE_TRY(hipMalloc(&H->starts, nb * 4));
    BPE_TRY(hipMalloc(&H->flag, nb));
    BPE_TRY(hipMalloc(&H->len, (size_t)vocab_size * 4));
    BPE_TRY(hipMalloc(&H->nstarts, 4));
    BPE_TRY(hipMalloc(&H->best, 16));
    BPE_TRY(hipHostMalloc(&H->host, 24, hipHostMallocDefault));
    if (n_symbols > 0) {
        BPE_TRY(hipMemcpy(H->sym, symbols, n_symbols * 4, hipMemcpyHostToDevice));
        BPE_TRY(hipMemcpy(H->nxt, nxt.data(), n_symbols * 4, hipMemcpyHostToDevice));
        BPE_TRY(hipMemcpy(H->prv, prv.data(), n_symbols * 4, hipMemcpyHostToDevice));
        BPE_TRY(hipMemcpy(H->wc, wc.data(), n_symbols * 4, hipMemcpyHostToDevice));
    }
    BPE_TRY(hipMemsetAsync(H->flag, 0, nb, H->s));
    {
        std::vector<int> lens(vocab_size, 1);  // special tokens and the alphabet: one character each
        BPE_TRY(hipMemcpy(H->len, lens.data(), lens.size() * 4, hipMemcpyHostToDevice));
    }
    int dev_cu = 256;
    (void)hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, device);
    H->grid = std::max(64, dev_cu * 8);
    int rc = table_alloc(H->t, pow2_at_least(2ull * (unsigned long long)nb + 1024), H->s);
    if (rc) return rc;
    hipLaunchKernelGGL(count_pairs_kernel, dim3(H->grid), dim3(256), 0, H->s, H->sym, H->nxt, H->wc, H->n, H->t);
    BPE_TRY(hipGetLastError());
    BPE_TRY(hipMemcpyAsync(H->host + 1, H->t.nkeys, 8, hipMemcpyDeviceToHost, H->s));
    BPE_TRY(hipStreamSynchronize(H->s));
    // room for the pairs the merges will form: 4x the distinct initial pairs, at least 2^20 slots
    if ((rc = rehash(H, pow2_at_least(4ull * H->host[1] + (1ull << 20))))) return rc;
    *out = h.release();
    return MIMI_OK;
}

extern "C" int mimi_bpe_best(mimi_bpe* h, int32_t* left, int32_t* right, int64_t* count) {
    if (!h || !left || !right || !count) return fail(MIMI_ERR_INVALID_ARGUMENT, "null argument");
    BPE_TRY(hipSetDevice(h->device));
    BPE_TRY(hipMemsetAsync(h->best, 0, 16, h->s));
    const unsigned long long slots = h->t.mask + 1;
    const unsigned grid = (unsigned)std::min<unsigned long long>((slots + 255) / 256, (unsigned long long)h->grid);
    hipLaunchKernelGGL(best_kernel<false>, dim3(grid), dim3(256), 0, h->s, h->t, h->best);
    BPE_TRY(hipGetLastError());
    hipLaunchKernelGGL(best_kernel<true>, dim3(grid), dim3(256), 0, h->s, h->t, h->best);
    BPE_TRY(hipGetLastError());
    BPE_TRY(hipMemcpyAsync(h->host, h->best, 16, hipMemcpyDeviceToHost, h->s));
    BPE_TRY(hipMemcpyAsync(h->host + 2, h->t.nkeys, 8, hipMemcpyDeviceToHost, h->s));
    BPE_TRY(hipStreamSynchronize(h->s));
    const unsigned long long c = h->host[0], m = h->host[1];
    *count = (int64_t)c;
    *left = c ? (int32_t)(kMaxId - ((m >> kIdBits) & kMaxId)) : -1;
    *right = c ? (int32_t)(kMaxId - (m & kMaxId)) : -1;
    // keep the load factor under 1/2 (the merges' new pairs); a rehash also drops the merged (zero) pairs
    if (2 * h->host[2] > slots) {
        int rc = rehash(h, slots * 2);
        if (rc) return rc;
    }
    return MIMI_OK;
}

extern "C" int mimi_bpe_merge(mimi_bpe* h, int32_t left, int32_t right, int32_t new_id, int32_t new_len) {
    if (!h) return fail(MIMI_ERR_INVALID_ARGUMENT, "null handle");
    if (left < 0 || right < 0 || new_id < 0 || left >= h->vocab || right >= h->vocab || new_id >= h->vocab ||
        new_len < 2)
        return fail(MIMI_ERR_INVALID_ARGUMENT, "merge (%d, %d) -> %d out of range", left, right, new_id);
    BPE_TRY(hipSetDevice(h->device));
    BPE_TRY(hipMemsetAsync(h->nstarts, 0, 4, h->s));
    const unsigned g = (unsigned)h->grid;
    if (h->n > 0) {
        hipLaunchKernelGGL(mark_kernel, dim3(g), dim3(256), 0, h->s, h->sym, h->nxt, h->prv, h->n, left, right,
                           h->flag, h->starts, h->nstarts);
        BPE_TRY(hipGetLastError());
        MergeArgs m{left, right, new_id, new_len, h->maxlen, h->len};
        hipLaunchKernelGGL(delta_kernel, dim3(g), dim3(256), 0, h->s, h->sym, h->nxt, h->prv, h->wc, h->flag,
                           h->starts, h->nstarts, m, h->t);
        BPE_TRY(hipGetLastError());
        hipLaunchKernelGGL(relink_kernel, dim3(g), dim3(256), 0, h->s, h->sym, h->nxt, h->prv, h->flag, h->starts,
                           h->nstarts, new_id, new_len, h->len);
        BPE_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(zero_pair_kernel, dim3(1), dim3(1), 0, h->s, h->t,
                       ((unsigned long long)(unsigned)left << 32) | (unsigned)right);
    BPE_TRY(hipGetLastError());
    return MIMI_OK;
}
