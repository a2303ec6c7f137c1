// FLAC decoder for the host-ingest path (libmimi_hip.so, C ABI mimi_flac_*).
//
// Replaces the libFLAC decode behind librosa.load -> soundfile -> libsndfile on the LibriSpeech path
// (librispeech-mimi/process_librispeech_dev-test.py:136 loads the corpus' .flac files; utils.py:84-87).
// Written from the format specification (RFC 9639): STREAMINFO, frame headers (fixed / variable block size,
// coded numbers, CRC-8), CONSTANT / VERBATIM / FIXED / LPC subframes with wasted bits, Rice and Rice2 residual
// partitions with escapes, the three stereo decorrelations, CRC-16 frame footers.  Output: planar int32
// samples at the stream's bit depth (the float conversion and librosa's channel mean stay in numpy,
// mimi_hip/ingest.py, shared with the WAV path).
//
// FLAC decoding is a serial bit-stream walk per frame (Rice lengths chain every partition's position, LPC
// restoration is a recursion over the block), so it stays on the host CPU like the reference's libsndfile;
// callers decode many files on a thread pool (the call holds no global state).
#include <cstdint>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/mimi_hip.h"

namespace mimi {
int set_last_error(int code, const std::string& msg);  // engine.cpp
}

namespace {

int fail(const std::string& m, int code = MIMI_ERR_IO) { return mimi::set_last_error(code, m); }

// MSB-first bit reader over a byte buffer: a 64-bit window refilled 8 bytes at a time; reading past the end
// yields zeros and sets `over`
struct BitReader {
    const uint8_t* p;
    size_t n;             // bytes
    size_t byte = 0;      // next byte to enter the window
    uint64_t cache = 0;   // valid bits left-aligned, zeros below
    int cbits = 0;
    bool over = false;

    BitReader(const uint8_t* d, size_t nb) : p(d), n(nb) {}
    size_t pos() const { return byte * 8 - (size_t)cbits; }
    __attribute__((always_inline)) inline void refill() {
        if (cbits > 56) return;
        if (byte + 8 <= n) {
            uint64_t w;
            memcpy(&w, p + byte, 8);
            w = __builtin_bswap64(w);
            const int take = (64 - cbits) >> 3;  // whole bytes that fit
            cache |= (take == 8 ? w : w >> (64 - 8 * take)) << (64 - cbits - 8 * take);
            cbits += 8 * take;
            byte += take;
        } else {
            while (cbits <= 56) {
                const uint64_t b = byte < n ? p[byte] : 0;
                cache |= b << (56 - cbits);
                cbits += 8;
                ++byte;
            }
        }
        if (byte > n && pos() > n * 8) over = true;
    }
    __attribute__((always_inline)) inline uint64_t bits(int k) {  // k <= 57
        if (k == 0) return 0;
        refill();
        const uint64_t v = cache >> (64 - k);
        cache <<= k;
        cbits -= k;
        if (byte > n && pos() > n * 8) over = true;
        return v;
    }
    __attribute__((always_inline)) inline int64_t sbits(int k) {  // two's complement, k <= 57
        if (k == 0) return 0;
        const uint64_t u = bits(k);
        return (int64_t)(u << (64 - k)) >> (64 - k);
    }
    __attribute__((always_inline)) inline uint32_t unary() {  // zeros before the next 1
        uint32_t q = 0;
        for (;;) {
            refill();
            if (cache == 0) {
                q += (uint32_t)cbits;
                cache = 0;
                cbits = 0;
                if (byte >= n) {
                    over = true;
                    return q;
                }
                continue;
            }
            const int z = __builtin_clzll(cache);
            cache <<= z + 1;
            cbits -= z + 1;
            if (byte > n && pos() > n * 8) over = true;
            return q + (uint32_t)z;
        }
    }
    // one Rice-coded value (unary quotient, k-bit remainder); fast path when both lie in the window
    __attribute__((always_inline)) inline uint64_t rice(int k) {
        refill();
        if (cache) {
            const int z = __builtin_clzll(cache);
            const int need = z + 1 + k;
            if (need <= cbits) {
                const uint64_t rest = z < 63 ? cache << (z + 1) : 0;
                const uint64_t v = ((uint64_t)z << k) | (k ? rest >> (64 - k) : 0);
                cache = need < 64 ? cache << need : 0;
                cbits -= need;
                return v;
            }
        }
        const uint64_t q = unary();
        return (q << k) | bits(k);
    }
    void align() {
        const int drop = cbits & 7;
        cache <<= drop;
        cbits -= drop;
    }
};

struct CrcTables {  // FLAC's CRC-8 (poly 0x07) and CRC-16 (poly 0x8005), MSB first, init 0
    uint8_t c8[256];
    uint16_t c16[8][256];  // c16[m][b]: CRC-16 of byte b followed by m zero bytes (slicing by 8)
    CrcTables() {
        for (int i = 0; i < 256; ++i) {
            uint8_t c = (uint8_t)i;
            for (int b = 0; b < 8; ++b) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
            c8[i] = c;
            uint16_t d = (uint16_t)(i << 8);
            for (int b = 0; b < 8; ++b) d = (uint16_t)((d & 0x8000) ? (d << 1) ^ 0x8005 : (d << 1));
            c16[0][i] = d;
        }
        for (int m = 1; m < 8; ++m)
            for (int i = 0; i < 256; ++i) {
                const uint16_t c = c16[m - 1][i];
                c16[m][i] = (uint16_t)((c << 8) ^ c16[0][c >> 8]);
            }
    }
};
const CrcTables kCrc;

uint8_t crc8(const uint8_t* d, size_t n) {
    uint8_t c = 0;
    for (size_t i = 0; i < n; ++i) c = kCrc.c8[c ^ d[i]];
    return c;
}

uint16_t crc16(const uint8_t* d, size_t n) {
    uint16_t c = 0;
    size_t i = 0;
    for (; i + 8 <= n; i += 8)  // the running CRC folds into the first two bytes of each 8-byte slice
        c = (uint16_t)(kCrc.c16[7][d[i] ^ (c >> 8)] ^ kCrc.c16[6][d[i + 1] ^ (c & 0xff)] ^ kCrc.c16[5][d[i + 2]] ^
                       kCrc.c16[4][d[i + 3]] ^ kCrc.c16[3][d[i + 4]] ^ kCrc.c16[2][d[i + 5]] ^ kCrc.c16[1][d[i + 6]] ^
                       kCrc.c16[0][d[i + 7]]);
    for (; i < n; ++i) c = (uint16_t)((c << 8) ^ kCrc.c16[0][(c >> 8) ^ d[i]]);
    return c;
}

struct StreamInfo {
    int min_block = 0, max_block = 0, rate = 0, channels = 0, bps = 0;
    int64_t total = 0;
};

// metadata: "fLaC", blocks until the last-block flag; returns the offset of the first frame
int parse_header(const uint8_t* d, size_t n, StreamInfo& si, size_t& first_frame) {
    size_t off = 0;
    if (n >= 10 && d[0] == 'I' && d[1] == 'D' && d[2] == '3') {  // ID3v2 tag in front (syncsafe size)
        const size_t sz = ((size_t)(d[6] & 0x7f) << 21) | ((size_t)(d[7] & 0x7f) << 14) | ((size_t)(d[8] & 0x7f) << 7) |
                          (size_t)(d[9] & 0x7f);
        off = 10 + sz + ((d[5] & 0x10) ? 10 : 0);
    }
    if (off + 4 > n || memcmp(d + off, "fLaC", 4) != 0) return fail("not a FLAC stream (no fLaC marker)");
    off += 4;
    bool seen_info = false, last = false;
    while (!last) {
        if (off + 4 > n) return fail("truncated metadata");
        last = (d[off] & 0x80) != 0;
        const int type = d[off] & 0x7f;
        const size_t len = ((size_t)d[off + 1] << 16) | ((size_t)d[off + 2] << 8) | d[off + 3];
        off += 4;
        if (off + len > n) return fail("truncated metadata block");
        if (type == 127) return fail("invalid metadata block type");
        if (type == 0) {
            if (len < 34) return fail("short STREAMINFO");
            BitReader br(d + off, len);
            si.min_block = (int)br.bits(16);
            si.max_block = (int)br.bits(16);
            br.bits(24);
            br.bits(24);
            si.rate = (int)br.bits(20);
            si.channels = (int)br.bits(3) + 1;
            si.bps = (int)br.bits(5) + 1;
            si.total = (int64_t)br.bits(36);
            seen_info = true;
        } else if (!seen_info) {
            return fail("STREAMINFO must be the first metadata block");
        }
        off += len;
    }
    if (!seen_info) return fail("no STREAMINFO");
    if (si.bps < 4 || si.bps > 32) return fail("unsupported bits per sample");
    first_frame = off;
    return MIMI_OK;
}

// residual of one subframe into res[order .. bs)
bool read_residual(BitReader& br, int bs, int order, int64_t* out) {
    const int method = (int)br.bits(2);
    if (method > 1) return false;
    const int pbits = method == 0 ? 4 : 5, esc = (1 << pbits) - 1;
    const int porder = (int)br.bits(4);
    const int parts = 1 << porder;
    if ((bs >> porder) << porder != bs) return false;
    const int psize = bs >> porder;
    if (psize < order) return false;
    int i = order;
    BitReader r = br;  // a local copy: its window stays in registers across the stores to `out`
    for (int pt = 0; pt < parts; ++pt) {
        const int cnt = pt == 0 ? psize - order : psize;
        const int k = (int)r.bits(pbits);
        if (k == esc) {
            const int nb = (int)r.bits(5);
            for (int j = 0; j < cnt; ++j) out[i++] = r.sbits(nb);
        } else {
            for (int j = 0; j < cnt; ++j) {
                const uint64_t v = r.rice(k);
                out[i++] = (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
            }
        }
        if (r.over) return false;
    }
    br = r;
    return true;
}

// s[i] += (sum_j coef[j] s[i-1-j]) >> shift, coefficient j applying to the sample j + 1 back.  The products and
// sums wrap in uint64 (two's complement, the same bits as int64 wherever a valid stream keeps them in range, and
// defined behaviour on a corrupt one, whose garbage the frame CRC-16 then rejects; tools/asan runs this under UBSan)
template <int ORDER>
void lpc_restore(int64_t* s, int bs, const int64_t* coef, int shift) {
    for (int i = ORDER; i < bs; ++i) {
        uint64_t sum = 0;
#pragma unroll
        for (int j = 0; j < ORDER; ++j) sum += (uint64_t)coef[j] * (uint64_t)s[i - 1 - j];
        s[i] = (int64_t)((uint64_t)s[i] + (uint64_t)((int64_t)sum >> shift));
    }
}

template <int... O>
void lpc_dispatch(int order, int64_t* s, int bs, const int64_t* coef, int shift, std::integer_sequence<int, O...>) {
    using Fn = void (*)(int64_t*, int, const int64_t*, int);
    static const Fn fns[] = {lpc_restore<O + 1>...};
    fns[order - 1](s, bs, coef, shift);
}

// one subframe of `bs` samples at `bps` bits into s[0..bs)
bool read_subframe(BitReader& br, int bs, int bps, int64_t* s) {
    if (br.bits(1) != 0) return false;  // padding bit
    const int type = (int)br.bits(6);
    int wasted = 0;
    if (br.bits(1)) wasted = (int)br.unary() + 1;
    const int b = bps - wasted;
    if (b <= 0) return false;
    if (type == 0) {  // CONSTANT
        const int64_t v = br.sbits(b);
        for (int i = 0; i < bs; ++i) s[i] = v;
    } else if (type == 1) {  // VERBATIM
        BitReader r = br;
        for (int i = 0; i < bs; ++i) s[i] = r.sbits(b);
        br = r;
    } else if (type >= 8 && type <= 12) {  // FIXED, order 0..4
        const int order = type - 8;
        if (order > bs) return false;
        for (int i = 0; i < order; ++i) s[i] = br.sbits(b);
        if (!read_residual(br, bs, order, s)) return false;
        for (int i = order; i < bs; ++i) {
            uint64_t pred = 0;  // (wrapping: see lpc_restore)
            const uint64_t a = (uint64_t)s[i - 1 < 0 ? 0 : i - 1], b2 = order >= 2 ? (uint64_t)s[i - 2] : 0,
                           c = order >= 3 ? (uint64_t)s[i - 3] : 0, d = order >= 4 ? (uint64_t)s[i - 4] : 0;
            switch (order) {
                case 1: pred = a; break;
                case 2: pred = 2 * a - b2; break;
                case 3: pred = 3 * a - 3 * b2 + c; break;
                case 4: pred = 4 * a - 6 * b2 + 4 * c - d; break;
                default: break;
            }
            s[i] = (int64_t)((uint64_t)s[i] + pred);
        }
    } else if (type >= 32) {  // LPC, order 1..32
        const int order = type - 31;
        if (order > bs) return false;
        for (int i = 0; i < order; ++i) s[i] = br.sbits(b);
        const int prec = (int)br.bits(4) + 1;
        if (prec == 16) return false;
        const int shift = (int)br.sbits(5);
        if (shift < 0) return false;
        int64_t coef[32];
        for (int j = 0; j < order; ++j) coef[j] = br.sbits(prec);
        if (!read_residual(br, bs, order, s)) return false;
        lpc_dispatch(order, s, bs, coef, shift, std::make_integer_sequence<int, 32>());
    } else {
        return false;  // reserved
    }
    if (wasted)
        for (int i = 0; i < bs; ++i) s[i] = (int64_t)((uint64_t)s[i] << wasted);
    return !br.over;
}

const int kRates[12] = {0, 88200, 176400, 192000, 8000, 16000, 22050, 24000, 32000, 44100, 48000, 96000};
const int kBps[8] = {0, 8, 12, -1, 16, 20, 24, 32};

}  // namespace

extern "C" {

int mimi_flac_info(const uint8_t* data, int64_t nbytes, int32_t* sample_rate, int32_t* channels,
                   int32_t* bits_per_sample, int64_t* total_samples) {
    if (!data || nbytes <= 0) return fail("empty buffer", MIMI_ERR_INVALID_ARGUMENT);
    StreamInfo si;
    size_t ff = 0;
    const int st = parse_header(data, (size_t)nbytes, si, ff);
    if (st) return st;
    if (sample_rate) *sample_rate = si.rate;
    if (channels) *channels = si.channels;
    if (bits_per_sample) *bits_per_sample = si.bps;
    if (total_samples) *total_samples = si.total;
    return MIMI_OK;
}

int mimi_flac_decode(const uint8_t* data, int64_t nbytes, int32_t* out, int64_t cap_per_channel,
                     int64_t* n_samples) {
    if (!data || nbytes <= 0 || !n_samples) return fail("bad arguments", MIMI_ERR_INVALID_ARGUMENT);
    StreamInfo si;
    size_t off = 0;
    int st = parse_header(data, (size_t)nbytes, si, off);
    if (st) return st;
    const size_t n = (size_t)nbytes;
    const int C = si.channels;
    std::vector<int64_t> buf;
    int64_t done = 0;
    while (off < n) {
        // ---- frame header
        if (off + 2 > n) break;
        if (data[off] != 0xFF || (data[off + 1] & 0xFE) != 0xF8) {
            if (si.total > 0 && done >= si.total) break;  // trailing garbage / tag after the last frame
            return fail("lost frame sync at byte " + std::to_string(off));
        }
        BitReader br(data + off, n - off);
        br.bits(15);
        br.bits(1);  // blocking strategy: the coded number is a frame or a sample number; unused here
        const int bs_code = (int)br.bits(4), sr_code = (int)br.bits(4), ch_code = (int)br.bits(4),
                  sz_code = (int)br.bits(3);
        if (br.bits(1) != 0) return fail("reserved frame header bit set");
        {  // coded number (UTF-8-like, up to 7 bytes)
            const uint32_t b0 = (uint32_t)br.bits(8);
            int extra = 0;
            if (b0 >= 0xFE) extra = 6;
            else if (b0 >= 0xFC) extra = 5;
            else if (b0 >= 0xF8) extra = 4;
            else if (b0 >= 0xF0) extra = 3;
            else if (b0 >= 0xE0) extra = 2;
            else if (b0 >= 0xC0) extra = 1;
            else if (b0 >= 0x80) return fail("bad coded number");
            for (int i = 0; i < extra; ++i)
                if ((br.bits(8) & 0xC0) != 0x80) return fail("bad coded number");
        }
        int bs = 0;
        if (bs_code == 0) return fail("reserved block size");
        if (bs_code == 1) bs = 192;
        else if (bs_code <= 5) bs = 576 << (bs_code - 2);
        else if (bs_code == 6) bs = (int)br.bits(8) + 1;
        else if (bs_code == 7) bs = (int)br.bits(16) + 1;
        else bs = 256 << (bs_code - 8);
        int rate = si.rate;
        if (sr_code >= 1 && sr_code <= 11) rate = kRates[sr_code];
        else if (sr_code == 12) rate = (int)br.bits(8) * 1000;
        else if (sr_code == 13) rate = (int)br.bits(16);
        else if (sr_code == 14) rate = (int)br.bits(16) * 10;
        else if (sr_code == 15) return fail("invalid sample rate code");
        (void)rate;
        int bps = sz_code == 0 ? si.bps : kBps[sz_code];
        if (bps < 0) return fail("reserved sample size");
        int fch = 0;
        if (ch_code <= 7) fch = ch_code + 1;
        else if (ch_code <= 10) fch = 2;
        else return fail("reserved channel assignment");
        if (fch != C) return fail("frame channel count differs from STREAMINFO");
        const size_t hdr_bytes = br.pos() / 8;
        const uint8_t want8 = (uint8_t)br.bits(8);
        if (br.over || crc8(data + off, hdr_bytes) != want8) return fail("frame header CRC-8 mismatch");
        // ---- subframes
        if ((int64_t)buf.size() < (int64_t)bs * C) buf.resize((size_t)bs * C);
        for (int c = 0; c < C; ++c) {
            int b = bps;
            if ((ch_code == 8 && c == 1) || (ch_code == 9 && c == 0) || (ch_code == 10 && c == 1)) b += 1;  // side
            if (!read_subframe(br, bs, b, buf.data() + (size_t)c * bs))
                return fail("malformed subframe in frame at byte " + std::to_string(off));
        }
        br.align();
        const size_t body = br.pos() / 8;
        const uint16_t want16 = (uint16_t)br.bits(16);
        if (br.over || crc16(data + off, body) != want16) return fail("frame CRC-16 mismatch");
        int64_t* a = buf.data();
        int64_t* s2 = buf.data() + bs;
        for (int i = 0; i < bs && C == 2; ++i) {
            if (ch_code == 8) {          // left, side
                s2[i] = a[i] - s2[i];
            } else if (ch_code == 9) {   // side, right
                a[i] = a[i] + s2[i];
            } else if (ch_code == 10) {  // mid, side
                const int64_t side = s2[i];
                const int64_t mid = (int64_t)((uint64_t)a[i] << 1) | (side & 1);
                a[i] = (mid + side) >> 1;
                s2[i] = (mid - side) >> 1;
            }
        }
        if (out) {
            if (done + bs > cap_per_channel) return fail("output capacity exceeded", MIMI_ERR_INVALID_ARGUMENT);
            for (int c = 0; c < C; ++c)
                for (int i = 0; i < bs; ++i) out[(size_t)c * cap_per_channel + done + i] = (int32_t)buf[(size_t)c * bs + i];
        }
        done += bs;
        off += br.pos() / 8;
    }
    if (si.total > 0 && done != si.total)
        return fail("decoded " + std::to_string(done) + " samples, STREAMINFO says " + std::to_string(si.total));
    *n_samples = done;
    return MIMI_OK;
}

}  // extern "C"
