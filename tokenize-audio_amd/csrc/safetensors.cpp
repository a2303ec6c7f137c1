// Host-side safetensors reader for mimi_load_safetensors (engine.cpp).  A checkpoint is untrusted bytes: every
// offset, size and shape is checked against the file before anything is read or allocated, and a malformed or
// truncated file is MIMI_ERR_IO, never a crash.  Host code only (no HIP), so tools/asan builds it under
// AddressSanitizer / UBSan together with flac.cpp.
//
// Format (safetensors v0.4, huggingface/safetensors README): u64 little-endian header length N, N bytes of JSON
// {"name": {"dtype": "F32", "shape": [..], "data_offsets": [begin, end]}, ..., "__metadata__": {..}}, then the
// tensor bytes, offsets relative to the end of the header.  The kyutai/mimi checkpoint (model.safetensors of the
// HF repo MimiModel.from_pretrained("kyutai/mimi") reads: emilia-mimi/process_shard.py:57) stores F32 tensors.
#include "host_io.h"

#include <cctype>
#include <cstring>
#include <fstream>
#include <limits>

#include "../../include/mimi_hip.h"

namespace mimi {
namespace {

struct JsonCursor {
    const std::string& s;
    size_t i = 0;
    explicit JsonCursor(const std::string& str) : s(str) {}
    void ws() {
        while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\t' || s[i] == '\r')) ++i;
    }
    bool eat(char c) {
        ws();
        if (i < s.size() && s[i] == c) {
            ++i;
            return true;
        }
        return false;
    }
    bool str(std::string& out) {
        ws();
        if (i >= s.size() || s[i] != '"') return false;
        ++i;
        out.clear();
        while (i < s.size() && s[i] != '"') {
            if (s[i] == '\\') {
                if (++i >= s.size()) return false;
            }
            out.push_back(s[i++]);
        }
        if (i >= s.size()) return false;
        ++i;
        return true;
    }
    // a non-negative integer that fits int64 (safetensors offsets and dims are unsigned)
    bool num(int64_t& v) {
        ws();
        size_t j = i;
        v = 0;
        while (j < s.size() && std::isdigit((unsigned char)s[j])) {
            const int d = s[j] - '0';
            if (v > (std::numeric_limits<int64_t>::max() - d) / 10) return false;
            v = v * 10 + d;
            ++j;
        }
        if (j == i) return false;
        i = j;
        return true;
    }
    bool skip_value(int depth = 0) {  // any JSON value (used for __metadata__ and unknown fields)
        ws();
        if (i >= s.size() || depth > 64) return false;
        const char ch = s[i];
        if (ch == '"') {
            std::string t;
            return str(t);
        }
        if (ch == '{' || ch == '[') {
            const char close = ch == '{' ? '}' : ']';
            ++i;
            if (eat(close)) return true;
            do {
                if (ch == '{') {
                    std::string k;
                    if (!str(k) || !eat(':')) return false;
                }
                if (!skip_value(depth + 1)) return false;
            } while (eat(','));
            return eat(close);
        }
        const size_t j = i;
        while (i < s.size() && s[i] != ',' && s[i] != '}' && s[i] != ']' && !std::isspace((unsigned char)s[i])) ++i;
        return i > j;
    }
    bool int_list(std::vector<int64_t>& v) {
        v.clear();
        if (!eat('[')) return false;
        if (eat(']')) return true;
        do {
            int64_t x;
            if (!num(x) || v.size() >= 16) return false;
            v.push_back(x);
        } while (eat(','));
        return eat(']');
    }
};

int dtype_size(const std::string& d) {
    if (d == "F64" || d == "I64" || d == "U64") return 8;
    if (d == "F32" || d == "I32" || d == "U32") return 4;
    if (d == "F16" || d == "BF16" || d == "I16" || d == "U16") return 2;
    if (d == "I8" || d == "U8" || d == "BOOL" || d == "F8_E4M3" || d == "F8_E5M2") return 1;
    return 0;
}

}  // namespace

bool st_parse_header(const std::string& hdr, int64_t data_bytes, std::map<std::string, StTensor>& out,
                     std::string& err) {
    out.clear();
    JsonCursor c(hdr);
    if (!c.eat('{')) return err = "header is not a JSON object", false;
    if (c.eat('}')) {
        c.ws();
        return c.i == hdr.size() ? true : (err = "bytes after the header object", false);
    }
    do {
        std::string key;
        if (!c.str(key) || !c.eat(':')) return err = "bad key", false;
        if (key == "__metadata__") {
            if (!c.skip_value()) return err = "bad __metadata__", false;
            continue;
        }
        StTensor en;
        bool has_dtype = false, has_shape = false, has_off = false;
        if (!c.eat('{')) return err = "entry " + key + " is not an object", false;
        if (!c.eat('}')) {
            do {
                std::string f;
                if (!c.str(f) || !c.eat(':')) return err = "bad field in " + key, false;
                if (f == "dtype") {
                    if (!c.str(en.dtype)) return err = "bad dtype in " + key, false;
                    has_dtype = true;
                } else if (f == "shape") {
                    if (!c.int_list(en.shape)) return err = "bad shape in " + key, false;
                    has_shape = true;
                } else if (f == "data_offsets") {
                    std::vector<int64_t> o;
                    if (!c.int_list(o) || o.size() != 2) return err = "bad data_offsets in " + key, false;
                    en.begin = o[0];
                    en.end = o[1];
                    has_off = true;
                } else if (!c.skip_value()) {
                    return err = "bad value in " + key, false;
                }
            } while (c.eat(','));
            if (!c.eat('}')) return err = "unterminated entry " + key, false;
        }
        if (!has_dtype || !has_shape || !has_off) return err = "entry " + key + " lacks dtype/shape/data_offsets", false;
        const int es = dtype_size(en.dtype);
        if (es == 0) return err = "entry " + key + ": unknown dtype " + en.dtype, false;
        int64_t numel = 1;
        for (int64_t d : en.shape) {
            if (d != 0 && numel > std::numeric_limits<int64_t>::max() / es / d) return err = key + ": shape overflows", false;
            numel *= d;
        }
        en.numel = numel;
        if (en.begin > en.end || en.end > data_bytes)
            return err = key + ": data_offsets outside the file (truncated?)", false;
        if (en.end - en.begin != numel * es) return err = key + ": data_offsets do not match dtype x shape", false;
        if (out.count(key)) return err = "duplicate entry " + key, false;
        out[key] = en;
    } while (c.eat(','));
    if (!c.eat('}')) return err = "unterminated header", false;
    c.ws();
    if (c.i != hdr.size()) return err = "bytes after the header object", false;
    return true;
}

int st_load(const char* path, const std::function<bool(const std::string&)>& wanted,
            std::map<std::string, std::vector<float>>& out, std::string& err) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) return err = std::string("cannot open ") + path, MIMI_ERR_IO;
    const int64_t fsize = (int64_t)f.tellg();
    f.seekg(0);
    uint64_t hlen = 0;
    unsigned char lb[8];
    f.read(reinterpret_cast<char*>(lb), 8);
    if (!f || fsize < 8) return err = std::string(path) + ": not a safetensors file (shorter than 8 bytes)", MIMI_ERR_IO;
    for (int i = 7; i >= 0; --i) hlen = hlen << 8 | lb[i];
    if (hlen < 2 || hlen > (uint64_t)(fsize - 8) || hlen > (1ull << 30))
        return err = std::string(path) + ": bad safetensors header length (truncated?)", MIMI_ERR_IO;
    std::string hdr((size_t)hlen, '\0');
    f.read(&hdr[0], (std::streamsize)hlen);
    if (!f) return err = std::string(path) + ": truncated header", MIMI_ERR_IO;
    const int64_t data0 = 8 + (int64_t)hlen;
    std::map<std::string, StTensor> entries;
    std::string perr;
    if (!st_parse_header(hdr, fsize - data0, entries, perr)) return err = std::string(path) + ": " + perr, MIMI_ERR_IO;
    for (const auto& kv : entries) {
        if (!wanted(kv.first)) continue;
        const StTensor& en = kv.second;
        if (en.dtype != "F32")
            return err = kv.first + ": dtype " + en.dtype + " (the engine reads F32 checkpoints)", MIMI_ERR_WEIGHTS;
        std::vector<float> buf((size_t)en.numel);
        f.seekg(data0 + en.begin);
        if (en.numel) f.read(reinterpret_cast<char*>(buf.data()), en.numel * 4);
        if (!f) return err = std::string(path) + ": truncated data for " + kv.first, MIMI_ERR_IO;
        out[kv.first] = std::move(buf);
    }
    return MIMI_OK;
}

}  // namespace mimi
