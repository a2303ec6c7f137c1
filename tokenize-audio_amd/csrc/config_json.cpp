// Host-side checkpoint-directory reading for the one-call constructor mimi_create_from_dir (engine.cpp):
// config.json -> mimi_config, and the directory scan that picks the safetensors file.  Untrusted bytes like the
// checkpoint itself: a bounded recursive-descent JSON parser, every failure a status + message, never a crash.  Host
// code only (no HIP), so tools/asan builds it under AddressSanitizer / UBSan beside flac.cpp and safetensors.cpp.
//
// What it restates (the Python host's MimiConfig.from_json + validate_supported + config_from_py, which follow the
// reference's MimiConfig, TF/configuration_mimi.py:86-175):
//   - the HF config.json keys of the encode path, unknown keys ignored (MimiConfig(**config_dict) keeps them as
//     attributes the encode never reads);
//   - rope_theta at the top level or inside rope_parameters (transformers 5.x writes the latter);
//   - head_dim null or absent -> hidden_size / num_attention_heads (TF/configuration_mimi.py:139);
//   - frame_rate present and not null -> the override; else sampling_rate / frame_size, with frame_size
//     = prod(upsampling_ratios) * 2 for one residual layer per stage (TF/configuration_mimi.py:152-175);
//   - the downsample conv's kernel = 2 * int(encodec_frame_rate / frame_rate), encodec_frame_rate
//     = ceil(sampling_rate / prod(upsampling_ratios)) (TF/modeling_mimi.py:1223-1233, configuration_mimi.py:143);
//   - the architecture checks of MimiConfig.validate_supported (causal convs, constant padding, one residual layer,
//     no conv shortcut, GELU, no attention bias, no GQA).
#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../../include/mimi_hip.h"
#include "host_io.h"

namespace mimi {
int set_last_error(int code, const std::string& msg);  // engine.cpp (thread-local, behind mimi_last_error)

namespace {

struct JVal {
    enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<JVal> arr;
    std::vector<std::pair<std::string, JVal>> obj;
    const JVal* get(const char* key) const {
        if (kind != OBJ) return nullptr;
        for (const auto& kv : obj)
            if (kv.first == key) return &kv.second;  // (duplicate keys: the first, like most readers)
        return nullptr;
    }
};

constexpr int kMaxDepth = 64;
constexpr size_t kMaxConfigBytes = 1 << 20;

class JsonParser {
  public:
    explicit JsonParser(const std::string& s) : s_(s) {}
    bool parse(JVal& out, std::string& err) {
        if (!value(out, 0)) {
            err = "config.json: " + err_ + " at byte " + std::to_string(i_);
            return false;
        }
        ws();
        if (i_ != s_.size()) {
            err = "config.json: trailing bytes at byte " + std::to_string(i_);
            return false;
        }
        return true;
    }

  private:
    const std::string& s_;
    size_t i_ = 0;
    std::string err_;

    bool fail(const char* m) {
        err_ = m;
        return false;
    }
    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\t' || s_[i_] == '\r')) ++i_;
    }
    bool lit(const char* w) {
        const size_t n = std::strlen(w);
        if (s_.compare(i_, n, w) != 0) return fail("invalid literal");
        i_ += n;
        return true;
    }
    static int hex(char c) {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    }
    bool u4(unsigned& cp) {
        if (i_ + 4 > s_.size()) return fail("truncated \\u escape");
        cp = 0;
        for (int k = 0; k < 4; ++k) {
            const int h = hex(s_[i_ + k]);
            if (h < 0) return fail("bad \\u escape");
            cp = cp * 16 + (unsigned)h;
        }
        i_ += 4;
        return true;
    }
    static void utf8(unsigned cp, std::string& o) {
        if (cp < 0x80) {
            o.push_back((char)cp);
        } else if (cp < 0x800) {
            o.push_back((char)(0xC0 | (cp >> 6)));
            o.push_back((char)(0x80 | (cp & 0x3F)));
        } else if (cp < 0x10000) {
            o.push_back((char)(0xE0 | (cp >> 12)));
            o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            o.push_back((char)(0x80 | (cp & 0x3F)));
        } else {
            o.push_back((char)(0xF0 | (cp >> 18)));
            o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
            o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            o.push_back((char)(0x80 | (cp & 0x3F)));
        }
    }
    bool string(std::string& o) {
        if (i_ >= s_.size() || s_[i_] != '"') return fail("expected a string");
        ++i_;
        o.clear();
        while (true) {
            if (i_ >= s_.size()) return fail("unterminated string");
            const char c = s_[i_++];
            if (c == '"') return true;
            if ((unsigned char)c < 0x20) return fail("control character in string");
            if (c != '\\') {
                o.push_back(c);
                continue;
            }
            if (i_ >= s_.size()) return fail("unterminated escape");
            const char e = s_[i_++];
            switch (e) {
                case '"': o.push_back('"'); break;
                case '\\': o.push_back('\\'); break;
                case '/': o.push_back('/'); break;
                case 'b': o.push_back('\b'); break;
                case 'f': o.push_back('\f'); break;
                case 'n': o.push_back('\n'); break;
                case 'r': o.push_back('\r'); break;
                case 't': o.push_back('\t'); break;
                case 'u': {
                    unsigned cp;
                    if (!u4(cp)) return false;
                    if (cp >= 0xD800 && cp < 0xDC00 && i_ + 6 <= s_.size() && s_[i_] == '\\' && s_[i_ + 1] == 'u') {
                        i_ += 2;
                        unsigned lo;
                        if (!u4(lo)) return false;
                        if (lo < 0xDC00 || lo >= 0xE000) return fail("unpaired surrogate");
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    } else if (cp >= 0xD800 && cp < 0xE000) {
                        return fail("unpaired surrogate");
                    }
                    utf8(cp, o);
                    break;
                }
                default: return fail("bad escape");
            }
        }
    }
    bool number(double& v) {
        const size_t b = i_;
        if (i_ < s_.size() && s_[i_] == '-') ++i_;
        if (i_ >= s_.size() || !std::isdigit((unsigned char)s_[i_])) return fail("bad number");
        if (s_[i_] == '0') {
            ++i_;
        } else {
            while (i_ < s_.size() && std::isdigit((unsigned char)s_[i_])) ++i_;
        }
        if (i_ < s_.size() && s_[i_] == '.') {
            ++i_;
            if (i_ >= s_.size() || !std::isdigit((unsigned char)s_[i_])) return fail("bad fraction");
            while (i_ < s_.size() && std::isdigit((unsigned char)s_[i_])) ++i_;
        }
        if (i_ < s_.size() && (s_[i_] == 'e' || s_[i_] == 'E')) {
            ++i_;
            if (i_ < s_.size() && (s_[i_] == '+' || s_[i_] == '-')) ++i_;
            if (i_ >= s_.size() || !std::isdigit((unsigned char)s_[i_])) return fail("bad exponent");
            while (i_ < s_.size() && std::isdigit((unsigned char)s_[i_])) ++i_;
        }
        const std::string tok = s_.substr(b, i_ - b);
        v = std::strtod(tok.c_str(), nullptr);
        return true;
    }
    bool value(JVal& v, int depth) {
        if (depth > kMaxDepth) return fail("nesting too deep");
        ws();
        if (i_ >= s_.size()) return fail("unexpected end");
        const char c = s_[i_];
        if (c == '{') {
            ++i_;
            v.kind = JVal::OBJ;
            ws();
            if (i_ < s_.size() && s_[i_] == '}') {
                ++i_;
                return true;
            }
            while (true) {
                ws();
                std::string k;
                if (!string(k)) return false;
                ws();
                if (i_ >= s_.size() || s_[i_] != ':') return fail("expected ':'");
                ++i_;
                v.obj.emplace_back(std::move(k), JVal());
                if (!value(v.obj.back().second, depth + 1)) return false;
                ws();
                if (i_ < s_.size() && s_[i_] == ',') {
                    ++i_;
                    continue;
                }
                if (i_ < s_.size() && s_[i_] == '}') {
                    ++i_;
                    return true;
                }
                return fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            ++i_;
            v.kind = JVal::ARR;
            ws();
            if (i_ < s_.size() && s_[i_] == ']') {
                ++i_;
                return true;
            }
            while (true) {
                v.arr.emplace_back();
                if (!value(v.arr.back(), depth + 1)) return false;
                ws();
                if (i_ < s_.size() && s_[i_] == ',') {
                    ++i_;
                    continue;
                }
                if (i_ < s_.size() && s_[i_] == ']') {
                    ++i_;
                    return true;
                }
                return fail("expected ',' or ']'");
            }
        }
        if (c == '"') {
            v.kind = JVal::STR;
            return string(v.str);
        }
        if (c == 't') {
            v.kind = JVal::BOOL;
            v.b = true;
            return lit("true");
        }
        if (c == 'f') {
            v.kind = JVal::BOOL;
            v.b = false;
            return lit("false");
        }
        if (c == 'n') {
            v.kind = JVal::NUL;
            return lit("null");
        }
        v.kind = JVal::NUM;
        return number(v.num);
    }
};

// field readers: absent (or, for `nullable`, null) leaves *dst alone
int get_int(const JVal& root, const char* key, int32_t* dst, bool nullable = false) {
    const JVal* v = root.get(key);
    if (!v || (nullable && v->kind == JVal::NUL)) return MIMI_OK;
    if (v->kind == JVal::BOOL) {  // Python: True == 1 (not a config anyone writes, but the same value)
        *dst = v->b ? 1 : 0;
        return MIMI_OK;
    }
    if (v->kind != JVal::NUM || v->num != std::floor(v->num) || std::fabs(v->num) > 2147483647.0)
        return set_last_error(MIMI_ERR_IO, std::string("config.json: ") + key + " must be an integer");
    *dst = (int32_t)v->num;
    return MIMI_OK;
}

int get_num(const JVal& root, const char* key, double* dst) {
    const JVal* v = root.get(key);
    if (!v) return MIMI_OK;
    if (v->kind != JVal::NUM) return set_last_error(MIMI_ERR_IO, std::string("config.json: ") + key + " must be a number");
    *dst = v->num;
    return MIMI_OK;
}

// a boolean / string architecture switch that must have the kyutai/mimi value when present
int require_bool(const JVal& root, const char* key, bool want, const char* msg) {
    const JVal* v = root.get(key);
    if (!v) return MIMI_OK;
    const bool val = v->kind == JVal::BOOL ? v->b : (v->kind == JVal::NUM ? v->num != 0.0 : false);
    if ((v->kind != JVal::BOOL && v->kind != JVal::NUM) || val != want)
        return set_last_error(MIMI_ERR_UNSUPPORTED, std::string("unsupported Mimi config: ") + msg);
    return MIMI_OK;
}
int require_str(const JVal& root, const char* key, const char* want, const char* msg) {
    const JVal* v = root.get(key);
    if (!v) return MIMI_OK;
    if (v->kind != JVal::STR || v->str != want)
        return set_last_error(MIMI_ERR_UNSUPPORTED, std::string("unsupported Mimi config: ") + msg);
    return MIMI_OK;
}

bool is_dir(const std::string& p) {
    struct stat st;
    return ::stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}
bool is_file(const std::string& p) {
    struct stat st;
    return ::stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

}  // namespace

int config_from_json_text(const std::string& text, mimi_config* cfg) {
    JVal root;
    std::string err;
    if (!JsonParser(text).parse(root, err)) return set_last_error(MIMI_ERR_IO, err);
    if (root.kind != JVal::OBJ) return set_last_error(MIMI_ERR_IO, "config.json: not a JSON object");
    mimi_config c;
    mimi_config_default(&c);
    int rc = MIMI_OK;
#define INT_FIELD(key, field) \
    if ((rc = get_int(root, key, &c.field))) return rc;
    INT_FIELD("sampling_rate", sampling_rate)
    INT_FIELD("audio_channels", audio_channels)
    INT_FIELD("hidden_size", hidden_size)
    INT_FIELD("num_filters", num_filters)
    INT_FIELD("kernel_size", kernel_size)
    INT_FIELD("last_kernel_size", last_kernel_size)
    INT_FIELD("residual_kernel_size", residual_kernel_size)
    INT_FIELD("compress", compress)
    INT_FIELD("codebook_size", codebook_size)
    INT_FIELD("codebook_dim", codebook_dim)
    INT_FIELD("num_quantizers", num_quantizers)
    INT_FIELD("num_semantic_quantizers", num_semantic_quantizers)
    INT_FIELD("vector_quantization_hidden_dimension", vq_hidden_dim)
    INT_FIELD("num_hidden_layers", num_hidden_layers)
    INT_FIELD("intermediate_size", intermediate_size)
    INT_FIELD("num_attention_heads", num_attention_heads)
    INT_FIELD("sliding_window", sliding_window)
#undef INT_FIELD
    if (const JVal* r = root.get("upsampling_ratios")) {
        if (r->kind != JVal::NUL) {  // null / empty: the default [8, 6, 5, 4] (TF/configuration_mimi.py:128)
            if (r->kind != JVal::ARR || r->arr.size() > 8)
                return set_last_error(MIMI_ERR_UNSUPPORTED, "config.json: upsampling_ratios must be a list of <= 8 ints");
            if (!r->arr.empty()) {
                c.num_ratios = (int32_t)r->arr.size();
                for (size_t k = 0; k < r->arr.size(); ++k) {
                    const JVal& x = r->arr[k];
                    if (x.kind != JVal::NUM || x.num != std::floor(x.num) || x.num < 1 || x.num > 1024)
                        return set_last_error(MIMI_ERR_IO, "config.json: upsampling_ratios must hold positive ints");
                    c.upsampling_ratios[k] = (int32_t)x.num;
                }
                for (size_t k = r->arr.size(); k < 8; ++k) c.upsampling_ratios[k] = 0;
            }
        }
    }
    int32_t head_dim = 0, kv_heads = c.num_attention_heads, residual_layers = 1;
    if ((rc = get_int(root, "head_dim", &head_dim, true))) return rc;
    if ((rc = get_int(root, "num_key_value_heads", &kv_heads))) return rc;
    if ((rc = get_int(root, "num_residual_layers", &residual_layers))) return rc;
    if (c.num_attention_heads <= 0) return set_last_error(MIMI_ERR_UNSUPPORTED, "config.json: num_attention_heads must be > 0");
    c.head_dim = head_dim ? head_dim : c.hidden_size / c.num_attention_heads;
    double eps = c.norm_eps, theta = c.rope_theta;
    if ((rc = get_num(root, "norm_eps", &eps))) return rc;
    if (const JVal* rp = root.get("rope_parameters"); rp && rp->kind == JVal::OBJ)
        if ((rc = get_num(*rp, "rope_theta", &theta))) return rc;
    if ((rc = get_num(root, "rope_theta", &theta))) return rc;
    c.norm_eps = (float)eps;
    c.rope_theta = (float)theta;

    // MimiConfig.validate_supported (the Python host's check, same order and wording)
    std::vector<std::string> problems;
    auto note = [&](int st) {
        if (st) problems.push_back(mimi_last_error() + std::strlen("unsupported Mimi config: "));
    };
    if (c.audio_channels != 1) problems.push_back("audio_channels must be 1 (mono)");
    note(require_bool(root, "use_causal_conv", true, "use_causal_conv must be True"));
    note(require_str(root, "pad_mode", "constant", "pad_mode must be 'constant'"));
    note(require_bool(root, "use_conv_shortcut", false, "use_conv_shortcut must be False"));
    if (residual_layers != 1) problems.push_back("num_residual_layers must be 1");
    note(require_str(root, "hidden_act", "gelu", "hidden_act must be 'gelu'"));
    note(require_bool(root, "attention_bias", false, "attention_bias must be False"));
    if (kv_heads != c.num_attention_heads)
        problems.push_back("GQA (num_key_value_heads != num_attention_heads) is not supported");
    if (c.head_dim * c.num_attention_heads != c.hidden_size)
        problems.push_back("head_dim * num_attention_heads must equal hidden_size");
    if (!problems.empty()) {
        std::string m = "unsupported Mimi config: ";
        for (size_t k = 0; k < problems.size(); ++k) m += (k ? "; " : "") + problems[k];
        return set_last_error(MIMI_ERR_UNSUPPORTED, m);
    }

    // the downsample conv's kernel from the frame rates (Python float arithmetic = double)
    double prod = 1.0;
    for (int k = 0; k < c.num_ratios; ++k) prod *= c.upsampling_ratios[k];
    if (c.sampling_rate <= 0) return set_last_error(MIMI_ERR_UNSUPPORTED, "config.json: sampling_rate must be > 0");
    const double encodec_rate = std::ceil((double)c.sampling_rate / prod);
    double frame_rate = (double)c.sampling_rate / (prod * 2.0);
    if (const JVal* fr = root.get("frame_rate"); fr && fr->kind != JVal::NUL) {
        if (fr->kind != JVal::NUM || !(fr->num > 0)) return set_last_error(MIMI_ERR_IO, "config.json: frame_rate must be a positive number");
        frame_rate = fr->num;
    }
    const double ratio = encodec_rate / frame_rate;
    if (!(ratio >= 1.0 && ratio < 64.0)) return set_last_error(MIMI_ERR_UNSUPPORTED, "config.json: frame_rate out of range");
    c.downsample_kernel = 2 * (int32_t)ratio;
    c.downsample_stride = 2;
    *cfg = c;
    return MIMI_OK;
}

int find_checkpoint(const char* path, std::string& config_json, std::string& safetensors) {
    config_json.clear();
    safetensors.clear();
    const std::string p(path);
    if (is_file(p)) {  // a .safetensors file on its own: the default config (MimiHipModel.from_pretrained)
        safetensors = p;
        return MIMI_OK;
    }
    if (!is_dir(p)) return set_last_error(MIMI_ERR_IO, "checkpoint " + p + " does not exist");
    if (is_file(p + "/config.json")) config_json = p + "/config.json";
    std::unique_ptr<DIR, int (*)(DIR*)> d(::opendir(p.c_str()), ::closedir);
    if (!d) return set_last_error(MIMI_ERR_IO, "cannot list " + p);
    std::vector<std::string> files;
    while (const dirent* ent = ::readdir(d.get())) {
        const std::string n = ent->d_name;
        const std::string suf = ".safetensors";
        if (n.empty() || n[0] == '.' || n.size() <= suf.size()) continue;  // (glob skips dot files)
        if (n.compare(n.size() - suf.size(), suf.size(), suf) == 0 && is_file(p + "/" + n)) files.push_back(n);
    }
    if (files.empty()) return set_last_error(MIMI_ERR_IO, "no .safetensors file in " + p);
    std::sort(files.begin(), files.end());  // sorted(glob(...))[0]
    safetensors = p + "/" + files[0];
    return MIMI_OK;
}

}  // namespace mimi

extern "C" void mimi_config_default(mimi_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->sampling_rate = 24000;
    c->audio_channels = 1;
    c->hidden_size = 512;
    c->num_filters = 64;
    c->num_ratios = 4;
    c->upsampling_ratios[0] = 8;
    c->upsampling_ratios[1] = 6;
    c->upsampling_ratios[2] = 5;
    c->upsampling_ratios[3] = 4;
    c->kernel_size = 7;
    c->last_kernel_size = 3;
    c->residual_kernel_size = 3;
    c->compress = 2;
    c->codebook_size = 2048;
    c->codebook_dim = 256;
    c->num_quantizers = 32;
    c->num_semantic_quantizers = 1;
    c->vq_hidden_dim = 256;
    c->num_hidden_layers = 8;
    c->intermediate_size = 2048;
    c->num_attention_heads = 8;
    c->head_dim = 64;
    c->sliding_window = 250;
    c->downsample_kernel = 4;
    c->downsample_stride = 2;
    c->norm_eps = 1e-5f;
    c->rope_theta = 10000.0f;
    c->codebook_eps = 1e-5f;
}

extern "C" int mimi_config_from_json(const char* path, mimi_config* cfg) {
    if (!path || !cfg) return mimi::set_last_error(MIMI_ERR_INVALID_ARGUMENT, "null argument");
    std::string p(path);
    if (mimi::is_dir(p)) p += "/config.json";
    std::ifstream f(p, std::ios::binary);
    if (!f) return mimi::set_last_error(MIMI_ERR_IO, "cannot open " + p);
    std::string text;
    char buf[65536];
    while (f.read(buf, sizeof(buf)) || f.gcount() > 0) {
        text.append(buf, (size_t)f.gcount());
        if (text.size() > mimi::kMaxConfigBytes) return mimi::set_last_error(MIMI_ERR_IO, p + ": larger than 1 MiB");
    }
    return mimi::config_from_json_text(text, cfg);
}
