// Sanitizer harness for the host code that parses untrusted bytes: the FLAC decoder (csrc/flac.cpp), the
// safetensors checkpoint reader (csrc/safetensors.cpp) and the config.json reader (csrc/config_json.cpp), built with -fsanitize=address,undefined by
// tools/asan/Makefile and driven by tests/test_sanitizers.py (CPU only: the GPU pool has no GPU sanitizers).
//
//   host_fuzz [--mutations N] file...
//
// Each file is decoded as is, then N deterministic mutations of it (byte flips, truncations, inserted and deleted
// bytes, a corrupted length field) -- every call must return a status, never read or write out of bounds (the
// sanitizers abort the process on any such access).  For a well-formed input the first line per file reports the
// status and a checksum of the decoded output, so the test can compare it with the expected PCM / tensors.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <algorithm>
#include <fstream>
#include <iterator>
#include <map>
#include <string>
#include <vector>

#include "../../include/mimi_hip.h"
#include "../../tokenize-audio_amd/csrc/host_io.h"

namespace mimi {
// engine.cpp's thread-local last error (not linked here)
static std::string g_err;
int set_last_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
}  // namespace mimi
extern "C" const char* mimi_last_error(void) { return mimi::g_err.c_str(); }

static uint64_t fnv(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

static bool ends_with(const std::string& s, const char* suf) {
    const size_t n = std::strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

static std::string tmp_path() {
    const char* d = std::getenv("TMPDIR");
    return std::string(d ? d : "/tmp") + "/host_fuzz_" + std::to_string(::getpid()) + ".safetensors";
}

// returns the status and a checksum of the decoded content
static int run_flac(const std::vector<uint8_t>& d, uint64_t* sum) {
    int32_t rate = 0, ch = 0, bps = 0;
    int64_t total = 0;
    int st = mimi_flac_info(d.data(), (int64_t)d.size(), &rate, &ch, &bps, &total);
    if (st) return st;
    int64_t n = 0;
    st = mimi_flac_decode(d.data(), (int64_t)d.size(), nullptr, 0, &n);
    if (st) return st;
    if (n < 0 || ch < 1 || ch > 8 || n > (int64_t)1 << 26) return -1;
    std::vector<int32_t> pcm((size_t)(ch * n) + 1);
    st = mimi_flac_decode(d.data(), (int64_t)d.size(), pcm.data(), n, &n);
    if (st) return st;
    *sum = fnv(pcm.data(), (size_t)(ch * n) * 4);
    return 0;
}

static int run_st(const std::vector<uint8_t>& d, uint64_t* sum) {
    const std::string p = tmp_path();
    {
        std::ofstream f(p, std::ios::binary | std::ios::trunc);
        f.write(reinterpret_cast<const char*>(d.data()), (std::streamsize)d.size());
    }
    std::map<std::string, std::vector<float>> out;
    std::string err;
    const int st = mimi::st_load(p.c_str(), [](const std::string&) { return true; }, out, err);
    std::remove(p.c_str());
    uint64_t h = 1469598103934665603ull;
    for (const auto& kv : out) {
        h = fnv(kv.first.data(), kv.first.size(), h);
        h = fnv(kv.second.data(), kv.second.size() * 4, h);
    }
    *sum = h;
    return st;
}

// config.json (config_json.cpp): the status and a checksum of the struct it fills
static int run_cfg(const std::vector<uint8_t>& d, uint64_t* sum) {
    mimi_config c;
    std::memset(&c, 0, sizeof(c));
    const int st = mimi::config_from_json_text(std::string(d.begin(), d.end()), &c);
    *sum = st ? 0 : fnv(&c, sizeof(c));
    return st;
}

int main(int argc, char** argv) {
    int mutations = 200;
    std::vector<std::string> files;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--mutations") && i + 1 < argc)
            mutations = std::atoi(argv[++i]);
        else
            files.push_back(argv[i]);
    }
    uint64_t rng = 0x9E3779B97F4A7C15ull;
    auto next = [&]() {
        rng ^= rng << 13;
        rng ^= rng >> 7;
        rng ^= rng << 17;
        return rng;
    };
    long runs = 0;
    for (const auto& fn : files) {
        std::ifstream f(fn, std::ios::binary);
        std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        const bool flac = ends_with(fn, ".flac"), json = ends_with(fn, ".json");
        auto run = [&](const std::vector<uint8_t>& x, uint64_t* s) {
            return flac ? run_flac(x, s) : json ? run_cfg(x, s) : run_st(x, s);
        };
        uint64_t sum = 0;
        const int st = run(d, &sum);
        std::printf("%s status=%d sum=%016llx\n", fn.c_str(), st, (unsigned long long)sum);
        int failed = 0;
        for (int m = 0; m < mutations; ++m) {
            std::vector<uint8_t> x = d;
            const int kind = (int)(next() % 6);
            const size_t n = x.size();
            if (n == 0) break;
            const size_t at = (size_t)(next() % n);
            if (kind == 0) {
                x[at] ^= (uint8_t)(1u << (next() % 8));
            } else if (kind == 1) {
                x.resize(at);
            } else if (kind == 2) {
                x.insert(x.begin() + (long)at, (uint8_t)next());
            } else if (kind == 3) {
                x.erase(x.begin() + (long)at);
            } else if (kind == 4) {  // a multi-byte field overwritten (lengths, counts, offsets)
                for (size_t k = at; k < std::min(n, at + 8); ++k) x[k] = (uint8_t)next();
            } else {  // header region: the first 64 bytes
                x[at % std::min<size_t>(n, 64)] = (uint8_t)next();
            }
            uint64_t s2 = 0;
            if (run(x, &s2) != 0) ++failed;
            ++runs;
        }
        std::printf("%s mutations=%d rejected=%d\n", fn.c_str(), mutations, failed);
    }
    std::printf("runs=%ld ok\n", runs);
    return 0;
}
