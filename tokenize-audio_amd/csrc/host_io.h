// Host-only readers of untrusted input (no HIP): the safetensors checkpoint reader (safetensors.cpp).  Kept out of
// the HIP translation units so tools/asan can build them under AddressSanitizer / UBSan (with flac.cpp).
#pragma once
#include <cstdint>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "../../include/mimi_hip.h"

namespace mimi {

struct StTensor {
    std::string dtype;
    std::vector<int64_t> shape;
    int64_t begin = 0, end = 0, numel = 0;
};

// Parses a safetensors JSON header; every entry's offsets must lie inside the data_bytes that follow the header
// and match dtype x shape.  false + err on anything malformed.
bool st_parse_header(const std::string& hdr, int64_t data_bytes, std::map<std::string, StTensor>& out,
                     std::string& err);

// Reads every tensor `wanted` accepts from the safetensors file at path as fp32 into out.  MIMI_OK, MIMI_ERR_IO
// (unreadable / malformed / truncated) or MIMI_ERR_WEIGHTS (a wanted tensor that is not F32), with err set.
int st_load(const char* path, const std::function<bool(const std::string&)>& wanted,
            std::map<std::string, std::vector<float>>& out, std::string& err);

// config_json.cpp: config.json text -> mimi_config (MIMI_OK, MIMI_ERR_IO for malformed JSON or a field of the
// wrong type, MIMI_ERR_UNSUPPORTED for an architecture the engine does not implement), and the checkpoint scan of
// mimi_create_from_dir: a directory's config.json (empty when absent) and its first *.safetensors in byte order, or
// a lone file as the checkpoint.
int config_from_json_text(const std::string& text, ::mimi_config* cfg);
int find_checkpoint(const char* path, std::string& config_json, std::string& safetensors);

}  // namespace mimi
