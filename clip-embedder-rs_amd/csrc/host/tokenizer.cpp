// placeholder, replaced by the CLIP BPE tokenizer
#include <cstdint>
#include "../../../include/clipgpu.h"
#include "api_util.hpp"
using namespace clipgpu;
struct clipgpu_tokenizer { int dummy; };
extern "C" {
int clipgpu_tokenizer_create(const char*, int, int64_t, clipgpu_tokenizer** out) {
  return guarded([&]() { if (out) *out = nullptr; throw ClipErr(CLIPGPU_ERR_TOKENIZER, "tokenizer not built"); });
}
void clipgpu_tokenizer_destroy(clipgpu_tokenizer* t) { delete t; }
int clipgpu_tokenize(clipgpu_tokenizer*, const char* const*, int64_t, int, int64_t*, int64_t*) {
  return guarded([&]() { throw ClipErr(CLIPGPU_ERR_TOKENIZER, "tokenizer not built"); });
}
int64_t clipgpu_tokenizer_token_id(const clipgpu_tokenizer*, const char*) { return -1; }
int64_t clipgpu_tokenizer_vocab_size(const clipgpu_tokenizer*) { return -1; }
}
