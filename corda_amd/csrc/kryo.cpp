// Native Kryo leaf encoder, host entry point: the leaf
// preimages that serializedHash hashes (MerkleTransaction.kt:16-18), written by
// the encoder core shared with the GPU (kryo_core.hpp). Each leaf is built in a
// per-thread buffer and copied to its place in the caller's output while it has
// room; past that only the sizes are kept (CORDAHIP_ERR_BUFFER_TOO_SMALL with
// off[n] = the bytes needed).
#include <cstdint>
#include <cstring>
#include <vector>

#include "kryo_core.hpp"

namespace {

using cordahip::kryo::Kout;
using cordahip::kryo::kLevelBytes;

// one leaf into `leaf` (grown when a first pass did not fit); false for an
// invalid item
bool encode(const cordahip_kryo_item& it, std::vector<uint8_t>& leaf, uint64_t& size) {
  thread_local std::vector<uint8_t> levels(kLevelBytes);
  for (;;) {
    Kout o(leaf.data(), leaf.size(), levels.data());
    if (!cordahip::kryo::encode_leaf(o, it)) return false;
    size = o.pos;
    if (o.pos <= leaf.size()) return true;
    leaf.resize(o.pos);
  }
}

}  // namespace

extern "C" int cordahip_kryo_encode(const cordahip_kryo_item* items, uint64_t n, uint8_t* out, uint64_t cap,
                                    uint64_t* off) {
  if ((n && !items) || !off) return CORDAHIP_ERR_INVALID_ARG;
  thread_local std::vector<uint8_t> leaf(1 << 16);
  uint64_t pos = 0;
  off[0] = 0;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t size = 0;
    if (!encode(items[i], leaf, size)) return CORDAHIP_ERR_INVALID_ARG;
    if (out && pos + size <= cap && size) std::memcpy(out + pos, leaf.data(), size);
    pos += size;
    off[i + 1] = pos;
  }
  if (pos > cap || (pos && !out)) return CORDAHIP_ERR_BUFFER_TOO_SMALL;
  return CORDAHIP_SUCCESS;
}
