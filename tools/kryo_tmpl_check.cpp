// Host check of the GPU encoder's template scheme (kryo_template.hpp), built by
// tests/test_kryo_template.py with g++: groups items by shape exactly as the
// GPU does (shape_hash_of picks the slot, the first item's ShapeRec is the
// slot's record, shape_matches confirms the others), traces the first item of each shape
// (trace_leaf) and rebuilds EVERY item of the shape from those symbols
// (sym_byte), comparing with the direct encoder (encode_leaf) byte for byte.
// stats: [0] shapes, [1] items rebuilt from a template, [2] items without a
// shape (direct encoder), [3] items of invalid shapes, [4] mismatches,
// [5] items whose template was unusable (trace beyond its buffer).
#include <cstdint>
#include <cstring>
#include <vector>

#include "../corda_amd/csrc/kryo_template.hpp"

using namespace cordahip::kryo;

namespace {

struct Rep {
  uint64_t hash;
  ShapeRec rec;
  int64_t size;  // -1 invalid, -2 no template
  std::vector<uint32_t> syms;
};

bool direct(const cordahip_kryo_item& it, std::vector<uint8_t>& leaf) {
  std::vector<uint8_t> levels(kLevelBytes);
  for (;;) {
    Kout o(leaf.data(), leaf.size(), levels.data());
    if (!encode_leaf(o, it)) return false;
    if (o.pos <= leaf.size()) {
      leaf.resize(o.pos);
      return true;
    }
    leaf.resize(o.pos);
  }
}

}  // namespace

extern "C" int kryo_template_check(const cordahip_kryo_item* items, uint64_t n, uint64_t cap_syms,
                                   uint64_t* stats) {
  std::vector<Rep> reps;
  std::vector<uint32_t> levels(kLevelBytes);
  for (int i = 0; i < 6; i++) stats[i] = 0;
  for (uint64_t i = 0; i < n; i++) {
    const cordahip_kryo_item& it = items[i];
    uint64_t h = 0;
    std::vector<uint8_t> want(1 << 12);
    const bool ok = direct(it, want);
    if (!shape_hash_of(it, h)) {
      stats[2]++;
      continue;
    }
    Rep* r = nullptr;
    for (Rep& x : reps)
      if (x.hash == h) {
        r = &x;
        break;
      }
    if (!r) {
      Rep x;
      x.hash = h;
      ShapeRecord rv(x.rec);
      shape_walk(it, rv);
      x.syms.assign(cap_syms, 0);
      x.size = x.rec.ok ? trace_leaf(it, x.syms.data(), cap_syms, levels.data()) : -2;
      reps.push_back(std::move(x));
      r = &reps.back();
      stats[0]++;
    }
    if (!shape_matches(it, r->rec)) {  // a hash collision, or a shape too big to record: direct encoder
      stats[2]++;
      continue;
    }
    if (r->size == -1) {  // invalid shape: the direct encoder must reject the item too
      stats[3]++;
      if (ok) stats[4]++;
      continue;
    }
    if (r->size == -2) {
      stats[5]++;
      continue;
    }
    stats[1]++;
    if (!ok || (int64_t)want.size() != r->size) {
      stats[4]++;
      continue;
    }
    for (int64_t p = 0; p < r->size; p++)
      if (sym_byte(r->syms[p], it.data, it.value) != want[p]) {
        stats[4]++;
        break;
      }
  }
  return stats[4] == 0 ? 0 : 1;
}
