// Mutation fuzzer of the Kryo encoder core (kryo_core.hpp, kryo_template.hpp) on the
// host, built by tests/test_kryo_fuzz.py with g++ -fsanitize=address,undefined
// together with the host entry point (corda_amd/csrc/kryo.cpp) and the template
// check (tools/kryo_tmpl_check.cpp). The same core runs on the GPU; the items come
// from the JVM, so every payload byte, length, kind and class id is untrusted.
//
// Seeds: a file of valid items (kind u32, class_id u32, value i64, len u64, nbytes
// u64, payload) the test writes with corda_amd._lib.kryo_pack. Each round takes a
// seed and builds a batch of mutants of it -- byte flips, truncated or extended
// lengths, another kind / class id / value, a missing payload, or the seed
// unchanged (so batches share shapes and the template path runs) -- each payload
// in its own heap block of exactly the bytes the item may read (len, or 2 len for
// String / kotlin_object), so any read past it is an ASan report. Per batch:
//   1. cordahip_kryo_encode item by item: the size pass (out = NULL), the write
//      into an exact buffer (off[1] must agree), a write into a buffer one byte
//      short (BUFFER_TOO_SMALL, nothing past cap touched);
//   2. the whole batch at once (INVALID_ARG exactly when some item is invalid);
//   3. kryo_template_check: every item rebuilt from its shape's template equals
//      the direct encoder's leaf (the GPU's scheme against the direct encoder).
// Exit 0 when every check holds; a sanitizer report aborts the process.
//
// usage: kryo_fuzz SEEDS_FILE ROUNDS RNG_SEED [--dump OUT]
//   --dump: also write every mutant and the host encoder's result for it (kind u32,
//   class_id u32, value i64, len u64, nbytes u64, has_data u8, payload; valid u8,
//   leaf size u64, leaf, templated u8 (the item alone rebuilds from a template, or a
//   valid RAW item), shape hash u64 (0: none), exact-shape fingerprint u64) for the device encoder's agreement run
//   (tools/agree_kryo_fuzz.py).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "../corda_amd/csrc/kryo_template.hpp"

extern "C" int kryo_template_check(const cordahip_kryo_item* items, uint64_t n, uint64_t cap_syms, uint64_t* stats);

namespace {

struct Seed {
  uint32_t kind, class_id;
  int64_t value;
  uint64_t len;
  std::vector<uint8_t> bytes;
};

struct Rng {
  uint64_t s;
  uint64_t next() {  // splitmix64
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

bool wide(uint32_t kind) { return kind == CORDAHIP_KRYO_STRING || kind == CORDAHIP_KRYO_KOTLIN_OBJECT; }

// the bytes an item of this kind and len may read
uint64_t payload_bytes(uint32_t kind, uint64_t len) { return wide(kind) ? 2 * len : len; }

struct Mutant {
  cordahip_kryo_item it;
  std::unique_ptr<uint8_t[]> buf;  // exactly payload_bytes (nullptr when 0 or dropped)
};

Mutant mutate(const Seed& sd, Rng& r) {
  Mutant m;
  uint32_t kind = sd.kind, cls = sd.class_id;
  int64_t value = sd.value;
  uint64_t len = sd.len;
  std::vector<uint8_t> b = sd.bytes;
  bool drop = false;
  const uint64_t nops = 1 + r.below(3) * r.below(2);  // mostly one mutation, up to three stacked
  for (uint64_t q = 0; q < nops; q++) {
    const uint64_t op = r.below(10);
    if (op == 0 || op == 1) {  // byte flips, more often near the front (headers, counts, lengths)
      const uint64_t k = 1 + r.below(4);
      for (uint64_t j = 0; j < k && !b.empty(); j++) {
        const uint64_t p = r.below(2) ? r.below(b.size() < 16 ? b.size() : 16) : r.below(b.size());
        b[p] ^= (uint8_t)(1u << r.below(8));
        if (r.below(4) == 0) b[p] = (uint8_t)r.next();
      }
    } else if (op == 2) {  // truncated
      len = r.below(len + 1);
    } else if (op == 3) {  // extended with random bytes
      len += 1 + r.below(r.below(8) ? 16 : 600);
    } else if (op == 4) {  // another kind (its own payload semantics over these bytes)
      kind = (uint32_t)r.below(18);
    } else if (op == 5) {
      cls = r.below(2) ? (uint32_t)r.below(300) : (uint32_t)r.next();
    } else if (op == 6) {
      value = r.below(2) ? (int64_t)r.next() : (int64_t)r.below(300) - 150;
    } else if (op == 7) {
      drop = true;  // data = NULL with the seed's len
    }  // 8, 9: the seed unchanged
  }
  const uint64_t nb = payload_bytes(kind, len);
  if (nb > (1u << 20)) len = 0;  // keep blocks small
  const uint64_t nbytes = payload_bytes(kind, len);
  b.resize(nbytes);
  for (uint64_t p = sd.bytes.size(); p < nbytes; p++) b[p] = (uint8_t)r.next();
  m.it.kind = kind;
  m.it.class_id = cls;
  m.it.value = value;
  m.it.len = len;
  m.it.data = nullptr;
  if (!drop && nbytes) {
    m.buf.reset(new uint8_t[nbytes]);
    std::memcpy(m.buf.get(), b.data(), nbytes);
    m.it.data = m.buf.get();
  } else if (!drop && sd.bytes.size() && r.below(2)) {
    m.buf.reset(new uint8_t[1]);  // len 0 with a non-null pointer to a 1-byte block
    m.it.data = m.buf.get();
  }
  return m;
}

bool read_seeds(const char* path, std::vector<Seed>& out) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  for (;;) {
    Seed s;
    uint64_t nbytes = 0;
    if (std::fread(&s.kind, 4, 1, f) != 1) break;
    if (std::fread(&s.class_id, 4, 1, f) != 1 || std::fread(&s.value, 8, 1, f) != 1 ||
        std::fread(&s.len, 8, 1, f) != 1 || std::fread(&nbytes, 8, 1, f) != 1) {
      std::fclose(f);
      return false;
    }
    s.bytes.resize(nbytes);
    if (nbytes && std::fread(s.bytes.data(), 1, nbytes, f) != nbytes) {
      std::fclose(f);
      return false;
    }
    out.push_back(std::move(s));
  }
  std::fclose(f);
  return !out.empty();
}

int fail(const char* what, uint64_t round, uint64_t i) {
  std::fprintf(stderr, "kryo_fuzz: %s (round %llu, item %llu)\n", what, (unsigned long long)round,
               (unsigned long long)i);
  return 1;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 4 && !(argc == 6 && std::strcmp(argv[4], "--dump") == 0)) {
    std::fprintf(stderr, "usage: kryo_fuzz SEEDS ROUNDS RNG_SEED [--dump OUT]\n");
    return 2;
  }
  FILE* dump = argc == 6 ? std::fopen(argv[5], "wb") : nullptr;
  if (argc == 6 && !dump) return fail("cannot open the dump file", 0, 0);
  std::vector<Seed> seeds;
  if (!read_seeds(argv[1], seeds)) return fail("bad seeds file", 0, 0);
  const uint64_t rounds = std::strtoull(argv[2], nullptr, 10);
  Rng r{std::strtoull(argv[3], nullptr, 10)};
  uint64_t items = 0, valid = 0, templated = 0, shapes = 0, bytes = 0;
  for (uint64_t round = 0; round < rounds; round++) {
    const Seed& sd = seeds[r.below(seeds.size())];
    const uint64_t n = 1 + r.below(24);
    std::vector<Mutant> ms;
    std::vector<cordahip_kryo_item> batch;
    for (uint64_t i = 0; i < n; i++) {
      ms.push_back(mutate(sd, r));
      batch.push_back(ms.back().it);
    }
    bool all_ok = true;
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; i++) {
      uint64_t off[2] = {7, 7};
      const int rc = cordahip_kryo_encode(&batch[i], 1, nullptr, 0, off);
      if (dump) {
        const cordahip_kryo_item& it = batch[i];
        const uint64_t nbytes = it.data ? payload_bytes(it.kind, it.len) : 0;
        const uint8_t has = it.data != nullptr;
        std::fwrite(&it.kind, 4, 1, dump);
        std::fwrite(&it.class_id, 4, 1, dump);
        std::fwrite(&it.value, 8, 1, dump);
        std::fwrite(&it.len, 8, 1, dump);
        std::fwrite(&nbytes, 8, 1, dump);
        std::fwrite(&has, 1, 1, dump);
        if (nbytes) std::fwrite(it.data, 1, nbytes, dump);
        const uint8_t valid = rc != CORDAHIP_ERR_INVALID_ARG;
        const uint64_t size = valid ? off[1] : 0;
        std::vector<uint8_t> leaf(size ? size : 1);
        if (size && cordahip_kryo_encode(&it, 1, leaf.data(), size, off) != CORDAHIP_SUCCESS)
          return fail("dump write", round, i);
        std::fwrite(&valid, 1, 1, dump);
        std::fwrite(&size, 8, 1, dump);
        if (size) std::fwrite(leaf.data(), 1, size, dump);
        uint64_t tst[6], h = 0;
        // 4096: the GPU arena's template size (kryo_device.hip kTmplSyms)
        const bool templ = kryo_template_check(&it, 1, 4096, tst) == 0 && tst[1] == 1;
        const uint8_t tb = templ || (valid && it.kind == CORDAHIP_KRYO_RAW);
        if (!cordahip::kryo::shape_hash_of(it, h)) h = 0;
        // the exact shape (the record the GPU compares), FNV-1a over its used part: two
        // shapes under one hash make the second one go direct
        uint64_t fp = 1469598103934665603ull;
        if (h) {
          cordahip::kryo::ShapeRec rec;
          std::memset(&rec, 0, sizeof rec);
          cordahip::kryo::ShapeRecord rv(rec);
          cordahip::kryo::shape_walk(it, rv);
          auto mix = [&](const void* p, size_t nb) {
            for (size_t q = 0; q < nb; q++) fp = (fp ^ static_cast<const uint8_t*>(p)[q]) * 1099511628211ull;
          };
          mix(&rec.nw, 16);
          mix(rec.w, 4 * (rec.nw < rec.kWords ? rec.nw : rec.kWords));
          mix(rec.sl, 4 * (rec.ns < rec.kSpans ? rec.ns : rec.kSpans));
          mix(rec.so, 4 * (rec.ns < rec.kSpans ? rec.ns : rec.kSpans));
          mix(rec.bytes, rec.nb < rec.kBytes ? rec.nb : rec.kBytes);
        }
        std::fwrite(&tb, 1, 1, dump);
        std::fwrite(&h, 8, 1, dump);
        std::fwrite(&fp, 8, 1, dump);
      }
      if (rc == CORDAHIP_ERR_INVALID_ARG) {
        all_ok = false;
        continue;
      }
      if (off[0] != 0) return fail("off[0] != 0", round, i);
      const uint64_t size = off[1];
      if (size == 0 ? rc != CORDAHIP_SUCCESS : rc != CORDAHIP_ERR_BUFFER_TOO_SMALL)
        return fail("size pass status", round, i);
      std::unique_ptr<uint8_t[]> out(new uint8_t[size ? size : 1]);
      uint64_t off2[2];
      if (cordahip_kryo_encode(&batch[i], 1, out.get(), size, off2) != CORDAHIP_SUCCESS || off2[1] != size)
        return fail("exact write", round, i);
      if (size) {  // one byte short: BUFFER_TOO_SMALL, the same size, no write past cap (ASan)
        std::unique_ptr<uint8_t[]> shortb(new uint8_t[size - 1 ? size - 1 : 1]);
        if (cordahip_kryo_encode(&batch[i], 1, shortb.get(), size - 1, off2) != CORDAHIP_ERR_BUFFER_TOO_SMALL ||
            off2[1] != size)
          return fail("short write", round, i);
      }
      valid++;
      total += size;
    }
    std::vector<uint64_t> off(n + 1);
    const int rc = cordahip_kryo_encode(batch.data(), n, nullptr, 0, off.data());
    if (all_ok ? (rc != (total ? CORDAHIP_ERR_BUFFER_TOO_SMALL : CORDAHIP_SUCCESS) || off[n] != total)
               : rc != CORDAHIP_ERR_INVALID_ARG)
      return fail("batch status", round, 0);
    uint64_t st[6];
    if (kryo_template_check(batch.data(), n, 1 << 14, st) != 0) return fail("template != direct encoder", round, 0);
    items += n;
    templated += st[1];
    shapes += st[0];
    bytes += total;
  }
  if (dump) std::fclose(dump);
  std::printf("{\"rounds\": %llu, \"items\": %llu, \"valid\": %llu, \"templated\": %llu, \"shapes\": %llu, "
              "\"leaf_bytes\": %llu}\n",
              (unsigned long long)rounds, (unsigned long long)items, (unsigned long long)valid,
              (unsigned long long)templated, (unsigned long long)shapes, (unsigned long long)bytes);
  return 0;
}
