// Leaf shapes and templates for the GPU Kryo encoder (kryo_device.hip), on top
// of the encoder core (kryo_core.hpp).
//
// The bytes of a leaf depend on its item in two ways: through *structure* --
// the kind, the class ids, every length the encoder branches on (key, name,
// reference, currency-code lengths, the varint length of the value), flags,
// whether the owner and issuer keys are equal -- and through *content* bytes
// that the encoder copies verbatim (key bytes, X.500 name bytes, the reference,
// the legal-contract hash) or writes from the item's value (the quantity /
// nonce varlong, a primitive's big-endian bytes). Items with equal structure
// ("one shape") produce leaves of the same length whose bytes differ only where
// content lands, and the positions of that content are the same. So the GPU
// encodes ONE representative per shape in trace mode (KoutT<true>: every byte
// a symbol naming its source) and writes every other item of the shape from
// those symbols -- no per-item encoder run, no level buffers.
//
// The rule that makes this exact: any input the encoder *branches* on, or
// validates, is part of the shape; only bytes it copies verbatim or derives
// from `value` are content. Content that the encoder inspects is therefore put
// in the shape whole (the command class name, the currency code, STRING and
// KOTLIN_OBJECT text) or in part (the DER header of an X.500 name, which the
// party decode validates). same_shape() compares structure words and those
// spans byte for byte; the hash only picks the table slot.
// tests/test_kryo_template.py checks, on the host, every item of randomised
// batches rebuilt from its shape representative's symbols against the direct
// encoder.
#pragma once
#include "kryo_core.hpp"

namespace cordahip {
namespace kryo {

struct Shape {
  static constexpr uint32_t kWords = 32, kSpans = 4;
  uint32_t w[kWords];
  uint32_t nw = 0;
  const uint8_t* sp[kSpans];
  uint32_t sl[kSpans];
  uint32_t ns = 0;
  bool ok = true;  // false: no template (the item goes through the direct encoder)
  KRYO_HD void word(uint32_t x) {
    if (nw < kWords) w[nw++] = x;
    else ok = false;
  }
  KRYO_HD void span(const uint8_t* p, uint32_t n) {
    if (ns < kSpans && (p || !n)) {
      sp[ns] = p;
      sl[ns++] = n;
    } else {
      ok = false;
    }
  }
};

// bytes of Output.writeVarLong(zigzag(v)) (1..9): part of the shape of a VALUE_ZZ kind
KRYO_HD inline uint32_t varlong_zz_len(int64_t x) {
  uint64_t v = ((uint64_t)x << 1) ^ (uint64_t)(x >> 63);
  uint32_t m = 1;
  for (int i = 0; i < 8 && (v >> 7); i++) {
    v >>= 7;
    m++;
  }
  return m;
}

// a party of a CASH_STATE payload: its structure, and the DER header of its
// name (Reader::party validates the name's TLV)
KRYO_HD inline void shape_party(Shape& s, const PartyRef& p) {
  s.word(p.key_class);
  s.word(p.key_len);
  s.word(p.name_len);
  s.span(p.name, p.name_len < 6 ? p.name_len : 6);
}

// The shape of an item, or ok = false when it has none (RAW leaves are copied
// directly; unknown kinds, malformed payloads and outsized content go to the
// direct encoder, which also decides their validity).
KRYO_HD inline Shape shape_of(const cordahip_kryo_item& it) {
  Shape s;
  s.word(it.kind);
  s.word(it.class_id);
  switch (it.kind) {
    case CORDAHIP_KRYO_CHAR:
    case CORDAHIP_KRYO_SHORT:
    case CORDAHIP_KRYO_INT:
    case CORDAHIP_KRYO_LONG:
    case CORDAHIP_KRYO_BYTE:
    case CORDAHIP_KRYO_FLOAT:
    case CORDAHIP_KRYO_DOUBLE: break;  // value bytes only
    case CORDAHIP_KRYO_BOOLEAN: s.word(it.value != 0); break;
    case CORDAHIP_KRYO_STRING:
    case CORDAHIP_KRYO_KOTLIN_OBJECT:  // the text is transcoded (UTF-16 -> Kryo string): all of it is shape
      if (it.len > 512 || (it.len && !it.data)) {
        s.ok = false;
        break;
      }
      s.word((uint32_t)it.len);
      s.span(it.data, (uint32_t)(2 * it.len));
      break;
    case CORDAHIP_KRYO_ED25519_KEY:
    case CORDAHIP_KRYO_PUBLIC_KEY:
      if (!it.data || it.len >= kMaxPayloadOff) s.ok = false;
      s.word((uint32_t)it.len);
      break;
    case CORDAHIP_KRYO_PARTY:
      if (!it.data || it.len >= kMaxPayloadOff) {
        s.ok = false;
        break;
      }
      s.word((uint32_t)it.value);  // the key class (its varint is written)
      s.word((uint32_t)it.len);
      s.span(it.data, it.len < 6 ? (uint32_t)it.len : 6);  // der_tlv_len splits name | key on these
      break;
    case CORDAHIP_KRYO_ISSUE_COMMAND: {
      if (!it.data || it.len < 2 || it.len >= kMaxPayloadOff) {
        s.ok = false;
        break;
      }
      Reader r(it.data, it.data + it.len);
      const uint32_t nlen = r.u8();
      const uint8_t* nm = r.span(nlen);
      const uint32_t nkeys = r.u8();
      s.word(varlong_zz_len(it.value));
      s.word(nlen);
      s.span(nm, nlen);  // the class name: written, compared, and cut for the field name
      s.word(nkeys);
      for (uint32_t i = 0; i < nkeys && r.ok; i++) {
        s.word(r.u16());
        s.word(r.u16());
        r.span(s.w[s.nw - 1]);
      }
      if (!r.ok || r.p != r.end) s.ok = false;
      break;
    }
    case CORDAHIP_KRYO_CASH_STATE: {
      if (!it.data || it.len >= kMaxPayloadOff) {
        s.ok = false;
        break;
      }
      Reader r(it.data, it.data + it.len);
      const PartyRef issuer = r.party();
      const uint32_t ref_len = r.u8();
      r.span(ref_len);
      const PartyRef owner = r.party();
      const PartyRef notary = r.party();
      const uint32_t code_len = r.u8();
      const uint8_t* code = r.span(code_len);
      const uint32_t scale = r.u8();
      r.span(32);
      const uint32_t flags = r.u8();
      const uint8_t* enc = r.span(4);
      if (!r.ok || r.p != r.end) {
        s.ok = false;
        break;
      }
      s.word(varlong_zz_len(it.value));
      shape_party(s, issuer);
      s.word(ref_len);
      shape_party(s, owner);
      shape_party(s, notary);
      s.word(code_len);
      s.span(code, code_len);  // ASCII-checked, written as a string
      s.word(scale);
      s.word(flags);
      s.word((flags & 1u) ? (uint32_t)(enc[0] | (enc[1] << 8) | (enc[2] << 16) | ((uint32_t)enc[3] << 24)) : 0);
      s.word(same_key(owner, issuer));  // exitKeys has one element or two
      break;
    }
    default: s.ok = false;  // RAW (copied directly) and unknown kinds
  }
  return s;
}

KRYO_HD inline uint64_t shape_hash(const Shape& s) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a over the words and the span bytes
  auto mix = [&](uint32_t x) {
    h ^= x;
    h *= 1099511628211ull;
  };
  for (uint32_t i = 0; i < s.nw; i++) mix(s.w[i]);
  for (uint32_t j = 0; j < s.ns; j++) {
    mix(0x100 | s.sl[j]);
    for (uint32_t i = 0; i < s.sl[j]; i++) mix(s.sp[j][i]);
  }
  return h ^ (h >> 29);
}

KRYO_HD inline bool same_shape(const Shape& a, const Shape& b) {
  if (!a.ok || !b.ok || a.nw != b.nw || a.ns != b.ns) return false;
  for (uint32_t i = 0; i < a.nw; i++)
    if (a.w[i] != b.w[i]) return false;
  for (uint32_t j = 0; j < a.ns; j++) {
    if (a.sl[j] != b.sl[j]) return false;
    if (a.sp[j] == b.sp[j]) continue;
    for (uint32_t i = 0; i < a.sl[j]; i++)
      if (a.sp[j][i] != b.sp[j][i]) return false;
  }
  return true;
}

// One leaf byte of an item from its shape's symbol.
KRYO_HD inline uint8_t sym_byte(uint32_t sym, const uint8_t* data, int64_t value) {
  const uint32_t j = (sym >> 8) & 15;
  switch (sym & kSymTypeMask) {
    case kSymConst: return (uint8_t)sym;
    case kSymPayload: return (uint8_t)(data[(sym >> 8) & (kMaxPayloadOff - 1)] | ((sym & kSymOr80) ? 0x80 : 0));
    case kSymValZz: {  // byte j of Output.writeVarLong(zigzag(value)) (varlong_zigzag)
      const uint64_t u = ((uint64_t)value << 1) ^ (uint64_t)(value >> 63);
      if (j >= 8) return (uint8_t)(u >> 56);
      const uint64_t x = u >> (7 * j);
      return (x >> 7) ? (uint8_t)((x & 0x7f) | 0x80) : (uint8_t)x;
    }
    default: return (uint8_t)((uint64_t)value >> (8 * j));  // byte j (little-endian index) of a big-endian write
  }
}

// The representative's leaf as symbols (trace mode): out = at least `cap`
// symbols, levels = kLevelBytes symbols. Returns the leaf size, or -1 when the
// item is invalid (the encoder rejects it: every item of the shape is invalid),
// or -2 when the leaf is longer than cap (no template: the direct encoder).
KRYO_HD inline int64_t trace_leaf(const cordahip_kryo_item& it, uint32_t* out, uint64_t cap, uint32_t* levels) {
  KoutT<true> o(out, cap, levels);
  o.src = it.data;
  o.src_len = it.data ? it.len : 0;
  if (!encode_leaf(o, it)) return -1;  // as the direct encoder: shape_of bounds payload offsets
  if (o.pos > cap) return -2;
  return (int64_t)o.pos;
}

}  // namespace kryo
}  // namespace cordahip
