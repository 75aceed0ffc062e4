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
// party decode validates). shape_matches() compares an item's structure words
// and those spans byte for byte with a recorded shape; the hash only picks the
// table slot.
// tests/test_kryo_template.py checks, on the host, every item of randomised
// batches rebuilt from its shape representative's symbols against the direct
// encoder.
#pragma once
#include "kryo_core.hpp"

namespace cordahip {
namespace kryo {

// ---- shapes ---------------------------------------------------------------------
// shape_walk visits an item's shape -- its structure words and the content
// spans the encoder inspects -- in a fixed order through a visitor V
// (V::word(x), V::span(p, n)), so hashing, recording and comparing shapes
// stream over the payload without arrays. Returns false when the item has no
// shape (RAW leaves are copied directly; unknown kinds, malformed payloads and
// outsized content go to the direct encoder, which also decides their
// validity).

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
template <class V>
KRYO_HD inline void shape_party(V& v, const PartyRef& p) {
  v.word(p.key_class);
  v.word(p.key_len);
  v.word(p.name_len);
  v.span(p.name, p.name_len < 6 ? p.name_len : 6);
}

template <class V>
KRYO_HD inline bool shape_walk(const cordahip_kryo_item& it, V& v) {
  v.word(it.kind);
  v.word(it.class_id);
  switch (it.kind) {
    case CORDAHIP_KRYO_CHAR:
    case CORDAHIP_KRYO_SHORT:
    case CORDAHIP_KRYO_INT:
    case CORDAHIP_KRYO_LONG:
    case CORDAHIP_KRYO_BYTE:
    case CORDAHIP_KRYO_FLOAT:
    case CORDAHIP_KRYO_DOUBLE: return true;  // value bytes only
    case CORDAHIP_KRYO_BOOLEAN: v.word(it.value != 0); return true;
    case CORDAHIP_KRYO_STRING:
    case CORDAHIP_KRYO_KOTLIN_OBJECT:  // the text is transcoded (UTF-16 -> Kryo string): all of it is shape
      if (it.len > 512 || (it.len && !it.data)) return false;
      v.word((uint32_t)it.len);
      v.span(it.data, (uint32_t)(2 * it.len));
      return true;
    case CORDAHIP_KRYO_ED25519_KEY:
    case CORDAHIP_KRYO_PUBLIC_KEY:
      if (!it.data || it.len >= kMaxPayloadOff) return false;
      v.word((uint32_t)it.len);
      return true;
    case CORDAHIP_KRYO_PARTY:
      if (!it.data || it.len >= kMaxPayloadOff) return false;
      v.word((uint32_t)it.value);  // the key class (its varint is written)
      v.word((uint32_t)it.len);
      v.span(it.data, it.len < 6 ? (uint32_t)it.len : 6);  // der_tlv_len splits name | key on these
      return true;
    case CORDAHIP_KRYO_ISSUE_COMMAND: {
      if (!it.data || it.len < 2 || it.len >= kMaxPayloadOff) return false;
      Reader r(it.data, it.data + it.len);
      const uint32_t nlen = r.u8();
      const uint8_t* nm = r.span(nlen);
      const uint32_t nkeys = r.u8();
      if (!r.ok || nkeys > 12) return false;
      v.word(varlong_zz_len(it.value));
      v.word(nlen);
      v.span(nm, nlen);  // the class name: written, compared, and cut for the field name
      v.word(nkeys);
      for (uint32_t i = 0; i < nkeys && r.ok; i++) {
        v.word(r.u16());
        const uint32_t kl = r.u16();
        v.word(kl);
        r.span(kl);
      }
      return r.ok && r.p == r.end;
    }
    case CORDAHIP_KRYO_CASH_STATE: {
      if (!it.data || it.len >= kMaxPayloadOff) return false;
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
      if (!r.ok || r.p != r.end) return false;
      v.word(varlong_zz_len(it.value));
      shape_party(v, issuer);
      v.word(ref_len);
      shape_party(v, owner);
      shape_party(v, notary);
      v.word(code_len);
      v.span(code, code_len);  // ASCII-checked, written as a string
      v.word(scale);
      v.word(flags);
      v.word((flags & 1u) ? (uint32_t)(enc[0] | (enc[1] << 8) | (enc[2] << 16) | ((uint32_t)enc[3] << 24)) : 0);
      v.word(same_key(owner, issuer));  // exitKeys has one element or two
      return true;
    }
    default: return false;  // RAW (copied directly) and unknown kinds
  }
}

// Up to 16 bytes p[0 .. min(n, 16)) as 4 little-endian words, zero-padded. On
// the GPU: at most two aligned 16-byte loads, each holding one of the wanted
// bytes (so both are mapped), and a funnel shift -- the shape walks read long
// spans (class names, TransactionType's text) 16 bytes per load.
KRYO_HD inline void span16(const uint8_t* p, uint32_t n, uint32_t w[4]) {
  const uint32_t m = n < 16 ? n : 16;
#if defined(__HIP_DEVICE_COMPILE__)
  w[0] = w[1] = w[2] = w[3] = 0;
  if (!m) return;
  const uintptr_t qa = (uintptr_t)p, ca = qa & ~(uintptr_t)15;
  const uint32_t s = (uint32_t)(qa - ca);
  uint4 u0 = *reinterpret_cast<const uint4*>(ca), u1 = make_uint4(0, 0, 0, 0);
  if (s + m - 1 >= 16) u1 = *reinterpret_cast<const uint4*>(ca + 16);
  const uint32_t d[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
  const uint32_t dw = s >> 2, sb = s & 3;
  uint32_t e[5];
#pragma unroll
  for (int i = 0; i < 5; i++)
    e[i] = dw == 0 ? d[i] : dw == 1 ? d[i + 1] : dw == 2 ? d[i + 2] : (i + 3 < 8 ? d[i + 3] : 0);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t x = __builtin_amdgcn_alignbyte(e[i + 1], e[i], sb);
    const uint32_t k = m > 4 * (uint32_t)i ? m - 4 * i : 0;  // wanted bytes of word i
    w[i] = k >= 4 ? x : (k ? x & ((1u << (8 * k)) - 1) : 0);
  }
#else
  for (int i = 0; i < 4; i++) w[i] = 0;
  for (uint32_t i = 0; i < m; i++) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
#endif
}

// FNV-1a over the words and each span's length, first 16 and last 16 bytes
// (the hash only picks a table slot; shape_matches compares every byte)
struct ShapeHash {
  uint64_t h = 1469598103934665603ull;
  KRYO_HD void mix(uint32_t x) {
    h ^= x;
    h *= 1099511628211ull;
  }
  KRYO_HD void word(uint32_t x) { mix(x); }
  KRYO_HD void span(const uint8_t* p, uint32_t n) {
    mix(0x100 | n);
    uint32_t w[4];
    span16(p, n, w);
    for (int i = 0; i < 4; i++) mix(w[i]);
    if (n > 16) {
      span16(p + n - 16, 16, w);
      for (int i = 0; i < 4; i++) mix(w[i]);
    }
  }
  KRYO_HD uint64_t value() const { return h ^ (h >> 29); }
};

// A shape as data: the GPU keeps one per table slot (the words and the span
// BYTES, so the record outlives the call whose item it came from), and items
// are compared with it as they are walked (ShapeCmp). Each span's bytes start
// 16-byte aligned in `bytes`, zero-padded, so a compare reads them 16 at a time.
struct ShapeRec {
  static constexpr uint32_t kWords = 48, kSpans = 8, kBytes = 256;
  uint32_t nw, ns, nb, ok;
  uint32_t w[kWords];
  uint32_t sl[kSpans];
  uint32_t so[kSpans];
  uint8_t bytes[kBytes];
};

struct ShapeRecord {  // visitor: fills a record (ok = 0 when it does not fit)
  ShapeRec& r;
  KRYO_HD explicit ShapeRecord(ShapeRec& x) : r(x) { r.nw = r.ns = r.nb = 0, r.ok = 1; }
  KRYO_HD void word(uint32_t x) {
    if (r.nw < ShapeRec::kWords) r.w[r.nw++] = x;
    else r.ok = 0;
  }
  KRYO_HD void span(const uint8_t* p, uint32_t n) {
    const uint32_t padded = (n + 15) / 16 * 16;
    if (r.ns >= ShapeRec::kSpans || r.nb + padded > ShapeRec::kBytes) {
      r.ok = 0;
      return;
    }
    r.sl[r.ns] = n;
    r.so[r.ns++] = r.nb;
    for (uint32_t i = 0; i < padded; i++) r.bytes[r.nb + i] = i < n ? p[i] : 0;
    r.nb += padded;
  }
};

struct ShapeCmp {  // visitor: eq stays true while the walk matches the record
  const ShapeRec& r;
  uint32_t iw = 0, is = 0;
  uint32_t buf[4] = {0, 0, 0, 0};  // record words iw & ~3 .. + 3 (read 4 at a time)
  bool eq = true;
  KRYO_HD explicit ShapeCmp(const ShapeRec& x) : r(x) {}
  KRYO_HD void word(uint32_t x) {
    if (iw >= ShapeRec::kWords) {
      eq = false;
      return;
    }
    if ((iw & 3) == 0) {
#if defined(__HIP_DEVICE_COMPILE__)
      const uint4 q = *reinterpret_cast<const uint4*>(&r.w[iw]);
      buf[0] = q.x, buf[1] = q.y, buf[2] = q.z, buf[3] = q.w;
#else
      for (int i = 0; i < 4; i++) buf[i] = r.w[iw + i];
#endif
    }
    const uint32_t k = iw & 3;
    const uint32_t y = k == 0 ? buf[0] : k == 1 ? buf[1] : k == 2 ? buf[2] : buf[3];
    eq = eq && iw < r.nw && y == x;
    iw++;
  }
  KRYO_HD void span(const uint8_t* p, uint32_t n) {
    eq = eq && is < r.ns && r.sl[is] == n;
    const uint32_t o = eq ? r.so[is] : 0;
    for (uint32_t i = 0; eq && i < n; i += 16) {
      uint32_t w[4];
      span16(p + i, n - i, w);
#if defined(__HIP_DEVICE_COMPILE__)
      const uint4 q = *reinterpret_cast<const uint4*>(&r.bytes[o + i]);
      eq = q.x == w[0] && q.y == w[1] && q.z == w[2] && q.w == w[3];
#else
      for (int k = 0; k < 4; k++) {
        uint32_t y = 0;
        for (int b = 0; b < 4; b++) y |= (uint32_t)r.bytes[o + i + 4 * k + b] << (8 * b);
        eq = eq && y == w[k];
      }
#endif
    }
    is++;
  }
  KRYO_HD bool done() const { return eq && iw == r.nw && is == r.ns; }
};

// hash of an item's shape; false: no shape
KRYO_HD inline bool shape_hash_of(const cordahip_kryo_item& it, uint64_t& h) {
  ShapeHash v;
  const bool ok = shape_walk(it, v);
  h = v.value();
  return ok;
}
// The encoder (kryo_core.hpp encode_leaf) rejects the item before writing a
// byte: an unknown kind, or a payload that is missing (after ItemSrc's bounds
// check) or of a length the kind never accepts. Mirrors encode_leaf's early
// returns; the shape pass gives such items status 1 at once instead of sending
// them to the direct encoder (or, in the templates-only chain, counting a miss
// that would redo the whole call).
KRYO_HD inline bool rejected_outright(const cordahip_kryo_item& it) {
  switch (it.kind) {
    case CORDAHIP_KRYO_CHAR: case CORDAHIP_KRYO_SHORT: case CORDAHIP_KRYO_INT: case CORDAHIP_KRYO_LONG:
    case CORDAHIP_KRYO_BYTE: case CORDAHIP_KRYO_BOOLEAN: case CORDAHIP_KRYO_FLOAT: case CORDAHIP_KRYO_DOUBLE:
      return false;
    case CORDAHIP_KRYO_RAW:
    case CORDAHIP_KRYO_STRING: return it.len && !it.data;
    case CORDAHIP_KRYO_ED25519_KEY: return !it.data || it.len != 32;
    case CORDAHIP_KRYO_PUBLIC_KEY: return !it.data || it.len == 0 || it.len > 0x7fffffffull;
    case CORDAHIP_KRYO_KOTLIN_OBJECT: return !it.data || it.len == 0;
    case CORDAHIP_KRYO_PARTY: return !it.data || it.len < 3;
    case CORDAHIP_KRYO_ISSUE_COMMAND: return !it.data || it.len < 2;
    case CORDAHIP_KRYO_CASH_STATE: return !it.data;
    default: return true;
  }
}
// the item has exactly the recorded shape
KRYO_HD inline bool shape_matches(const cordahip_kryo_item& it, const ShapeRec& rec) {
  ShapeCmp v(rec);
  return rec.ok && shape_walk(it, v) && v.done();
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
