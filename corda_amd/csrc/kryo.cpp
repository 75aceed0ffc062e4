// Native Kryo leaf encoder: the p2p Kryo preimages of
// transaction components, i.e. what serializedHash hashes
// (core/.../transactions/MerkleTransaction.kt:16-18):
//   "corda\0\0\1" (Kryo.kt:101) + kryo.writeClassAndObject(x) (Kryo.kt:165-176)
// with references off (withoutReferences). Wire primitives restate Kryo 4.0.0's
// published Output format (writeVarInt, writeString, big-endian fixed-width
// writes); class headers are DefaultClassResolver.writeClass (registered: id + 2;
// implicitly registered Kotlin objects: NAME + 2, name id, class name), the
// bodies are Corda's serializers (Kryo.kt:383-393, :441-451) or Kryo's default
// primitive serializers. Host code only; see include/cordahip.h for the kinds.
#include <algorithm>
#include <cstdint>
#include <functional>
#include <cstring>
#include <initializer_list>
#include <string>
#include <vector>

#include "../../include/cordahip.h"

namespace {

// Kryo 4 default registrations (Kryo constructor): int 0, String 1, float 2,
// boolean 3, byte 4, char 5, short 6, long 7, double 8, void 9; boxed types
// share their primitive's registration.
constexpr uint32_t kIdInt = 0, kIdString = 1, kIdFloat = 2, kIdBoolean = 3, kIdByte = 4, kIdChar = 5, kIdShort = 6,
                   kIdLong = 7, kIdDouble = 8;
constexpr uint32_t kName = static_cast<uint32_t>(-1);  // DefaultClassResolver.NAME

// ---- nested OutputChunked framing (Kryo 4.0.0 Output / OutputChunked) --------
// CompatibleFieldSerializer.write (DefaultKryoCustomizer.kt:56-58 makes it the
// default serializer, EXTENDED cached field names) writes, the first time its
// class is written in an object graph, varint(field count) and every field's
// "DeclaringSimpleName.field" (fields sorted by that name); then it wraps its
// Output in `new OutputChunked(output, 1024)` and writes each field into it
// followed by endChunks(). A field whose value is itself written by a
// CompatibleFieldSerializer nests a second OutputChunked over the first, and
// the framing of the nest is NOT one self-contained chunk per field:
//   OutputChunked.flush() = if (position > 0) { writeChunkSize() (varint, byte
//     by byte, to its stream); Output.flush() }, and Output.flush() writes the
//     buffer to its stream and then calls the STREAM's flush();
//   endChunks() = flush(); stream.write(0).
// The stream of a nested OutputChunked is the enclosing one, so every inner
// flush also flushes every enclosing level: each enclosing field is cut into a
// chunk at that point, and the inner 0 terminator starts a new chunk of the
// enclosing field (e.g. an issue command's value field is [len(A)] A, then
// [01 00], then the field's own 0: ADVICE r03). A level's buffer holds 1024
// bytes: Output.require(n) flushes it when fewer than n are free (varints and
// fixed-width writes are atomic, writeBytes / ASCII strings fill it first). The
// leaf's own Output (Kryo.kt:165-176: a 64 KiB buffer over a
// ByteArrayOutputStream) flushes in order, so level 0 is kept unbounded.
constexpr size_t kChunk = 1024;

struct Kout {
  std::vector<std::vector<uint8_t>> lv{1};  // lv[0]: the leaf; lv[k]: the k-th nested OutputChunked
  void require(size_t k, size_t n) {
    if (k > 0 && kChunk - lv[k].size() < n) flush(k);
  }
  void prim(size_t k, const uint8_t* p, size_t n) {  // an atomic write (require(n), then copy)
    require(k, n);
    lv[k].insert(lv[k].end(), p, p + n);
  }
  void byte(size_t k, uint32_t v) {
    const uint8_t b = (uint8_t)v;
    prim(k, &b, 1);
  }
  void bytes(size_t k, const uint8_t* p, size_t n) {  // Output.writeBytes: fill, flush, continue
    if (k == 0) {
      lv[0].insert(lv[0].end(), p, p + n);
      return;
    }
    size_t c = std::min(kChunk - lv[k].size(), n);
    for (;;) {
      lv[k].insert(lv[k].end(), p, p + c);
      p += c;
      n -= c;
      if (n == 0) return;
      c = std::min(kChunk, n);
      require(k, c);
    }
  }
  void varint(size_t k, uint32_t v) {  // Output.writeVarInt(v, true)
    uint8_t t[5];
    size_t m = 0;
    while (v >> 7) {
      t[m++] = (uint8_t)((v & 0x7f) | 0x80);
      v >>= 7;
    }
    t[m++] = (uint8_t)v;
    prim(k, t, m);
  }
  void varlong_zigzag(size_t k, int64_t x) {  // Output.writeVarLong(v, false)
    uint64_t v = ((uint64_t)x << 1) ^ (uint64_t)(x >> 63);
    uint8_t t[9];
    size_t m = 0;
    for (int i = 0; i < 8 && (v >> 7); i++) {
      t[m++] = (uint8_t)((v & 0x7f) | 0x80);
      v >>= 7;
    }
    t[m++] = (uint8_t)v;
    prim(k, t, m);
  }
  void varint_zigzag(size_t k, int32_t x) {  // Output.writeVarInt(v, false)
    varint(k, ((uint32_t)x << 1) ^ (uint32_t)(x >> 31));
  }
  // OutputChunked.flush at level k: its chunk (varint size, then the bytes) to
  // level k - 1, whose own flush follows (Output.flush flushes the stream)
  void flush(size_t k) {
    if (k == 0) return;
    if (!lv[k].empty()) {
      std::vector<uint8_t> data;
      data.swap(lv[k]);
      uint32_t sz = (uint32_t)data.size();
      while (sz >> 7) {  // writeChunkSize: one stream.write(int) per byte
        byte(k - 1, (sz & 0x7f) | 0x80);
        sz >>= 7;
      }
      byte(k - 1, sz);
      bytes(k - 1, data.data(), data.size());
    }
    flush(k - 1);
  }
  void end_chunks(size_t k) {
    flush(k);
    byte(k - 1, 0);
  }
  // Output.writeString over UTF-16 code units (Java String semantics)
  void string(size_t k, const uint16_t* c, uint64_t n) {
    if (n == 0) {
      byte(k, 1 | 0x80);  // empty string
      return;
    }
    bool ascii = n > 1 && n < 64;
    for (uint64_t i = 0; ascii && i < n; i++) ascii = c[i] <= 127;
    if (ascii) {
      std::vector<uint8_t> t(c, c + n);
      bytes(k, t.data(), n);
      lv[k].back() |= 0x80;  // the last byte carries the end mark
      return;
    }
    utf8_length(k, (uint32_t)n + 1);
    uint64_t i = 0;
    if (k == 0 || kChunk - lv[k].size() >= n)  // the 8-bit fast path while it fits
      for (; i < n && c[i] <= 127; i++) lv[k].push_back((uint8_t)c[i]);
    for (; i < n; i++) {  // writeString_slow
      if (k > 0 && lv[k].size() == kChunk) require(k, std::min<uint64_t>(kChunk, n - i));
      const uint32_t x = c[i];
      if (x <= 0x7f) {
        lv[k].push_back((uint8_t)x);
      } else if (x > 0x7ff) {
        lv[k].push_back((uint8_t)(0xe0 | ((x >> 12) & 0x0f)));
        require(k, 2);
        lv[k].push_back((uint8_t)(0x80 | ((x >> 6) & 0x3f)));
        lv[k].push_back((uint8_t)(0x80 | (x & 0x3f)));
      } else {
        lv[k].push_back((uint8_t)(0xc0 | ((x >> 6) & 0x1f)));
        require(k, 1);
        lv[k].push_back((uint8_t)(0x80 | (x & 0x3f)));
      }
    }
  }
  // Output.writeUtf8Length: bit 8 of the first byte flags UTF-8, bit 7 "more"
  void utf8_length(size_t k, uint32_t v) {
    uint8_t t[5];
    size_t m = 0;
    if ((v >> 6) == 0) {
      t[m++] = (uint8_t)(v | 0x80);
    } else {
      t[m++] = (uint8_t)(v | 0x40 | 0x80);
      v >>= 6;
      while (v >> 7 && m < 4) {
        t[m++] = (uint8_t)((v & 0x7f) | 0x80);
        v >>= 7;
      }
      t[m++] = (uint8_t)v;
    }
    prim(k, t, m);
  }
  void ascii(size_t k, const char* s, uint64_t n) {
    std::vector<uint16_t> c(s, s + n);
    string(k, c.data(), n);
  }
};

// One object graph (Kryo.writeClassAndObject resets both at the top level):
// DefaultClassResolver's class-name ids and CompatibleFieldSerializer's
// "header written" marks.
struct Graph {
  std::vector<std::string> names;
  std::vector<std::string> headers;
  // DefaultClassResolver.writeClass for a registered class: varint(id + 2)
  static void class_id(Kout& o, size_t k, uint32_t id) { o.varint(k, id + 2); }
  // DefaultClassResolver.writeName: NAME + 2, the graph's name id, and the class
  // name the first time the class occurs in the graph
  void class_name(Kout& o, size_t k, const std::string& name) {
    o.varint(k, kName + 2);
    for (size_t i = 0; i < names.size(); i++)
      if (names[i] == name) {
        o.varint(k, (uint32_t)i);
        return;
      }
    names.push_back(name);
    o.varint(k, (uint32_t)(names.size() - 1));
    o.ascii(k, name.data(), name.size());
  }
  // CompatibleFieldSerializer.write of one object of class `cls` at level k:
  // header (once per graph), then each field (sorted by EXTENDED name) through
  // the OutputChunked at level k + 1
  using Field = std::pair<std::string, std::function<void(size_t)>>;
  void cfs(Kout& o, size_t k, const std::string& cls, std::vector<Field> fields) {
    std::sort(fields.begin(), fields.end(), [](const Field& a, const Field& b) { return a.first < b.first; });
    if (std::find(headers.begin(), headers.end(), cls) == headers.end()) {
      headers.push_back(cls);
      o.varint(k, (uint32_t)fields.size());
      for (const Field& f : fields) o.ascii(k, f.first.data(), f.first.size());
    }
    o.lv.emplace_back();
    const size_t c = k + 1;
    for (const Field& f : fields) {
      f.second(c);
      o.end_chunks(c);
    }
    o.lv.pop_back();
  }
};

// a public key as a field / element of unknown concrete type: its class
// (registered: Ed25519PublicKeySerializer or PublicKeySerializer, Kryo.kt:383-393,
// :441-451), then writeBytesWithLength (Kryo.kt:305-308: writeInt(size, true) +
// writeBytes) -- the same bytes for both serializers
void key_value(Kout& o, size_t k, uint32_t key_class, const uint8_t* key, uint64_t n) {
  Graph::class_id(o, k, key_class);
  o.varint(k, (uint32_t)n);
  o.bytes(k, key, n);
}

// Length of a DER TLV at p (definite form), 0 if malformed / longer than n.
uint64_t der_tlv_len(const uint8_t* p, uint64_t n) {
  if (n < 2) return 0;
  uint64_t len = p[1], hdr = 2;
  if (len & 0x80) {
    const uint32_t k = len & 0x7f;
    if (k == 0 || k > 4 || n < 2 + k) return 0;
    len = 0;
    for (uint32_t i = 0; i < k; i++) len = (len << 8) | p[2 + i];
    hdr += k;
  }
  return hdr + len <= n ? hdr + len : 0;
}

std::vector<uint16_t> utf16(const uint8_t* p, uint64_t n) {
  std::vector<uint16_t> c(n);
  for (uint64_t i = 0; i < n; i++) c[i] = (uint16_t)(p[2 * i] | (p[2 * i + 1] << 8));
  return c;
}

// A party of a CASH_STATE payload: u16 LE key class id, u16 LE key length, the
// key, u16 LE X.500 name length, the name's DER (length 0: an AnonymousParty).
struct PartyRef {
  uint32_t key_class = 0;
  const uint8_t* key = nullptr;
  uint32_t key_len = 0;
  const uint8_t* name = nullptr;
  uint32_t name_len = 0;
};

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  uint32_t u8() { return take(1) ? p[-1] : 0; }
  uint32_t u16() { return take(2) ? (uint32_t)(p[-2] | (p[-1] << 8)) : 0; }
  const uint8_t* span(uint64_t n) { return take(n) ? p - n : nullptr; }
  bool take(uint64_t n) {
    if (!ok || (uint64_t)(end - p) < n) return ok = false;
    p += n;
    return true;
  }
  PartyRef party() {
    PartyRef r;
    r.key_class = u16();
    r.key_len = u16();
    r.key = span(r.key_len);
    r.name_len = u16();
    r.name = span(r.name_len);
    if (r.key_len == 0 || (r.name_len && (der_tlv_len(r.name, r.name_len) != r.name_len || r.name[0] != 0x30)))
      ok = false;
    return r;
  }
};

// net.corda.core.identity.Party(name: X500Name, owningKey: PublicKey) (identity/Party.kt,
// AbstractParty.kt) or AnonymousParty(owningKey) (AnonymousParty.kt): the class (when
// written) by implicit NAME registration (CordaClassResolver.registerImplicit), then
// CompatibleFieldSerializer over AbstractParty.owningKey and Party.name; the name
// through X500NameSerializer (Kryo.kt:615-624: writeBytes(encoded), no length).
void party_body(Kout& o, Graph& g, size_t k, const PartyRef& p, uint32_t x500_class) {
  std::vector<Graph::Field> f;
  f.push_back({"AbstractParty.owningKey", [&](size_t c) { key_value(o, c, p.key_class, p.key, p.key_len); }});
  if (p.name_len)
    f.push_back({"Party.name", [&](size_t c) {
                   Graph::class_id(o, c, x500_class);
                   o.bytes(c, p.name, p.name_len);
                 }});
  g.cfs(o, k, p.name_len ? "net.corda.core.identity.Party" : "net.corda.core.identity.AnonymousParty", f);
}
void party_class_and_object(Kout& o, Graph& g, size_t k, const PartyRef& p, uint32_t x500_class) {
  g.class_name(o, k, p.name_len ? "net.corda.core.identity.Party" : "net.corda.core.identity.AnonymousParty");
  party_body(o, g, k, p, x500_class);
}

// net.corda.core.utilities.OpaqueBytes / SecureHash$SHA256 (utilities/ByteArrays.kt:16,
// crypto/SecureHash.kt:13-15): one field OpaqueBytes.bytes, a byte[] (a final
// class: no class written; ByteArraySerializer accepts null, so no null marker):
// varint(length + 1), the bytes
void opaque_bytes(Kout& o, Graph& g, size_t k, const char* cls, const uint8_t* b, uint64_t n) {
  g.class_name(o, k, cls);
  g.cfs(o, k, cls, {{"OpaqueBytes.bytes", [&](size_t c) {
                       o.varint(c, (uint32_t)n + 1);
                       o.bytes(c, b, n);
                     }}});
}

bool same_key(const PartyRef& a, const PartyRef& b) {
  return a.key_class == b.key_class && a.key_len == b.key_len && std::memcmp(a.key, b.key, a.key_len) == 0;
}

// TransactionState<Cash.State> -- the output component of a cash-issue
// transaction (Cash.generateIssue, Cash.kt:166-167: TransactionState(State(amount,
// owner), notary)). Fields and their writes (Kryo 4.0.0 FieldSerializer: a field of a
// final class is written as NOT_NULL + body, of any other class as class + body):
//   TransactionState (Structures.kt:95-117): data (ContractState: class + body),
//     encumbrance (Integer: NULL, or NOT_NULL + writeInt(v, false)), notary (Party, final)
//   Cash.State (Cash.kt:92-103): amount (Amount, final), contract (Cash, final: its
//     one field Cash.legalContractReference, Cash.kt:62, a SecureHash$SHA256),
//     exitKeys (setOf(owner key, issuer key): java.util.LinkedHashSet through
//     CollectionSerializer: varint(size), each key class + bytes), owner
//     (AbstractParty), participants (listOf(owner): Collections$SingletonList,
//     CollectionsSingletonListSerializer: the element's class + body)
//   Amount (Amount.kt:37): displayTokenSize (java.math.BigDecimal, BigDecimalSerializer:
//     unscaled BigInteger as varint(len + 1) + two's-complement bytes, then
//     writeInt(scale, false)), quantity (long: writeVarLong(v, false)), token (Issued)
//   Issued (Structures.kt:132): issuer (PartyAndReference, final), product
//     (java.util.Currency, CurrencySerializer: writeString(code))
//   PartyAndReference (Structures.kt:268): party (AbstractParty), reference (OpaqueBytes)
// Classes without a registration go by implicit NAME registration: each name's
// string is written at its first occurrence in the graph (DefaultWhitelist.kt
// whitelists LinkedHashSet, Currency, SingletonList, BigDecimal).
bool cash_state(Kout& o, const cordahip_kryo_item& it) {
  Reader r{it.data, it.data + it.len};
  const PartyRef issuer = r.party();
  const uint32_t ref_len = r.u8();
  const uint8_t* ref = r.span(ref_len);
  const PartyRef owner = r.party();
  const PartyRef notary = r.party();
  const uint32_t code_len = r.u8();
  const uint8_t* code = r.span(code_len);
  const uint32_t scale = r.u8();
  const uint8_t* legal = r.span(32);
  const uint32_t flags = r.u8();
  const uint8_t* enc = r.span(4);
  if (!r.ok || r.p != r.end || ref_len == 0 || code_len == 0 || notary.name_len == 0 || (flags & ~1u)) return false;
  for (uint32_t i = 0; i < code_len; i++)
    if (code[i] > 127) return false;
  const uint32_t x500 = it.class_id;
  const int64_t quantity = it.value;
  Graph g;
  g.class_name(o, 0, "net.corda.core.contracts.TransactionState");
  g.cfs(o, 0, "net.corda.core.contracts.TransactionState", {
    {"TransactionState.data", [&](size_t k1) {
       g.class_name(o, k1, "net.corda.contracts.asset.Cash$State");
       g.cfs(o, k1, "net.corda.contracts.asset.Cash$State", {
         {"State.amount", [&](size_t k2) {
            o.byte(k2, 1);  // NOT_NULL
            g.cfs(o, k2, "net.corda.core.contracts.Amount", {
              {"Amount.displayTokenSize", [&](size_t k3) {
                 g.class_name(o, k3, "java.math.BigDecimal");
                 o.varint(k3, 2);  // BigInteger.ONE.toByteArray() = {1}: varint(1 + 1), 01
                 o.byte(k3, 1);
                 o.varint_zigzag(k3, (int32_t)(int8_t)scale);  // Currency: ONE.scaleByPowerOfTen(-digits), Amount.kt:70-80
               }},
              {"Amount.quantity", [&](size_t k3) { o.varlong_zigzag(k3, quantity); }},
              {"Amount.token", [&](size_t k3) {
                 g.class_name(o, k3, "net.corda.core.contracts.Issued");
                 g.cfs(o, k3, "net.corda.core.contracts.Issued", {
                   {"Issued.issuer", [&](size_t k4) {
                      o.byte(k4, 1);  // NOT_NULL
                      g.cfs(o, k4, "net.corda.core.contracts.PartyAndReference", {
                        {"PartyAndReference.party", [&](size_t k5) { party_class_and_object(o, g, k5, issuer, x500); }},
                        {"PartyAndReference.reference",
                         [&](size_t k5) { opaque_bytes(o, g, k5, "net.corda.core.utilities.OpaqueBytes", ref, ref_len); }},
                      });
                    }},
                   {"Issued.product", [&](size_t k4) {
                      g.class_name(o, k4, "java.util.Currency");
                      o.ascii(k4, (const char*)code, code_len);
                    }},
                 });
               }},
            });
          }},
         {"State.contract", [&](size_t k2) {
            o.byte(k2, 1);  // NOT_NULL
            g.cfs(o, k2, "net.corda.contracts.asset.Cash", {
              {"Cash.legalContractReference",
               [&](size_t k3) { opaque_bytes(o, g, k3, "net.corda.core.crypto.SecureHash$SHA256", legal, 32); }},
            });
          }},
         {"State.exitKeys", [&](size_t k2) {
            g.class_name(o, k2, "java.util.LinkedHashSet");
            const bool one = same_key(owner, issuer);  // a set: one element when the keys are equal
            o.varint(k2, one ? 1 : 2);
            key_value(o, k2, owner.key_class, owner.key, owner.key_len);
            if (!one) key_value(o, k2, issuer.key_class, issuer.key, issuer.key_len);
          }},
         {"State.owner", [&](size_t k2) { party_class_and_object(o, g, k2, owner, x500); }},
         {"State.participants", [&](size_t k2) {
            g.class_name(o, k2, "java.util.Collections$SingletonList");
            party_class_and_object(o, g, k2, owner, x500);
          }},
       });
     }},
    {"TransactionState.encumbrance", [&](size_t k1) {
       if (flags & 1u) {
         o.byte(k1, 1);  // NOT_NULL, then IntSerializer: writeInt(v, false)
         o.varint_zigzag(k1, (int32_t)(enc[0] | (enc[1] << 8) | (enc[2] << 16) | ((uint32_t)enc[3] << 24)));
       } else {
         o.byte(k1, 0);  // NULL
       }
     }},
    {"TransactionState.notary", [&](size_t k1) {
       o.byte(k1, 1);  // NOT_NULL (Party is final)
       party_body(o, g, k1, notary, x500);
     }},
  });
  return true;
}

// one component's leaf preimage; false for an unknown kind / missing payload
bool encode(const cordahip_kryo_item& it, std::vector<uint8_t>& out) {
  if (it.kind == CORDAHIP_KRYO_RAW) {
    if (it.len && !it.data) return false;
    out.insert(out.end(), it.data, it.data + it.len);
    return true;
  }
  static const uint8_t kHeader[8] = {'c', 'o', 'r', 'd', 'a', 0, 0, 1};  // KryoHeaderV0_1
  Kout o;
  o.bytes(0, kHeader, 8);
  const uint64_t v = (uint64_t)it.value;
  auto be = [&](uint64_t x, int n) {
    for (int i = n - 1; i >= 0; i--) o.byte(0, (uint32_t)(x >> (8 * i)));
  };
  bool ok = true;
  switch (it.kind) {
    case CORDAHIP_KRYO_CHAR: Graph::class_id(o, 0, kIdChar); be(v, 2); break;
    case CORDAHIP_KRYO_SHORT: Graph::class_id(o, 0, kIdShort); be(v, 2); break;
    case CORDAHIP_KRYO_INT: Graph::class_id(o, 0, kIdInt); be(v, 4); break;
    case CORDAHIP_KRYO_LONG: Graph::class_id(o, 0, kIdLong); be(v, 8); break;
    case CORDAHIP_KRYO_BYTE: Graph::class_id(o, 0, kIdByte); be(v, 1); break;
    case CORDAHIP_KRYO_BOOLEAN: Graph::class_id(o, 0, kIdBoolean); o.byte(0, v ? 1 : 0); break;
    case CORDAHIP_KRYO_FLOAT: Graph::class_id(o, 0, kIdFloat); be(v, 4); break;     // writeFloat: floatToIntBits
    case CORDAHIP_KRYO_DOUBLE: Graph::class_id(o, 0, kIdDouble); be(v, 8); break;   // writeDouble: doubleToLongBits
    case CORDAHIP_KRYO_STRING: {
      if (it.len && !it.data) return false;
      const std::vector<uint16_t> c = utf16(it.data, it.len);
      Graph::class_id(o, 0, kIdString);
      o.string(0, c.data(), c.size());
      break;
    }
    case CORDAHIP_KRYO_ED25519_KEY:  // Ed25519PublicKeySerializer: writeBytesWithLength(abyte)
      if (!it.data || it.len != 32) return false;
      key_value(o, 0, it.class_id, it.data, 32);
      break;
    case CORDAHIP_KRYO_PUBLIC_KEY:  // PublicKeySerializer: writeBytesWithLength(key.encoded)
      if (!it.data || it.len == 0 || it.len > 0x7fffffffull) return false;
      key_value(o, 0, it.class_id, it.data, it.len);
      break;
    case CORDAHIP_KRYO_KOTLIN_OBJECT: {  // NAME registration, KotlinObjectSerializer writes no body
      if (!it.data || it.len == 0) return false;
      const std::vector<uint16_t> c = utf16(it.data, it.len);
      o.varint(0, kName + 2);  // = 1
      o.varint(0, 0);          // first class name of this object graph: name id 0
      o.string(0, c.data(), c.size());
      break;
    }
    case CORDAHIP_KRYO_PARTY: {
      // the notary Party as a component: data = the X.500 name's DER, then the key
      if (!it.data || it.len < 3) return false;
      const uint64_t dn = der_tlv_len(it.data, it.len);
      if (dn == 0 || dn >= it.len || it.data[0] != 0x30 || it.len - dn > 0xffff) return false;
      PartyRef p;
      p.key_class = (uint32_t)it.value;
      p.key = it.data + dn;
      p.key_len = (uint32_t)(it.len - dn);
      p.name = it.data;
      p.name_len = (uint32_t)dn;
      Graph g;
      party_class_and_object(o, g, 0, p, it.class_id);
      break;
    }
    case CORDAHIP_KRYO_ISSUE_COMMAND: {
      // net.corda.core.contracts.Command(value, signers) (contracts/Structures.kt:285)
      // as TransactionBuilder.addCommand(data, vararg keys) builds it
      // (TransactionBuilder.kt:124: listOf(*keys) = java.util.Arrays$ArrayList
      // over a PublicKey[]), value = an issue command data class with one
      // `nonce: Long` field (Cash / CommodityContract / Obligation
      // Commands.Issue, e.g. Cash.kt:148; OnLedgerAsset.generateIssue,
      // OnLedgerAsset.kt:208-219). data = u8 name length, the command class's
      // binary name, u8 key count, per key u16 LE registration id, u16 LE
      // length, the key bytes; class_id = the Arrays$ArrayList registration
      // (ArraysAsListSerializer); value = the nonce.
      if (!it.data || it.len < 2) return false;
      Reader r{it.data, it.data + it.len};
      const uint32_t nlen = r.u8();
      const uint8_t* nm = r.span(nlen);
      const uint32_t nkeys = r.u8();
      if (!r.ok || nlen < 2 || nkeys == 0) return false;  // Command: require(signers.isNotEmpty())
      std::vector<PartyRef> keys(nkeys);
      for (auto& kk : keys) {
        kk.key_class = r.u16();
        kk.key_len = r.u16();
        kk.key = r.span(kk.key_len);
        if (kk.key_len == 0) r.ok = false;
      }
      if (!r.ok || r.p != r.end) return false;
      const std::string name((const char*)nm, nlen);
      const size_t cut = name.find_last_of("$.");
      const std::string simple = (cut == std::string::npos ? name : name.substr(cut + 1)) + ".nonce";
      Graph g;
      g.class_name(o, 0, "net.corda.core.contracts.Command");
      g.cfs(o, 0, "net.corda.core.contracts.Command", {
        {"Command.signers", [&](size_t k) {
           // ArraysAsListSerializer (kryo-serializers 0.41): writeInt(length, true),
           // writeClass(component type) -- java.security.PublicKey, implicit NAME --
           // then writeClassAndObject per element
           Graph::class_id(o, k, it.class_id);
           o.varint(k, nkeys);
           g.class_name(o, k, "java.security.PublicKey");
           for (const auto& kk : keys) key_value(o, k, kk.key_class, kk.key, kk.key_len);
         }},
        {"Command.value", [&](size_t k) {
           // the command data: implicit NAME, its own CompatibleFieldSerializer (a
           // primitive long nonce: writeVarLong(v, false)) -- a nested OutputChunked
           g.class_name(o, k, name);
           g.cfs(o, k, name, {{simple, [&](size_t c) { o.varlong_zigzag(c, it.value); }}});
         }},
      });
      break;
    }
    case CORDAHIP_KRYO_CASH_STATE:
      if (!it.data) return false;
      ok = cash_state(o, it);
      break;
    default: return false;
  }
  if (!ok) return false;
  out.insert(out.end(), o.lv[0].begin(), o.lv[0].end());
  return true;
}

}  // namespace

extern "C" int cordahip_kryo_encode(const cordahip_kryo_item* items, uint64_t n, uint8_t* out, uint64_t cap,
                                    uint64_t* off) {
  if ((n && !items) || !off) return CORDAHIP_ERR_INVALID_ARG;
  std::vector<uint8_t> o;
  off[0] = 0;
  for (uint64_t i = 0; i < n; i++) {
    if (!encode(items[i], o)) return CORDAHIP_ERR_INVALID_ARG;
    off[i + 1] = o.size();
  }
  if (o.size() > cap || (o.size() && !out)) return CORDAHIP_ERR_BUFFER_TOO_SMALL;
  if (o.size()) std::memcpy(out, o.data(), o.size());
  return CORDAHIP_SUCCESS;
}
