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
#include <cstdint>
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

struct Out {
  std::vector<uint8_t> b;
  void byte(uint32_t v) { b.push_back((uint8_t)v); }
  // Output.writeVarInt(value, true): 7-bit groups, least significant first
  void varint(uint32_t v) {
    while (v >> 7) {
      byte((v & 0x7f) | 0x80);
      v >>= 7;
    }
    byte(v);
  }
  void be(uint64_t v, int bytes) {
    for (int i = bytes - 1; i >= 0; i--) byte((uint32_t)(v >> (8 * i)));
  }
  void bytes(const uint8_t* p, uint64_t n) { b.insert(b.end(), p, p + n); }
  // Output.writeUtf8Length: bit 8 of the first byte flags UTF-8, bit 7 "more"
  void utf8_length(uint32_t v) {
    if ((v >> 6) == 0) {
      byte(v | 0x80);
    } else if ((v >> 13) == 0) {
      byte(v | 0x40 | 0x80);
      byte(v >> 6);
    } else if ((v >> 20) == 0) {
      byte(v | 0x40 | 0x80);
      byte((v >> 6) | 0x80);
      byte(v >> 13);
    } else if ((v >> 27) == 0) {
      byte(v | 0x40 | 0x80);
      byte((v >> 6) | 0x80);
      byte((v >> 13) | 0x80);
      byte(v >> 20);
    } else {
      byte(v | 0x40 | 0x80);
      byte((v >> 6) | 0x80);
      byte((v >> 13) | 0x80);
      byte((v >> 20) | 0x80);
      byte(v >> 27);
    }
  }
  // Output.writeString over UTF-16 code units (Java String semantics)
  void string(const uint16_t* c, uint64_t n) {
    if (n == 0) {
      byte(1 | 0x80);  // empty string
      return;
    }
    bool ascii = n > 1 && n < 64;
    for (uint64_t i = 0; ascii && i < n; i++) ascii = c[i] <= 127;
    if (ascii) {
      for (uint64_t i = 0; i < n; i++) byte(c[i]);
      b.back() |= 0x80;  // the last byte carries the end mark
      return;
    }
    utf8_length((uint32_t)n + 1);
    for (uint64_t i = 0; i < n; i++) {
      const uint32_t x = c[i];
      if (x <= 0x7f) {
        byte(x);
      } else if (x > 0x7ff) {
        byte(0xe0 | ((x >> 12) & 0x0f));
        byte(0x80 | ((x >> 6) & 0x3f));
        byte(0x80 | (x & 0x3f));
      } else {
        byte(0xc0 | ((x >> 6) & 0x1f));
        byte(0x80 | (x & 0x3f));
      }
    }
  }
  void class_id(uint32_t id) { varint(id + 2); }  // DefaultClassResolver.writeClass, registered
  // DefaultClassResolver.writeName: NAME + 2, then the graph's name id, then
  // (first use of the class in this object graph) the class name
  void class_name(uint32_t name_id, const char* name) {
    varint(kName + 2);
    varint(name_id);
    ascii(name, strlen(name));
  }
  void ascii(const char* s, uint64_t n) {
    std::vector<uint16_t> c(s, s + n);
    string(c.data(), n);
  }
  // Output.writeVarLong(v, false): zig-zag, 7-bit groups, a 9th byte of 8 bits
  void varlong_zigzag(int64_t x) {
    uint64_t v = ((uint64_t)x << 1) ^ (uint64_t)(x >> 63);
    for (int i = 0; i < 8; i++) {
      if ((v >> 7) == 0) {
        byte((uint32_t)v);
        return;
      }
      byte((uint32_t)(v & 0x7f) | 0x80);
      v >>= 7;
    }
    byte((uint32_t)v);
  }
  // OutputChunked(output, 1024) + endChunks: the data in chunks of at most 1024
  // bytes, each preceded by its varint length, then a zero-length chunk
  void chunked(const Out& field) {
    const uint64_t n = field.b.size();
    for (uint64_t p = 0; p < n; p += 1024) {
      const uint64_t c = n - p < 1024 ? n - p : 1024;
      varint((uint32_t)c);
      bytes(field.b.data() + p, c);
    }
    byte(0);
  }
};

// CompatibleFieldSerializer.write (Kryo 4.0.0; DefaultKryoCustomizer.kt:56-58
// sets it as the default serializer with EXTENDED cached field names): the
// first time a class's serializer writes in an object graph it writes
// varint(field count) and every field's "DeclaringSimpleName.field" (fields
// sorted by that name); then each field's value through OutputChunked.
void fields_header(Out& o, std::initializer_list<const char*> names) {
  o.varint((uint32_t)names.size());
  for (const char* nm : names) o.ascii(nm, strlen(nm));
}

// a public key as a field / list element of unknown concrete type: its class
// (registered: Ed25519PublicKeySerializer or PublicKeySerializer, Kryo.kt:383-393,
// :441-451), then writeBytesWithLength -- the same bytes for both serializers
void key_value(Out& o, uint32_t key_class, const uint8_t* key, uint64_t n) {
  o.class_id(key_class);
  o.varint((uint32_t)n);
  o.bytes(key, n);
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

// one component's leaf preimage; false for an unknown kind / missing payload
bool encode(const cordahip_kryo_item& it, Out& o) {
  if (it.kind == CORDAHIP_KRYO_RAW) {
    if (it.len && !it.data) return false;
    o.bytes(it.data, it.len);
    return true;
  }
  static const uint8_t kHeader[8] = {'c', 'o', 'r', 'd', 'a', 0, 0, 1};  // KryoHeaderV0_1
  o.bytes(kHeader, 8);
  const uint64_t v = (uint64_t)it.value;
  switch (it.kind) {
    case CORDAHIP_KRYO_CHAR: o.class_id(kIdChar); o.be(v, 2); return true;
    case CORDAHIP_KRYO_SHORT: o.class_id(kIdShort); o.be(v, 2); return true;
    case CORDAHIP_KRYO_INT: o.class_id(kIdInt); o.be(v, 4); return true;
    case CORDAHIP_KRYO_LONG: o.class_id(kIdLong); o.be(v, 8); return true;
    case CORDAHIP_KRYO_BYTE: o.class_id(kIdByte); o.be(v, 1); return true;
    case CORDAHIP_KRYO_BOOLEAN: o.class_id(kIdBoolean); o.byte(v ? 1 : 0); return true;
    case CORDAHIP_KRYO_FLOAT: o.class_id(kIdFloat); o.be(v, 4); return true;     // writeFloat: floatToIntBits
    case CORDAHIP_KRYO_DOUBLE: o.class_id(kIdDouble); o.be(v, 8); return true;   // writeDouble: doubleToLongBits
    case CORDAHIP_KRYO_STRING: {
      if (it.len && !it.data) return false;
      const std::vector<uint16_t> c = utf16(it.data, it.len);
      o.class_id(kIdString);
      o.string(c.data(), c.size());
      return true;
    }
    case CORDAHIP_KRYO_ED25519_KEY:  // Ed25519PublicKeySerializer: writeBytesWithLength(abyte)
      if (!it.data || it.len != 32) return false;
      o.class_id(it.class_id);
      o.varint(32);
      o.bytes(it.data, 32);
      return true;
    case CORDAHIP_KRYO_PUBLIC_KEY:  // PublicKeySerializer: writeBytesWithLength(key.encoded)
      if (!it.data || it.len == 0 || it.len > 0x7fffffffull) return false;
      o.class_id(it.class_id);
      o.varint((uint32_t)it.len);
      o.bytes(it.data, it.len);
      return true;
    case CORDAHIP_KRYO_KOTLIN_OBJECT: {  // NAME registration, KotlinObjectSerializer writes no body
      if (!it.data || it.len == 0) return false;
      const std::vector<uint16_t> c = utf16(it.data, it.len);
      o.varint(kName + 2);  // = 1
      o.varint(0);          // first class name of this object graph: name id 0
      o.string(c.data(), c.size());
      return true;
    }
    case CORDAHIP_KRYO_PARTY: {
      // net.corda.core.identity.Party(name: X500Name, owningKey: PublicKey)
      // (identity/Party.kt, AbstractParty.kt): implicit NAME registration
      // (CordaClassResolver.registerImplicit), CompatibleFieldSerializer over
      // AbstractParty.owningKey and Party.name; the name through
      // X500NameSerializer (Kryo.kt:615-624: writeBytes(obj.encoded), no length)
      if (!it.data || it.len < 3) return false;
      const uint64_t dn = der_tlv_len(it.data, it.len);
      if (dn == 0 || dn >= it.len || it.data[0] != 0x30) return false;
      o.class_name(0, "net.corda.core.identity.Party");
      fields_header(o, {"AbstractParty.owningKey", "Party.name"});
      Out f;
      key_value(f, (uint32_t)it.value, it.data + dn, it.len - dn);
      o.chunked(f);
      Out g;
      g.class_id(it.class_id);
      g.bytes(it.data, dn);
      o.chunked(g);
      return true;
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
      const uint8_t* p = it.data;
      const uint8_t* end = it.data + it.len;
      const uint32_t nlen = *p++;
      if (nlen < 2 || p + nlen + 1 > end) return false;
      const std::string name((const char*)p, nlen);
      p += nlen;
      const uint32_t nkeys = *p++;
      if (nkeys == 0) return false;  // Command: require(signers.isNotEmpty())
      Out sig;
      sig.class_id(it.class_id);  // java.util.Arrays$ArrayList
      sig.varint(nkeys);          // ArraysAsListSerializer: array length,
      sig.class_name(1, "java.security.PublicKey");  // component type (implicit NAME, name id 1)
      for (uint32_t k = 0; k < nkeys; k++) {
        if (p + 4 > end) return false;
        const uint32_t kid = p[0] | (p[1] << 8), kl = p[2] | (p[3] << 8);
        p += 4;
        if (kl == 0 || p + kl > end) return false;
        key_value(sig, kid, p, kl);  // writeClassAndObject per element
        p += kl;
      }
      if (p != end) return false;
      // the command data: implicit NAME (name id 2), its own CompatibleFieldSerializer
      // (field "<SimpleName>.nonce", a primitive long: writeLong(v, false))
      const size_t cut = name.find_last_of("$.");
      const std::string simple = (cut == std::string::npos ? name : name.substr(cut + 1)) + ".nonce";
      Out val;
      val.class_name(2, name.c_str());
      fields_header(val, {simple.c_str()});
      Out nonce;
      nonce.varlong_zigzag(it.value);
      val.chunked(nonce);
      o.class_name(0, "net.corda.core.contracts.Command");
      fields_header(o, {"Command.signers", "Command.value"});
      o.chunked(sig);
      o.chunked(val);
      return true;
    }
    default: return false;
  }
}

}  // namespace

extern "C" int cordahip_kryo_encode(const cordahip_kryo_item* items, uint64_t n, uint8_t* out, uint64_t cap,
                                    uint64_t* off) {
  if ((n && !items) || !off) return CORDAHIP_ERR_INVALID_ARG;
  Out o;
  off[0] = 0;
  for (uint64_t i = 0; i < n; i++) {
    if (!encode(items[i], o)) return CORDAHIP_ERR_INVALID_ARG;
    off[i + 1] = o.b.size();
  }
  if (o.b.size() > cap || (o.b.size() && !out)) return CORDAHIP_ERR_BUFFER_TOO_SMALL;
  if (o.b.size()) std::memcpy(out, o.b.data(), o.b.size());
  return CORDAHIP_SUCCESS;
}
