// Kryo leaf encoder core, shared by the host entry point (kryo.cpp,
// cordahip_kryo_encode) and the GPU one (kryo_device.hip, cordahip_kryo_encode_device):
// the p2p Kryo preimages of transaction components, i.e. what serializedHash
// hashes (core/.../transactions/MerkleTransaction.kt:16-18):
//   "corda\0\0\1" (Kryo.kt:101) + kryo.writeClassAndObject(x) (Kryo.kt:165-176)
// with references off (withoutReferences). Wire primitives restate Kryo 4.0.0's
// published Output format (writeVarInt, writeString, big-endian fixed-width
// writes); class headers are DefaultClassResolver.writeClass (registered: id + 2;
// implicitly registered Kotlin objects: NAME + 2, name id, class name), the
// bodies are Corda's serializers (Kryo.kt:383-393, :441-451) or Kryo's default
// primitive serializers. See include/cordahip.h for the kinds.
//
// Written once for both sides: no allocation, no std::string, no recursion but
// the bounded flush cascade, fixed-size level buffers supplied by the caller
// (a thread_local array on the host, a slice of a workspace on the GPU), and a
// counting mode (no buffers, no output) that yields a leaf's exact size.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/cordahip.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define KRYO_HD __host__ __device__
#else
#define KRYO_HD
#endif

namespace cordahip {
namespace kryo {

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
constexpr uint32_t kChunk = 1024;
constexpr uint32_t kMaxDepth = 8;                   // levels 0..7 (a cash-state leaf uses 0..6)
constexpr uint32_t kLevelBytes = (kMaxDepth - 1) * kChunk;  // per-encoder level buffers: levels 1..7

KRYO_HD inline uint32_t kmin(uint32_t a, uint32_t b) { return a < b ? a : b; }


// a byte string view that works on both sides (names are ASCII literals or
// caller bytes)
struct Sv {
  const char* p;
  uint32_t n;
  KRYO_HD Sv() : p(""), n(0) {}
  template <uint32_t N>
  KRYO_HD Sv(const char (&s)[N]) : p(s), n(N - 1) {}  // NOLINT: implicit from literals
  KRYO_HD Sv(const char* s) : p(s), n(0) {  // NOLINT: a runtime C string
    while (s[n]) n++;
  }
  KRYO_HD Sv(const char* s, uint32_t m) : p(s), n(m) {}
};
KRYO_HD inline bool operator==(const Sv& a, const Sv& b) {
  if (a.n != b.n) return false;
  if (a.p == b.p) return true;  // the same literal (class names are compared often)
  // class names share long prefixes ("net.corda.core.contracts."): test the end first
  if (a.n && a.p[a.n - 1] != b.p[a.n - 1]) return false;
  for (uint32_t i = 0; i < a.n; i++)
    if (a.p[i] != b.p[i]) return false;
  return true;
}
KRYO_HD inline bool operator<(const Sv& a, const Sv& b) {  // std::string order (bytes as unsigned)
  const uint32_t m = kmin(a.n, b.n);
  for (uint32_t i = 0; i < m; i++)
    if (a.p[i] != b.p[i]) return (uint8_t)a.p[i] < (uint8_t)b.p[i];
  return a.n < b.n;
}

// ---- trace symbols (KoutT<true>) -------------------------------------------
// The GPU encoder builds one template per leaf *shape* (kryo_template.hpp): it
// encodes a representative item once with every byte as a 32-bit symbol that
// says where the byte comes from -- a constant of the shape, byte `off` of the
// item's payload (optionally with bit 7 set: the last byte of an ASCII string),
// or byte j of the item's `value` as Kryo writes it (zig-zag varlong, or
// big-endian fixed width) -- and every item of that shape is then written from
// the symbols (sym_byte) without running the encoder.
constexpr uint32_t kSymConst = 0u << 30, kSymPayload = 1u << 30, kSymValZz = 2u << 30, kSymValBe = 3u << 30;
constexpr uint32_t kSymTypeMask = 3u << 30;
constexpr uint32_t kSymOr80 = 1u << 29;
constexpr uint32_t kMaxPayloadOff = 1u << 21;  // payload offsets a symbol can name (bits 8..28)

// Level-0 byte sink (KoutT's Sink): NoSink for the leaf in memory (or counting);
// kryo_device.hip's hashing sink takes the leaf's bytes as they are written and
// compresses them into a SHA-256 state (the direct encoder's leaves then need no
// buffer). A sink keeps at least the last byte written until the next one
// arrives: mark() sets bit 7 of it (an ASCII string's end mark).
struct NoSink {
  static constexpr bool kActive = false;
  KRYO_HD void put(uint8_t) {}
  KRYO_HD void write(const uint8_t*, uint64_t) {}
  KRYO_HD void mark() {}
};

template <bool Trace, class Sink = NoSink>
struct KoutT {
  using Sym = typename std::conditional<Trace, uint32_t, uint8_t>::type;
  Sink* sink = nullptr;  // level 0 into this sink instead of `out` (out must be nullptr, buf set)
  Sym* out;          // level 0 (the leaf); nullptr: counting
  uint64_t pos = 0;  // level-0 bytes so far (also past cap)
  uint64_t cap;      // writes at or beyond cap are dropped (pos still counts them)
  Sym* buf;          // levels 1..kMaxDepth-1, kChunk each (kLevelBytes symbols); nullptr: counting
  uint32_t len[kMaxDepth];
  uint32_t depth = 0;   // the deepest level in use
  bool failed = false;  // nesting or a graph beyond the fixed tables, a bad payload
  // trace only: the item's payload (bytes copied from it become PAYLOAD symbols)
  // and the value tag of the bytes being written (VAL_* | byte index << 8)
  const uint8_t* src = nullptr;
  uint64_t src_len = 0;
  uint32_t vtag = 0;
  KRYO_HD KoutT(Sym* o, uint64_t c, Sym* levels) : out(o), cap(c), buf(levels) { len[0] = 0; }
  KRYO_HD Sym& at(uint32_t k, uint32_t i) { return buf[(size_t)(k - 1) * kChunk + i]; }  // k >= 1
  KRYO_HD void set_vtag(uint32_t t) {
    if constexpr (Trace) vtag = t;
    else (void)t;
  }
  // the symbol of byte p[j] (the byte itself when not tracing)
  KRYO_HD Sym sym(const uint8_t* p, uint32_t j) {
    if constexpr (Trace) {
      const uint8_t b = p[j];
      const uintptr_t a = (uintptr_t)(p + j), lo = (uintptr_t)src;
      if (src && a >= lo && a - lo < src_len) {
        if (a - lo >= kMaxPayloadOff) failed = true;
        return kSymPayload | ((uint32_t)(a - lo) << 8) | b;
      }
      return vtag ? ((vtag + (j << 8)) | b) : (uint32_t)b;
    } else {
      return p[j];
    }
  }
  KRYO_HD static void mark(Sym& x) {
    x |= 0x80;
    if constexpr (Trace)
      if ((x & kSymTypeMask) == kSymPayload) x |= kSymOr80;
  }
  KRYO_HD uint32_t push_level() {
    if (depth + 1 >= kMaxDepth) {
      failed = true;
      return depth;  // keeps writing into the deepest level; the leaf is rejected
    }
    len[++depth] = 0;
    return depth;
  }
  KRYO_HD void pop_level() {
    if (!failed && depth > 0) depth--;
  }
  KRYO_HD void put0(uint8_t b) {
    if constexpr (Sink::kActive) sink->put(b);
    else if (out && pos < cap) out[pos] = b;
    pos++;
  }
  KRYO_HD void put(uint32_t k, uint8_t b) {  // raw append (the caller has made room)
    if (k == 0) {
      put0(b);
    } else {
      if (buf) at(k, len[k]) = b;
      len[k]++;
    }
  }
  KRYO_HD void mark_last(uint32_t k) {  // the last byte written carries the end mark (ASCII strings)
    if (k == 0) {
      if constexpr (Sink::kActive) sink->mark();
      else if (out && pos - 1 < cap) mark(out[pos - 1]);
    } else if (buf) {
      mark(at(k, len[k] - 1));
    }
  }
  KRYO_HD void copy(uint32_t k, const uint8_t* p, uint32_t n) {  // n bytes that fit
    if (k == 0) {
      if constexpr (Sink::kActive) {
        sink->write(p, n);
      } else if (out) {
        bool done = false;
        if constexpr (!Trace) {
          if (pos + n <= cap) {
            __builtin_memcpy(out + pos, p, n);
            done = true;
          }
        }
        if (!done)
          for (uint32_t i = 0; i < n; i++)
            if (pos + i < cap) out[pos + i] = sym(p, i);
      }
      pos += n;
    } else {
      if (buf) {
        if constexpr (!Trace) {
          __builtin_memcpy(&at(k, len[k]), p, n);
        } else {
          for (uint32_t i = 0; i < n; i++) at(k, len[k] + i) = sym(p, i);
        }
      }
      len[k] += n;
    }
  }
  KRYO_HD void put_syms0(const Sym* p, uint32_t n) {  // a flushed level-1 chunk into the leaf
    if constexpr (Sink::kActive) {
      if constexpr (Trace) {
        for (uint32_t i = 0; i < n; i++) sink->put((uint8_t)p[i]);
      } else {
        sink->write(p, n);
      }
    } else if (out) {
      if (pos + n <= cap) {
        __builtin_memcpy(out + pos, p, (size_t)n * sizeof(Sym));
      } else {
        for (uint32_t i = 0; i < n; i++)
          if (pos + i < cap) out[pos + i] = p[i];
      }
    }
    pos += n;
  }
  // Output.require(n) at level k. A flush writes into the level below, which may
  // itself need a flush there, and so on: D counts that nesting, so the call
  // graph is a fixed chain of instances (no recursion: the GPU side gets a
  // static stack) -- at most one nested flush per level
  template <uint32_t D = 0>
  KRYO_HD void require(uint32_t k, uint32_t n) {
    if (k > 0 && kChunk - len[k] < n) {
      if constexpr (D <= kMaxDepth) flush<D>(k);
      else failed = true;  // unreachable: a nested flush is always one level lower
    }
  }
  KRYO_HD void prim(uint32_t k, const uint8_t* p, uint32_t n) {  // an atomic write (require(n), then copy)
    require(k, n);
    copy(k, p, n);
  }
  KRYO_HD void byte(uint32_t k, uint32_t v) {
    const uint8_t b = (uint8_t)v;
    prim(k, &b, 1);
  }
  KRYO_HD void bytes(uint32_t k, const uint8_t* p, uint64_t n) {  // Output.writeBytes: fill, flush, continue
    if (k == 0) {
      while (n) {
        const uint32_t c = (uint32_t)(n < kChunk ? n : kChunk);
        copy(0, p, c);
        p += c;
        n -= c;
      }
      return;
    }
    uint32_t c = (uint32_t)(n < (uint64_t)(kChunk - len[k]) ? n : kChunk - len[k]);
    for (;;) {
      copy(k, p, c);
      p += c;
      n -= c;
      if (n == 0) return;
      c = (uint32_t)(n < kChunk ? n : kChunk);
      require(k, c);
    }
  }
  KRYO_HD void varint(uint32_t k, uint32_t v) {  // Output.writeVarInt(v, true)
    uint8_t t[5];
    uint32_t m = 0;
    while (v >> 7) {
      t[m++] = (uint8_t)((v & 0x7f) | 0x80);
      v >>= 7;
    }
    t[m++] = (uint8_t)v;
    prim(k, t, m);
  }
  KRYO_HD void varlong_zigzag(uint32_t k, int64_t x) {  // Output.writeVarLong(v, false)
    uint64_t v = ((uint64_t)x << 1) ^ (uint64_t)(x >> 63);
    uint8_t t[9];
    uint32_t m = 0;
    for (int i = 0; i < 8 && (v >> 7); i++) {
      t[m++] = (uint8_t)((v & 0x7f) | 0x80);
      v >>= 7;
    }
    t[m++] = (uint8_t)v;
    prim(k, t, m);
  }
  KRYO_HD void varint_zigzag(uint32_t k, int32_t x) {  // Output.writeVarInt(v, false)
    varint(k, ((uint32_t)x << 1) ^ (uint32_t)(x >> 31));
  }
  // OutputChunked.flush at level k: its chunk (varint size, then the bytes) to
  // level k - 1, whose own flush follows (Output.flush flushes the stream). The
  // writes into k - 1 can only flush levels below k, so level k's buffer stays
  // intact while it is copied out; the cascade is at most kMaxDepth deep.
  template <uint32_t D = 0>
  KRYO_HD void flush(uint32_t k) {
    for (; k > 0; k--) {
      if (len[k] == 0) continue;
      const uint32_t n = len[k];
      len[k] = 0;
      uint32_t sz = n;
      while (sz >> 7) {  // writeChunkSize: one stream.write(int) per byte
        require<D + 1>(k - 1, 1);
        put(k - 1, (uint8_t)((sz & 0x7f) | 0x80));
        sz >>= 7;
      }
      require<D + 1>(k - 1, 1);
      put(k - 1, (uint8_t)sz);
      chunk_bytes<D + 1>(k - 1, k, n);
    }
  }
  // writeBytes of level `from`'s flushed chunk (its first n bytes) into level k = from - 1
  template <uint32_t D>
  KRYO_HD void chunk_bytes(uint32_t k, uint32_t from, uint32_t n) {
    uint32_t s = 0;  // next source byte
    if (k == 0) {
      if (!buf) pos += n;
      else put_syms0(&at(from, 0), n);
      return;
    }
    uint32_t c = kmin(kChunk - len[k], n);
    for (;;) {
      if (buf) __builtin_memcpy(&at(k, len[k]), &at(from, s), (size_t)c * sizeof(Sym));
      len[k] += c;
      s += c;
      n -= c;
      if (n == 0) return;
      c = kmin(kChunk, n);
      require<D>(k, c);
    }
  }
  KRYO_HD void end_chunks(uint32_t k) {
    flush(k);
    byte(k - 1, 0);
  }
  // Output.writeString over code units unit(i), i < n (Java String semantics:
  // UTF-16 units, or the bytes of an ASCII name)
  template <class U>
  KRYO_HD void string(uint32_t k, U unit, uint64_t n) {
    if (n == 0) {
      byte(k, 1 | 0x80);  // empty string
      return;
    }
    bool ascii = n > 1 && n < 64;
    for (uint64_t i = 0; ascii && i < n; i++) ascii = unit(i) <= 127;
    if (ascii) {
      uint8_t t[64];
      for (uint64_t i = 0; i < n; i++) t[i] = (uint8_t)unit(i);
      bytes(k, t, n);
      mark_last(k);
      return;
    }
    utf8_length(k, (uint32_t)n + 1);
    uint64_t i = 0;
    if (k == 0 || kChunk - len[k] >= n)  // the 8-bit fast path while it fits
      for (; i < n && unit(i) <= 127; i++) put(k, (uint8_t)unit(i));
    for (; i < n; i++) {  // writeString_slow
      if (k > 0 && len[k] == kChunk) require(k, (uint32_t)(n - i < kChunk ? n - i : kChunk));
      const uint32_t x = unit(i);
      if (x <= 0x7f) {
        put(k, (uint8_t)x);
      } else if (x > 0x7ff) {
        put(k, (uint8_t)(0xe0 | ((x >> 12) & 0x0f)));
        require(k, 2);
        put(k, (uint8_t)(0x80 | ((x >> 6) & 0x3f)));
        put(k, (uint8_t)(0x80 | (x & 0x3f)));
      } else {
        put(k, (uint8_t)(0xc0 | ((x >> 6) & 0x1f)));
        require(k, 1);
        put(k, (uint8_t)(0x80 | (x & 0x3f)));
      }
    }
  }
  // Output.writeUtf8Length: bit 8 of the first byte flags UTF-8, bit 7 "more"
  KRYO_HD void utf8_length(uint32_t k, uint32_t v) {
    uint8_t t[5];
    uint32_t m = 0;
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
  KRYO_HD void ascii(uint32_t k, const Sv& s) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(s.p);
    bool fast = s.n > 1 && s.n < 64;  // writeString's ASCII path, straight from the name's bytes
    for (uint32_t i = 0; fast && i < s.n; i++) fast = p[i] <= 127;
    if (fast) {
      bytes(k, p, s.n);
      mark_last(k);
      return;
    }
    string(k, [&](uint64_t i) { return (uint32_t)p[i]; }, s.n);
  }
  KRYO_HD void utf16le(uint32_t k, const uint8_t* p, uint64_t n) {  // Java String from UTF-16LE units
    string(k, [&](uint64_t i) { return (uint32_t)(p[2 * i] | (p[2 * i + 1] << 8)); }, n);
  }
};
using Kout = KoutT<false>;

// One object graph (Kryo.writeClassAndObject resets both at the top level):
// DefaultClassResolver's class-name ids and CompatibleFieldSerializer's
// "header written" marks.
struct Graph {
  static constexpr uint32_t kMaxNames = 16;  // a cash-state graph names 11 classes
  Sv names[kMaxNames] = {};
  uint32_t nnames = 0;
  Sv headers[kMaxNames] = {};
  uint32_t nheaders = 0;
  KRYO_HD Graph() {}
  // DefaultClassResolver.writeClass for a registered class: varint(id + 2)
  template <class O>
  KRYO_HD static void class_id(O& o, uint32_t k, uint32_t id) { o.varint(k, id + 2); }
  // DefaultClassResolver.writeName: NAME + 2, the graph's name id, and the class
  // name the first time the class occurs in the graph
  template <class O>
  KRYO_HD void class_name(O& o, uint32_t k, const Sv& name) {
    o.varint(k, kName + 2);
    for (uint32_t i = 0; i < nnames; i++)
      if (names[i] == name) {
        o.varint(k, i);
        return;
      }
    if (nnames == kMaxNames) {
      o.failed = true;
      return;
    }
    names[nnames++] = name;
    o.varint(k, nnames - 1);
    o.ascii(k, name);
  }
  // CompatibleFieldSerializer.write of one object of class `cls` at level k:
  // header (once per graph), then each field through the OutputChunked at level
  // k + 1. The fields come in sorted EXTENDED-name order (checked: an unsorted
  // list fails the leaf rather than mis-frame it).
  template <class O, uint32_t N, class... F>
  KRYO_HD void cfs(O& o, uint32_t k, const Sv& cls, const Sv (&fields)[N], F&&... write) {
    static_assert(N == sizeof...(F), "one writer per field");
    for (uint32_t i = 1; i < N; i++)
      if (!(fields[i - 1] < fields[i])) o.failed = true;
    bool seen = false;
    for (uint32_t i = 0; i < nheaders && !seen; i++) seen = headers[i] == cls;
    if (!seen) {
      if (nheaders == kMaxNames) {
        o.failed = true;
        return;
      }
      headers[nheaders++] = cls;
      o.varint(k, N);
      for (uint32_t i = 0; i < N; i++) o.ascii(k, fields[i]);
    }
    const uint32_t c = o.push_level();
    ((write(c), o.end_chunks(c)), ...);
    o.pop_level();
  }
};

// a public key as a field / element of unknown concrete type: its class
// (registered: Ed25519PublicKeySerializer or PublicKeySerializer, Kryo.kt:383-393,
// :441-451), then writeBytesWithLength (Kryo.kt:305-308: writeInt(size, true) +
// writeBytes) -- the same bytes for both serializers
template <class O>
KRYO_HD inline void key_value(O& o, uint32_t k, uint32_t key_class, const uint8_t* key, uint64_t n) {
  Graph::class_id(o, k, key_class);
  o.varint(k, (uint32_t)n);
  o.bytes(k, key, n);
}

// Length of a DER TLV at p (definite form), 0 if malformed / longer than n.
KRYO_HD inline uint64_t der_tlv_len(const uint8_t* p, uint64_t n) {
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
  KRYO_HD Reader(const uint8_t* a, const uint8_t* b) : p(a), end(b) {}
  KRYO_HD bool take(uint64_t n) {
    if (!ok || (uint64_t)(end - p) < n) return ok = false;
    p += n;
    return true;
  }
  KRYO_HD uint32_t u8() { return take(1) ? p[-1] : 0; }
  KRYO_HD uint32_t u16() { return take(2) ? (uint32_t)(p[-2] | (p[-1] << 8)) : 0; }
  KRYO_HD const uint8_t* span(uint64_t n) { return take(n) ? p - n : nullptr; }
  KRYO_HD PartyRef party() {
    PartyRef r;
    r.key_class = u16();
    r.key_len = u16();
    r.key = span(r.key_len);
    r.name_len = u16();
    r.name = span(r.name_len);
    // a truncated payload leaves name null with name_len set: test ok first
    if (!ok || r.key_len == 0 || (r.name_len && (der_tlv_len(r.name, r.name_len) != r.name_len || r.name[0] != 0x30)))
      ok = false;
    return r;
  }
};

// net.corda.core.identity.Party(name: X500Name, owningKey: PublicKey) (identity/Party.kt,
// AbstractParty.kt) or AnonymousParty(owningKey) (AnonymousParty.kt): the class (when
// written) by implicit NAME registration (CordaClassResolver.registerImplicit), then
// CompatibleFieldSerializer over AbstractParty.owningKey and Party.name; the name
// through X500NameSerializer (Kryo.kt:615-624: writeBytes(encoded), no length).
template <class O>
KRYO_HD inline void party_body(O& o, Graph& g, uint32_t k, const PartyRef& p, uint32_t x500_class) {
  auto key = [&](uint32_t c) { key_value(o, c, p.key_class, p.key, p.key_len); };
  if (p.name_len)
    g.cfs(o, k, "net.corda.core.identity.Party", {"AbstractParty.owningKey", "Party.name"}, key, [&](uint32_t c) {
      Graph::class_id(o, c, x500_class);
      o.bytes(c, p.name, p.name_len);
    });
  else
    g.cfs(o, k, "net.corda.core.identity.AnonymousParty", {"AbstractParty.owningKey"}, key);
}
template <class O>
KRYO_HD inline void party_class_and_object(O& o, Graph& g, uint32_t k, const PartyRef& p, uint32_t x500_class) {
  g.class_name(o, k, p.name_len ? "net.corda.core.identity.Party" : "net.corda.core.identity.AnonymousParty");
  party_body(o, g, k, p, x500_class);
}

// net.corda.core.utilities.OpaqueBytes / SecureHash$SHA256 (utilities/ByteArrays.kt:16,
// crypto/SecureHash.kt:13-15): one field OpaqueBytes.bytes, a byte[] (a final
// class: no class written; ByteArraySerializer accepts null, so no null marker):
// varint(length + 1), the bytes
template <class O>
KRYO_HD inline void opaque_bytes(O& o, Graph& g, uint32_t k, const Sv& cls, const uint8_t* b, uint64_t n) {
  g.class_name(o, k, cls);
  g.cfs(o, k, cls, {"OpaqueBytes.bytes"}, [&](uint32_t c) {
    o.varint(c, (uint32_t)n + 1);
    o.bytes(c, b, n);
  });
}

KRYO_HD inline bool same_key(const PartyRef& a, const PartyRef& b) {
  if (a.key_class != b.key_class || a.key_len != b.key_len) return false;
  for (uint32_t i = 0; i < a.key_len; i++)
    if (a.key[i] != b.key[i]) return false;
  return true;
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
template <class O>
KRYO_HD inline bool cash_state(O& o, const cordahip_kryo_item& it) {
  Reader r(it.data, it.data + it.len);
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
  g.cfs(o, 0, "net.corda.core.contracts.TransactionState",
        {"TransactionState.data", "TransactionState.encumbrance", "TransactionState.notary"},
        [&](uint32_t k1) {  // data
          g.class_name(o, k1, "net.corda.contracts.asset.Cash$State");
          g.cfs(o, k1, "net.corda.contracts.asset.Cash$State",
                {"State.amount", "State.contract", "State.exitKeys", "State.owner", "State.participants"},
                [&](uint32_t k2) {  // amount
                  o.byte(k2, 1);    // NOT_NULL
                  g.cfs(o, k2, "net.corda.core.contracts.Amount",
                        {"Amount.displayTokenSize", "Amount.quantity", "Amount.token"},
                        [&](uint32_t k3) {
                          g.class_name(o, k3, "java.math.BigDecimal");
                          o.varint(k3, 2);  // BigInteger.ONE.toByteArray() = {1}: varint(1 + 1), 01
                          o.byte(k3, 1);
                          // Currency: ONE.scaleByPowerOfTen(-digits), Amount.kt:70-80
                          o.varint_zigzag(k3, (int32_t)(int8_t)scale);
                        },
                        [&](uint32_t k3) {  // the item's value: VALUE symbols when tracing
                          o.set_vtag(kSymValZz);
                          o.varlong_zigzag(k3, quantity);
                          o.set_vtag(0);
                        },
                        [&](uint32_t k3) {  // token
                          g.class_name(o, k3, "net.corda.core.contracts.Issued");
                          g.cfs(o, k3, "net.corda.core.contracts.Issued", {"Issued.issuer", "Issued.product"},
                                [&](uint32_t k4) {
                                  o.byte(k4, 1);  // NOT_NULL
                                  g.cfs(o, k4, "net.corda.core.contracts.PartyAndReference",
                                        {"PartyAndReference.party", "PartyAndReference.reference"},
                                        [&](uint32_t k5) { party_class_and_object(o, g, k5, issuer, x500); },
                                        [&](uint32_t k5) {
                                          opaque_bytes(o, g, k5, "net.corda.core.utilities.OpaqueBytes", ref, ref_len);
                                        });
                                },
                                [&](uint32_t k4) {
                                  g.class_name(o, k4, "java.util.Currency");
                                  o.ascii(k4, Sv((const char*)code, code_len));
                                });
                        });
                },
                [&](uint32_t k2) {  // contract
                  o.byte(k2, 1);    // NOT_NULL
                  g.cfs(o, k2, "net.corda.contracts.asset.Cash", {"Cash.legalContractReference"}, [&](uint32_t k3) {
                    opaque_bytes(o, g, k3, "net.corda.core.crypto.SecureHash$SHA256", legal, 32);
                  });
                },
                [&](uint32_t k2) {  // exitKeys
                  g.class_name(o, k2, "java.util.LinkedHashSet");
                  const bool one = same_key(owner, issuer);  // a set: one element when the keys are equal
                  o.varint(k2, one ? 1 : 2);
                  key_value(o, k2, owner.key_class, owner.key, owner.key_len);
                  if (!one) key_value(o, k2, issuer.key_class, issuer.key, issuer.key_len);
                },
                [&](uint32_t k2) { party_class_and_object(o, g, k2, owner, x500); },  // owner
                [&](uint32_t k2) {  // participants
                  g.class_name(o, k2, "java.util.Collections$SingletonList");
                  party_class_and_object(o, g, k2, owner, x500);
                });
        },
        [&](uint32_t k1) {  // encumbrance
          if (flags & 1u) {
            o.byte(k1, 1);  // NOT_NULL, then IntSerializer: writeInt(v, false)
            o.varint_zigzag(k1, (int32_t)(enc[0] | (enc[1] << 8) | (enc[2] << 16) | ((uint32_t)enc[3] << 24)));
          } else {
            o.byte(k1, 0);  // NULL
          }
        },
        [&](uint32_t k1) {  // notary
          o.byte(k1, 1);    // NOT_NULL (Party is final)
          party_body(o, g, k1, notary, x500);
        });
  return true;
}

// net.corda.core.contracts.Command(value, signers) (contracts/Structures.kt:285)
// as TransactionBuilder.addCommand(data, vararg keys) builds it
// (TransactionBuilder.kt:124: listOf(*keys) = java.util.Arrays$ArrayList over a
// PublicKey[]), value = an issue command data class with one `nonce: Long` field
// (Cash / CommodityContract / Obligation Commands.Issue, e.g. Cash.kt:148;
// OnLedgerAsset.generateIssue, OnLedgerAsset.kt:208-219). data = u8 name length,
// the command class's binary name, u8 key count, per key u16 LE registration id,
// u16 LE length, the key bytes; class_id = the Arrays$ArrayList registration
// (ArraysAsListSerializer); value = the nonce.
template <class O>
KRYO_HD inline bool issue_command(O& o, const cordahip_kryo_item& it) {
  if (!it.data || it.len < 2) return false;
  Reader r(it.data, it.data + it.len);
  const uint32_t nlen = r.u8();
  const uint8_t* nm = r.span(nlen);
  const uint32_t nkeys = r.u8();
  if (!r.ok || nlen < 2 || nkeys == 0) return false;  // Command: require(signers.isNotEmpty())
  const uint8_t* keys = r.p;  // validated here, read again while writing
  for (uint32_t i = 0; i < nkeys; i++) {
    r.u16();
    const uint32_t kl = r.u16();
    if (!r.span(kl) || kl == 0) return false;
  }
  if (!r.ok || r.p != r.end) return false;
  const Sv name((const char*)nm, nlen);
  uint32_t cut = nlen;  // the simple name follows the last '$' or '.'
  while (cut > 0 && nm[cut - 1] != '$' && nm[cut - 1] != '.') cut--;
  // "<Simple>.nonce" (EXTENDED field name) in a small local buffer
  char field[264];
  const uint32_t sl = nlen - cut;
  if (sl + 6 > sizeof(field)) return false;
  for (uint32_t i = 0; i < sl; i++) field[i] = (char)nm[cut + i];
  const char* suffix = ".nonce";
  for (uint32_t i = 0; i < 6; i++) field[sl + i] = suffix[i];
  const Sv simple(field, sl + 6);
  Graph g;
  g.class_name(o, 0, "net.corda.core.contracts.Command");
  g.cfs(o, 0, "net.corda.core.contracts.Command", {"Command.signers", "Command.value"},
        [&](uint32_t k) {
          // ArraysAsListSerializer (kryo-serializers 0.41): writeInt(length, true),
          // writeClass(component type) -- java.security.PublicKey, implicit NAME --
          // then writeClassAndObject per element
          Graph::class_id(o, k, it.class_id);
          o.varint(k, nkeys);
          g.class_name(o, k, "java.security.PublicKey");
          Reader kr(keys, it.data + it.len);
          for (uint32_t i = 0; i < nkeys; i++) {
            const uint32_t kc = kr.u16(), kl = kr.u16();
            key_value(o, k, kc, kr.span(kl), kl);
          }
        },
        [&](uint32_t k) {
          // the command data: implicit NAME, its own CompatibleFieldSerializer (a
          // primitive long nonce: writeVarLong(v, false)) -- a nested OutputChunked
          g.class_name(o, k, name);
          g.cfs(o, k, name, {simple}, [&](uint32_t c) {
            o.set_vtag(kSymValZz);  // the item's value: VALUE symbols when tracing
            o.varlong_zigzag(c, it.value);
            o.set_vtag(0);
          });
        });
  return true;
}

// One component's leaf preimage through o (RAW: the bytes as given); false for
// an unknown kind or a missing / malformed payload.
template <class O>
KRYO_HD inline bool encode_leaf(O& o, const cordahip_kryo_item& it) {
  if (it.kind == CORDAHIP_KRYO_RAW) {
    if (it.len && !it.data) return false;
    o.bytes(0, it.data, it.len);
    return true;
  }
  const uint8_t header[8] = {'c', 'o', 'r', 'd', 'a', 0, 0, 1};  // KryoHeaderV0_1
  o.bytes(0, header, 8);
  const uint64_t v = (uint64_t)it.value;
  auto be = [&](uint64_t x, int n) {  // the item's value, big-endian: VALUE symbols when tracing
    for (int i = n - 1; i >= 0; i--) {
      o.set_vtag(kSymValBe | ((uint32_t)i << 8));
      o.byte(0, (uint32_t)(x >> (8 * i)));
    }
    o.set_vtag(0);
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
    case CORDAHIP_KRYO_STRING:
      if (it.len && !it.data) return false;
      Graph::class_id(o, 0, kIdString);
      o.utf16le(0, it.data, it.len);
      break;
    case CORDAHIP_KRYO_ED25519_KEY:  // Ed25519PublicKeySerializer: writeBytesWithLength(abyte)
      if (!it.data || it.len != 32) return false;
      key_value(o, 0, it.class_id, it.data, 32);
      break;
    case CORDAHIP_KRYO_PUBLIC_KEY:  // PublicKeySerializer: writeBytesWithLength(key.encoded)
      if (!it.data || it.len == 0 || it.len > 0x7fffffffull) return false;
      key_value(o, 0, it.class_id, it.data, it.len);
      break;
    case CORDAHIP_KRYO_KOTLIN_OBJECT:  // NAME registration, KotlinObjectSerializer writes no body
      if (!it.data || it.len == 0) return false;
      o.varint(0, kName + 2);  // = 1
      o.varint(0, 0);          // first class name of this object graph: name id 0
      o.utf16le(0, it.data, it.len);
      break;
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
    case CORDAHIP_KRYO_ISSUE_COMMAND: ok = issue_command(o, it); break;
    case CORDAHIP_KRYO_CASH_STATE: ok = it.data && cash_state(o, it); break;
    default: return false;
  }
  return ok && !o.failed;
}

}  // namespace kryo
}  // namespace cordahip
