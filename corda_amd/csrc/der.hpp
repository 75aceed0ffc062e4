// Strict DER decoding of an ECDSA signature, BouncyCastle 1.57 rules
// (StdDSAEncoder.decode, reached from DSABase.engineVerify):
// SEQUENCE of exactly two INTEGERs, definite minimal lengths, nothing after
// the SEQUENCE, non-empty minimal INTEGER contents. Any violation is
// SignatureException("error decoding signature bytes.") = MALFORMED_SIG.
// Negative or oversized INTEGERs are well-formed DER: they fail the range
// check r, s in [1, n-1] later (BAD_SIG), exactly as ECDSASigner does.
//
// Shared by the GPU kernel (one lane per signature) and the host runtime
// (signatures longer than the kernel's 72-byte slot).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define CHD __host__ __device__ inline
#else
#define CHD inline
#endif

namespace cordahip {

struct DerInt {
  uint32_t v[8];  // magnitude (little-endian limbs) when fits
  bool neg;       // INTEGER encodes a negative value
  bool big;       // more than 32 significant bytes (>= 2^256)
};

CHD bool der_read_len(const uint8_t* b, uint32_t n, uint32_t& i, uint32_t& out) {
  if (i >= n) return false;
  const uint8_t l0 = b[i++];
  if (l0 < 0x80) {
    out = l0;
    return true;
  }
  const uint32_t nb = l0 & 0x7f;
  if (nb == 0 || nb > 4 || i + nb > n) return false;  // indefinite / oversized
  if (b[i] == 0) return false;                        // leading zero length byte: not minimal
  uint32_t v = 0;
  for (uint32_t k = 0; k < nb; k++) v = (v << 8) | b[i++];
  if (v < 0x80) return false;  // long form for a short length: not DER
  out = v;
  return true;
}

// returns false if malformed
CHD bool der_decode_sig(const uint8_t* sig, uint32_t n, DerInt& r, DerInt& s) {
  uint32_t i = 1, len = 0;
  if (n < 2 || sig[0] != 0x30) return false;
  if (!der_read_len(sig, n, i, len) || i + len != n) return false;
  for (int k = 0; k < 2; k++) {
    DerInt& d = k == 0 ? r : s;
    if (i >= n || sig[i++] != 0x02) return false;
    uint32_t l = 0;
    if (!der_read_len(sig, n, i, l) || l == 0 || i + l > n) return false;
    const uint8_t* body = sig + i;
    if (l > 1 && ((body[0] == 0 && body[1] < 0x80) || (body[0] == 0xff && body[1] >= 0x80))) return false;
    d.neg = body[0] >= 0x80;
    // more than 32 significant bytes: a nonzero byte above significance 31
    uint32_t hi = 0;
    for (uint32_t t = 0; t + 32 < l; t++) hi |= body[t];
    d.big = hi != 0;
    // the low 32 bytes by significance k (unrolled: every limb index is a
    // compile-time constant, so the limbs stay in registers on the GPU instead
    // of a scratch-memory array written byte by byte)
#pragma unroll
    for (int q = 0; q < 8; q++) d.v[q] = 0;
#pragma unroll
    for (int k = 0; k < 32; k++) {
      const bool in = (uint32_t)k < l;
      const uint32_t b = body[in ? l - 1 - k : 0] & (in ? 0xffu : 0u);  // address always inside the body
      d.v[k >> 2] |= b << (8 * (k & 3));
    }
    if (d.big) {
#pragma unroll
      for (int q = 0; q < 8; q++) d.v[q] = 0;
    }
    i += l;
  }
  return i == n;  // exactly two elements
}

}  // namespace cordahip
