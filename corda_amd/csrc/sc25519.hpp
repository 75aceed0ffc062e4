// Scalars modulo L = 2^252 + 27742317777372353535851937790883648493 and the
// scalar recodings the verify kernel uses.
//
// Semantics that must match the reference engine (i2p eddsa 0.2.0,
// SURVEY.md Appendix A.1, restated in oracle/i2p_ed25519.py):
//   * h = SHA-512(R || Abyte || M) reduced mod L        (ScalarOps.reduce)
//   * S is NOT range checked; its effective value is what GroupElement.slide()
//     encodes, i.e. S, or S - 2^256 when slide's carry runs past bit 255
//     (slide_drops_carry below). Since B has order L, only S_eff mod L matters,
//     so the kernel is free to use a different (fixed-window, SIMD-uniform)
//     recoding of S_eff mod L for the actual multiplication.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef CDEV
#define CDEV __device__ __forceinline__
#endif

namespace cordahip {

// L, mu = floor(2^512 / L), 2^256 mod L as little-endian 32-bit words
CDEV uint32_t sc_L(int i) {
  const uint32_t c[8] = {0x5cf5d3ed, 0x5812631a, 0xa2f79cd6, 0x14def9de, 0x0, 0x0, 0x0, 0x10000000};
  return c[i];
}
CDEV uint32_t sc_mu(int i) {
  const uint32_t c[9] = {0x0a2c131b, 0xed9ce5a3, 0x086329a7, 0x2106215d, 0xffffffeb,
                         0xffffffff, 0xffffffff, 0xffffffff, 0xf};
  return c[i];
}
CDEV uint32_t sc_2p256(int i) {
  const uint32_t c[8] = {0x8d98951d, 0xd6ec3174, 0x737dcf70, 0xc6ef5bf4,
                         0xfffffffe, 0xffffffff, 0xffffffff, 0x0fffffff};
  return c[i];
}

// r (9 words) >= L ?  (branch-free borrow chain)
CDEV bool sc_geq_L9(const uint32_t r[9]) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) br = (uint32_t)(((uint64_t)r[i] - sc_L(i) - br) >> 63);
  return r[8] != 0 || br == 0;
}

CDEV void sc_sub_L9(uint32_t r[9]) {
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint64_t d = (uint64_t)r[i] - (i < 8 ? sc_L(i) : 0u) - borrow;
    r[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
}

// Barrett reduction (HAC 14.42, b = 2^32, k = 8) of a 512-bit x mod L.
CDEV void sc_reduce512(uint32_t out[8], const uint32_t x[16]) {
  // q2 = (x >> 224) * mu ; only words >= 9 are used (q3 = q2 >> 288)
  uint32_t p[18];
#pragma unroll
  for (int i = 0; i < 18; i++) p[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const uint64_t t = (uint64_t)x[7 + i] * sc_mu(j) + p[i + j] + carry;
      p[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    p[i + 9] = (uint32_t)carry;
  }
  // r2 = (q3 * L) mod 2^288 ; q3 = p[9..17]
  uint32_t r2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) r2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (i + j >= 9) break;
      const uint64_t t = (uint64_t)p[9 + i] * sc_L(j) + r2[i + j] + carry;
      r2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    if (i + 8 < 9) r2[i + 8] += (uint32_t)carry;
  }
  // r = x mod 2^288 - r2 (mod 2^288)
  uint32_t r[9];
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint64_t d = (uint64_t)x[i] - r2[i] - borrow;
    r[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
  if (sc_geq_L9(r)) sc_sub_L9(r);
  if (sc_geq_L9(r)) sc_sub_L9(r);
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = r[i];
}

// ---- exact emulation of i2p GroupElement.slide()'s carry drop -------------
// State: T = the bits at positions > i (positions <= i already became
// digits). At a set bit i the inner loop either absorbs bit i+b into the
// digit (clears it), or subtracts 2^b from the digit and adds 2^(i+b) to the
// upper bits (the Java carry loop), or stops. The carry loop never touches
// positions below i+b (they are zero at that moment), so it is exactly a
// 256-bit add of 2^(i+b) to T; its carry out of bit 255 is the dropped carry.
CDEV uint32_t word_sel(const uint32_t t[8], int w) {
  uint32_t r = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) r = (q == w) ? t[q] : r;
  return r;
}
CDEV uint32_t bit_at(const uint32_t t[8], int k) { return (word_sel(t, k >> 5) >> (k & 31)) & 1u; }
CDEV void clear_bit(uint32_t t[8], int k) {
  const int w = k >> 5;
  const uint32_t m = ~(1u << (k & 31));
#pragma unroll
  for (int q = 0; q < 8; q++) t[q] = (q == w) ? (t[q] & m) : t[q];
}
// t += 2^k ; returns carry out of bit 255
CDEV uint32_t add_pow2(uint32_t t[8], int k) {
  const int w = k >> 5;
  const uint32_t a = 1u << (k & 31);
  uint32_t c = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint32_t add = (q == w) ? a : 0u;
    const uint64_t s = (uint64_t)t[q] + add + c;
    t[q] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
  return c;
}

// A carry can only run out of bit 255 when bit 255 of S is set: checked
// exhaustively for every S of the same recoding at widths 8..19
// (tests/test_oracle.py::test_slide_drop_needs_top_bit), so lanes with
// S < 2^255 — every honest signature — skip the emulation.
CDEV bool slide_drops_carry(const uint32_t s[8]) {
  if (!(s[7] >> 31)) return false;
  uint32_t t[8];
#pragma unroll
  for (int q = 0; q < 8; q++) t[q] = s[q];
  uint32_t dropped = 0;
  for (int w = 0; w < 8; w++) {
    // skip zero bits a word at a time
    while (true) {
      const uint32_t cur = word_sel(t, w);
      if (cur == 0) break;
      const int i = w * 32 + __builtin_ctz(cur);
      clear_bit(t, i);
      int v = 1;
      for (int b = 1; b <= 6 && i + b < 256; b++) {
        if (!bit_at(t, i + b)) continue;
        if (v + (1 << b) <= 15) {
          v += 1 << b;
          clear_bit(t, i + b);
        } else if (v - (1 << b) >= -15) {
          v -= 1 << b;
          dropped |= add_pow2(t, i + b);
        } else {
          break;
        }
      }
    }
  }
  return dropped != 0;
}

// S_eff mod L where S_eff = S - 2^256 * dropped
CDEV void sc_effective_S(uint32_t out[8], const uint32_t s[8], bool dropped) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x[i] = s[i];
    x[8 + i] = 0;
  }
  uint32_t r[8];
  sc_reduce512(r, x);
  if (dropped) {
    // r = r - (2^256 mod L) mod L
    uint32_t d[9];
    uint64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint64_t t = (uint64_t)r[i] - sc_2p256(i) - borrow;
      d[i] = (uint32_t)t;
      borrow = (t >> 63) & 1;
    }
    if (borrow) {  // add L back
      uint64_t c = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const uint64_t t = (uint64_t)d[i] + sc_L(i) + c;
        d[i] = (uint32_t)t;
        c = t >> 32;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = d[i];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = r[i];
}

// Booth (signed fixed-window) digit j of width W for a scalar < 2^(256-1):
// d_j = b_{Wj-1} + sum_{t<W-1} 2^t b_{Wj+t} - 2^(W-1) b_{Wj+W-1}, in [-2^(W-1), 2^(W-1)].
// Uniform digit positions across lanes -> no divergence in the ladder.
template <int W>
CDEV int booth_digit(const uint32_t k[8], int j) {
  const int lo = W * j - 1;  // may be -1
  // gather W+1 bits starting at lo (bit -1 == 0)
  uint32_t v;
  if (lo < 0) {
    v = (k[0] << 1) & ((1u << (W + 1)) - 1);
  } else {
    const int w = lo >> 5, sh = lo & 31;
    const uint64_t pair = ((uint64_t)word_sel(k, w + 1 > 7 ? 7 : w + 1) << 32) | word_sel(k, w);
    const uint64_t hi_valid = (w + 1 > 7) ? 0 : 1;
    const uint64_t p2 = hi_valid ? pair : (pair & 0xffffffffull);
    v = (uint32_t)(p2 >> sh) & ((1u << (W + 1)) - 1);
  }
  return (int)((v + 1) >> 1) - (int)((v >> W) << W);
}

}  // namespace cordahip
