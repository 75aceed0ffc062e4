// Base-field arithmetic of the two ECDSA curves (secp256k1, P-256) for
// gfx950 lanes: kernel K2's ladder, point tables and key decode.
//
// Representation: 9 unsigned 32-bit limbs in radix 2^29 (261 bits),
// Montgomery form with R = 2^261. Why this shape on CDNA4: a 32x32->64
// v_mad_u64_u32 issues at the same rate as an add (profiles/r01_int_rates.jsonl),
// so a field product costs its instruction count. With 29-bit limbs every
// column of the product AND of the Montgomery reduction (<= 9 + 9 terms of
// < 2^60) stays below 2^64: each partial product is ONE v_mad_u64_u32 into a
// 64-bit column accumulator, no carry instruction, and the column carry rides
// in the next column's addend. The saturated 8 x 32-bit Montgomery product
// (mp256.hpp, still used for the scalar field mod n) needs a v_addc_co_u32
// per partial product: ~1.5-2x the instructions.
//
// Lazy reduction (all bounds exact; modelled limb for limb, with assertions,
// by tests/test_fp29_model.py):
//   "norm"  limbs 0..7 < 2^29 (limbs 0, 1 may exceed it by < 2^15 after
//           f29_red), value < 2p. Outputs of f29_mul / f29_sqr / f29_red.
//   f29_mul(a, b): needs a * b < 2^261 p (e.g. a, b < 4p, or 2p x 16p) and
//           limb products <= 2^60.5 (both limbs <= 2^30.25, or one <= 2^29 and
//           the other <= 2^31.5). Output norm, < 2p.
//   f29_add: limb-wise, no carry (values and limb bounds add).
//   f29_sub(a, b) = a + 2p - b with one carry pass: b norm (value <= 2p),
//           a limbs < 2^31; output limbs normalised, value < a + 2p.
//   f29_red(a): limbs < 2^31.5, value < 2^260 -> norm (< 2p), by folding the
//           bits above 2^256 with 2^256 == 2^256 - p (mod p).
//   f29_canon: norm input -> the canonical residue in [0, p).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef CDEV
#define CDEV __device__ __forceinline__
#endif

namespace cordahip {

static constexpr uint32_t kMask29 = (1u << 29) - 1;

struct f29 {
  uint32_t v[9];
};

// A compile-time constant moved into an SGPR behind an empty asm: q * m then
// stays one v_mad_u64_u32 per limb (with the constant visible, InstCombine
// rewrites q * (2^29 - 1) as a 64-bit shift-subtract and factors equal
// constants out of a column's sum).
CDEV uint32_t sconst(uint32_t x) {
  asm("" : "+s"(x));
  return x;
}

// ---- Montgomery reduction in special form (both curves) --------------------
// r = (a b + Q p) / 2^261 with Q = sum q_k 2^(29 k) chosen column by column so
// that the low 261 bits vanish (product scanning: column k accumulates the
// a_j b_(k-j) and the q terms that land in it). The q_k and the result are
// those of a generic REDC over p's 9 limbs; only the q terms are cheaper:
//   P-256: p = 2^256 - 2^224 + 2^192 + 2^96 - 1 == -1 (mod 2^29), so
//     q_k = column mod 2^29 and its -q_k term clears exactly those bits (the
//     shift does it, no instruction); the rest is q_k 2^9 in column k+3, q_k 2^18
//     in k+6, q_k m7 in k+7 and q_k m8 in k+8 (m7 2^203 + m8 2^232 = 2^256 - 2^224):
//     4 products per q instead of 7.
//   secp256k1: p = m0 + m1 2^29 + (2^232 - 2^58) + m8 2^232; the six all-ones
//     limbs (2^232 - 2^58) become -q_k in column k+2 and +q_k in column k+8
//     (there with m8: q_k 2^24). The -q_k is added as (2^29 - 1 - q_k) >= 0 with
//     the bias carried upwards (2^29 - q_0 in column 2, 2^29 - 1 in columns
//     11..15, -1 in column 16: sum 0), so no column value is ever negative:
//     4 products per q instead of 9.
// Column sums stay < 2^64 for f29_mul's operand bounds (tests/test_fp29_asm.py
// checks every column exactly; fp29_asm.hpp is the same schedule in asm pairs).
template <class F>
CDEV void f29_redc_terms(uint64_t& acc, const uint32_t* q, const uint32_t* qn, int k) {
  if constexpr (F::kRed == 1) {
    if (k >= 1 && k <= 9) acc += (uint64_t)q[k - 1] * sconst(F::m(1));
    if (k >= 2 && k <= 10) acc += qn[k - 2];
    if (k >= 11 && k <= 15) acc += kMask29;
    if (k == 16) acc -= 1;
    if (k >= 8) acc += (uint64_t)q[k - 8] * sconst(1u << 24);
  } else {
    if (k >= 3 && k <= 11) acc += (uint64_t)q[k - 3] * sconst(1u << 9);
    if (k >= 6 && k <= 14) acc += (uint64_t)q[k - 6] * sconst(1u << 18);
    if (k >= 7 && k <= 15) acc += (uint64_t)q[k - 7] * sconst(F::m(7));
    if (k >= 8) acc += (uint64_t)q[k - 8] * sconst(F::m(8));
  }
}
// column k < 9: pick q_k (and clear the column's low 29 bits)
template <class F>
CDEV void f29_redc_q(uint64_t& acc, uint32_t* q, uint32_t* qn, int k) {
  if constexpr (F::kRed == 1) {
    q[k] = ((uint32_t)acc * F::kMinv) & kMask29;
    qn[k] = (k == 0 ? (1u << 29) : kMask29) - q[k];
    acc += (uint64_t)q[k] * sconst(F::m(0));
  } else {
    q[k] = (uint32_t)acc & kMask29;  // acc - q_k: the p == -1 term
  }
}

// r = a b R^-1 mod p (norm, < 2p)
template <class F>
CDEV void f29_mul(f29& r, const f29& a, const f29& b) {
  uint32_t q[9], qn[9];
  uint64_t acc = 0;
  f29 t;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int j = (k > 8 ? k - 8 : 0); j <= (k < 8 ? k : 8); j++) acc += (uint64_t)a.v[j] * b.v[k - j];
    f29_redc_terms<F>(acc, q, qn, k);
    if (k < 9) f29_redc_q<F>(acc, q, qn, k);
    else t.v[k - 9] = (uint32_t)acc & kMask29;
    acc >>= 29;
  }
  t.v[8] = (uint32_t)acc;
  r = t;  // r may alias a or b
}

// r = a^2 R^-1 mod p: 45 distinct limb products (off-diagonal ones doubled)
template <class F>
CDEV void f29_sqr(f29& r, const f29& a) {
  uint32_t q[9], qn[9], a2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) a2[i] = a.v[i] << 1;
  uint64_t acc = 0;
  f29 t;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int j = (k > 8 ? k - 8 : 0); 2 * j < k; j++) acc += (uint64_t)a2[j] * a.v[k - j];
    if ((k & 1) == 0) acc += (uint64_t)a.v[k / 2] * a.v[k / 2];
    f29_redc_terms<F>(acc, q, qn, k);
    if (k < 9) f29_redc_q<F>(acc, q, qn, k);
    else t.v[k - 9] = (uint32_t)acc & kMask29;
    acc >>= 29;
  }
  t.v[8] = (uint32_t)acc;
  r = t;
}

CDEV void f29_add(f29& r, const f29& a, const f29& b) {
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + b.v[i];
}

// r = a + 2p - b, one carry pass. F::sub2p is 2p written with limbs 0..7 >=
// 2^29 - 1 (each borrowed from the limb above), so no limb goes negative for a
// norm b; the top limb may wrap transiently, the total stays >= 0.
template <class F>
CDEV void f29_sub(f29& r, const f29& a, const f29& b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t t = a.v[i] + F::sub2p(i) - b.v[i] + c;
    r.v[i] = t & kMask29;
    c = t >> 29;
  }
  r.v[8] = a.v[8] + F::sub2p(8) - b.v[8] + c;
}

// conditional negation (2p - a for a norm a), branch-free
template <class F>
CDEV void f29_cneg(f29& r, bool neg) {
  f29 z, n;
#pragma unroll
  for (int i = 0; i < 9; i++) z.v[i] = 0;
  f29_sub<F>(n, z, r);
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = neg ? n.v[i] : r.v[i];
}

// a - b + 4p limb by limb, no carry pass (F::sub4p's limbs exceed a norm b's):
// value < a + 4p, limbs < a's + 2^31.4. Only as the operand of a product whose
// other operand is norm (columns < 2^63.9; tests/test_fp29_model.py): the
// doublings' 4 beta - X3 (P-256) and D - X3 (secp256k1).
template <class F>
CDEV void f29_sub_loose(f29& r, const f29& a, const f29& b) {
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + F::sub4p(i) - b.v[i];
}

// The y of a mixed addition's affine point, conditionally negated without a
// carry pass: 4p - a limb by limb (F::sub4p's limbs exceed those of any norm a,
// so none goes negative). The result (value < 4p, limbs < 2^31.4) is only ever
// the first operand of jmadd's y2 * Z1 product, whose column sums stay below
// 2^64 (checked exactly by tests/test_fp29_model.py). 18 instructions instead
// of f29_cneg's carry pass + select (~50).
template <class F>
CDEV void f29_cneg_loose(f29& r, bool neg) {
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = neg ? F::sub4p(i) - r.v[i] : r.v[i];
}

// limbs 0..7 of r normalised (< 2^29), top = the value's bits >= 2^232 (value
// < 2^260)  ->  r norm, value < 2p: folds the bits >= 2^256.
template <class F>
CDEV void f29_fold(f29& r, uint32_t top) {
  const uint32_t q = top >> 24;  // the value's bits >= 2^256 (q < 16)
  r.v[8] = top & 0xffffffu;
  if (F::kRed == 1) {
    // secp256k1: 2^256 == 2^32 + 977 (mod p); 2^32 = 2^29 * 8
    r.v[0] += q * 977u;
    r.v[1] += q << 3;
  } else {
    // P-256: 2^256 == 2^224 - 2^192 - 2^96 + 1 (mod p); bit 96 is limb 3 bit 9,
    // bit 192 limb 6 bit 18, bit 224 limb 7 bit 21. Limbs 3 and 6 may go
    // negative: one signed carry pass over limbs 3..7 (the total is >= 0).
    r.v[0] += q;
    r.v[3] -= q << 9;
    r.v[6] -= q << 18;
    r.v[7] += q << 21;
#pragma unroll
    for (int i = 3; i < 8; i++) {
      const int32_t cs = (int32_t)r.v[i] >> 29;
      r.v[i] &= kMask29;
      r.v[i + 1] += (uint32_t)cs;
    }
  }
}

// limbs < 2^31.5, value < 2^260  ->  norm, value < 2p
template <class F>
CDEV void f29_red(f29& r, const f29& a) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t t = a.v[i] + c;
    r.v[i] = t & kMask29;
    c = t >> 29;
  }
  f29_fold<F>(r, a.v[8] + c);
}

// The point formulas' "subtract, subtract, reduce" steps in ONE carry pass:
// r = red(a + 2p - b), red(a + 4p - b - c), red(a + 6p - b - c - d). The
// subtrahends are norm (value <= 2p, limbs < 2^29 + 2^15), the minuend's limbs
// < 2^30.5 (a product output or a sum of two norms); F::sub4p / sub6p keep
// every limb in [0, 2^32) (tools/gen_fp29_consts.py subkp). Value < a + 6p
// < 2^260, so the fold applies. Same residue as the f29_sub / f29_red chains
// they replace (another representative: every comparison goes through f29_canon).
template <class F>
CDEV void f29_sub_red(f29& r, const f29& a, const f29& b) {
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t t = a.v[i] + F::sub2p(i) - b.v[i] + cy;
    r.v[i] = t & kMask29;
    cy = t >> 29;
  }
  f29_fold<F>(r, a.v[8] + F::sub2p(8) - b.v[8] + cy);
}
template <class F>
CDEV void f29_sub2_red(f29& r, const f29& a, const f29& b, const f29& c) {
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t t = a.v[i] + F::sub4p(i) - b.v[i] - c.v[i] + cy;
    r.v[i] = t & kMask29;
    cy = t >> 29;
  }
  f29_fold<F>(r, a.v[8] + F::sub4p(8) - b.v[8] - c.v[8] + cy);
}
template <class F>
CDEV void f29_sub3_red(f29& r, const f29& a, const f29& b, const f29& c, const f29& d) {
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t t = a.v[i] + F::sub6p(i) - b.v[i] - c.v[i] - d.v[i] + cy;
    r.v[i] = t & kMask29;
    cy = t >> 29;
  }
  f29_fold<F>(r, a.v[8] + F::sub6p(8) - b.v[8] - c.v[8] - d.v[8] + cy);
}
// r = red(K a), K <= 4, a norm
template <class F, int K>
CDEV void f29_mulk_red(f29& r, const f29& a) {
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t t = a.v[i] * K + cy;
    r.v[i] = t & kMask29;
    cy = t >> 29;
  }
  f29_fold<F>(r, a.v[8] * K + cy);
}
// r = K a with one carry pass and NO fold: limbs 0..7 < 2^29, the top limb
// keeps the bits >= 2^232. For a REDC output a (value < 1.5p when its operands
// were < 4p each) and K = 3: value < 4.5p, top < 2^26.2 -- the P-256
// doubling's alpha, whose products alpha^2 (< 20.25 p^2) and alpha (4 beta - X3)
// (< 27 p^2) stay under the Montgomery bound R p ~ 32 p^2 (the fold's ~25
// instructions per doubling saved; tests/test_fp29_model.py checks the columns).
template <class F, int K>
CDEV void f29_mulk_carry(f29& r, const f29& a) {
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t t = a.v[i] * K + cy;
    r.v[i] = t & kMask29;
    cy = t >> 29;
  }
  r.v[8] = a.v[8] * K + cy;
}

// r = 4p - 2a for a norm a, one carry pass: limbs 0..7 < 2^29, value < 4p
// (F::sub4p's limbs exceed 2a's, so no limb goes negative; the top limb is
// the value's bits >= 2^232, >= 0). The mixed addition's Y1 (4p - 2J) operand.
template <class F>
CDEV void f29_neg2_norm(f29& r, const f29& a) {
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t t = F::sub4p(i) - 2 * a.v[i] + cy;
    r.v[i] = t & kMask29;
    cy = t >> 29;
  }
  r.v[8] = F::sub4p(8) - 2 * a.v[8] + cy;
}

// canonical residue in [0, p), limbs fully normalised
template <class F>
CDEV void f29_canon(f29& r, const f29& a) {
  f29 t;
  f29_red<F>(t, a);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t s = t.v[i] + c;
    t.v[i] = s & kMask29;
    c = s >> 29;
  }
  t.v[8] += c;
  f29 d;  // t - p, kept when there is no borrow
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint32_t s = t.v[i] - F::m(i) - br;
    d.v[i] = s & kMask29;
    br = s >> 31;
  }
  const bool ge = br == 0;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = ge ? d.v[i] : t.v[i];
}

template <class F>
CDEV bool f29_iszero(const f29& a) {
  f29 c;
  f29_canon<F>(c, a);
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) x |= c.v[i];
  return x == 0;
}

// a == 0 (mod p) for a NORM a (value < 2p, as every f29_*_red output): one
// carry pass gives the unique radix-2^29 limbs of the value, which is then 0
// or p. No fold and no conditional subtraction (f29_iszero canonicalises any
// a < 2^260): the additions' exceptional-case test on H runs once per addition.
template <class F>
CDEV bool f29_iszero_norm(const f29& a) {
  uint32_t c = 0, z = 0, dp = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t s = a.v[i] + c;
    const uint32_t l = s & kMask29;
    c = s >> 29;
    z |= l;
    dp |= l ^ F::m(i);
  }
  const uint32_t top = a.v[8] + c;
  z |= top;
  dp |= top ^ F::m(8);
  return z == 0 || dp == 0;
}

template <class F>
CDEV bool f29_eq(const f29& a, const f29& b) {
  f29 x, y;
  f29_canon<F>(x, a);
  f29_canon<F>(y, b);
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) d |= x.v[i] ^ y.v[i];
  return d == 0;
}

// 8 little-endian 32-bit words (value < 2^256) <-> 29-bit limbs
CDEV void f29_from_words(f29& r, const uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int lo = 29 * i, wi = lo >> 5, sh = lo & 31;
    const uint64_t x = (uint64_t)w[wi] | (wi + 1 < 8 ? (uint64_t)w[wi + 1] << 32 : 0ull);
    r.v[i] = (uint32_t)(x >> sh) & kMask29;
  }
}
// a: canonical (fully normalised limbs, value < 2^256)
CDEV void f29_to_words(uint32_t w[8], const f29& a) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int lo = 32 * k, li = lo / 29, sh = lo % 29;
    uint64_t x = (uint64_t)a.v[li] >> sh;
    x |= (uint64_t)a.v[li + 1] << (29 - sh);
    if (li + 2 < 9 && 58 - sh < 32) x |= (uint64_t)a.v[li + 2] << (58 - sh);
    w[k] = (uint32_t)x;
  }
}

template <class F>
CDEV void f29_const_one(f29& r) {  // R mod p: 1 in Montgomery form
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = F::one(i);
}

// plain x < 2^256  ->  Montgomery form x R mod p (norm)
template <class F>
CDEV void f29_to_mont(f29& r, const f29& x) {
  f29 r2;
#pragma unroll
  for (int i = 0; i < 9; i++) r2.v[i] = F::r2(i);
  f29_mul<F>(r, x, r2);
}
// Montgomery form -> canonical plain residue
template <class F>
CDEV void f29_from_mont(f29& r, const f29& a) {
  f29 one;
#pragma unroll
  for (int i = 0; i < 9; i++) one.v[i] = i == 0;
  f29_mul<F>(r, a, one);
  f29_canon<F>(r, r);
}

// a^e for a compile-time exponent E (8 x 32-bit limbs)
template <class F, class E>
CDEV void f29_pow_const(f29& r, const f29& a) {
  f29 acc = a;
  int top = 255;
  while (top > 0 && !((E::limb(top >> 5) >> (top & 31)) & 1)) top--;
#pragma unroll 1
  for (int i = top - 1; i >= 0; i--) {
    f29_sqr<F>(acc, acc);
    if ((E::limb(i >> 5) >> (i & 31)) & 1) f29_mul<F>(acc, acc, a);
  }
  r = acc;
}

}  // namespace cordahip
