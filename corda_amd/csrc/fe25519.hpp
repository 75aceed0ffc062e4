// GF(2^255 - 19) arithmetic for gfx950 lanes.
//
// Representation: 10 unsigned 32-bit limbs in radix 2^25.5 (limb i holds
// 26 bits when i is even, 25 when odd; weights 2^0,2^26,2^51,...,2^230).
// Why this radix on CDNA4 (measured, tools/microbench/int_rates.hip →
// profiles/r01_int_rates.jsonl): v_mad_u64_u32 issues at the same rate as
// v_add_co_u32 / v_addc_co_u32 (~60 lane-ops per CU-cycle), so a radix-2^32
// product costs mad + addc per limb product, while here every partial
// product column stays below 2^64 and accumulates with ONE v_mad_u64_u32
// and no carry instruction. Additions/subtractions are carry-free
// v_add_u32 (full rate, ~110/CU-cycle).
//
// Bounds (all arithmetic is exact, no overflow):
//   tight : even limbs <= 2^26 + 2^10, odd limbs <= 2^25 + 2^17
//           (outputs of fe_mul/fe_sq/fe_carry/fe_sub)
//   loose : <= 3.3 x the tight bound (sum of up to three tight values)
//   fe_mul/fe_sq accept loose inputs: 19*g < 2^32 and every 64-bit column
//   sum < 2^62.5.
//   fe_sub(a, b) = a + 4p - b followed by a 32-bit carry pass: b may be
//   loose (4p limbs >= 2^27), output tight.
//   fe_mul(r, f, g) is asymmetric: g (scaled by 19) must stay <= 3.3x tight,
//   f may be up to ~5x (column sums then stay below 2^63). The group
//   formulas use carry-free fe_sub_loose / fe_neg_loose wherever the
//   result only feeds such an operand (bounds: tools/proto/fe_bounds.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CDEV __device__ __forceinline__

namespace cordahip {

struct fe {
  uint32_t v[10];
};

static constexpr uint32_t M26 = (1u << 26) - 1;
static constexpr uint32_t M25 = (1u << 25) - 1;

CDEV constexpr int limb_bits(int i) { return (i & 1) ? 25 : 26; }

CDEV void fe_set(fe& r, uint32_t x) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = 0;
  r.v[0] = x;
}

CDEV void fe_add(fe& r, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = a.v[i] + b.v[i];
}

// 32-bit carry pass; limbs in < 2^31 -> tight
CDEV void fe_carry(fe& r) {
  uint32_t c;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    c = r.v[i] >> limb_bits(i);
    r.v[i] &= (i & 1) ? M25 : M26;
    r.v[i + 1] += c;
  }
  c = r.v[9] >> 25;
  r.v[9] &= M25;
  r.v[0] += c * 19;
  c = r.v[0] >> 26;
  r.v[0] &= M26;
  r.v[1] += c;
}

// 4p in this radix: even limb 0: 4*(2^26-19), odd: 4*(2^25-1), even: 4*(2^26-1)
CDEV void fe_sub(fe& r, const fe& a, const fe& b) {
  r.v[0] = a.v[0] + (4u * ((1u << 26) - 19)) - b.v[0];
#pragma unroll
  for (int i = 1; i < 10; i++) r.v[i] = a.v[i] + ((i & 1) ? 4u * M25 : 4u * M26) - b.v[i];
  fe_carry(r);
}

// r = a + 2p - b with NO carry pass: b must be tight (2p limbs >= tight
// limbs); the result is at most a + 2p. Only for values that go straight into
// fe_mul / fe_sq within the operand bounds checked in tools/proto/fe_bounds.py.
CDEV void fe_sub_loose(fe& r, const fe& a, const fe& b) {
  r.v[0] = a.v[0] + (2u * ((1u << 26) - 19)) - b.v[0];
#pragma unroll
  for (int i = 1; i < 10; i++) r.v[i] = a.v[i] + ((i & 1) ? 2u * M25 : 2u * M26) - b.v[i];
}
// r = 2p - a (a tight), no carry: <= 2x tight
CDEV void fe_neg_loose(fe& r, const fe& a) {
  r.v[0] = (2u * ((1u << 26) - 19)) - a.v[0];
#pragma unroll
  for (int i = 1; i < 10; i++) r.v[i] = ((i & 1) ? 2u * M25 : 2u * M26) - a.v[i];
}

CDEV void fe_neg(fe& r, const fe& a) {
  fe z;
  fe_set(z, 0);
  fe_sub(r, z, a);
}

// conditional select: r = c ? a : r  (c is 0/1 per lane)
CDEV void fe_cmov(fe& r, const fe& a, bool c) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = c ? a.v[i] : r.v[i];
}

// Carry-chained column reduction: column k's 64-bit accumulator STARTS at the
// carry out of column k-1, so the carry costs no add (it rides in
// v_mad_u64_u32's 64-bit addend) — one shift and one mask per limb, plus one
// fold of 19 * carry(limb 9) into limbs 0/1. Bounds: column sums < 2^62.5 plus
// a carry < 2^38; the final carry c < 2^38, 19c < 2^42.3, so limb 1 grows by
// < 2^16.4 -> output tight. (LLVM still re-associates the carry into an extra
// 64-bit add per column; the group formulas' paired products avoid that with
// generated asm, fe25519_asm.hpp.)

// 19 * x, opaque to LLVM: with a visible constant factor InstCombine
// factors sums of wrapped products as 19 * (64-bit sum), which costs a 64x32
// multiply per column instead of one 32-bit multiply per limb.
CDEV uint32_t mul19(uint32_t x) {
  uint32_t r;
  asm("v_mul_lo_u32 %0, %1, 19" : "=v"(r) : "v"(x));
  return r;
}

CDEV uint64_t mac64(uint32_t a, uint32_t b, uint64_t acc) { return acc + (uint64_t)a * b; }

CDEV void fe_fold_top(fe& r, uint64_t c) {
  const uint64_t t = (uint64_t)r.v[0] + c * 19u;
  r.v[0] = (uint32_t)t & M26;
  r.v[1] += (uint32_t)(t >> 26);
}

// h = f * g. Column k collects f_i g_j with i + j == k (mod 10); wrapped
// terms carry 2^255 == 19, and odd*odd terms carry an extra 2 (radix 2^25.5).
CDEV void fe_mul(fe& r, const fe& f, const fe& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g19[i] = mul19(g.v[i]);
    f2[i] = f.v[i] << 1;
  }
  fe o;
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t acc = c;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const int j = (k - i + 10) % 10;
      const bool wrap = (i + j) >= 10;
      const bool oo = (i & 1) && (j & 1);
      const uint32_t a = oo ? f2[i] : f.v[i];
      const uint32_t b = wrap ? g19[j] : g.v[j];
      acc = mac64(a, b, acc);
    }
    o.v[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
    c = acc >> limb_bits(k);
  }
  fe_fold_top(o, c);
  r = o;  // r may alias f or g
}

// h = f^2 (55 products)
CDEV void fe_sq(fe& r, const fe& f) {
  uint32_t f2[10], f4[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    f2[i] = f.v[i] << 1;
    f4[i] = f.v[i] << 2;
    f19[i] = mul19(f.v[i]);
  }
  fe o;
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t acc = c;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const int j = (k - i + 10) % 10;
      if (j < i) continue;
      const bool wrap = (i + j) >= 10;
      const bool oo = (i & 1) && (j & 1);
      const int mult = (i < j ? 2 : 1) * (oo ? 2 : 1);  // 1, 2 or 4
      const uint32_t a = mult == 1 ? f.v[i] : (mult == 2 ? f2[i] : f4[i]);
      const uint32_t b = wrap ? f19[j] : f.v[j];
      acc = mac64(a, b, acc);
    }
    o.v[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
    c = acc >> limb_bits(k);
  }
  fe_fold_top(o, c);
  r = o;  // r may alias f or g
}

// n squarings, kept as a loop: a fully unrolled chain lets the scheduler
// interleave successive squarings and blows the register budget.
CDEV void fe_sqn(fe& r, const fe& a, int n) {
  fe_sq(r, a);
#pragma unroll 1
  for (int i = 1; i < n; i++) fe_sq(r, r);
}

// z^(2^250 - 1) and z^11 (shared prefix of invert and pow22523)
CDEV void fe_pow2_250_1(fe& out, fe& z11, const fe& z) {
  fe z2, z9, t, a, b;
  fe_sq(z2, z);
  fe_sqn(t, z2, 2);
  fe_mul(z9, t, z);
  fe_mul(z11, z9, z2);
  fe_sq(t, z11);
  fe_mul(a, t, z9);          // 2^5 - 1
  fe_sqn(t, a, 5);
  fe_mul(a, t, a);           // 2^10 - 1
  fe_sqn(t, a, 10);
  fe_mul(b, t, a);           // 2^20 - 1
  fe_sqn(t, b, 20);
  fe_mul(t, t, b);           // 2^40 - 1
  fe_sqn(t, t, 10);
  fe_mul(a, t, a);           // 2^50 - 1
  fe_sqn(t, a, 50);
  fe_mul(b, t, a);           // 2^100 - 1
  fe_sqn(t, b, 100);
  fe_mul(t, t, b);           // 2^200 - 1
  fe_sqn(t, t, 50);
  fe_mul(out, t, a);         // 2^250 - 1
}

CDEV void fe_invert(fe& r, const fe& z) {
  fe t, z11;
  fe_pow2_250_1(t, z11, z);
  fe_sqn(t, t, 5);
  fe_mul(r, t, z11);  // 2^255 - 21
}

CDEV void fe_pow22523(fe& r, const fe& z) {
  fe t, z11;
  fe_pow2_250_1(t, z11, z);
  fe_sqn(t, t, 2);
  fe_mul(r, t, z);  // 2^252 - 3
}

// Canonical little-endian 32-bit words of a tight value (fully reduced mod p).
CDEV void fe_tobytes(uint32_t w[8], const fe& a) {
  fe t = a;
  fe_carry(t);
  fe_carry(t);
  // q = 1 iff t >= p  (carry out of t + 19 at bit 255)
  uint32_t q = (t.v[0] + 19) >> 26;
#pragma unroll
  for (int i = 1; i < 10; i++) q = (t.v[i] + q) >> limb_bits(i);
  t.v[0] += 19 * q;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint32_t c = t.v[i] >> limb_bits(i);
    t.v[i] &= (i & 1) ? M25 : M26;
    t.v[i + 1] += c;
  }
  t.v[9] &= M25;
  // pack limbs (offsets 0,26,51,77,102,128,153,179,204,230) into 8 words
  w[0] = t.v[0] | (t.v[1] << 26);
  w[1] = (t.v[1] >> 6) | (t.v[2] << 19);
  w[2] = (t.v[2] >> 13) | (t.v[3] << 13);
  w[3] = (t.v[3] >> 19) | (t.v[4] << 6);
  w[4] = t.v[5] | (t.v[6] << 25);
  w[5] = (t.v[6] >> 7) | (t.v[7] << 19);
  w[6] = (t.v[7] >> 13) | (t.v[8] << 12);
  w[7] = (t.v[8] >> 20) | (t.v[9] << 6);
}

// ref10 fe_frombytes semantics: bit 255 ignored, value NOT reduced below p.
CDEV void fe_frombytes(fe& r, const uint32_t w[8]) {
  r.v[0] = w[0] & M26;
  r.v[1] = ((w[0] >> 26) | (w[1] << 6)) & M25;
  r.v[2] = ((w[1] >> 19) | (w[2] << 13)) & M26;
  r.v[3] = ((w[2] >> 13) | (w[3] << 19)) & M25;
  r.v[4] = (w[3] >> 6) & M26;
  r.v[5] = w[4] & M25;
  r.v[6] = ((w[4] >> 25) | (w[5] << 7)) & M26;
  r.v[7] = ((w[5] >> 19) | (w[6] << 13)) & M25;
  r.v[8] = ((w[6] >> 12) | (w[7] << 20)) & M26;
  r.v[9] = (w[7] >> 6) & M25;
}

CDEV bool fe_iszero(const fe& a) {
  uint32_t w[8];
  fe_tobytes(w, a);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) acc |= w[i];
  return acc == 0;
}

CDEV uint32_t fe_isnegative(const fe& a) {
  uint32_t w[8];
  fe_tobytes(w, a);
  return w[0] & 1;
}

// curve constants (radix 2^25.5 limbs; values from RFC 8032 §5.1)
CDEV void fe_const_d(fe& r) {
  const uint32_t c[10] = {0x35978a3, 0xd37284, 0x3156ebd, 0x6a0a0e, 0x1c029,
                          0x179e898, 0x3a03cbb, 0x1ce7198, 0x2e2b6ff, 0x1480db3};
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = c[i];
}
CDEV void fe_const_d2(fe& r) {
  const uint32_t c[10] = {0x2b2f159, 0x1a6e509, 0x22add7a, 0xd4141d, 0x38052,
                          0xf3d130, 0x3407977, 0x19ce331, 0x1c56dff, 0x901b67};
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = c[i];
}
CDEV void fe_const_sqrtm1(fe& r) {
  const uint32_t c[10] = {0x20ea0b0, 0x186c9d2, 0x8f189d, 0x35697f, 0xbd0c60,
                          0x1fbd7a7, 0x2804c9e, 0x1e16569, 0x4fc1d, 0xae0c92};
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = c[i];
}

}  // namespace cordahip
