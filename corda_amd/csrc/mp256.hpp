// 256-bit modular arithmetic for gfx950 lanes (ECDSA, kernel K2).
//
// 8 x 32-bit limbs, little-endian. Montgomery multiplication in product-
// scanning (FIPS) form: every 32x32 partial product is ONE v_mad_u64_u32
// into a 64-bit column accumulator plus ONE v_addc_co_u32 catching its carry
// (the two instructions issue at the same rate on CDNA4 —
// profiles/r01_int_rates.jsonl). Modulus limbs are compile-time constants, so
// zero limbs (P-256's p has three) cost nothing and unit limbs cost an add.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef CDEV
#define CDEV __device__ __forceinline__
#endif

namespace cordahip {

struct u256 {
  uint32_t v[8];
};

// acc(64) : hi(32) += a * b
CDEV void mac(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(hi)
      : "v"(a), "v"(b)
      : "vcc");
}
// acc(64) : hi(32) += x (32-bit)
CDEV void acc_add(uint64_t& acc, uint32_t& hi, uint32_t x) {
  const uint64_t s = acc + x;
  hi += (s < acc);
  acc = s;
}

template <class M>
CDEV void mac_const(uint64_t& acc, uint32_t& hi, uint32_t q, int j) {
  const uint32_t m = M::limb(j);
  if (m == 0) return;
  if (m == 1) {
    acc_add(acc, hi, q);
    return;
  }
  mac(acc, hi, q, m);
}

// a >= b: no borrow out of a - b (branch-free; a short-circuit word compare
// becomes divergent control flow on the GPU)
CDEV bool u256_geq(const u256& a, const u256& b) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) br = (uint32_t)(((uint64_t)a.v[i] - b.v[i] - br) >> 63);
  return br == 0;
}
CDEV bool u256_iszero(const u256& a) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x |= a.v[i];
  return x == 0;
}
CDEV bool u256_eq(const u256& a, const u256& b) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x |= a.v[i] ^ b.v[i];
  return x == 0;
}
// r = a + b, returns carry
CDEV uint32_t u256_add(u256& r, const u256& a, const u256& b) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c += (uint64_t)a.v[i] + b.v[i];
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)c;
}
// r = a - b, returns borrow
CDEV uint32_t u256_sub(u256& r, const u256& a, const u256& b) {
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t d = (uint64_t)a.v[i] - b.v[i] - br;
    r.v[i] = (uint32_t)d;
    br = (d >> 63) & 1;
  }
  return (uint32_t)br;
}

template <class M>
CDEV u256 mod_m() {
  u256 m;
#pragma unroll
  for (int i = 0; i < 8; i++) m.v[i] = M::limb(i);
  return m;
}

// r = (x + carry*2^256) mod m for x + carry*2^256 < 2m
template <class M>
CDEV void cond_sub_m(u256& r, const u256& x, uint32_t carry) {
  u256 t;
  const uint32_t br = u256_sub(t, x, mod_m<M>());
  const bool use = carry || !br;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = use ? t.v[i] : x.v[i];
}

template <class M>
CDEV void mod_add(u256& r, const u256& a, const u256& b) {
  u256 s;
  const uint32_t c = u256_add(s, a, b);
  cond_sub_m<M>(r, s, c);
}
template <class M>
CDEV void mod_sub(u256& r, const u256& a, const u256& b) {
  u256 d, t;
  const uint32_t br = u256_sub(d, a, b);
  u256_add(t, d, mod_m<M>());
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = br ? t.v[i] : d.v[i];
}
template <class M>
CDEV void mod_neg(u256& r, const u256& a) {
  u256 z;
#pragma unroll
  for (int i = 0; i < 8; i++) z.v[i] = 0;
  mod_sub<M>(r, z, a);
}

// Montgomery product r = a b 2^-256 mod m, inputs < m (FIPS, product scanning)
template <class M>
CDEV void mont_mul(u256& r, const u256& a, const u256& b) {
  uint32_t q[8];
  uint64_t acc = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      mac(acc, hi, a.v[j], b.v[i - j]);
      mac_const<M>(acc, hi, q[j], i - j);
    }
    mac(acc, hi, a.v[i], b.v[0]);
    q[i] = (uint32_t)acc * M::kMinv;
    mac_const<M>(acc, hi, q[i], 0);  // zeroes the low word
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  u256 t;
#pragma unroll
  for (int i = 8; i < 15; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) {
      mac(acc, hi, a.v[j], b.v[i - j]);
      mac_const<M>(acc, hi, q[j], i - j);
    }
    t.v[i - 8] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t.v[7] = (uint32_t)acc;
  cond_sub_m<M>(r, t, (uint32_t)(acc >> 32));
}

template <class M>
CDEV void mont_sqr(u256& r, const u256& a) {
  mont_mul<M>(r, a, a);
}

// a^e for a compile-time exponent given as 8 limbs (Montgomery domain)
template <class M, class E>
CDEV void mont_pow_const(u256& r, const u256& a) {
  u256 acc = a;  // top bit of every exponent used here is 1
  int top = 255;
  while (top > 0 && !((E::limb(top >> 5) >> (top & 31)) & 1)) top--;
  for (int i = top - 1; i >= 0; i--) {
    mont_sqr<M>(acc, acc);
    if ((E::limb(i >> 5) >> (i & 31)) & 1) mont_mul<M>(acc, acc, a);
  }
  r = acc;
}

// big-endian 32 bytes -> limbs
CDEV void u256_from_be_bytes(u256& r, const uint8_t* p) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint8_t* b = p + 28 - 4 * i;
    r.v[i] = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
  }
}

}  // namespace cordahip
