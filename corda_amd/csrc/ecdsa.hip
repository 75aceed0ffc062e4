// ECDSA (ECDSA_SECP256K1_SHA256 = 2, ECDSA_SECP256R1_SHA256 = 3) batch
// verification for gfx950 — kernel K2.
//
// Replaces, per lane, Crypto.isValid for the two ECDSA schemes
// (core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:91-116, :534-541)
// -> JCA "SHA256withECDSA" -> BouncyCastle 1.57 DSABase.engineVerify /
// ECDSASigner.verifySignature (semantics: SURVEY App. A.2, restated in
// oracle/bc_ecdsa.py and oracle/c/ecdsa.c):
//   key: SEC1 point, coordinates < p, on the curve (else BAD_KEY);
//   sig: strict DER (der.hpp) else MALFORMED_SIG; r, s in [1, n-1] else BAD_SIG;
//   e = SHA-256(msg); w = s^-1; P = (e w) G + (r w) Q; accept iff P != O and
//   x(P) mod n == r, checked inversion-free as X == r Z^2 or (r + n) Z^2.
// Arithmetic: the base field in fp29.hpp (9 x 29-bit limbs, Montgomery
// R = 2^261, lazy reduction), the scalar field mod n in mp256.hpp.
// secp256k1 lanes split both scalars with the GLV endomorphism
// (u = k1 + k2 lambda with |k1|, |k2| < 2^129; phi(x, y) = (beta x, y) =
// [lambda](x, y)), so their ladder runs 128 doublings instead of 252.
// One lane per signature; lanes are permuted so each wave holds one curve
// (device-side partition kernels below), so the two curves' code never
// diverges inside a wave except at the single boundary wave.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <string>

#include "der.hpp"
#include "fp29.hpp"
#include "fp29_asm.hpp"
#include "fp29_consts.hpp"
#include "mp256.hpp"
#include "sc25519.hpp"
#include "sha2_device.hpp"
#include "status.hpp"

namespace cordahip {

#define CH_LIMBS(name, a0, a1, a2, a3, a4, a5, a6, a7)                                              \
  CDEV static constexpr uint32_t name(int i) {                                                      \
    return i == 0 ? a0 : i == 1 ? a1 : i == 2 ? a2 : i == 3 ? a3 : i == 4 ? a4 : i == 5 ? a5 : i == 6 ? a6 : a7; \
  }

// 8 x 32-bit moduli: p for range checks, n (with R^2 = 2^512 mod n) for the
// scalar-field Montgomery arithmetic of mp256.hpp
struct K1P {
  CH_LIMBS(limb, 0xfffffc2fu, 0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu)
};
struct K1N {
  CH_LIMBS(limb, 0xd0364141u, 0xbfd25e8cu, 0xaf48a03bu, 0xbaaedce6u, 0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu)
  CH_LIMBS(r2, 0x67d7d140u, 0x896cf214u, 0x0e7cf878u, 0x741496c2u, 0x5bcd07c6u, 0xe697f5e4u, 0x81c69bc5u, 0x9d671cd5u)
  static constexpr uint32_t kMinv = 0x5588b13fu;
};
struct R1P {
  CH_LIMBS(limb, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u, 0x00000001u, 0xffffffffu)
};
struct R1N {
  CH_LIMBS(limb, 0xfc632551u, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu, 0xffffffffu, 0xffffffffu, 0u, 0xffffffffu)
  CH_LIMBS(r2, 0xbe79eea2u, 0x83244c95u, 0x49bd6fa6u, 0x4699799cu, 0x2b6bec59u, 0x2845b239u, 0xf3d95620u, 0x66e12d94u)
  static constexpr uint32_t kMinv = 0xee00bc4fu;
};
// exponents: (p+1)/4 (square root, p = 3 mod 4), p-2 and n-2 (Fermat inversion)
struct K1Sqrt { CH_LIMBS(limb, 0xbfffff0cu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x3fffffffu) };
struct K1Pm2 { CH_LIMBS(limb, 0xfffffc2du, 0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu) };
struct K1Nm2 { CH_LIMBS(limb, 0xd036413fu, 0xbfd25e8cu, 0xaf48a03bu, 0xbaaedce6u, 0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu) };
struct R1Sqrt { CH_LIMBS(limb, 0u, 0u, 0x40000000u, 0u, 0u, 0x40000000u, 0xc0000000u, 0x3fffffffu) };
struct R1Pm2 { CH_LIMBS(limb, 0xfffffffdu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u, 0x00000001u, 0xffffffffu) };
struct R1Nm2 { CH_LIMBS(limb, 0xfc63254fu, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu, 0xffffffffu, 0xffffffffu, 0u, 0xffffffffu) };
// p - n (x(P) mod n == r also holds for x = r + n when r < p - n)
struct K1PmN { CH_LIMBS(limb, 0x22fc9baeu, 0x402da172u, 0x50b75fc4u, 0x45512319u, 0x00000001u, 0u, 0u, 0u) };
struct R1PmN { CH_LIMBS(limb, 0x039cdaaeu, 0x0c46353du, 0x58e8617bu, 0x43190553u, 0u, 0u, 0u, 0u) };

template <int SCHEME>
struct Curve;
template <>
struct Curve<2> {  // secp256k1: y^2 = x^3 + 7
  using P = K1P;
  using N = K1N;
  using F = K1F;
  using Sqrt = K1Sqrt;
  using Pm2 = K1Pm2;
  using Nm2 = K1Nm2;
  using PmN = K1PmN;
  static constexpr bool kAm3 = false;
  static constexpr bool kGlv = true;
};
template <>
struct Curve<3> {  // secp256r1 / P-256: y^2 = x^3 - 3x + b
  using P = R1P;
  using N = R1N;
  using F = R1F;
  using Sqrt = R1Sqrt;
  using Pm2 = R1Pm2;
  using Nm2 = R1Nm2;
  using PmN = R1PmN;
  static constexpr bool kAm3 = true;
  static constexpr bool kGlv = false;
};

template <class Fc>
CDEV u256 limbs_of() {
  u256 r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = Fc::limb(i);
  return r;
}

// scalar field (mod n) Montgomery conversions
template <class M>
CDEV void to_mont(u256& r, const u256& a) {
  u256 r2;
#pragma unroll
  for (int i = 0; i < 8; i++) r2.v[i] = M::r2(i);
  mont_mul<M>(r, a, r2);
}

// ---- Jacobian points, coordinates in fp29 Montgomery form (norm, < 2p) -----
struct jpt {
  f29 X, Y, Z;
  bool inf;
};

// Two independent field products. EC_USE_ASM2 (default): one generated asm
// block per pair (fp29_asm.hpp, tools/gen_fp29_asm.py), bit-identical to two
// f29_mul / f29_sqr calls; results may alias any operand. Only kernels with a
// >= 164-VGPR budget (amdgpu_waves_per_eu(2) or fewer waves) may use them: the
// asm's column accumulators are v160..v163.
#ifndef EC_USE_ASM2
#define EC_USE_ASM2 1
#endif
// single products of the ladder's formulas (no partner): one asm chain each
template <class F>
CDEV void f29_mul1(f29& r, const f29& a, const f29& b) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_mul_k1(r, a, b);
  else f29a_mul_r1(r, a, b);
#else
  f29_mul<F>(r, a, b);
#endif
}
template <class F>
CDEV void f29_sqr1(f29& r, const f29& a) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_sqr_k1(r, a);
  else f29a_sqr_r1(r, a);
#else
  f29_sqr<F>(r, a);
#endif
}
template <class F>
CDEV void f29_mul_pair(f29& r0, const f29& a0, const f29& b0, f29& r1, const f29& a1, const f29& b1) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_mul_mul_k1(r0, a0, b0, r1, a1, b1);
  else f29a_mul_mul_r1(r0, a0, b0, r1, a1, b1);
#else
  f29 t0, t1;
  f29_mul<F>(t0, a0, b0);
  f29_mul<F>(t1, a1, b1);
  r0 = t0;
  r1 = t1;
#endif
}
template <class F>
CDEV void f29_sqr_pair(f29& r0, const f29& a0, f29& r1, const f29& a1) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_sqr_sqr_k1(r0, a0, r1, a1);
  else f29a_sqr_sqr_r1(r0, a0, r1, a1);
#else
  f29 t0, t1;
  f29_sqr<F>(t0, a0);
  f29_sqr<F>(t1, a1);
  r0 = t0;
  r1 = t1;
#endif
}
template <class F>  // r0 = a0^2, r1 = a1 b1
CDEV void f29_sqr_mul_pair(f29& r0, const f29& a0, f29& r1, const f29& a1, const f29& b1) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_sqr_mul_k1(r0, a0, r1, a1, b1);
  else f29a_sqr_mul_r1(r0, a0, r1, a1, b1);
#else
  f29 t0, t1;
  f29_sqr<F>(t0, a0);
  f29_mul<F>(t1, a1, b1);
  r0 = t0;
  r1 = t1;
#endif
}

// Products minus norm subtrahends with the subtraction folded into the REDC's
// output columns (fp29_asm.hpp *_sub variants): red(a b + 4p - s0 - s1), or
// + 6p with three subtrahends; the C versions (EC_USE_ASM2 0) compute the same
// limbs as a product and one f29_sub*_red pass with the same multiple of p.
template <class F>  // r0 = a0 b0 - s00, r1 = a1 b1 - s10 (+4p each)
CDEV void f29_mul_pair_s1s1(f29& r0, const f29& a0, const f29& b0, const f29& s00, f29& r1, const f29& a1,
                            const f29& b1, const f29& s10) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_mul_mul_s1s1_k1(r0, a0, b0, s00, r1, a1, b1, s10);
  else f29a_mul_mul_s1s1_r1(r0, a0, b0, s00, r1, a1, b1, s10);
#else
  f29 t0, t1, z;
  for (int i = 0; i < 9; i++) z.v[i] = 0;
  f29_mul<F>(t0, a0, b0);
  f29_mul<F>(t1, a1, b1);
  f29_sub2_red<F>(r0, t0, s00, z);
  f29_sub2_red<F>(r1, t1, s10, z);
#endif
}
template <class F>  // r0 = a0^2 - s00 - s01 (+4p), r1 = a1 b1
CDEV void f29_sqr_mul_pair_s2(f29& r0, const f29& a0, const f29& s00, const f29& s01, f29& r1, const f29& a1,
                              const f29& b1) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_sqr_mul_s2_k1(r0, a0, s00, s01, r1, a1, b1);
  else f29a_sqr_mul_s2_r1(r0, a0, s00, s01, r1, a1, b1);
#else
  f29 t0, t1;
  f29_sqr<F>(t0, a0);
  f29_mul<F>(t1, a1, b1);
  f29_sub2_red<F>(r0, t0, s00, s01);
  r1 = t1;
#endif
}
template <class F>  // r0 = a0^2 - s00 - s01 - s02 (+6p), r1 = a1 b1
CDEV void f29_sqr_mul_pair_s3(f29& r0, const f29& a0, const f29& s00, const f29& s01, const f29& s02, f29& r1,
                              const f29& a1, const f29& b1) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_sqr_mul_s3_k1(r0, a0, s00, s01, s02, r1, a1, b1);
  else f29a_sqr_mul_s3_r1(r0, a0, s00, s01, s02, r1, a1, b1);
#else
  f29 t0, t1;
  f29_sqr<F>(t0, a0);
  f29_mul<F>(t1, a1, b1);
  f29_sub3_red<F>(r0, t0, s00, s01, s02);
  r1 = t1;
#endif
}
template <class F>  // r0 = a0^2, r1 = a1 b1 - 2 r0 (+4p)
CDEV void f29_sqr_mul_pair_o2(f29& r0, const f29& a0, f29& r1, const f29& a1, const f29& b1) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_sqr_mul_o2_k1(r0, a0, r1, a1, b1);
  else f29a_sqr_mul_o2_r1(r0, a0, r1, a1, b1);
#else
  f29 t0, t1;
  f29_sqr<F>(t0, a0);
  f29_mul<F>(t1, a1, b1);
  f29_sub2_red<F>(r1, t1, t0, t0);
  r0 = t0;
#endif
}
template <class F>  // r0 = a0 b0 - s00 - s01 (+4p)
CDEV void f29_mul1_s2(f29& r0, const f29& a0, const f29& b0, const f29& s00, const f29& s01) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_mul_s2_k1(r0, a0, b0, s00, s01);
  else f29a_mul_s2_r1(r0, a0, b0, s00, s01);
#else
  f29 t0;
  f29_mul<F>(t0, a0, b0);
  f29_sub2_red<F>(r0, t0, s00, s01);
#endif
}

template <class F>  // r0 = a0^2 - s00 - s01, r1 = a1^2 - s10 - s11 (+4p each)
CDEV void f29_sqr_pair_s2s2(f29& r0, const f29& a0, const f29& s00, const f29& s01, f29& r1, const f29& a1,
                            const f29& s10, const f29& s11) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_sqr_sqr_s2s2_k1(r0, a0, s00, s01, r1, a1, s10, s11);
  else f29a_sqr_sqr_s2s2_r1(r0, a0, s00, s01, r1, a1, s10, s11);
#else
  f29 t0, t1;
  f29_sqr<F>(t0, a0);
  f29_sqr<F>(t1, a1);
  f29_sub2_red<F>(r0, t0, s00, s01);
  f29_sub2_red<F>(r1, t1, s10, s11);
#endif
}
template <class F>  // r0 = a0^2 - s00 - s01, r1 = a1 b1 - s10 - s11 (+4p each)
CDEV void f29_sqr_mul_pair_s2s2(f29& r0, const f29& a0, const f29& s00, const f29& s01, f29& r1, const f29& a1,
                                const f29& b1, const f29& s10, const f29& s11) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_sqr_mul_s2s2_k1(r0, a0, s00, s01, r1, a1, b1, s10, s11);
  else f29a_sqr_mul_s2s2_r1(r0, a0, s00, s01, r1, a1, b1, s10, s11);
#else
  f29 t0, t1;
  f29_sqr<F>(t0, a0);
  f29_mul<F>(t1, a1, b1);
  f29_sub2_red<F>(r0, t0, s00, s01);
  f29_sub2_red<F>(r1, t1, s10, s11);
#endif
}

template <class F>  // r0 = a0 b0 + c0 d0 with ONE REDC (the column sums stay < 2^64 for the
                    // mixed addition's operands: tests/test_fp29_model.py)
CDEV void f29_mul2(f29& r0, const f29& a0, const f29& b0, const f29& c0, const f29& d0) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_mul2_k1(r0, a0, b0, c0, d0);
  else f29a_mul2_r1(r0, a0, b0, c0, d0);
#else
  f29 t0, t1, z;
  for (int i = 0; i < 9; i++) z.v[i] = 0;
  f29_mul<F>(t0, a0, b0);
  f29_mul<F>(t1, c0, d0);
  f29_add(t0, t0, t1);  // another representative of the same residue (< 4p)
  f29_sub2_red<F>(r0, t0, z, z);
#endif
}
template <class F>  // r0 = a0^2 - s00 - s01 - s02 (+6p)
CDEV void f29_sqr1_s3(f29& r0, const f29& a0, const f29& s00, const f29& s01, const f29& s02) {
#if EC_USE_ASM2
  if constexpr (F::kRed == 1) f29a_sqr_s3_k1(r0, a0, s00, s01, s02);
  else f29a_sqr_s3_r1(r0, a0, s00, s01, s02);
#else
  f29 t0;
  f29_sqr<F>(t0, a0);
  f29_sub3_red<F>(r0, t0, s00, s01, s02);
#endif
}

// 2P. a = -3: dbl-2001-b (3M + 5S); a = 0: dbl-2009-l (2M + 5S) with
// D = 4XB as one product (3M + 4S). Prime-order
// curves have no 2-torsion, so only the point at infinity is exceptional.
// Every f29_sub / f29_red below respects fp29.hpp's operand bounds (value
// bounds in units of p in the comments; modelled in tests/test_fp29_model.py).
// Independent products are issued in pairs (same operands as the formulas'
// sequential statement, so the results are unchanged).
template <class C>
CDEV void jdbl(jpt& r, const jpt& p) {
  using F = typename C::F;
  if (p.inf) {
    r.inf = true;
    return;
  }
  f29 x3, y3, z3, t, u;
  if constexpr (C::kAm3) {
    f29 delta, gamma, x4, a3, b4, yz;
    f29_sqr_pair<F>(delta, p.Z, gamma, p.Y);
    f29_sub<F>(t, p.X, delta);  // < 4p
    f29_add(u, p.X, delta);     // < 4p
    f29_add(x4, p.X, p.X);
    f29_add(x4, x4, x4);        // 4X < 8p, limbs < 2^31: (4X) gamma < 16 p^2 < R p
    f29_mul_pair<F>(b4, x4, gamma, a3, t, u);  // 4 beta directly (no f29_mulk_red pass)
    f29_mulk_carry<F, 3>(a3, a3);  // alpha = 3 (X - delta)(X + delta) < 4.5p, unfolded
    // Z3 = 2 Y Z as one product instead of (Y + Z)^2 - gamma - delta (4M + 4S;
    // equal time with the square form once both subtractions ride in REDCs,
    // fewer instructions: profiles/r03_ec_glue_ab/)
    f29_add(yz, p.Y, p.Y);  // 2Y < 4p, limbs < 2^30.1
    f29_sqr_mul_pair_s2<F>(x3, a3, b4, b4, z3, yz, p.Z);  // X3 = alpha^2 - 8 beta
    f29_sub_loose<F>(u, b4, x3);  // < 6p, only the operand of alpha * u
    f29_add(t, gamma, gamma);
    f29_sqr_mul_pair_o2<F>(t, t, y3, a3, u);  // Y3 = alpha (4 beta - X3) - 2 (2 gamma)^2
  } else {
    f29 A, B, Cc, D, E, x4;
    f29_sqr_pair<F>(A, p.X, B, p.Y);
    f29_add(x4, p.X, p.X);
    f29_add(x4, x4, x4);         // 4X < 8p, limbs < 2^31: (4X) B < 16 p^2 < R p
    // D = 2 ((X + B)^2 - A - C) = 4 X B as one product: cheaper than the
    // square, the subtract pass and the doubling pass it replaces
    f29_sqr_mul_pair<F>(Cc, B, D, x4, B);
    f29_mulk_carry<F, 3>(E, A);  // E = 3 A < 3.4p, unfolded (A < 1.125p: a square of a norm X)
    f29_add(t, p.Y, p.Y);
    f29_sqr_mul_pair_s2<F>(x3, E, D, D, z3, t, p.Z);  // X3 = E^2 - 2 D, Z3 = 2 Y Z
    f29_sub_loose<F>(t, D, x3);  // < 6p, only the operand of E * t
    f29_mulk_red<F, 4>(u, Cc);   // 4 C
    f29_mul1_s2<F>(y3, E, t, u, u);  // Y3 = E (D - X3) - 8 C
  }
  r.X = x3;
  r.Y = y3;
  r.Z = z3;
  r.inf = false;
}

// P + Q, both Jacobian (add-2007-bl, 11M + 5S), with the exceptional cases
template <class C>
CDEV void jadd(jpt& r, const jpt& p, const jpt& q) {
  using F = typename C::F;
  if (p.inf) {
    r = q;
    return;
  }
  if (q.inf) {
    r = p;
    return;
  }
  f29 z1z1, z2z2, u1, u2, s1, s2, h, rr, t;
  f29_sqr<F>(z1z1, p.Z);
  f29_sqr<F>(z2z2, q.Z);
  f29_mul<F>(u1, p.X, z2z2);
  f29_mul<F>(u2, q.X, z1z1);
  f29_mul<F>(t, p.Y, q.Z);
  f29_mul<F>(s1, t, z2z2);
  f29_mul<F>(t, q.Y, p.Z);
  f29_mul<F>(s2, t, z1z1);
  f29_sub<F>(t, u2, u1);
  f29_red<F>(h, t);
  f29_sub<F>(t, s2, s1);
  f29_red<F>(rr, t);
  if (f29_iszero<F>(h)) {
    if (f29_iszero<F>(rr)) {
      jdbl<C>(r, p);
    } else {
      r.inf = true;
    }
    return;
  }
  f29 i, j, v, x3, y3, z3;
  f29_add(t, h, h);
  f29_sqr<F>(i, t);             // I = (2H)^2
  f29_mul<F>(j, h, i);          // J = H I
  f29_add(rr, rr, rr);          // r = 2 (S2 - S1), < 4p
  f29_mul<F>(v, u1, i);         // V = U1 I
  f29_sqr<F>(x3, rr);
  f29_sub<F>(x3, x3, j);
  f29_sub<F>(x3, x3, v);
  f29_sub<F>(t, x3, v);         // < 8p
  f29_red<F>(x3, t);            // X3 = r^2 - J - 2V
  f29_sub<F>(t, v, x3);
  f29_mul<F>(y3, rr, t);
  f29_mul<F>(t, s1, j);
  f29_sub<F>(y3, y3, t);
  f29_sub<F>(y3, y3, t);
  f29_red<F>(y3, y3);           // Y3 = r (V - X3) - 2 S1 J
  f29_add(t, p.Z, q.Z);
  f29_sqr<F>(t, t);
  f29_sub<F>(t, t, z1z1);
  f29_sub<F>(t, t, z2z2);       // < 6p
  f29_mul<F>(z3, t, h);         // Z3 = ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H
  r.X = x3;
  r.Y = y3;
  r.Z = z3;
  r.inf = false;
}

// P + (x2, y2) affine (madd-2007-bl, 7M + 4S), products paired as in jdbl
template <class C>
CDEV void jmadd(jpt& r, const jpt& p, const f29& x2, const f29& y2) {
  using F = typename C::F;
  if (p.inf) {
    r.X = x2;
    f29_red<F>(r.Y, y2);  // y2 may be f29_cneg_loose's 4p - y: back to norm
    f29_const_one<F>(r.Z);
    r.inf = false;
    return;
  }
  // every subtraction after a product rides in that product's REDC (*_s blocks)
  f29 z1z1, u2, h, hh, i, j, rr, v, t, x3, y3, z3;
  f29_sqr_mul_pair<F>(z1z1, p.Z, t, y2, p.Z);
  f29_mul_pair_s1s1<F>(h, x2, z1z1, p.X, rr, t, z1z1, p.Y);  // H = U2 - X1, R = S2 - Y1
  if (f29_iszero_norm<F>(h)) {  // h, rr norm (folded outputs)
    if (f29_iszero_norm<F>(rr)) {
      jdbl<C>(r, p);
    } else {
      r.inf = true;
    }
    return;
  }
  f29_add(rr, rr, rr);
  f29_add(t, p.Z, p.Z);
  f29_sqr_mul_pair<F>(hh, h, z3, t, h);  // HH, Z3 = 2 Z1 H (= (Z1 + H)^2 - Z1Z1 - HH)
  f29_add(i, hh, hh);
  f29_add(i, i, i);             // I = 4 HH, < 8p
  f29_mul_pair<F>(j, h, i, v, p.X, i);
  // Y1 J is only ever subtracted: Y3 = r (V - X3) + Y1 (4p - 2J) as ONE REDC
  // (-0.8% P-256, -1.5% secp256k1 ladder time, profiles/r03_ec_y3_ab/)
  f29_sqr1_s3<F>(x3, rr, j, v, v);  // X3 = r^2 - J - 2 V
  f29_sub<F>(u2, v, x3);
  f29_neg2_norm<F>(t, j);
  f29_mul2<F>(y3, rr, u2, p.Y, t);
  r.X = x3;
  r.Y = y3;
  r.Z = z3;
  r.inf = false;
}

// ---- G tables: entry k = [k]G affine (Montgomery, canonical) ---------------
// Booth windows of kGBits over the fixed base: 20-bit digits (|d| <= 2^19)
// cut the ladder's G additions from 32 to 13 (P-256) and from 34 to 14
// (secp256k1's two 129-bit halves) for tables of 2^19 + 1 affine entries
// (42 MB each, gathered from MALL; 12-bit windows measured 2.2% slower than
// 16-bit ones, profiles/r02_c3_field_ab.json, and 20-bit ones +0.9% on C3,
// profiles/r03_ec_g20_ab/); the window is a multiple of the 4-bit Q window so
// both share the doublings. Tables [0, kGEntries) = [k]G and, for
// secp256k1, [kGEntries, 2 kGEntries) = [k](lambda G) = (beta x, y).
#ifndef EC_G_BITS
#define EC_G_BITS 20
#endif
static constexpr int kGBits = EC_G_BITS;
static_assert(kGBits % 4 == 0, "G windows must share the 4-bit Q windows' doublings");
static constexpr int kGEntries = (1 << (kGBits - 1)) + 1;
static constexpr int kGEntryWords = 20;  // x[9], y[9], 2 pad: five 16-B loads
static constexpr int kGTables = 2;

template <class C>
__global__ void __launch_bounds__(64) ecdsa_gtable_kernel(uint32_t* __restrict__ tab) {
  using F = typename C::F;
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= kGTables * kGEntries) return;
  const int k = g % kGEntries;
  uint32_t* o = tab + g * kGEntryWords;
  if (k == 0 || (g >= kGEntries && !C::kGlv)) {
    for (int i = 0; i < kGEntryWords; i++) o[i] = 0;
    return;
  }
  jpt G, R;
  for (int i = 0; i < 9; i++) {
    G.X.v[i] = F::gxm(i);
    G.Y.v[i] = F::gym(i);
  }
  f29_const_one<F>(G.Z);
  G.inf = false;
  R.inf = true;
  for (int bit = kGBits - 1; bit >= 0; bit--) {
    jdbl<C>(R, R);
    if ((k >> bit) & 1) jadd<C>(R, R, G);
  }
  f29 zi, zi2, x, y;
  f29_pow_const<F, typename C::Pm2>(zi, R.Z);
  f29_sqr<F>(zi2, zi);
  f29_mul<F>(x, R.X, zi2);
  f29_mul<F>(zi2, zi2, zi);
  f29_mul<F>(y, R.Y, zi2);
  if (g >= kGEntries) {
    f29 b;
    for (int i = 0; i < 9; i++) b.v[i] = F::betam(i);
    f29_mul<F>(x, x, b);
  }
  f29_canon<F>(x, x);
  f29_canon<F>(y, y);
  for (int i = 0; i < 9; i++) {
    o[i] = x.v[i];
    o[9 + i] = y.v[i];
  }
  o[18] = 0;
  o[19] = 0;
}

CDEV void load_g(f29& x, f29& y, const uint32_t* __restrict__ tab, int idx) {
  const uint4* e = reinterpret_cast<const uint4*>(tab + idx * kGEntryWords);
  uint32_t w[20];
#pragma unroll
  for (int q = 0; q < 5; q++) {
    const uint4 v = e[q];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 9; i++) {
    x.v[i] = w[i];
    y.v[i] = w[9 + i];
  }
}

// SEC1 point decode + validation (BC ECCurve.decodePoint); Montgomery form
template <class C>
CDEV bool decode_key(jpt& Q, const uint8_t* __restrict__ key, uint32_t len) {
  using P = typename C::P;
  using F = typename C::F;
  const u256 pm = mod_m<P>();
  const bool unc = (len == 65 && key[0] == 4);
  const bool cmp = (len == 33 && (key[0] == 2 || key[0] == 3));
  if (!unc && !cmp) return false;
  u256 x, y;
  u256_from_be_bytes(x, key + 1);
  if (u256_geq(x, pm)) return false;
  f29 xm, rhs, t, ym;
  f29_from_words(t, x.v);
  f29_to_mont<F>(xm, t);
  // rhs = x^3 + a x + b
  f29_sqr<F>(rhs, xm);
  f29_mul<F>(rhs, rhs, xm);
  if constexpr (C::kAm3) {
    f29_add(t, xm, xm);
    f29_add(t, t, xm);
    f29_red<F>(t, t);
    f29_sub<F>(rhs, rhs, t);
  }
#pragma unroll
  for (int i = 0; i < 9; i++) t.v[i] = F::bm(i);
  f29_add(rhs, rhs, t);
  f29_red<F>(rhs, rhs);
  if (unc) {
    u256_from_be_bytes(y, key + 33);
    if (u256_geq(y, pm)) return false;
    f29_from_words(t, y.v);
    f29_to_mont<F>(ym, t);
  } else {
    f29_pow_const<F, typename C::Sqrt>(ym, rhs);
    f29 yp;
    f29_from_mont<F>(yp, ym);
    f29_cneg<F>(ym, (yp.v[0] & 1) != (uint32_t)(key[0] & 1));
  }
  f29_sqr<F>(t, ym);
  if (!f29_eq<F>(t, rhs)) return false;
  Q.X = xm;
  Q.Y = ym;
  f29_const_one<F>(Q.Z);
  Q.inf = false;
  return true;
}

// scalar k < n -> (k' < 2^255, neg) with [k]X = neg ? -[k']X : [k']X
template <class N>
CDEV void split_sign(u256& out, bool& neg, const u256& k) {
  neg = (k.v[7] >> 31) != 0;
  u256 t;
  u256_sub(t, mod_m<N>(), k);
#pragma unroll
  for (int i = 0; i < 8; i++) out.v[i] = neg ? t.v[i] : k.v[i];
}

// round(k g / 2^384) for k, g < 2^256 (bits 384.. of the product, rounded at bit 383)
CDEV void mul_shift_384(u256& c, const u256& k, const u256& g) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t t = (uint64_t)k.v[i] * g.v[j] + x[i + j] + carry;
      x[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    x[i + 8] = (uint32_t)carry;
  }
  uint64_t s = (uint64_t)x[12] + (x[11] >> 31);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (i) s += x[12 + i];
    c.v[i] = (uint32_t)s;
    s >>= 32;
  }
  c.v[4] = (uint32_t)s;
  c.v[5] = c.v[6] = c.v[7] = 0;
}

// secp256k1 GLV split: k == k1 + k2 lambda (mod n), returned as magnitudes
// < 2^129 with signs (split_sign convention). Basis, rounding constants and
// the bound: tools/gen_fp29_consts.py (Gallant-Lambert-Vanstone 2001).
CDEV void glv_split(u256& k1, bool& neg1, u256& k2, bool& neg2, const u256& k) {
  using N = K1N;
  u256 c1, c2, t1, t2, r1, r2;
  mul_shift_384(c1, k, limbs_of<K1G1>());
  mul_shift_384(c2, k, limbs_of<K1G2>());
  mont_mul<N>(t1, c1, limbs_of<K1MB1M>());   // c1 (-b1) mod n
  mont_mul<N>(t2, c2, limbs_of<K1MB2M>());   // c2 (-b2) mod n
  mod_add<N>(r2, t1, t2);
  mont_mul<N>(t1, r2, limbs_of<K1MLamM>());  // -lambda r2
  mod_add<N>(r1, t1, k);
  split_sign<N>(k1, neg1, r1);
  split_sign<N>(k2, neg2, r2);
}

// ---- per-lane workspace record (split path) and its layout ------------------
// Slots are the curve-partitioned order (perm), processed in chunks of
// ws_slots; each slot owns a 1 KiB record in HBM.
static constexpr int kEcPtWords = 28;           // X, Y, Z (9 limbs each) + 1 pad: seven 16-B accesses
static constexpr int kEcTab = 0;                // [k]Q, k = 1..8, Jacobian
static constexpr int kEcS = 8 * kEcPtWords;     // s, Montgomery form mod n (batch-inversion input)
static constexpr int kEcW = kEcS + 8;           // prefix products, then w = s^-1 (Montgomery form mod n)
static constexpr int kEcE = kEcW + 8;           // e = SHA-256(msg) mod n
static constexpr int kEcR = kEcE + 8;           // r
static constexpr int kEcZ = kEcR + 8;           // prod of the table's Z (k = 2..8), Montgomery mod p (12 words)
static constexpr int kEcZW = kEcZ + 12;         // prefix products, then that product's inverse (12 words)
static constexpr int kEcWords = kEcZW + 12;     // 280 words = 1120 B
static constexpr int kEcInvBatch = 64;          // signatures per thread in the batch inversion
static constexpr uint8_t kEcPending = 0xff;     // slot whose verdict the ladder decides

CDEV void st256(uint32_t* __restrict__ o, const u256& v) {
  uint4* o4 = reinterpret_cast<uint4*>(o);
  o4[0] = make_uint4(v.v[0], v.v[1], v.v[2], v.v[3]);
  o4[1] = make_uint4(v.v[4], v.v[5], v.v[6], v.v[7]);
}
CDEV void ld256(u256& v, const uint32_t* __restrict__ p) {
  const uint4* p4 = reinterpret_cast<const uint4*>(p);
  const uint4 a = p4[0], b = p4[1];
  v.v[0] = a.x; v.v[1] = a.y; v.v[2] = a.z; v.v[3] = a.w;
  v.v[4] = b.x; v.v[5] = b.y; v.v[6] = b.z; v.v[7] = b.w;
}
CDEV void st_f29(uint32_t* __restrict__ o, const f29& a) {
  uint4* o4 = reinterpret_cast<uint4*>(o);
  o4[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
  o4[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
  o4[2] = make_uint4(a.v[8], 0u, 0u, 0u);
}
CDEV void ld_f29(f29& a, const uint32_t* __restrict__ o) {
  const uint4* o4 = reinterpret_cast<const uint4*>(o);
  const uint4 x = o4[0], y = o4[1], z = o4[2];
  a.v[0] = x.x; a.v[1] = x.y; a.v[2] = x.z; a.v[3] = x.w;
  a.v[4] = y.x; a.v[5] = y.y; a.v[6] = y.z; a.v[7] = y.w; a.v[8] = z.x;
}
// Z of a Jacobian table slot: words 18..26, read as the three aligned 16-B
// vectors covering words 16..27 (slots start 16-B aligned)
CDEV void ld_slot_z(f29& z, const uint32_t* __restrict__ slot) {
  const uint4* o4 = reinterpret_cast<const uint4*>(slot + 16);
  const uint4 a = o4[0], b = o4[1], c = o4[2];
  z.v[0] = a.z; z.v[1] = a.w;
  z.v[2] = b.x; z.v[3] = b.y; z.v[4] = b.z; z.v[5] = b.w;
  z.v[6] = c.x; z.v[7] = c.y; z.v[8] = c.z;
}
// affine table entry: X, Y in the first 18 words of a kEcPtWords slot (five 16-B loads)
CDEV void ld_aff(f29& x, f29& y, const uint32_t* __restrict__ o) {
  const uint4* o4 = reinterpret_cast<const uint4*>(o);
  uint32_t w[20];
#pragma unroll
  for (int q = 0; q < 5; q++) {
    const uint4 v = o4[q];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 9; i++) {
    x.v[i] = w[i];
    y.v[i] = w[9 + i];
  }
}

CDEV void st_jpt(uint32_t* __restrict__ o, const jpt& p) {
  uint32_t w[28];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    w[i] = p.X.v[i];
    w[9 + i] = p.Y.v[i];
    w[18 + i] = p.Z.v[i];
  }
  w[27] = 0;
  uint4* o4 = reinterpret_cast<uint4*>(o);
#pragma unroll
  for (int q = 0; q < 7; q++) o4[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
CDEV void ld_jpt(jpt& p, const uint32_t* __restrict__ o) {
  const uint4* o4 = reinterpret_cast<const uint4*>(o);
  uint32_t w[28];
#pragma unroll
  for (int q = 0; q < 7; q++) {
    const uint4 v = o4[q];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 9; i++) {
    p.X.v[i] = w[i];
    p.Y.v[i] = w[9 + i];
    p.Z.v[i] = w[18 + i];
  }
  p.inf = false;
}

// x(P) mod n == r  <=>  X == r Z^2  or (r < p - n and X == (r + n) Z^2)
template <class C>
CDEV uint8_t x_check(const jpt& acc, const u256& r) {
  using F = typename C::F;
  if (acc.inf) return kStatusBadSig;
  f29 z2, rm, t;
  f29_sqr<F>(z2, acc.Z);
  f29_from_words(t, r.v);
  f29_to_mont<F>(rm, t);
  f29_mul<F>(t, rm, z2);
  const bool eq0 = f29_eq<F>(t, acc.X);
  u256 rn;
  u256_add(rn, r, mod_m<typename C::N>());
  const bool alt = !u256_geq(r, limbs_of<typename C::PmN>());
  f29_from_words(t, rn.v);
  f29_to_mont<F>(rm, t);
  f29_mul<F>(t, rm, z2);
  const bool eq1 = f29_eq<F>(t, acc.X);
  return (eq0 || (alt && eq1)) ? kStatusOk : kStatusBadSig;
}

// Everything before the scalar multiplication, in the reference's order (key
// decode, Crypto.doVerify's require()s, DER, range checks), then e, s, r and
// the [k]Q table go to the slot's record. Decided lanes store s = 1 so the
// batch product stays invertible.
template <class C>
CDEV uint8_t ecdsa_prep_lane(const uint8_t* __restrict__ key, uint32_t key_len, const uint8_t* __restrict__ sig,
                             uint32_t sig_len, const uint8_t* __restrict__ msg, uint64_t msg_len, uint8_t pre_status,
                             bool empty_is_error, uint32_t* __restrict__ rec) {
  using N = typename C::N;
  using F = typename C::F;
  f29 zprod;
  f29_const_one<F>(zprod);
  u256 sm;
  {
    u256 one;
#pragma unroll
    for (int q = 0; q < 8; q++) one.v[q] = q == 0;
    to_mont<N>(sm, one);
  }
  jpt Q;
  uint8_t st = kEcPending;
  u256 r, s;
  if (!decode_key<C>(Q, key, key_len)) {
    st = kStatusBadKey;  // key built before verify
  } else if (pre_status != kStatusOk) {
    st = pre_status;
  } else if (empty_is_error && (sig_len == 0 || msg_len == 0)) {
    st = kStatusEmpty;  // doVerify: Crypto.kt:475-476 (isValid: DER decode / hash as usual)
  } else {
    DerInt dr, ds;
    if (!der_decode_sig(sig, sig_len, dr, ds)) {
      st = kStatusMalformedSig;
    } else {
#pragma unroll
      for (int q = 0; q < 8; q++) {
        r.v[q] = dr.v[q];
        s.v[q] = ds.v[q];
      }
      const u256 nm = mod_m<N>();
      if (dr.neg || dr.big || ds.neg || ds.big || u256_iszero(r) || u256_iszero(s) || u256_geq(r, nm) ||
          u256_geq(s, nm))
        st = kStatusBadSig;
    }
  }
  if (st == kEcPending) {
    uint32_t hw[8];
    sha256_bytes(hw, msg, msg_len);
    u256 e, t;
#pragma unroll
    for (int q = 0; q < 8; q++) e.v[q] = hw[7 - q];
    if (!u256_sub(t, e, mod_m<N>())) e = t;
    to_mont<N>(sm, s);
    st256(rec + kEcE, e);
    st256(rec + kEcR, r);
    st_jpt(rec + kEcTab, Q);
    jpt T;
    jdbl<C>(T, Q);
    st_jpt(rec + kEcTab + kEcPtWords, T);
    zprod = T.Z;
    for (int k = 3; k <= 8; k++) {
      jmadd<C>(T, T, Q.X, Q.Y);  // Q has Z = 1
      st_jpt(rec + kEcTab + kEcPtWords * (k - 1), T);
      f29_mul<F>(zprod, zprod, T.Z);
    }
  }
  st256(rec + kEcS, sm);
  st_f29(rec + kEcZ, zprod);  // decided lanes: 1, so the batch product stays invertible
  return st;
}

// P = u1 G + u2 Q with w = s^-1 from the record; x(P) mod n == r
template <class C>
CDEV uint8_t ecdsa_ladder_lane(const uint32_t* __restrict__ rec, const uint32_t* __restrict__ gtab) {
  using F = typename C::F;
  using N = typename C::N;
  u256 w, e, r, u1, u2;
  ld256(w, rec + kEcW);
  ld256(e, rec + kEcE);
  ld256(r, rec + kEcR);
  mont_mul<N>(u1, e, w);  // plain e * s^-1 (one Montgomery factor cancels)
  mont_mul<N>(u2, r, w);
  const uint32_t* tab = rec + kEcTab;
  jpt acc;
  acc.inf = true;
  if constexpr (C::kGlv) {
    // u1 G = [a1]G + [a2](lambda G), u2 Q = [b1]Q + [b2]phi(Q): 33 windows of 4 bits
    u256 a1, a2, b1, b2;
    bool na1, na2, nb1, nb2;
    glv_split(a1, na1, a2, na2, u1);
    glv_split(b1, nb1, b2, nb2, u2);
    f29 beta;
#pragma unroll
    for (int i = 0; i < 9; i++) beta.v[i] = F::betam(i);
    const uint32_t* gtab2 = gtab + kGEntries * kGEntryWords;
    for (int j = 32; j >= 0; j--) {
      const int d1 = booth_digit<4>(b1.v, j), d2 = booth_digit<4>(b2.v, j);
      const int e1 = d1 < 0 ? -d1 : d1, e2 = d2 < 0 ? -d2 : d2;
      f29 x1, y1, x2, y2;  // affine [k]Q; issued before the doublings, consumed after them
      ld_aff(x1, y1, tab + kEcPtWords * (e1 > 0 ? e1 - 1 : 0));
      ld_aff(x2, y2, tab + kEcPtWords * (e2 > 0 ? e2 - 1 : 0));
      if (j != 32) {
        jdbl<C>(acc, acc);
        jdbl<C>(acc, acc);
        jdbl<C>(acc, acc);
        jdbl<C>(acc, acc);
      }
      if (e1) {
        f29_cneg_loose<F>(y1, (d1 < 0) != nb1);
        jmadd<C>(acc, acc, x1, y1);
      }
      if (e2) {
        f29_mul1<F>(x2, x2, beta);  // phi([e2]Q)
        f29_cneg_loose<F>(y2, (d2 < 0) != nb2);
        jmadd<C>(acc, acc, x2, y2);
      }
      if (j % (kGBits / 4) == 0) {
        const int g1 = booth_digit<kGBits>(a1.v, j / (kGBits / 4)), g2 = booth_digit<kGBits>(a2.v, j / (kGBits / 4));
        f29 gx, gy;
        if (g1) {
          load_g(gx, gy, gtab, g1 < 0 ? -g1 : g1);
          f29_cneg_loose<F>(gy, (g1 < 0) != na1);
          jmadd<C>(acc, acc, gx, gy);
        }
        if (g2) {
          load_g(gx, gy, gtab2, g2 < 0 ? -g2 : g2);
          f29_cneg_loose<F>(gy, (g2 < 0) != na2);
          jmadd<C>(acc, acc, gx, gy);
        }
      }
    }
  } else {
    bool neg1, neg2;
    split_sign<N>(u1, neg1, u1);
    split_sign<N>(u2, neg2, u2);
    for (int j = 63; j >= 0; j--) {
      const int dq = booth_digit<4>(u2.v, j);
      const int aq = dq < 0 ? -dq : dq;
      f29 tx, ty;  // affine [aq]Q; issued before the doublings, consumed after them
      ld_aff(tx, ty, tab + kEcPtWords * (aq > 0 ? aq - 1 : 0));
      if (j != 63) {
        jdbl<C>(acc, acc);
        jdbl<C>(acc, acc);
        jdbl<C>(acc, acc);
        jdbl<C>(acc, acc);
      }
      if (aq) {
        f29_cneg_loose<F>(ty, (dq < 0) != neg2);
        jmadd<C>(acc, acc, tx, ty);
      }
      if (j % (kGBits / 4) == 0) {
        const int dg = booth_digit<kGBits>(u1.v, j / (kGBits / 4));
        if (dg) {
          f29 gx, gy;
          load_g(gx, gy, gtab, dg < 0 ? -dg : dg);
          f29_cneg_loose<F>(gy, (dg < 0) != neg1);
          jmadd<C>(acc, acc, gx, gy);
        }
      }
    }
  }
  return x_check<C>(acc, r);
}

// ---- signing (corpus generation for the C3 / C5 benchmarks) -----------------
// d = SHA-256(seed) mod n, k = SHA-256(seed || msg) mod n (deterministic
// synthetic nonces: this is test-data generation, not a production signer).
template <class C>
CDEV void fixed_base_g(jpt& acc, const u256& k, const uint32_t* __restrict__ gtab) {
  using F = typename C::F;
  u256 kk;
  bool neg;
  split_sign<typename C::N>(kk, neg, k);
  acc.inf = true;
  for (int j = 31; j >= 0; j--) {
    if (j != 31)
      for (int t = 0; t < 8; t++) jdbl<C>(acc, acc);
    const int d = booth_digit<8>(kk.v, j);
    if (d != 0) {
      f29 gx, gy;
      load_g(gx, gy, gtab, d < 0 ? -d : d);
      f29_cneg_loose<F>(gy, (d < 0) != neg);
      jmadd<C>(acc, acc, gx, gy);
    }
  }
}

template <class C>
CDEV void to_affine(u256& x, u256& y, const jpt& p) {  // plain coordinates
  using F = typename C::F;
  f29 zi, zi2, X, Y;
  f29_pow_const<F, typename C::Pm2>(zi, p.Z);
  f29_sqr<F>(zi2, zi);
  f29_mul<F>(X, p.X, zi2);
  f29_mul<F>(zi2, zi2, zi);
  f29_mul<F>(Y, p.Y, zi2);
  f29_from_mont<F>(X, X);
  f29_from_mont<F>(Y, Y);
  f29_to_words(x.v, X);
  f29_to_words(y.v, Y);
}

CDEV void put_be32(uint8_t* o, const u256& v) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t w = v.v[7 - i];
    o[4 * i] = w >> 24;
    o[4 * i + 1] = w >> 16;
    o[4 * i + 2] = w >> 8;
    o[4 * i + 3] = w;
  }
}
// minimal DER INTEGER of a positive value < 2^256; returns bytes written
CDEV uint32_t der_put_int(uint8_t* o, const u256& v) {
  uint8_t be[32];
  put_be32(be, v);
  int start = 0;
  while (start < 31 && be[start] == 0) start++;
  const bool pad = be[start] >= 0x80;
  const uint32_t len = (32 - start) + (pad ? 1 : 0);
  o[0] = 0x02;
  o[1] = (uint8_t)len;
  uint32_t p = 2;
  if (pad) o[p++] = 0;
  for (int i = start; i < 32; i++) o[p++] = be[i];
  return p;
}

template <class C>
CDEV u256 hash_mod_n(const uint8_t* p, uint64_t len) {
  uint32_t hw[8];
  sha256_bytes(hw, p, len);
  u256 e, t;
#pragma unroll
  for (int i = 0; i < 8; i++) e.v[i] = hw[7 - i];
  if (!u256_sub(t, e, mod_m<typename C::N>())) e = t;
  if (u256_iszero(e)) e.v[0] = 1;
  return e;
}

template <class C>
CDEV void ecdsa_sign_lane(const uint8_t* __restrict__ seed, const uint8_t* __restrict__ msg, uint32_t msg_len,
                          const uint32_t* __restrict__ gtab, uint8_t* key_out, uint8_t* key_len_out, uint8_t* sig_out,
                          uint8_t* sig_len_out) {
  using N = typename C::N;
  uint8_t buf[32 + 64];
  for (int i = 0; i < 32; i++) buf[i] = seed[i];
  const u256 d = hash_mod_n<C>(buf, 32);
  const uint32_t ml = msg_len <= 64 ? msg_len : 64;
  for (uint32_t i = 0; i < ml; i++) buf[32 + i] = msg[i];
  const u256 k = hash_mod_n<C>(buf, 32 + ml);
  jpt Q, R;
  fixed_base_g<C>(Q, d, gtab);
  fixed_base_g<C>(R, k, gtab);
  u256 qx, qy, rx, ry;
  to_affine<C>(qx, qy, Q);
  to_affine<C>(rx, ry, R);
  key_out[0] = 4;
  put_be32(key_out + 1, qx);
  put_be32(key_out + 33, qy);
  *key_len_out = 65;
  u256 r = rx, t;
  if (!u256_sub(t, r, mod_m<N>())) r = t;  // r = x mod n
  uint32_t hw[8];
  sha256_bytes(hw, msg, msg_len);
  u256 e;
#pragma unroll
  for (int i = 0; i < 8; i++) e.v[i] = hw[7 - i];
  if (!u256_sub(t, e, mod_m<N>())) e = t;
  // s = k^-1 (e + r d) mod n
  u256 km, kinv, rm, rd, sum, s;
  to_mont<N>(km, k);
  mont_pow_const<N, typename C::Nm2>(kinv, km);
  to_mont<N>(rm, r);
  mont_mul<N>(rd, rm, d);
  mod_add<N>(sum, e, rd);
  mont_mul<N>(s, kinv, sum);
  uint8_t body[70];
  uint32_t p = der_put_int(body, r);
  p += der_put_int(body + p, s);
  sig_out[0] = 0x30;
  sig_out[1] = (uint8_t)p;
  for (uint32_t i = 0; i < p; i++) sig_out[2 + i] = body[i];
  *sig_len_out = (uint8_t)(p + 2);
}

__global__ void __launch_bounds__(256) ecdsa_sign_kernel(const uint8_t* __restrict__ scheme,
                                                        const uint8_t* __restrict__ seeds,
                                                        const uint8_t* __restrict__ msgs, uint32_t msg_len,
                                                        uint64_t n, const uint32_t* __restrict__ gk1,
                                                        const uint32_t* __restrict__ gr1, uint8_t* __restrict__ keys,
                                                        uint8_t* __restrict__ key_len, uint8_t* __restrict__ sigs,
                                                        uint8_t* __restrict__ sig_len) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* msg = msgs + i * (uint64_t)msg_len;
  if (scheme[i] == 2)
    ecdsa_sign_lane<Curve<2>>(seeds + i * 32, msg, msg_len, gk1, keys + i * 65, key_len + i, sigs + i * 72,
                              sig_len + i);
  else
    ecdsa_sign_lane<Curve<3>>(seeds + i * 32, msg, msg_len, gr1, keys + i * 65, key_len + i, sigs + i * 72,
                              sig_len + i);
}

// ---- device-side scheme partition (wave-aggregated atomics) -----------------
// Partition classes: secp256k1 uncompressed / compressed, P-256 uncompressed /
// compressed, other. Compressed keys (33-byte SEC1) need a square root in
// prep (a 256-bit exponentiation, about half of prep's instructions); grouping
// them keeps that divergent branch inside ~10% of the waves instead of
// letting one compressed key per wave stall 63 lanes. Curve runs stay
// contiguous: [0, n0 + n1) secp256k1, then P-256, then the rest.
static constexpr int kPartClasses = 5;
CDEV int scheme_class(uint8_t s, uint8_t key_len) {
  const int comp = key_len == 33 ? 1 : 0;
  return s == 2 ? comp : s == 3 ? 2 + comp : 4;
}

// Each 256-thread block owns a tile of kPartTile lanes, visited in kPartIter
// coalesced strides. Counting: wave ballots -> per-wave totals -> LDS -> ONE
// atomic per class per block. Scatter: a wave first totals its kPartIter
// ballots per class, reserves its range with one atomic per class, then
// re-reads its (L1/L2-resident) scheme bytes and writes ranks. The previous
// one-atomic-per-wave-per-class form serialised ~800k atomics on three
// addresses (~6 ms per 2^24 lanes per kernel); this issues 16x fewer.
static constexpr int kPartIter = 16;
static constexpr int kPartTile = 256 * kPartIter;

__global__ void __launch_bounds__(256) ecdsa_count_kernel(const uint8_t* __restrict__ scheme,
                                                         const uint8_t* __restrict__ key_len, uint64_t n,
                                                         unsigned int* __restrict__ counts) {
  __shared__ unsigned int part[kPartClasses][4];
  const uint64_t tile = (uint64_t)blockIdx.x * kPartTile;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned int tot[kPartClasses] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll 4
  for (int it = 0; it < kPartIter; it++) {
    const uint64_t i = tile + (uint64_t)it * 256 + threadIdx.x;
    const int c = i < n ? scheme_class(scheme[i], key_len[i]) : -1;
#pragma unroll
    for (int k = 0; k < kPartClasses; k++) tot[k] += (unsigned int)__popcll(__ballot(c == k));
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < kPartClasses; k++) part[k][wave] = tot[k];
  }
  __syncthreads();
  if (threadIdx.x < kPartClasses) {
    const unsigned int t = part[threadIdx.x][0] + part[threadIdx.x][1] + part[threadIdx.x][2] + part[threadIdx.x][3];
    if (t) atomicAdd(&counts[threadIdx.x], t);
  }
}

__global__ void __launch_bounds__(256) ecdsa_scatter_kernel(const uint8_t* __restrict__ scheme,
                                                           const uint8_t* __restrict__ key_len, uint64_t n,
                                                           const unsigned int* __restrict__ counts,
                                                           unsigned int* __restrict__ cursors,
                                                           unsigned int* __restrict__ perm) {
  const uint64_t tile = (uint64_t)blockIdx.x * kPartTile;
  const int lane = threadIdx.x & 63;
  unsigned int tot[kPartClasses] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll 4
  for (int it = 0; it < kPartIter; it++) {
    const uint64_t i = tile + (uint64_t)it * 256 + threadIdx.x;
    const int c = i < n ? scheme_class(scheme[i], key_len[i]) : -1;
#pragma unroll
    for (int k = 0; k < kPartClasses; k++) tot[k] += (unsigned int)__popcll(__ballot(c == k));
  }
  unsigned int start[kPartClasses];
  unsigned int base = 0;
#pragma unroll
  for (int k = 0; k < kPartClasses; k++) {
    unsigned int s0 = 0;
    if (lane == 0 && tot[k]) s0 = atomicAdd(&cursors[k], tot[k]);
    start[k] = __shfl(s0, 0) + base;
    base += counts[k];
  }
  const unsigned long long below = (1ull << lane) - 1;
#pragma unroll 4
  for (int it = 0; it < kPartIter; it++) {
    const uint64_t i = tile + (uint64_t)it * 256 + threadIdx.x;
    const int c = i < n ? scheme_class(scheme[i], key_len[i]) : -1;
#pragma unroll
    for (int k = 0; k < kPartClasses; k++) {
      const unsigned long long m = __ballot(c == k);
      if (c == k) perm[start[k] + __popcll(m & below)] = (unsigned int)i;
      start[k] += (unsigned int)__popcll(m);
    }
  }
}

__global__ void __launch_bounds__(256) verdict_kernel(const uint8_t* __restrict__ status, uint64_t n,
                                                     unsigned long long* __restrict__ verdict) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long m = __ballot(i < n && status[i] == kStatusOk);
  if ((threadIdx.x & 63) == 0 && i < n) verdict[i >> 6] = m;
}

// ---- split verification (default): prep -> batch inversion -> ladder --------
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) ecdsa_prep_kernel(
    const unsigned int* __restrict__ perm, const uint8_t* __restrict__ scheme, const uint8_t* __restrict__ keys,
    const uint8_t* __restrict__ key_len, const uint8_t* __restrict__ sigs, const uint8_t* __restrict__ sig_len,
    const uint8_t* __restrict__ msgs, const uint64_t* __restrict__ msg_off, uint32_t msg_len, uint64_t base,
    uint64_t m, const uint8_t* __restrict__ pre_status, uint8_t* __restrict__ status, uint32_t* __restrict__ ws,
    uint32_t empty_is_error) {
  const uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= m) return;
  const uint64_t slot = base + li;
  const uint64_t i = perm ? perm[slot] : slot;
  const uint8_t sch = scheme[i];
  const uint8_t* key = keys + i * 65;
  const uint8_t* sig = sigs + i * 72;
  const uint8_t* msg = msg_off ? msgs + msg_off[i] : msgs + i * (uint64_t)msg_len;
  const uint64_t ml = msg_off ? msg_off[i + 1] - msg_off[i] : msg_len;
  uint8_t pre = pre_status ? pre_status[i] : kStatusOk;
  // a DER signature longer than its 72-byte slot is not representable in the
  // dense layout (r, s < n always fit 72 bytes, so BC would reject it too): the
  // lane is decided without reading past the slot. The generic CSR path decodes
  // such signatures exactly on the host (cordahip.cpp ecdsa_host_lanes).
  const uint32_t sl = sig_len[i];
  if (sl > 72 && pre == kStatusOk) pre = (ml == 0 && empty_is_error) ? kStatusEmpty : kStatusMalformedSig;
  uint32_t* rec = ws + li * kEcWords;
  uint8_t st;
  if (sch == 2)
    st = ecdsa_prep_lane<Curve<2>>(key, key_len[i], sig, sl > 72 ? 72 : sl, msg, ml, pre, empty_is_error, rec);
  else if (sch == 3)
    st = ecdsa_prep_lane<Curve<3>>(key, key_len[i], sig, sl > 72 ? 72 : sl, msg, ml, pre, empty_is_error, rec);
  else
    st = kStatusUnsupported;
  status[i] = st;
}

// Montgomery's trick over chunk-relative slots [a, b) of one curve: prefix
// products into W, ONE Fermat inversion, then back-substitution: every slot's
// W becomes s^-1, at 3 multiplications per slot plus 1/(b-a) of an inversion.
template <class C>
CDEV void ecdsa_inv_run(uint32_t* __restrict__ ws, uint64_t a, uint64_t b) {
  using N = typename C::N;
  u256 acc, x;
  ld256(acc, ws + a * kEcWords + kEcS);
  st256(ws + a * kEcWords + kEcW, acc);
  for (uint64_t j = a + 1; j < b; j++) {
    ld256(x, ws + j * kEcWords + kEcS);
    mont_mul<N>(acc, acc, x);
    st256(ws + j * kEcWords + kEcW, acc);
  }
  u256 inv;
  mont_pow_const<N, typename C::Nm2>(inv, acc);
  for (uint64_t j = b - 1; j > a; j--) {
    ld256(x, ws + (j - 1) * kEcWords + kEcW);
    u256 wj;
    mont_mul<N>(wj, inv, x);
    st256(ws + j * kEcWords + kEcW, wj);
    ld256(x, ws + j * kEcWords + kEcS);
    mont_mul<N>(inv, inv, x);
  }
  st256(ws + a * kEcWords + kEcW, inv);
}

// The same trick mod p over the slots' table-Z products (kEcZ -> kEcZW).
template <class C>
CDEV void ecdsa_zinv_run(uint32_t* __restrict__ ws, uint64_t a, uint64_t b) {
  using F = typename C::F;
  f29 acc, x;
  ld_f29(acc, ws + a * kEcWords + kEcZ);
  st_f29(ws + a * kEcWords + kEcZW, acc);
  for (uint64_t j = a + 1; j < b; j++) {
    ld_f29(x, ws + j * kEcWords + kEcZ);
    f29_mul<F>(acc, acc, x);
    st_f29(ws + j * kEcWords + kEcZW, acc);
  }
  f29 inv;
  f29_pow_const<F, typename C::Pm2>(inv, acc);
  for (uint64_t j = b - 1; j > a; j--) {
    ld_f29(x, ws + (j - 1) * kEcWords + kEcZW);
    f29 wj;
    f29_mul<F>(wj, inv, x);
    st_f29(ws + j * kEcWords + kEcZW, wj);
    ld_f29(x, ws + j * kEcWords + kEcZ);
    f29_mul<F>(inv, inv, x);
  }
  st_f29(ws + a * kEcWords + kEcZW, inv);
}

// kEcInvBatch consecutive slots per thread; curve runs from the partition
// counts (slots [0, c1) secp256k1, [c1, c1 + c2) P-256, the rest unsupported)
__global__ void __launch_bounds__(256) ecdsa_inv_kernel(uint64_t base, uint64_t m,
                                                       const unsigned int* __restrict__ counts,
                                                       uint32_t* __restrict__ ws) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t lo = t * kEcInvBatch;
  if (lo >= m) return;
  const uint64_t hi = lo + kEcInvBatch < m ? lo + kEcInvBatch : m;
  const uint64_t c1 = counts[0] + counts[1], c2 = c1 + counts[2] + counts[3];  // secp256k1 | P-256 runs
  const uint64_t k1_end = c1 > base ? (c1 - base < m ? c1 - base : m) : 0;
  const uint64_t r1_end = c2 > base ? (c2 - base < m ? c2 - base : m) : 0;
  {
    const uint64_t a = lo, b = hi < k1_end ? hi : k1_end;
    if (a < b) {
      ecdsa_inv_run<Curve<2>>(ws, a, b);
      ecdsa_zinv_run<Curve<2>>(ws, a, b);
    }
  }
  {
    const uint64_t a = lo > k1_end ? lo : k1_end, b = hi < r1_end ? hi : r1_end;
    if (a < b) {
      ecdsa_inv_run<Curve<3>>(ws, a, b);
      ecdsa_zinv_run<Curve<3>>(ws, a, b);
    }
  }
}

// Table [k]Q, k = 2..8, to affine with the inverse of their Z product from
// ecdsa_inv_kernel: per-entry Z^-1 by back-substitution (2M each), then
// x = X Z^-2, y = Y Z^-3 written over X, Y. The ladder then adds Q-multiples
// with jmadd (7M + 4S) instead of jadd (11M + 5S).
template <class C>
CDEV void ecdsa_affine_lane(uint32_t* __restrict__ rec) {
  using F = typename C::F;
  uint32_t* tab = rec + kEcTab;
  f29 pre[7];  // pre[k - 2] = Z_2 ... Z_k
  ld_slot_z(pre[0], tab + kEcPtWords * 1);
#pragma unroll
  for (int k = 3; k <= 8; k++) {
    f29 z;
    ld_slot_z(z, tab + kEcPtWords * (k - 1));
    f29_mul<F>(pre[k - 2], pre[k - 3], z);
  }
  f29 inv;
  ld_f29(inv, rec + kEcZW);  // (Z_2 ... Z_8)^-1
#pragma unroll
  for (int k = 8; k >= 2; k--) {
    f29 zi, z;
    if (k > 2) {
      ld_slot_z(z, tab + kEcPtWords * (k - 1));
      // Z_k^-1, (Z_2 ... Z_{k-1})^-1
      f29_mul_pair<F>(zi, inv, pre[k - 3], inv, inv, z);
    } else {
      zi = inv;
    }
    f29 z2, z3, x, y;
    ld_aff(x, y, tab + kEcPtWords * (k - 1));
    f29_sqr<F>(z2, zi);
    f29_mul_pair<F>(z3, z2, zi, x, x, z2);
    f29_mul<F>(y, y, z3);
    uint32_t w[20];
#pragma unroll
    for (int q = 0; q < 9; q++) {
      w[q] = x.v[q];
      w[9 + q] = y.v[q];
    }
    w[18] = w[19] = 0;
    uint4* o4 = reinterpret_cast<uint4*>(tab + kEcPtWords * (k - 1));
#pragma unroll
    for (int q = 0; q < 5; q++) o4[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
}

// One kernel per curve (launched over the whole chunk; the other curve's lanes
// exit at once, and the partition makes them whole waves): the register
// allocations differ (P-256 allocates 164 VGPRs = 3 waves per SIMD, secp256k1's
// GLV ladder 221 = 2 waves), and a combined kernel runs both at the larger one.
// amdgpu_waves_per_eu(2) is a lower bound on occupancy, i.e. a VGPR CAP of 256
// for both (the allocation itself sets 3 waves for P-256); every budget >= 164
// leaves room for fp29_asm.hpp's fixed accumulators v160..v163.
template <int S>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) ecdsa_ladder_kernel(
    const unsigned int* __restrict__ perm, const uint8_t* __restrict__ scheme, uint64_t base, uint64_t m,
    const uint32_t* __restrict__ gtab, uint32_t* __restrict__ ws, uint8_t* __restrict__ status) {
  const uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= m) return;
  const uint64_t slot = base + li;
  const uint64_t i = perm ? perm[slot] : slot;
  if (scheme[i] != S || status[i] != kEcPending) return;
  uint32_t* rec = ws + li * kEcWords;
  // table-to-affine pass fused into the ladder: as a kernel of its own its
  // uncoalesced record traffic cost 14.8 ms per 2^24 lanes; here it overlaps the
  // VALU-bound ladder of the SIMD's other waves (same thread writes, then reads)
  ecdsa_affine_lane<Curve<S>>(rec);
  status[i] = ecdsa_ladder_lane<Curve<S>>(rec, gtab);
}

// ---------------------------------------------------------------------------
size_t ecdsa_gtable_bytes() { return (size_t)kGTables * kGEntries * kGEntryWords * sizeof(uint32_t); }
size_t ecdsa_ws_slot_bytes() { return kEcWords * sizeof(uint32_t); }

hipError_t launch_ecdsa_sign(const uint8_t* scheme, const uint8_t* seeds, const uint8_t* msgs, uint32_t msg_len,
                             uint64_t n, const uint32_t* gk1, const uint32_t* gr1, uint8_t* keys, uint8_t* key_len,
                             uint8_t* sigs, uint8_t* sig_len, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(ecdsa_sign_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, scheme, seeds, msgs,
                     msg_len, n, gk1, gr1, keys, key_len, sigs, sig_len);
  return hipGetLastError();
}

hipError_t launch_ecdsa_gtables(uint32_t* k1, uint32_t* r1, hipStream_t s) {
  const dim3 g((kGTables * kGEntries + 63) / 64);
  hipLaunchKernelGGL(ecdsa_gtable_kernel<Curve<2>>, g, dim3(64), 0, s, k1);
  hipLaunchKernelGGL(ecdsa_gtable_kernel<Curve<3>>, g, dim3(64), 0, s, r1);
  return hipGetLastError();
}

// partition + verify + verdict; work: counts[5] + cursors[5] (zeroed here) and perm[n].
// ws (ws_slots * ecdsa_ws_slot_bytes() of device memory) selects the split
// path (prep -> batch inversion -> ladder per chunk of ws_slots); without it,
// a missing workspace is an error (the old single-kernel path is retired).
hipError_t launch_ecdsa_verify(const uint8_t* scheme, const uint8_t* keys, const uint8_t* key_len,
                               const uint8_t* sigs, const uint8_t* sig_len, const uint8_t* msgs,
                               const uint64_t* msg_off, uint32_t msg_len, uint64_t n, const uint32_t* gk1,
                               const uint32_t* gr1, const uint8_t* pre_status, uint8_t* status,
                               unsigned long long* verdict, unsigned int* counters6, unsigned int* perm,
                               uint32_t* ws, uint64_t ws_slots, uint32_t flags, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (!ws || ws_slots < 64) return hipErrorInvalidValue;  // the split path is the only verify path
  const dim3 grid((uint32_t)((n + 255) / 256));
  hipError_t e = hipMemsetAsync(counters6, 0, 2 * kPartClasses * sizeof(unsigned int), s);
  if (e != hipSuccess) return e;
  const dim3 pgrid((uint32_t)((n + kPartTile - 1) / kPartTile));
  hipLaunchKernelGGL(ecdsa_count_kernel, pgrid, dim3(256), 0, s, scheme, key_len, n, counters6);
  hipLaunchKernelGGL(ecdsa_scatter_kernel, pgrid, dim3(256), 0, s, scheme, key_len, n, counters6,
                     counters6 + kPartClasses, perm);
  for (uint64_t base = 0; base < n; base += ws_slots) {
    const uint64_t m = n - base < ws_slots ? n - base : ws_slots;
    const dim3 g((uint32_t)((m + 255) / 256));
    hipLaunchKernelGGL(ecdsa_prep_kernel, g, dim3(256), 0, s, perm, scheme, keys, key_len, sigs, sig_len, msgs,
                       msg_off, msg_len, base, m, pre_status, status, ws, (flags & 1u) ? 0u : 1u);
    const uint64_t nt = (m + kEcInvBatch - 1) / kEcInvBatch;
    hipLaunchKernelGGL(ecdsa_inv_kernel, dim3((uint32_t)((nt + 255) / 256)), dim3(256), 0, s, base, m, counters6,
                       ws);
    hipLaunchKernelGGL(ecdsa_ladder_kernel<2>, g, dim3(256), 0, s, perm, scheme, base, m, gk1, ws, status);
    hipLaunchKernelGGL(ecdsa_ladder_kernel<3>, g, dim3(256), 0, s, perm, scheme, base, m, gr1, ws, status);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (verdict) hipLaunchKernelGGL(verdict_kernel, grid, dim3(256), 0, s, status, n, verdict);
  return hipGetLastError();
}

}  // namespace cordahip
