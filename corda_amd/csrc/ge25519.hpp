// Edwards25519 group operations for gfx950 lanes (extended coordinates).
//
// Formulas: add-2008-hwcd-3 / dbl-2008-hwcd with a = -1 (Hisil-Wong-Carter-
// Dawson). Both are complete on edwards25519 (d non-square), so small-order
// and mixed-order keys — which i2p 0.2.0 accepts without a torsion check —
// go through the same straight-line code as honest keys (no exceptional
// branches, no lane divergence).
#pragma once
#include "fe25519.hpp"
#if FE_USE_ASM2
#include "fe25519_asm.hpp"
#endif

namespace cordahip {

// The group formulas compute their products in independent pairs. With
// FE_USE_ASM2 (per translation unit) a pair is ONE hand-scheduled asm block
// (fe25519_asm.hpp: carry in the MAC addend, the two chains interleaved);
// otherwise two fe_mul / fe_sq calls. Bit-identical either way.
#ifndef FE_USE_ASM2
#define FE_USE_ASM2 0
#endif
CDEV void fe_mul_pair(fe& r0, const fe& f0, const fe& g0, fe& r1, const fe& f1, const fe& g1) {
#if FE_USE_ASM2
  fe_mul2(r0, f0, g0, r1, f1, g1);
#else
  fe o0, o1;
  fe_mul(o0, f0, g0);
  fe_mul(o1, f1, g1);
  r0 = o0;
  r1 = o1;
#endif
}
CDEV void fe_sq_pair(fe& r0, const fe& f0, fe& r1, const fe& f1) {
#if FE_USE_ASM2
  fe_sq2(r0, f0, r1, f1);
#else
  fe o0, o1;
  fe_sq(o0, f0);
  fe_sq(o1, f1);
  r0 = o0;
  r1 = o1;
#endif
}

// Three and four independent products (the additions' first stage and every
// formula's output stage): with FE_USE_ASM2 and FE_QUAD (per translation unit;
// the ladder's) one asm block with three / four interleaved chains
// (fe25519_asm.hpp: two chains per wave leave the dependent v_mad_u64_u32
// latency partly exposed at two waves per SIMD; +1% on C2,
// profiles/r02_c2_quad_ab.json). The prep keeps pairs (register pressure).
#ifndef FE_QUAD
#define FE_QUAD 1
#endif

CDEV void fe_mul_triple(fe& r0, const fe& f0, const fe& g0, fe& r1, const fe& f1, const fe& g1, fe& r2,
                        const fe& f2, const fe& g2) {
#if FE_USE_ASM2 && FE_QUAD
  fe_mul3(r0, f0, g0, r1, f1, g1, r2, f2, g2);
#else
  fe o2;
  fe_mul(o2, f2, g2);
  fe_mul_pair(r0, f0, g0, r1, f1, g1);
  r2 = o2;
#endif
}
CDEV void fe_mul_quad(fe& r0, const fe& f0, const fe& g0, fe& r1, const fe& f1, const fe& g1, fe& r2,
                      const fe& f2, const fe& g2, fe& r3, const fe& f3, const fe& g3) {
#if FE_USE_ASM2 && FE_QUAD
  fe_mul4(r0, f0, g0, r1, f1, g1, r2, f2, g2, r3, f3, g3);
#else
  fe o2, o3;
  fe_mul_pair(o2, f2, g2, o3, f3, g3);
  fe_mul_pair(r0, f0, g0, r1, f1, g1);
  r2 = o2;
  r3 = o3;
#endif
}
// The formulas' output stage X = F E, Y = H G, Z = F G (, T = H E): F and H
// as f-operands, E and G as g-operands (F' may reach 5x, so it is never
// 19-scaled), as ONE outer-product block whose scaled operand copies are
// shared (fe25519_asm.hpp fe_mul3x / fe_mul4x; Y = H G and T = H E are
// bit-identical to G H and E H).
template <bool WANT_T, class P>
CDEV void ge_out_stage(P& r, const fe& f, const fe& e, const fe& g, const fe& h) {
#if FE_USE_ASM2 && FE_QUAD
  if (WANT_T) fe_mul4x(r.X, r.Y, r.Z, r.T, f, h, e, g);
  else fe_mul3x(r.X, r.Y, r.Z, f, h, e, g);
#else
  if (WANT_T) fe_mul_quad(r.X, f, e, r.Y, g, h, r.Z, f, g, r.T, e, h);
  else fe_mul_triple(r.X, f, e, r.Y, g, h, r.Z, f, g);
#endif
}

struct ge_p3 {      // x = X/Z, y = Y/Z, x*y = T/Z
  fe X, Y, Z, T;
};
struct ge_cached {  // (Y+X, Y-X, Z, 2d*T) of a projective point
  fe YpX, YmX, Z, T2d;
};
struct ge_niels {   // affine (y+x, y-x, 2d*x*y), Z = 1
  fe ypx, ymx, xy2d;
};

CDEV void ge_identity(ge_p3& r) {
  fe_set(r.X, 0);
  fe_set(r.Y, 1);
  fe_set(r.Z, 1);
  fe_set(r.T, 0);
}

CDEV void ge_to_cached(ge_cached& c, const ge_p3& p) {
  fe d2;
  fe_const_d2(d2);
  fe_add(c.YpX, p.Y, p.X);
  fe_sub(c.YmX, p.Y, p.X);
  c.Z = p.Z;
  fe_mul(c.T2d, p.T, d2);
}

// r = 2p. WANT_T: compute T (needed when an addition follows). The four
// squarings stay two pairs: as one 4-chain block they need more registers than
// the ladder has while its table gathers are in flight (and measured no faster
// where they fit).
template <bool WANT_T>
CDEV void ge_dbl(ge_p3& r, const ge_p3& p) {
  fe a, b, c, e, f, g, h, t;
  fe_add(t, p.X, p.Y);
  fe_sq_pair(a, p.X, b, p.Y);
  fe_sq_pair(c, p.Z, t, t);
  fe_add(h, a, b);         // H' = A + B          (= -H), 2x
  fe_sub(e, h, t);         // E' = A + B - (X+Y)^2 (= -E), tight
  fe_sub_loose(g, a, b);   // G' = A - B          (= -G), <= 3x
  fe_add(f, c, c);
  fe_add(f, f, g);         // F' = 2Z^2 + G'      (= -F), <= 5x: f-operand only
  ge_out_stage<WANT_T>(r, f, e, g, h);
}

// r = p + q (q cached). WANT_T as above.
template <bool WANT_T>
CDEV void ge_add(ge_p3& r, const ge_p3& p, const ge_cached& q) {
  fe a, b, c, d, e, f, g, h, t, u;
  fe_sub_loose(t, p.Y, p.X);  // <= 3x
  fe_add(u, p.Y, p.X);
  fe_mul_quad(a, t, q.YmX, b, u, q.YpX, c, p.T, q.T2d, d, p.Z, q.Z);
  fe_add(d, d, d);            // 2x
  fe_sub_loose(e, b, a);      // <= 3x
  fe_sub_loose(f, d, c);      // <= 4x: f-operand only
  fe_add(g, d, c);            // <= 3x
  fe_add(h, b, a);            // 2x
  ge_out_stage<WANT_T>(r, f, e, g, h);
}

// r = p + q (q affine niels: saves the Z multiplication)
template <bool WANT_T>
CDEV void ge_madd(ge_p3& r, const ge_p3& p, const ge_niels& q) {
  fe a, b, c, d, e, f, g, h, t, u;
  fe_sub_loose(t, p.Y, p.X);
  fe_add(u, p.Y, p.X);
  fe_mul_triple(a, t, q.ymx, b, u, q.ypx, c, p.T, q.xy2d);
  fe_add(d, p.Z, p.Z);
  fe_sub_loose(e, b, a);
  fe_sub_loose(f, d, c);
  fe_add(g, d, c);
  fe_add(h, b, a);
  ge_out_stage<WANT_T>(r, f, e, g, h);
}

// Canonical encoding (i2p GroupElement.toByteArray / ref10 ge_tobytes):
// y = Y/Z reduced mod p, bit 255 = parity of x = X/Z.
CDEV void ge_tobytes(uint32_t w[8], const ge_p3& p) {
  fe zi, x, y;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  fe_tobytes(w, y);
  w[7] ^= fe_isnegative(x) << 31;
}

// i2p 0.2.0 GroupElement(Curve, byte[] s) (ref10 ge_frombytes without the
// negation): y = s with bit 255 cleared, NOT range checked; x from
// u v^3 (u v^7)^((p-5)/8); fix with sqrt(-1) when v x^2 == -u; fail when
// neither; negate x if its parity differs from bit 255 (x = 0 with the bit
// set stays 0). Returns false on "not a valid GroupElement".
CDEV bool ge_frombytes_i2p(ge_p3& r, const uint32_t w[8]) {
  fe y, yy, u, v, v3, x, vxx, chk, dd, one;
  fe_set(one, 1);
  fe_const_d(dd);
  fe_frombytes(y, w);
  fe_sq(yy, y);
  fe_sub(u, yy, one);
  fe_mul(v, yy, dd);
  fe_add(v, v, one);
  fe_sq(v3, v);
  fe_mul(v3, v3, v);
  fe_sq(x, v3);
  fe_mul(x, x, v);
  fe_mul(x, x, u);
  fe_pow22523(x, x);
  fe_mul(x, x, v3);
  fe_mul(x, x, u);
  fe_sq(vxx, x);
  fe_mul(vxx, vxx, v);
  fe_sub(chk, vxx, u);
  bool ok = true;
  if (!fe_iszero(chk)) {
    fe_add(chk, vxx, u);
    if (!fe_iszero(chk)) {
      ok = false;
    } else {
      fe i;
      fe_const_sqrtm1(i);
      fe_mul(x, x, i);
    }
  }
  if (fe_isnegative(x) != (w[7] >> 31)) fe_neg(x, x);
  r.X = x;
  r.Y = y;
  fe_set(r.Z, 1);
  fe_mul(r.T, x, y);
  return ok;
}

// z^(2^252 - 3) for two independent inputs (the decompression exponent of
// ge_frombytes_i2p), every step a pair: the two square chains run interleaved
// instead of one serial chain per lane (fe25519.hpp fe_pow22523).
CDEV void fe_sqn_pair(fe& r0, const fe& a0, fe& r1, const fe& a1, int n) {
  fe_sq_pair(r0, a0, r1, a1);
#pragma unroll 1
  for (int i = 1; i < n; i++) fe_sq_pair(r0, r0, r1, r1);
}
CDEV void fe_pow22523_pair(fe& r0, const fe& z0, fe& r1, const fe& z1) {
  fe z2_0, z2_1, z9_0, z9_1, z11_0, z11_1, t0, t1, a0, a1, b0, b1;
  fe_sq_pair(z2_0, z0, z2_1, z1);
  fe_sqn_pair(t0, z2_0, t1, z2_1, 2);
  fe_mul_pair(z9_0, t0, z0, z9_1, t1, z1);
  fe_mul_pair(z11_0, z9_0, z2_0, z11_1, z9_1, z2_1);
  fe_sq_pair(t0, z11_0, t1, z11_1);
  fe_mul_pair(a0, t0, z9_0, a1, t1, z9_1);     // 2^5 - 1
  fe_sqn_pair(t0, a0, t1, a1, 5);
  fe_mul_pair(a0, t0, a0, a1, t1, a1);         // 2^10 - 1
  fe_sqn_pair(t0, a0, t1, a1, 10);
  fe_mul_pair(b0, t0, a0, b1, t1, a1);         // 2^20 - 1
  fe_sqn_pair(t0, b0, t1, b1, 20);
  fe_mul_pair(t0, t0, b0, t1, t1, b1);         // 2^40 - 1
  fe_sqn_pair(t0, t0, t1, t1, 10);
  fe_mul_pair(a0, t0, a0, a1, t1, a1);         // 2^50 - 1
  fe_sqn_pair(t0, a0, t1, a1, 50);
  fe_mul_pair(b0, t0, a0, b1, t1, a1);         // 2^100 - 1
  fe_sqn_pair(t0, b0, t1, b1, 100);
  fe_mul_pair(t0, t0, b0, t1, t1, b1);         // 2^200 - 1
  fe_sqn_pair(t0, t0, t1, t1, 50);
  fe_mul_pair(t0, t0, a0, t1, t1, a1);         // 2^250 - 1
  fe_sqn_pair(t0, t0, t1, t1, 2);
  fe_mul_pair(r0, t0, z0, r1, t1, z1);         // 2^252 - 3
}

// ge_frombytes_i2p for two encodings at once (the key A and the signature's R
// in the Ed25519 prep): the same steps and checks, every field product paired.
CDEV void ge_frombytes_i2p_pair(ge_p3& r0, bool& ok0, const uint32_t w0[8], ge_p3& r1, bool& ok1,
                                const uint32_t w1[8]) {
  fe y0, y1, yy0, yy1, u0, u1, v0, v1, v3_0, v3_1, x0, x1, vxx0, vxx1, chk, dd, one;
  fe_set(one, 1);
  fe_const_d(dd);
  fe_frombytes(y0, w0);
  fe_frombytes(y1, w1);
  fe_sq_pair(yy0, y0, yy1, y1);
  fe_sub(u0, yy0, one);
  fe_sub(u1, yy1, one);
  fe_mul_pair(v0, yy0, dd, v1, yy1, dd);
  fe_add(v0, v0, one);
  fe_add(v1, v1, one);
  fe_sq_pair(v3_0, v0, v3_1, v1);
  fe_mul_pair(v3_0, v3_0, v0, v3_1, v3_1, v1);
  fe_sq_pair(x0, v3_0, x1, v3_1);
  fe_mul_pair(x0, x0, v0, x1, x1, v1);
  fe_mul_pair(x0, x0, u0, x1, x1, u1);
  fe_pow22523_pair(x0, x0, x1, x1);
  fe_mul_pair(x0, x0, v3_0, x1, x1, v3_1);
  fe_mul_pair(x0, x0, u0, x1, x1, u1);
  fe_sq_pair(vxx0, x0, vxx1, x1);
  fe_mul_pair(vxx0, vxx0, v0, vxx1, vxx1, v1);
  fe i;
  fe_const_sqrtm1(i);
  // per encoding: v x^2 == u ok; == -u: x *= sqrt(-1); else not a point
  fe_sub(chk, vxx0, u0);
  const bool e0 = fe_iszero(chk);
  fe_add(chk, vxx0, u0);
  const bool n0 = fe_iszero(chk);
  fe_sub(chk, vxx1, u1);
  const bool e1 = fe_iszero(chk);
  fe_add(chk, vxx1, u1);
  const bool n1 = fe_iszero(chk);
  ok0 = e0 || n0;
  ok1 = e1 || n1;
  fe xi0, xi1;
  fe_mul_pair(xi0, x0, i, xi1, x1, i);
  fe_cmov(x0, xi0, !e0 && n0);
  fe_cmov(x1, xi1, !e1 && n1);
  if (fe_isnegative(x0) != (w0[7] >> 31)) fe_neg(x0, x0);
  if (fe_isnegative(x1) != (w1[7] >> 31)) fe_neg(x1, x1);
  r0.X = x0;
  r0.Y = y0;
  fe_set(r0.Z, 1);
  r1.X = x1;
  r1.Y = y1;
  fe_set(r1.Z, 1);
  fe_mul_pair(r0.T, x0, y0, r1.T, x1, y1);
}

}  // namespace cordahip
