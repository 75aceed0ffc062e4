// Edwards25519 group operations for gfx950 lanes (extended coordinates).
//
// Formulas: add-2008-hwcd-3 / dbl-2008-hwcd with a = -1 (Hisil-Wong-Carter-
// Dawson). Both are complete on edwards25519 (d non-square), so small-order
// and mixed-order keys — which i2p 0.2.0 accepts without a torsion check —
// go through the same straight-line code as honest keys (no exceptional
// branches, no lane divergence).
#pragma once
#include "fe25519.hpp"

namespace cordahip {

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

// r = 2p. WANT_T: compute T (needed when an addition follows).
template <bool WANT_T>
CDEV void ge_dbl(ge_p3& r, const ge_p3& p) {
  fe a, b, c, e, f, g, h, t;
  fe_sq(a, p.X);
  fe_sq(b, p.Y);
  fe_sq(c, p.Z);
  fe_add(t, p.X, p.Y);
  fe_sq(t, t);
  fe_add(h, a, b);         // H' = A + B          (= -H), 2x
  fe_sub(e, h, t);         // E' = A + B - (X+Y)^2 (= -E), tight
  fe_sub_loose(g, a, b);   // G' = A - B          (= -G), <= 3x
  fe_add(f, c, c);
  fe_add(f, f, g);         // F' = 2Z^2 + G'      (= -F), <= 5x: f-operand only
  fe_mul(r.X, f, e);
  fe_mul(r.Y, g, h);
  fe_mul(r.Z, f, g);
  if (WANT_T) fe_mul(r.T, e, h);
}

// r = p + q (q cached). WANT_T as above.
template <bool WANT_T>
CDEV void ge_add(ge_p3& r, const ge_p3& p, const ge_cached& q) {
  fe a, b, c, d, e, f, g, h, t;
  fe_sub_loose(t, p.Y, p.X);  // <= 3x
  fe_mul(a, t, q.YmX);
  fe_add(t, p.Y, p.X);
  fe_mul(b, t, q.YpX);
  fe_mul(c, p.T, q.T2d);
  fe_mul(d, p.Z, q.Z);
  fe_add(d, d, d);            // 2x
  fe_sub_loose(e, b, a);      // <= 3x
  fe_sub_loose(f, d, c);      // <= 4x: f-operand only
  fe_add(g, d, c);            // <= 3x
  fe_add(h, b, a);            // 2x
  fe_mul(r.X, f, e);
  fe_mul(r.Y, g, h);
  fe_mul(r.Z, f, g);
  if (WANT_T) fe_mul(r.T, e, h);
}

// r = p + q (q affine niels: saves the Z multiplication)
template <bool WANT_T>
CDEV void ge_madd(ge_p3& r, const ge_p3& p, const ge_niels& q) {
  fe a, b, c, d, e, f, g, h, t;
  fe_sub_loose(t, p.Y, p.X);
  fe_mul(a, t, q.ymx);
  fe_add(t, p.Y, p.X);
  fe_mul(b, t, q.ypx);
  fe_mul(c, p.T, q.xy2d);
  fe_add(d, p.Z, p.Z);
  fe_sub_loose(e, b, a);
  fe_sub_loose(f, d, c);
  fe_add(g, d, c);
  fe_add(h, b, a);
  fe_mul(r.X, f, e);
  fe_mul(r.Y, g, h);
  fe_mul(r.Z, f, g);
  if (WANT_T) fe_mul(r.T, e, h);
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

}  // namespace cordahip
