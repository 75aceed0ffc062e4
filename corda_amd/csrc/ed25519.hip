// Ed25519 (EDDSA_ED25519_SHA512) batch verification for gfx950 — kernel K1,
// first half (prep) plus the fixed-base table and the corpus signer.
//
// Replaces, per lane, the reference's
//   Crypto.isValid(EDDSA_ED25519_SHA512, key, sig, clear)   Crypto.kt:534-541
//   -> i2p eddsa 0.2.0 EdDSAEngine.engineVerify (3P, semantics SURVEY App. A.1)
// with bit-exact verdicts (status byte per lane + 64-bit verdict word per
// wave via ballot). Oracle: oracle/i2p_ed25519.py, oracle/c/ed25519.c.
//
// Two kernels per batch (layout shared in ed25519_ws.hpp):
//   ed25519_prep_half_kernel (here): decode A exactly as i2p (y not range
//     checked), decode R strictly, hash the canonical re-encoding of A,
//     h = SHA-512(R||Abyte||M) mod L, S_eff from an exact emulation of
//     slide()'s carry drop, the half-size scalars (c0, c1) and e = c1 S_eff,
//     and the per-lane tables [0..8](-A), [0..8](-R) -> HBM workspace record;
//   ed25519_ladder_half_kernel (ed25519_ladder.hip): [e]B + [c0](+-A) + [c1](-R) == O.
// field products in hand-scheduled pairs (ge25519.hpp fe_mul_pair, fe25519_asm.hpp)
#ifndef FE_QUAD
#define FE_QUAD 0  // prep keeps pairs (register pressure)
#endif
#ifndef FE_USE_ASM2
#define FE_USE_ASM2 1
#endif
#include <hip/hip_runtime.h>

#include <functional>
#include <stdint.h>
#include <stdlib.h>

#include "ed25519_ws.hpp"
#include "sha2_device.hpp"
#include "status.hpp"

namespace cordahip {

// ---------------------------------------------------------------------------
// B table (layout: ed25519_ws.hpp), built once per context by a kernel.
CDEV void ge_base(ge_p3& b) {
  const uint32_t bx[10] = {0x325d51a, 0x18b5823, 0xf6592a, 0x104a92d, 0x1a4b31d,
                           0x1d6dc5c, 0x27118fe, 0x7fd814, 0x13cd6e5, 0x85a4db};
  const uint32_t by[10] = {0x2666658, 0x1999999, 0xcccccc, 0x1333333, 0x1999999,
                           0x666666, 0x3333333, 0xcccccc, 0x2666666, 0x1999999};
  const uint32_t bt[10] = {0x1b7dda3, 0x1a2ace9, 0x25eadbb, 0x3ba8a, 0x83c27e,
                           0xabe37d, 0x1274732, 0xccacdd, 0xfd78b7, 0x19e1d7c};
#pragma unroll
  for (int i = 0; i < 10; i++) {
    b.X.v[i] = bx[i];
    b.Y.v[i] = by[i];
    b.T.v[i] = bt[i];
  }
  fe_set(b.Z, 1);
}

// tab: entries [0, kBTableEntries) = [k]B, then [k]B' with B' = [2^128]B
__global__ void __launch_bounds__(64) ed25519_btable_kernel(uint32_t* __restrict__ tab) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= 2 * kBTableEntries) return;
  const int k = g % kBTableEntries;
  ge_p3 B, P;
  ge_base(B);
  if (g >= kBTableEntries)
    for (int t = 0; t < kBDigits * kBBits; t++) ge_dbl<true>(B, B);
  ge_cached bc;
  ge_to_cached(bc, B);
  ge_identity(P);
  for (int bit = kBBits - 1; bit >= 0; bit--) {
    ge_dbl<true>(P, P);
    if ((k >> bit) & 1) ge_add<true>(P, P, bc);
  }
  fe zi, x, y, t, d2;
  fe_invert(zi, P.Z);
  fe_mul(x, P.X, zi);
  fe_mul(y, P.Y, zi);
  fe_const_d2(d2);
  ge_niels n;
  fe_add(n.ypx, y, x);
  fe_carry(n.ypx);
  fe_sub(n.ymx, y, x);
  fe_mul(t, x, y);
  fe_mul(n.xy2d, t, d2);
  uint32_t* o = tab + g * kBEntryWords;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    o[i] = n.ypx.v[i];
    o[10 + i] = n.ymx.v[i];
    o[20 + i] = n.xy2d.v[i];
  }
  o[30] = 0;
  o[31] = 0;
}


// ---------------------------------------------------------------------------
// SHA-512 over  seg0(32 B, registers) || seg1(32 B, registers, optional) || msg
// (global, msg_len bytes). Fast path: everything fits one block with msg_len
// a multiple of 8 bytes' worth of whole words read as registers.
CDEV uint32_t byte_of(const uint32_t w[8], int idx) { return (word_sel(w, idx >> 2) >> (8 * (idx & 3))) & 0xffu; }

CDEV void sha512_segments(uint32_t out_le[16], const uint32_t s0[8], const uint32_t s1[8], bool has_s1,
                          const uint8_t* __restrict__ msg, uint32_t msg_len) {
  uint64_t h[8];
  sha512_init(h);
  const uint32_t pre = has_s1 ? 64u : 32u;
  const uint64_t total = (uint64_t)pre + msg_len;
  uint64_t w[16];
  if (has_s1 && msg_len == 32) {
    // hot shape: R || A || txId = 96 bytes, one block
    const uint4* m4 = reinterpret_cast<const uint4*>(msg);
    const uint4 ma = m4[0], mb = m4[1];
    const uint32_t m[8] = {ma.x, ma.y, ma.z, ma.w, mb.x, mb.y, mb.z, mb.w};
#pragma unroll
    for (int q = 0; q < 4; q++) {
      w[q] = ((uint64_t)bswap32(s0[2 * q]) << 32) | bswap32(s0[2 * q + 1]);
      w[4 + q] = ((uint64_t)bswap32(s1[2 * q]) << 32) | bswap32(s1[2 * q + 1]);
      w[8 + q] = ((uint64_t)bswap32(m[2 * q]) << 32) | bswap32(m[2 * q + 1]);
    }
    w[12] = 0x8000000000000000ULL;
    w[13] = 0;
    w[14] = 0;
    w[15] = total * 8;
    sha512_block(h, w);
  } else {
#ifndef ED_NO_GENERIC_SHA
    const uint64_t nblocks = (total + 17 + 127) / 128;
    for (uint64_t b = 0; b < nblocks; b++) {
      for (int q = 0; q < 16; q++) {
        uint64_t word = 0;
        for (int k = 0; k < 8; k++) {
          const uint64_t pos = b * 128 + (uint64_t)q * 8 + k;
          uint32_t byte;
          if (pos < 32) byte = byte_of(s0, (int)pos);
          else if (pos < pre) byte = byte_of(s1, (int)(pos - 32));
          else if (pos < total) byte = msg[pos - pre];
          else if (pos == total) byte = 0x80;
          else if (b == nblocks - 1 && q == 15) byte = (uint32_t)(((total * 8) >> (8 * (7 - k))) & 0xff);
          else byte = 0;
          word = (word << 8) | byte;
        }
        w[q] = word;
      }
      sha512_block(h, w);
    }
#endif
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    out_le[2 * i] = bswap32((uint32_t)(h[i] >> 32));
    out_le[2 * i + 1] = bswap32((uint32_t)h[i]);
  }
}

// ---------------------------------------------------------------------------
// Half-size scalars. With R decoded strictly,
//   encode([S]B - [h]A) == R_bytes  <=>  P := [S]B - [h]A - R == O.
// For any (c0, c1) with c0 == c1*h (mod 8L) and c1 odd, c1 != 0 (mod L):
//   [c1]P == [c1*S mod L]B - [c0]A - [c1]R,   and   [c1]P == O <=> P == O
// (A, R may carry torsion: every point's order divides 8L, so the mod-8L
// congruence makes [c0]A == [c1 h]A exact; c1 odd kills no 2-power torsion;
// c1 != 0 mod L keeps the prime-order part). Extended Euclid on (8L, h),
// stopped below sqrt(8L), gives |c0|, |c1| ~ 2^128: the ladder needs ~128
// doublings instead of ~252 (idea: T. Pornin, ePrint 2020/454). The
// equivalence is checked on the golden catalogue in tools/proto/half_scalar.py.
// a >= b as the absence of a borrow out of a - b (branch-free: a
// short-circuit word compare becomes divergent control flow on the GPU)
CDEV bool mp8_ge(const uint32_t a[8], const uint32_t b[8]) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) br = (uint32_t)(((uint64_t)a[i] - b[i] - br) >> 63);
  return br == 0;
}
CDEV void mp8_add(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c += (uint64_t)a[i] + b[i];
    r[i] = (uint32_t)c;
    c >>= 32;
  }
}
CDEV void mp8_neg(uint32_t a[8]) {
  uint64_t c = 1;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c += (uint64_t)(~a[i]);
    a[i] = (uint32_t)c;
    c >>= 32;
  }
}
CDEV void mp8_copy(uint32_t d[8], const uint32_t s[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = s[i];
}
// |a| of a two's-complement value and its sign
CDEV int mp8_absbits(const uint32_t a[8]) {
  uint32_t t[8];
  mp8_copy(t, a);
  if (a[7] >> 31) mp8_neg(t);
  return mp8_bitlen(t);
}

// value of an 8-word integer as a double (relative error < 2^-49)
CDEV double mp8_f64(const uint32_t a[8]) {
  double d = (double)a[7];
#pragma unroll
  for (int i = 6; i >= 0; i--) d = fma(d, 4294967296.0, (double)a[i]);
  return d;
}
// a -= q * b  (mod 2^256), q < 2^32
CDEV void mp8_submul(uint32_t a[8], const uint32_t b[8], uint32_t q) {
  uint64_t pc = 0;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t p = (uint64_t)q * b[i] + pc;
    pc = p >> 32;
    const uint64_t d = (uint64_t)a[i] - (uint32_t)p - br;
    a[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
}
// o = b << k  (mod 2^256), 0 <= k < 256
CDEV void mp8_shl_dyn(uint32_t o[8], const uint32_t b[8], int k) {
  const int ws = k >> 5, bs = k & 31;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t lo = (i - ws >= 0) ? word_sel(b, i - ws) : 0u;
    const uint32_t lo2 = (i - ws - 1 >= 0) ? word_sel(b, i - ws - 1) : 0u;
    o[i] = bs ? ((lo << bs) | (lo2 >> (32 - bs))) : lo;
  }
}

// rp <- rp mod rc,  tp <- tp - (rp div rc) * tc   (mod 2^256), rc > 0.
// The quotient comes from a double-precision estimate scaled down by
// (1 - 2^-40): it never exceeds the true quotient (relative error of the
// estimate < 2^-48), so rp stays non-negative, and the loop repeats until
// rp < rc. Euclid's partial quotients are small (~1.7 bits per step), so one
// pass is the rule; a quotient >= 2^32 is taken 31 bits at a time.
CDEV void euclid_divstep(uint32_t rp[8], const uint32_t rc[8], uint32_t tp[8], const uint32_t tc[8]) {
  const double inv = 1.0 / mp8_f64(rc);
  while (mp8_ge(rp, rc)) {
    const double qd = mp8_f64(rp) * inv * (1.0 - 0x1p-40);
    if (qd < 4294967296.0) {
      uint32_t q = (uint32_t)qd;
      q = q ? q : 1u;
      mp8_submul(rp, rc, q);
      mp8_submul(tp, tc, q);
    } else {
      const int e = (int)((__double_as_longlong(qd) >> 52) & 0x7ff) - 1023;  // qd in [2^e, 2^(e+1))
      const int k = e - 31;
      const uint32_t q = (uint32_t)(qd * __longlong_as_double((long long)(1023 - k) << 52));  // qd / 2^k
      uint32_t bs[8], ts[8];
      mp8_shl_dyn(bs, rc, k);
      mp8_shl_dyn(ts, tc, k);
      mp8_submul(rp, bs, q);
      mp8_submul(tp, ts, q);
    }
  }
}

// floor(a / 2^s) as a double, exact for a < 2^(s+53)
CDEV double mp8_top(const uint32_t a[8], int s) {
  const int w = s >> 5, b = s & 31;
  const uint64_t lo = ((uint64_t)word_sel(a, w + 1) << 32) | word_sel(a, w);
  const uint64_t hi = word_sel(a, w + 2);
  return (double)((lo >> b) | (b ? hi << (64 - b) : 0ull));
}
// o = a*x + b*y (mod 2^256) for |a|, |b| < 2^31 of opposite signs (or one of
// them zero), as |a|x - |b|y, negated when the positive factor is b
CDEV void mp8_lincomb(uint32_t o[8], const uint32_t x[8], int a, const uint32_t y[8], int b) {
  const uint32_t ua = (uint32_t)(a < 0 ? -a : a), ub = (uint32_t)(b < 0 ? -b : b);
  uint64_t pc = 0, qc = 0;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t p = (uint64_t)ua * x[i] + pc;
    pc = p >> 32;
    const uint64_t q = (uint64_t)ub * y[i] + qc;
    qc = q >> 32;
    const uint64_t d = (uint64_t)(uint32_t)p - (uint32_t)q - br;
    o[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  if (b > 0 || (b == 0 && a < 0)) mp8_neg(o);
}

// (c0, c1): c0 == c1*h (mod 8L), c1 odd and positive; returns |c0| and its sign
CDEV void half_scalars(uint32_t c0abs[8], bool& c0neg, uint32_t c1[8], const uint32_t h[8]) {
  const uint32_t kM[8] = {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0u, 0u, 0u, 0x80000000u};  // 8L
  const uint32_t kS[8] = {0x754abea0u, 0x597d89b3u, 0xf9de6484u, 0xb504f333u, 0u, 0u, 0u, 0u};        // isqrt(8L)+1
  uint32_t rp[8], rc[8], tp[8], tc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    rp[i] = kM[i];
    rc[i] = h[i];
    tp[i] = 0;
    tc[i] = i == 0;
  }
  // Euclid on (8L, h) until the first remainder below sqrt(8L), run as Lehmer
  // rounds (Knuth TAOCP 4.5.2, Algorithm L): Euclid on the 52-bit leading
  // parts of rp, rc (exact in doubles) while both bracketing quotients agree,
  // so every quotient is Euclid's own, then the round's 2x2 cofactor matrix
  // is applied to the 256-bit remainders and cofactors once. A step is taken
  // only while the remainder it produces provably stays >= sqrt(8L) (its
  // true value is within max(|C|,|D|) units of the leading part), so one
  // exact step below finishes. ~6 rounds of ~12 double-precision steps replace
  // ~73 multiprecision steps; the state handed over is Euclid's exactly
  // (tools/proto/lehmer.py checks that on 5e4 random h).
  for (;;) {
    const int s = max(mp8_bitlen(rp) - 52, 0);
    double uh = mp8_top(rp, s), vh = mp8_top(rc, s);
    const double th = mp8_top(kS, s) + 1.0;
    double A = 1.0, B = 0.0, C = 0.0, D = 1.0;
    int n = 0;
    for (;;) {
      const double d1 = vh + C, d2 = vh + D;
      if (!(d1 > 0.0 && d2 > 0.0)) break;
      const double n1 = uh + A;
      double q = floor(n1 / d1);
      const double r1 = fma(-q, d1, n1);  // exact: |r1| < 2^53
      q = r1 < 0.0 ? q - 1.0 : (r1 >= d1 ? q + 1.0 : q);
      const double r2 = fma(-q, d2, uh + B);
      if (!(r2 >= 0.0 && r2 < d2)) break;  // the other bracket's quotient differs
      const double nC = fma(-q, C, A), nD = fma(-q, D, B), nv = fma(-q, vh, uh);
      const double mc = fmax(fabs(nC), fabs(nD));
      if (nv - mc < th || mc >= 0x1p30) break;
      A = C;
      B = D;
      C = nC;
      D = nD;
      uh = vh;
      vh = nv;
      n++;
    }
    if (n == 0) break;
    const int a = (int)A, b = (int)B, c = (int)C, d = (int)D;
    uint32_t x[8], y[8];
    mp8_lincomb(x, rp, a, rc, b);
    mp8_lincomb(y, rp, c, rc, d);
    mp8_copy(rp, x);
    mp8_copy(rc, y);
    mp8_lincomb(x, tp, a, tc, b);
    mp8_lincomb(y, tp, c, tc, d);
    mp8_copy(tp, x);
    mp8_copy(tc, y);
  }
  // the remaining exact step(s): (rc, tc) <- the first remainder below
  // sqrt(8L) and its cofactor, (rp, tp) <- the previous one
  while (mp8_ge(rc, kS)) {
    euclid_divstep(rp, rc, tp, tc);  // rp <- rp mod rc
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t a = rp[i], b = tp[i];
      rp[i] = rc[i];
      rc[i] = a;
      tp[i] = tc[i];
      tc[i] = b;
    }
  }
  uint32_t a0[8], a1[8];  // chosen (c0, c1), two's complement
  mp8_copy(a0, rc);
  mp8_copy(a1, tc);
  if (!(tc[0] & 1)) {
    // v1 = (rc, tc) has even c1; v3 = next Euclid vector has odd c1, and so do v1 +- v3
    uint32_t r3[8], t3[8];
    mp8_copy(r3, rp);
    mp8_copy(t3, tp);
    euclid_divstep(r3, rc, t3, tc);
    uint32_t p0[8], p1[8], m0[8], m1[8], nr3[8], nt3[8];
    mp8_add(p0, rc, r3);
    mp8_add(p1, tc, t3);
    mp8_copy(nr3, r3);
    mp8_neg(nr3);
    mp8_copy(nt3, t3);
    mp8_neg(nt3);
    mp8_add(m0, rc, nr3);
    mp8_add(m1, tc, nt3);
    int best = max(mp8_absbits(r3), mp8_absbits(t3));
    mp8_copy(a0, r3);
    mp8_copy(a1, t3);
    const int bp = max(mp8_absbits(p0), mp8_absbits(p1));
    if (bp < best) {
      best = bp;
      mp8_copy(a0, p0);
      mp8_copy(a1, p1);
    }
    const int bm = max(mp8_absbits(m0), mp8_absbits(m1));
    if (bm < best) {
      mp8_copy(a0, m0);
      mp8_copy(a1, m1);
    }
  }
  if (a1[7] >> 31) {  // make c1 positive: (c0, c1) -> (-c0, -c1)
    mp8_neg(a0);
    mp8_neg(a1);
  }
  c0neg = (a0[7] >> 31) != 0;
  if (c0neg) mp8_neg(a0);
  mp8_copy(c0abs, a0);
  mp8_copy(c1, a1);
}

// Strict R decode: the reference never decodes R, it compares encode(R')
// with the 32 bytes; those equal only when the bytes are the canonical
// encoding of a curve point: y < p, on the curve, not (x == 0 with bit 255).
// the extra conditions of a strict decode, given R = ge_frombytes_i2p(w) succeeded
CDEV bool ge_strict_ok(const ge_p3& R, const uint32_t w[8]) {
  uint32_t all_ones = (w[7] & 0x7fffffffu) == 0x7fffffffu;
#pragma unroll
  for (int i = 1; i < 7; i++) all_ones &= (w[i] == 0xffffffffu);
  if (all_ones && w[0] >= 0xffffffedu) return false;  // y >= p
  return !((w[7] >> 31) && fe_iszero(R.X));
}

CDEV void sc_muladd(uint32_t out[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]);

// an affine point (Z = 1) as X, Y, T (30 words, 16-B aligned slot of 40)
CDEV void store_point(uint32_t* __restrict__ o, const ge_p3& p) {
  uint4* o4 = reinterpret_cast<uint4*>(o);
  uint32_t w[32];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    w[i] = p.X.v[i];
    w[10 + i] = p.Y.v[i];
    w[20 + i] = p.T.v[i];
  }
  w[30] = w[31] = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) o4[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
CDEV void load_point(ge_p3& p, const uint32_t* __restrict__ o) {
  const uint4* o4 = reinterpret_cast<const uint4*>(o);
  uint32_t w[32];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint4 v = o4[q];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 10; i++) {
    p.X.v[i] = w[i];
    p.Y.v[i] = w[10 + i];
    p.T.v[i] = w[20 + i];
  }
  fe_set(p.Z, 1);
}

// entries [1..8]base of a per-lane table (entry 0, the identity, is shared:
// table_entry in ed25519_ws.hpp)
CDEV void store_table8(uint32_t* __restrict__ rec, const ge_p3& base) {
  ge_cached c, c1;
  ge_to_cached(c1, base);
  store_cached(rec, c1);
  ge_p3 Q;
  ge_dbl<true>(Q, base);
  ge_to_cached(c, Q);
  store_cached(rec + kWhEntryWords, c);
  for (int k = 3; k <= 8; k++) {
    ge_add<true>(Q, Q, c1);
    ge_to_cached(c, Q);
    store_cached(rec + kWhEntryWords * (k - 1), c);
  }
}

// ---------------------------------------------------------------------------
// Prep of the half-size-scalar verification: the ladder (ed25519_ladder.hip)
// decides [e]B + [c0](+-A) + [c1](-R) == O with ~128-bit c0, c1 (half_scalars):
// ~132 doublings instead of 252 and no final inversion (P == O is X == 0, Y == Z).
// Record layout: ed25519_ws.hpp (kWh*).

// Phases, each finished (and its table written to the workspace) before the
// next starts: decode A -> table [k](-A) | strict decode R -> table [k](-R) |
// SHA-512, h, S_eff, lattice reduction, e = c1 S_eff mod L. Lanes whose
// status is already decided run the phases on the identity / zero scalars.
#ifndef ED_PREP_WAVES
#define ED_PREP_WAVES 2
#endif
// Phase 1 of the prep (no message): decode A and R, the pre-engine statuses, the
// tables [k](-A), [k](-R). Returns the lane's status (kStatusPending: verify);
// abyte = EdDSAPublicKey.Abyte, Rw = R's bytes, both for the SHA-512 of phase 2.
CDEV uint8_t prep_keys_phase(const uint8_t* __restrict__ keys, const uint8_t* __restrict__ sigs, uint64_t i,
                             uint32_t msg_len, const uint8_t* __restrict__ pre_status, uint32_t empty_is_error,
                             uint32_t* __restrict__ rec, uint32_t abyte[8], uint32_t Rw[8]) {
  uint8_t st = kStatusPending;
  load8(Rw, reinterpret_cast<const uint32_t*>(sigs + i * 64));
  {
    // A (i2p decode: y not range checked) and R (strict decode: encode(R') ==
    // Rw only if Rw is a canonical point encoding) decompressed together: the
    // two square-root exponentiations run as interleaved chains
    uint32_t wa[8];
    load8(wa, reinterpret_cast<const uint32_t*>(keys + i * 32));
    ge_p3 A, R;
    bool okA, okR;
    ge_frombytes_i2p_pair(A, okA, wa, R, okR, Rw);
    if (!okA) st = kStatusBadKey;  // key decode precedes doVerify (Kryo.kt:389-392)
    else if (pre_status && pre_status[i] != kStatusOk) st = pre_status[i];
    else if (msg_len == 0 && empty_is_error) st = kStatusEmpty;  // doVerify: Crypto.kt:476 (isValid hashes it)
    fe_tobytes(abyte, A.Y);  // EdDSAPublicKey.Abyte = A.toByteArray(): canonical
    abyte[7] |= fe_isnegative(A.X) << 31;
    if (st == kStatusPending && !(okR && ge_strict_ok(R, Rw))) st = kStatusBadSig;  // no canonical point encodes to Rw
    if (st != kStatusPending) {
      ge_identity(A);
      ge_identity(R);
    }
    // -A, -R parked in the last entry of their table (Z = 1: X, Y, T), so the
    // table loop below holds one point at a time
    fe_neg(A.X, A.X);
    fe_neg(A.T, A.T);
    fe_neg(R.X, R.X);
    fe_neg(R.T, R.T);
    store_point(rec + kWhTabA + kWhEntryWords * 7, A);
    store_point(rec + kWhTabR + kWhEntryWords * 7, R);
  }
  PHASE_BARRIER();
  // tables [k](-A), [k](-R): one loop body keeps a single copy of the table
  // code in the I-cache
#pragma unroll 1
  for (int pass = 0; pass < 2; pass++) {
    uint32_t* tab = rec + (pass ? kWhTabR : kWhTabA);
    ge_p3 P;
    load_point(P, tab + kWhEntryWords * 7);  // read before store_table8 overwrites slot 8
    store_table8(tab, P);
    PHASE_BARRIER();
  }
  return st;
}

// Phase 2 (the message): SHA-512(R || A || M), h, S_eff, the lattice reduction,
// e = c1 S_eff mod L -> the record's scalars (zero for decided lanes).
CDEV void prep_msg_phase(const uint8_t* __restrict__ sigs, const uint8_t* __restrict__ msgs, uint32_t msg_len,
                         uint64_t i, uint8_t st, const uint32_t abyte[8], const uint32_t Rw[8],
                         uint32_t* __restrict__ rec) {
  uint32_t ka[8], kr[8], e[8];
  bool c0neg = false;
  if (st == kStatusPending) {
    uint32_t S[8], hd[16], h[8], se[8], zero[8];
    load8(S, reinterpret_cast<const uint32_t*>(sigs + i * 64 + 32));
    sha512_segments(hd, Rw, abyte, true, msgs + i * (uint64_t)msg_len, msg_len);
    sc_reduce512(h, hd);
    sc_effective_S(se, S, slide_drops_carry(S));
    half_scalars(ka, c0neg, kr, h);
#pragma unroll
    for (int q = 0; q < 8; q++) zero[q] = 0;
    sc_muladd(e, kr, se, zero);  // e = c1 S_eff mod L
  } else {
#pragma unroll
    for (int q = 0; q < 8; q++) ka[q] = kr[q] = e[q] = 0;
  }
  store8(rec + kWhKa, ka);
  store8(rec + kWhKr, kr);
  store8(rec + kWhE, e);
  reinterpret_cast<uint4*>(rec + kWhFlags)[0] = make_uint4(c0neg ? 1u : 0u, 0u, 0u, 0u);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ED_PREP_WAVES))) ed25519_prep_half_kernel(
    const uint8_t* __restrict__ keys, const uint8_t* __restrict__ sigs, const uint8_t* __restrict__ msgs,
    uint32_t msg_len, uint64_t base, uint64_t m, const uint8_t* __restrict__ pre_status,
    uint8_t* __restrict__ status, uint32_t* __restrict__ ws, uint32_t empty_is_error) {
  const uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= m) return;
  const uint64_t i = base + li;
  uint32_t* rec = ws + li * kWhLaneWords;
  uint32_t abyte[8], Rw[8];
  const uint8_t st = prep_keys_phase(keys, sigs, i, msg_len, pre_status, empty_is_error, rec, abyte, Rw);
  prep_msg_phase(sigs, msgs, msg_len, i, st, abyte, Rw, rec);
  status[i] = st;
}

// The same prep in two launches, for batches whose messages arrive after their
// keys and signatures (the signed-tx chunks: each message is its transaction's
// id, gathered on the device once the id slice is done): phase 1 needs no
// message and runs while the ids are computed; it leaves the lane's status in
// `status` and Abyte in the record's scalar words, which phase 2 overwrites.
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ED_PREP_WAVES))) ed25519_prep_keys_kernel(
    const uint8_t* __restrict__ keys, const uint8_t* __restrict__ sigs, uint32_t msg_len, uint64_t base, uint64_t m,
    const uint8_t* __restrict__ pre_status, uint8_t* __restrict__ status, uint32_t* __restrict__ ws,
    uint32_t empty_is_error) {
  const uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= m) return;
  const uint64_t i = base + li;
  uint32_t* rec = ws + li * kWhLaneWords;
  uint32_t abyte[8], Rw[8];
  status[i] = prep_keys_phase(keys, sigs, i, msg_len, pre_status, empty_is_error, rec, abyte, Rw);
  store8(rec + kWhKa, abyte);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ED_PREP_WAVES))) ed25519_prep_msg_kernel(const uint8_t* __restrict__ sigs,
                                                               const uint8_t* __restrict__ msgs, uint32_t msg_len,
                                                               uint64_t base, uint64_t m,
                                                               const uint8_t* __restrict__ status,
                                                               uint32_t* __restrict__ ws) {
  const uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= m) return;
  const uint64_t i = base + li;
  uint32_t* rec = ws + li * kWhLaneWords;
  uint32_t abyte[8], Rw[8];
  load8(abyte, rec + kWhKa);
  load8(Rw, reinterpret_cast<const uint32_t*>(sigs + i * 64));
  prep_msg_phase(sigs, msgs, msg_len, i, status[i], abyte, Rw, rec);
}

// ---------------------------------------------------------------------------
// RFC 8032 keygen + sign (Crypto.doSign / deriveKeyPairFromEntropy for
// Ed25519): the GPU corpus generator for bench.py and the C5 stream.
CDEV void fixed_base_mult(ge_p3& P, const uint32_t k[8], const uint32_t* __restrict__ btab) {
  ge_identity(P);
  for (int j = 31; j >= 0; j--) {
    if (j != 31) {
#pragma unroll
      for (int t = 0; t < 7; t++) ge_dbl<false>(P, P);
      ge_dbl<true>(P, P);
    }
    const int d = booth_digit<8>(k, j);
    ge_niels nb;
    load_niels(nb, btab, d < 0 ? -d : d);
    niels_cneg(nb, d < 0);
    ge_madd<true>(P, P, nb);
  }
}

CDEV void sc_muladd(uint32_t out[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t t = (uint64_t)a[i] * b[j] + x[i + j] + carry;
      x[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    x[i + 8] = (uint32_t)carry;
  }
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint64_t t = (uint64_t)x[i] + (i < 8 ? c[i] : 0u) + carry;
    x[i] = (uint32_t)t;
    carry = t >> 32;
  }
  sc_reduce512(out, x);
}

__global__ void __launch_bounds__(256) ed25519_sign_kernel(const uint8_t* __restrict__ seeds,
                                                          const uint8_t* __restrict__ msgs, uint32_t msg_len,
                                                          uint64_t n, const uint32_t* __restrict__ btab,
                                                          uint8_t* __restrict__ pubs, uint8_t* __restrict__ sigs) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t seed[8];
  {
    const uint4* s4 = reinterpret_cast<const uint4*>(seeds + i * 32);
    const uint4 a = s4[0], b = s4[1];
    seed[0] = a.x; seed[1] = a.y; seed[2] = a.z; seed[3] = a.w;
    seed[4] = b.x; seed[5] = b.y; seed[6] = b.z; seed[7] = b.w;
  }
  const uint8_t* msg = msgs + i * (uint64_t)msg_len;
  uint32_t hs[16], dummy[8];
#pragma unroll
  for (int q = 0; q < 8; q++) dummy[q] = 0;
  sha512_segments(hs, seed, dummy, false, msg, 0);
  uint32_t a[8], prefix[8];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    a[q] = hs[q];
    prefix[q] = hs[8 + q];
  }
  a[0] &= ~7u;
  a[7] &= 0x3fffffffu;
  a[7] |= 0x40000000u;
  uint32_t a16[16], ar[8];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    a16[q] = a[q];
    a16[8 + q] = 0;
  }
  sc_reduce512(ar, a16);
  ge_p3 A;
  fixed_base_mult(A, ar, btab);
  uint32_t pub[8];
  ge_tobytes(pub, A);
  uint32_t rh[16], r[8];
  sha512_segments(rh, prefix, dummy, false, msg, msg_len);
  sc_reduce512(r, rh);
  ge_p3 Rp;
  fixed_base_mult(Rp, r, btab);
  uint32_t R[8];
  ge_tobytes(R, Rp);
  uint32_t kh[16], k[8], S[8];
  sha512_segments(kh, R, pub, true, msg, msg_len);
  sc_reduce512(k, kh);
  sc_muladd(S, k, ar, r);
  uint4* p4 = reinterpret_cast<uint4*>(pubs + i * 32);
  p4[0] = make_uint4(pub[0], pub[1], pub[2], pub[3]);
  p4[1] = make_uint4(pub[4], pub[5], pub[6], pub[7]);
  uint4* s4 = reinterpret_cast<uint4*>(sigs + i * 64);
  s4[0] = make_uint4(R[0], R[1], R[2], R[3]);
  s4[1] = make_uint4(R[4], R[5], R[6], R[7]);
  s4[2] = make_uint4(S[0], S[1], S[2], S[3]);
  s4[3] = make_uint4(S[4], S[5], S[6], S[7]);
}

}  // namespace cordahip

// ---------------------------------------------------------------------------
// host-side launchers (called by cordahip.cpp)
namespace cordahip {
hipError_t launch_ed25519_btable(uint32_t* tab, hipStream_t s) {
  hipLaunchKernelGGL(ed25519_btable_kernel, dim3((2 * kBTableEntries + 63) / 64), dim3(64), 0, s, tab);
  return hipGetLastError();
}
size_t ed25519_btable_bytes() { return 2 * (size_t)kBTableEntries * kBEntryWords * sizeof(uint32_t); }

size_t ed25519_ws_lane_bytes() { return kWhLaneWords * sizeof(uint32_t); }

// Split verification, one prep/ladder launch pair per ws_lanes chunk (ws:
// ws_lanes * ed25519_ws_lane_bytes() of device memory, ws_lanes a multiple of
// 64; the caller orders the workspace's users). A missing workspace is an
// error: this is the only verification path.
hipError_t launch_ed25519_verify(const uint8_t* keys, const uint8_t* sigs, const uint8_t* msgs, uint32_t msg_len,
                                 uint64_t n, const uint32_t* btab, const uint8_t* pre_status, uint8_t* status,
                                 unsigned long long* verdict, uint32_t* ws, uint64_t ws_lanes, uint32_t flags,
                                 hipStream_t s, const std::function<hipError_t()>* before_msgs) {
  if (n == 0) return hipSuccess;
  if (!ws || ws_lanes < 64 || ws_lanes % 64) return hipErrorInvalidValue;
  bool msgs_ready = before_msgs == nullptr;
  for (uint64_t base = 0; base < n; base += ws_lanes) {
    const uint64_t m = n - base < ws_lanes ? n - base : ws_lanes;
    const uint32_t blocks = (uint32_t)((m + 255) / 256);
    hipError_t e = hipSuccess;
    if (msgs_ready) {
      hipLaunchKernelGGL(ed25519_prep_half_kernel, dim3(blocks), dim3(256), 0, s, keys, sigs, msgs, msg_len, base, m,
                         pre_status, status, ws, (flags & 1u) ? 0u : 1u);
      e = hipGetLastError();
    } else {
      // keys and R first; the messages' producer (enqueued by before_msgs on the same
      // stream) then runs beside this launch's tail, phase 2 after it
      hipLaunchKernelGGL(ed25519_prep_keys_kernel, dim3(blocks), dim3(256), 0, s, keys, sigs, msg_len, base, m,
                         pre_status, status, ws, (flags & 1u) ? 0u : 1u);
      e = hipGetLastError();
      e = e ? e : (*before_msgs)();
      msgs_ready = true;
      if (e == hipSuccess)
        hipLaunchKernelGGL(ed25519_prep_msg_kernel, dim3(blocks), dim3(256), 0, s, sigs, msgs, msg_len, base, m, status,
                           ws);
      e = e ? e : hipGetLastError();
    }
    if (e == hipSuccess) e = launch_ed25519_ladder(base, m, btab, ws, status, verdict, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_ed25519_sign(const uint8_t* seeds, const uint8_t* msgs, uint32_t msg_len, uint64_t n,
                               const uint32_t* btab, uint8_t* pubs, uint8_t* sigs, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(ed25519_sign_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, seeds, msgs, msg_len, n, btab,
                     pubs, sigs);
  return hipGetLastError();
}
}  // namespace cordahip
