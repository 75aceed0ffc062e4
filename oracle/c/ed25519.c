/* Ed25519 verification with i2p eddsa 0.2.0 semantics — ORACLE (test infra only).
 *
 * Restates, step for step, the algorithm of the third-party engine the
 * reference calls (Crypto.kt:119-132 scheme, :534-541 isValid → JCA →
 * net.i2p.crypto.eddsa.EdDSAEngine; jar not vendored):
 *   decode_i2p         GroupElement(Curve, byte[])      (y not range-checked)
 *   Abyte              EdDSAPublicKey: A.toByteArray()  (canonical re-encode)
 *   slide              GroupElement.slide               (carry out of bit 255 dropped)
 *   dsm_vartime        GroupElement.doubleScalarMultiplyVariableTime
 *   verify             EdDSAEngine.engineVerify: |sig|==64, no S<L check,
 *                      encode(R') == R byte-for-byte (cofactorless)
 * Field arithmetic: radix 2^51, 5 limbs, unsigned __int128 products (this is
 * the oracle's own representation; i2p uses 10 x int32 limbs — only the group
 * elements and bytes matter for parity).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef unsigned __int128 u128;
typedef struct { uint64_t v[5]; } fe;

#define MASK51 ((1ULL << 51) - 1)

static void fe_carry(fe* r) {
  uint64_t c;
  c = r->v[0] >> 51; r->v[0] &= MASK51; r->v[1] += c;
  c = r->v[1] >> 51; r->v[1] &= MASK51; r->v[2] += c;
  c = r->v[2] >> 51; r->v[2] &= MASK51; r->v[3] += c;
  c = r->v[3] >> 51; r->v[3] &= MASK51; r->v[4] += c;
  c = r->v[4] >> 51; r->v[4] &= MASK51; r->v[0] += c * 19;
  c = r->v[0] >> 51; r->v[0] &= MASK51; r->v[1] += c;
}
static void fe_0(fe* r) { memset(r, 0, sizeof *r); }
static void fe_1(fe* r) { fe_0(r); r->v[0] = 1; }
static void fe_add(fe* r, const fe* a, const fe* b) {
  for (int i = 0; i < 5; i++) r->v[i] = a->v[i] + b->v[i];
  fe_carry(r);
}
/* a - b computed as a + 4p - b (inputs weakly reduced: limbs < 2^52) */
static void fe_sub(fe* r, const fe* a, const fe* b) {
  r->v[0] = a->v[0] + 0x1FFFFFFFFFFFB4ULL - b->v[0];
  for (int i = 1; i < 5; i++) r->v[i] = a->v[i] + 0x1FFFFFFFFFFFFCULL - b->v[i];
  fe_carry(r);
}
static void fe_neg(fe* r, const fe* a) { fe z; fe_0(&z); fe_sub(r, &z, a); }
static void fe_mul(fe* r, const fe* a, const fe* b) {
  const uint64_t *x = a->v, *y = b->v;
  uint64_t y1 = y[1] * 19, y2 = y[2] * 19, y3 = y[3] * 19, y4 = y[4] * 19;
  u128 t0 = (u128)x[0] * y[0] + (u128)x[1] * y4 + (u128)x[2] * y3 + (u128)x[3] * y2 + (u128)x[4] * y1;
  u128 t1 = (u128)x[0] * y[1] + (u128)x[1] * y[0] + (u128)x[2] * y4 + (u128)x[3] * y3 + (u128)x[4] * y2;
  u128 t2 = (u128)x[0] * y[2] + (u128)x[1] * y[1] + (u128)x[2] * y[0] + (u128)x[3] * y4 + (u128)x[4] * y3;
  u128 t3 = (u128)x[0] * y[3] + (u128)x[1] * y[2] + (u128)x[2] * y[1] + (u128)x[3] * y[0] + (u128)x[4] * y4;
  u128 t4 = (u128)x[0] * y[4] + (u128)x[1] * y[3] + (u128)x[2] * y[2] + (u128)x[3] * y[1] + (u128)x[4] * y[0];
  t1 += (uint64_t)(t0 >> 51); uint64_t r0 = (uint64_t)t0 & MASK51;
  t2 += (uint64_t)(t1 >> 51); uint64_t r1 = (uint64_t)t1 & MASK51;
  t3 += (uint64_t)(t2 >> 51); uint64_t r2 = (uint64_t)t2 & MASK51;
  t4 += (uint64_t)(t3 >> 51); uint64_t r3 = (uint64_t)t3 & MASK51;
  uint64_t c = (uint64_t)(t4 >> 51); uint64_t r4 = (uint64_t)t4 & MASK51;
  r0 += c * 19; r1 += r0 >> 51; r0 &= MASK51;
  r->v[0] = r0; r->v[1] = r1; r->v[2] = r2; r->v[3] = r3; r->v[4] = r4;
}
static void fe_sq(fe* r, const fe* a) { fe_mul(r, a, a); }
static void fe_sqn(fe* r, const fe* a, int n) { fe_sq(r, a); for (int i = 1; i < n; i++) fe_sq(r, r); }

/* ref10 fe_frombytes semantics: bit 255 ignored, value NOT reduced below p. */
static void fe_frombytes(fe* r, const uint8_t s[32]) {
  uint64_t w[4];
  for (int i = 0; i < 4; i++) {
    uint64_t x = 0;
    for (int k = 7; k >= 0; k--) x = (x << 8) | s[8 * i + k];
    w[i] = x;
  }
  r->v[0] = w[0] & MASK51;
  r->v[1] = ((w[0] >> 51) | (w[1] << 13)) & MASK51;
  r->v[2] = ((w[1] >> 38) | (w[2] << 26)) & MASK51;
  r->v[3] = ((w[2] >> 25) | (w[3] << 39)) & MASK51;
  r->v[4] = (w[3] >> 12) & MASK51;
}
/* canonical (fully reduced) little-endian bytes */
static void fe_tobytes(uint8_t s[32], const fe* a) {
  fe t = *a;
  fe_carry(&t);
  fe_carry(&t);
  /* now t < 2^255 + small; subtract p if t >= p */
  uint64_t q = (t.v[0] + 19) >> 51;
  q = (t.v[1] + q) >> 51; q = (t.v[2] + q) >> 51; q = (t.v[3] + q) >> 51; q = (t.v[4] + q) >> 51;
  t.v[0] += 19 * q;
  uint64_t c;
  c = t.v[0] >> 51; t.v[0] &= MASK51; t.v[1] += c;
  c = t.v[1] >> 51; t.v[1] &= MASK51; t.v[2] += c;
  c = t.v[2] >> 51; t.v[2] &= MASK51; t.v[3] += c;
  c = t.v[3] >> 51; t.v[3] &= MASK51; t.v[4] += c;
  t.v[4] &= MASK51;
  uint64_t w0 = t.v[0] | (t.v[1] << 51), w1 = (t.v[1] >> 13) | (t.v[2] << 38);
  uint64_t w2 = (t.v[2] >> 26) | (t.v[3] << 25), w3 = (t.v[3] >> 39) | (t.v[4] << 12);
  uint64_t w[4] = {w0, w1, w2, w3};
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) s[8 * i + k] = (uint8_t)(w[i] >> (8 * k));
}
static int fe_isnonzero(const fe* a) {
  uint8_t s[32]; fe_tobytes(s, a);
  uint8_t acc = 0; for (int i = 0; i < 32; i++) acc |= s[i];
  return acc != 0;
}
static int fe_isnegative(const fe* a) { uint8_t s[32]; fe_tobytes(s, a); return s[0] & 1; }

/* z^(2^250 - 1) helper chain, shared by invert and pow22523 */
static void fe_pow2_250_1(fe* out, fe* z11, const fe* z) {
  fe z2, z9, t, z2_5_0, z2_10_0, z2_20_0, z2_50_0, z2_100_0;
  fe_sq(&z2, z);
  fe_sqn(&t, &z2, 2);
  fe_mul(&z9, &t, z);
  fe_mul(z11, &z9, &z2);
  fe_sq(&t, z11);
  fe_mul(&z2_5_0, &t, &z9);
  fe_sqn(&t, &z2_5_0, 5); fe_mul(&z2_10_0, &t, &z2_5_0);
  fe_sqn(&t, &z2_10_0, 10); fe_mul(&z2_20_0, &t, &z2_10_0);
  fe_sqn(&t, &z2_20_0, 20); fe_mul(&t, &t, &z2_20_0);
  fe_sqn(&t, &t, 10); fe_mul(&z2_50_0, &t, &z2_10_0);
  fe_sqn(&t, &z2_50_0, 50); fe_mul(&z2_100_0, &t, &z2_50_0);
  fe_sqn(&t, &z2_100_0, 100); fe_mul(&t, &t, &z2_100_0);
  fe_sqn(&t, &t, 50); fe_mul(out, &t, &z2_50_0);
}
static void fe_invert(fe* r, const fe* z) {
  fe t, z11;
  fe_pow2_250_1(&t, &z11, z);
  fe_sqn(&t, &t, 5);
  fe_mul(r, &t, &z11);
}
static void fe_pow22523(fe* r, const fe* z) {
  fe t, z11;
  fe_pow2_250_1(&t, &z11, z);
  fe_sqn(&t, &t, 2);
  fe_mul(r, &t, z);
}

/* constants (computed at first use from their defining equations) */
static fe FE_D, FE_D2, FE_SQRTM1;
typedef struct { fe X, Y, Z, T; } ge_p3;
typedef struct { fe YpX, YmX, Z, T2d; } ge_cached;
static ge_cached B_TABLE[8];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void fe_from_u64(fe* r, uint64_t x) { fe_0(r); r->v[0] = x & MASK51; r->v[1] = x >> 51; }

static void ge_to_cached(ge_cached* c, const ge_p3* p) {
  fe_add(&c->YpX, &p->Y, &p->X);
  fe_sub(&c->YmX, &p->Y, &p->X);
  c->Z = p->Z;
  fe_mul(&c->T2d, &p->T, &FE_D2);
}
/* extended addition (add-2008-hwcd-3), complete on Ed25519 */
static void ge_add(ge_p3* r, const ge_p3* p, const ge_cached* q) {
  fe a, b, c, d, e, f, g, h, t;
  fe_sub(&t, &p->Y, &p->X); fe_mul(&a, &t, &q->YmX);
  fe_add(&t, &p->Y, &p->X); fe_mul(&b, &t, &q->YpX);
  fe_mul(&c, &p->T, &q->T2d);
  fe_mul(&d, &p->Z, &q->Z); fe_add(&d, &d, &d);
  fe_sub(&e, &b, &a); fe_sub(&f, &d, &c); fe_add(&g, &d, &c); fe_add(&h, &b, &a);
  fe_mul(&r->X, &e, &f); fe_mul(&r->Y, &g, &h); fe_mul(&r->Z, &f, &g); fe_mul(&r->T, &e, &h);
}
static void ge_sub(ge_p3* r, const ge_p3* p, const ge_cached* q) {
  ge_cached n;
  n.YpX = q->YmX; n.YmX = q->YpX; n.Z = q->Z; fe_neg(&n.T2d, &q->T2d);
  ge_add(r, p, &n);
}
/* doubling (dbl-2008-hwcd, a = -1) */
static void ge_dbl(ge_p3* r, const ge_p3* p) {
  fe a, b, c, e, f, g, h, t;
  fe_sq(&a, &p->X); fe_sq(&b, &p->Y); fe_sq(&c, &p->Z); fe_add(&c, &c, &c);
  fe_add(&t, &p->X, &p->Y); fe_sq(&t, &t);
  fe_add(&h, &a, &b);           /* H = A + B */
  fe_sub(&e, &h, &t);           /* E = H - (X+Y)^2  (= -2XY) */
  fe_sub(&g, &a, &b);           /* G = A - B  (a=-1: -A + B negated consistently) */
  fe_add(&f, &c, &g);           /* F = C + G */
  /* with a = -1: X3 = E*F, Y3 = G*H, Z3 = F*G, T3 = E*H  (signs folded) */
  fe_mul(&r->X, &e, &f); fe_mul(&r->Y, &g, &h); fe_mul(&r->Z, &f, &g); fe_mul(&r->T, &e, &h);
}
static void ge_identity(ge_p3* r) { fe_0(&r->X); fe_1(&r->Y); fe_1(&r->Z); fe_0(&r->T); }
static void ge_tobytes(uint8_t s[32], const ge_p3* p) {
  fe zi, x, y;
  fe_invert(&zi, &p->Z);
  fe_mul(&x, &p->X, &zi); fe_mul(&y, &p->Y, &zi);
  fe_tobytes(s, &y);
  s[31] ^= (uint8_t)(fe_isnegative(&x) << 7);
}

/* i2p GroupElement(Curve, byte[] s); returns 0 on success, -1 = "not a valid GroupElement" */
static int ge_decode_i2p(ge_p3* r, const uint8_t s[32]) {
  fe y, yy, u, v, v3, x, vxx, chk;
  fe_frombytes(&y, s);
  fe_sq(&yy, &y);
  fe one; fe_1(&one);
  fe_sub(&u, &yy, &one);
  fe_mul(&v, &yy, &FE_D); fe_add(&v, &v, &one);
  fe_sq(&v3, &v); fe_mul(&v3, &v3, &v);
  fe_sq(&x, &v3); fe_mul(&x, &x, &v); fe_mul(&x, &x, &u);
  fe_pow22523(&x, &x);
  fe_mul(&x, &x, &v3); fe_mul(&x, &x, &u);
  fe_sq(&vxx, &x); fe_mul(&vxx, &vxx, &v);
  fe_sub(&chk, &vxx, &u);
  if (fe_isnonzero(&chk)) {
    fe_add(&chk, &vxx, &u);
    if (fe_isnonzero(&chk)) return -1;
    fe_mul(&x, &x, &FE_SQRTM1);
  }
  if (fe_isnegative(&x) != ((s[31] >> 7) & 1)) fe_neg(&x, &x);
  r->X = x; r->Y = y; fe_1(&r->Z); fe_mul(&r->T, &x, &y);
  return 0;
}

static void odd_multiples(ge_cached out[8], const ge_p3* p) {
  ge_p3 p2, acc = *p;
  ge_cached c2;
  ge_dbl(&p2, p);
  ge_to_cached(&c2, &p2);
  ge_to_cached(&out[0], &acc);
  for (int i = 1; i < 8; i++) {
    ge_add(&acc, &acc, &c2);
    ge_to_cached(&out[i], &acc);
  }
}

static void init_consts(void) {
  /* d = -121665/121666 */
  fe n, dd, inv;
  fe_from_u64(&n, 121665); fe_from_u64(&dd, 121666);
  fe_invert(&inv, &dd);
  fe_mul(&FE_D, &n, &inv); fe_neg(&FE_D, &FE_D);
  fe_add(&FE_D2, &FE_D, &FE_D);
  /* sqrt(-1) = 2^((p-1)/4) */
  fe two, t;
  fe_from_u64(&two, 2);
  /* (p-1)/4 = 2^253 - 5 : compute 2^(2^253-5) via square-and-multiply on bits */
  fe acc; fe_1(&acc);
  /* exponent bits of 2^253 - 5 = 0x1fff...ffb */
  for (int i = 252; i >= 0; i--) {
    fe_sq(&acc, &acc);
    int bit = (i == 2) ? 0 : 1; /* 2^253-5 = 111...1011 (bits 252..0, bit 2 clear) */
    if (bit) fe_mul(&acc, &acc, &two);
  }
  FE_SQRTM1 = acc;
  (void)t;
  /* base point: y = 4/5, x even */
  uint8_t by[32];
  fe four, five, fy;
  fe_from_u64(&four, 4); fe_from_u64(&five, 5); fe_invert(&inv, &five); fe_mul(&fy, &four, &inv);
  fe_tobytes(by, &fy);
  ge_p3 B;
  ge_decode_i2p(&B, by);
  odd_multiples(B_TABLE, &B);
}

int oracle_slide(const uint8_t a[32], int8_t r[256]) {
  int dropped = 0;
  for (int i = 0; i < 256; i++) r[i] = 1 & (a[i >> 3] >> (i & 7));
  for (int i = 0; i < 256; i++) {
    if (!r[i]) continue;
    for (int b = 1; b <= 6 && i + b < 256; b++) {
      if (!r[i + b]) continue;
      if (r[i] + (r[i + b] << b) <= 15) {
        r[i] += r[i + b] << b;
        r[i + b] = 0;
      } else if (r[i] - (r[i + b] << b) >= -15) {
        r[i] -= r[i + b] << b;
        int k;
        for (k = i + b; k < 256; k++) {
          if (!r[k]) { r[k] = 1; break; }
          r[k] = 0;
        }
        if (k == 256) dropped = 1;
      } else {
        break;
      }
    }
  }
  return dropped;
}

/* B.doubleScalarMultiplyVariableTime(Aneg, h, S) = [h]Aneg + [S]B */
static void dsm_vartime(ge_p3* r, const ge_p3* Aneg, const uint8_t h[32], const uint8_t s[32]) {
  int8_t as[256], bs[256];
  ge_cached at[8];
  oracle_slide(h, as);
  oracle_slide(s, bs);
  odd_multiples(at, Aneg);
  ge_identity(r);
  int i = 255;
  while (i >= 0 && !as[i] && !bs[i]) i--;
  for (; i >= 0; i--) {
    ge_dbl(r, r);
    if (as[i] > 0) ge_add(r, r, &at[as[i] / 2]);
    else if (as[i] < 0) ge_sub(r, r, &at[(-as[i]) / 2]);
    if (bs[i] > 0) ge_add(r, r, &B_TABLE[bs[i] / 2]);
    else if (bs[i] < 0) ge_sub(r, r, &B_TABLE[(-bs[i]) / 2]);
  }
}

/* --- scalars mod L (bitwise long division; oracle clarity over speed) --- */
static const uint64_t L64[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};

static void sc_reduce_words(uint64_t* x, int nw, uint8_t out[32]) {
  /* remainder r (5 words) built MSB-first */
  uint64_t r[5] = {0, 0, 0, 0, 0};
  for (int bit = nw * 64 - 1; bit >= 0; bit--) {
    /* r = 2r + bit */
    for (int k = 4; k > 0; k--) r[k] = (r[k] << 1) | (r[k - 1] >> 63);
    r[0] = (r[0] << 1) | ((x[bit / 64] >> (bit % 64)) & 1);
    /* if r >= L: r -= L */
    int ge = r[4] != 0;
    if (!ge) {
      ge = 1;
      for (int k = 3; k >= 0; k--) {
        if (r[k] != L64[k]) { ge = r[k] > L64[k]; break; }
      }
    }
    if (ge) {
      u128 borrow = 0;
      for (int k = 0; k < 4; k++) {
        u128 d = (u128)r[k] - L64[k] - borrow;
        r[k] = (uint64_t)d;
        borrow = (d >> 64) ? 1 : 0;
      }
      r[4] -= (uint64_t)borrow;
    }
  }
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) out[8 * i + k] = (uint8_t)(r[i] >> (8 * k));
}
static void sc_reduce64(uint8_t out[32], const uint8_t in[64]) {
  uint64_t x[8];
  for (int i = 0; i < 8; i++) {
    uint64_t v = 0;
    for (int k = 7; k >= 0; k--) v = (v << 8) | in[8 * i + k];
    x[i] = v;
  }
  sc_reduce_words(x, 8, out);
}

static void pthread_init(void) { init_consts(); }

static int ed_verify(const uint8_t* pub, size_t publen, const uint8_t* sig, size_t siglen, const uint8_t* msg,
                     size_t msglen, int is_valid) {
  pthread_once(&g_once, pthread_init);
  /* key decode happens at key construction (Kryo.kt:389-392), before verify */
  if (publen != 32) return ORACLE_BAD_KEY;
  ge_p3 A;
  if (ge_decode_i2p(&A, pub) != 0) return ORACLE_BAD_KEY;
  /* Crypto.doVerify require checks (Crypto.kt:475-476); Crypto.isValid (:534-541) has none */
  if (!is_valid && (siglen == 0 || msglen == 0)) return ORACLE_EMPTY;
  if (siglen != 64) return ORACLE_MALFORMED_SIG;
  uint8_t abyte[32];
  ge_tobytes(abyte, &A);
  /* h = SHA-512(R || Abyte || M) mod L */
  size_t hl = 64 + msglen;
  uint8_t stackbuf[512];
  uint8_t* buf = hl <= sizeof stackbuf ? stackbuf : (uint8_t*)malloc(hl);
  memcpy(buf, sig, 32);
  memcpy(buf + 32, abyte, 32);
  memcpy(buf + 64, msg, msglen);
  uint8_t hd[64], h[32];
  oracle_sha512(buf, hl, hd);
  if (buf != stackbuf) free(buf);
  sc_reduce64(h, hd);
  /* Aneg = -A */
  ge_p3 Aneg = A;
  fe_neg(&Aneg.X, &A.X);
  fe_neg(&Aneg.T, &A.T);
  ge_p3 R;
  dsm_vartime(&R, &Aneg, h, sig + 32);
  uint8_t rc[32];
  ge_tobytes(rc, &R);
  return memcmp(rc, sig, 32) == 0 ? ORACLE_OK : ORACLE_BAD_SIG;
}

int oracle_ed25519_verify(const uint8_t* pub, size_t publen, const uint8_t* sig, size_t siglen,
                          const uint8_t* msg, size_t msglen) {
  return ed_verify(pub, publen, sig, siglen, msg, msglen, 0);
}

int oracle_ed25519_is_valid(const uint8_t* pub, size_t publen, const uint8_t* sig, size_t siglen,
                            const uint8_t* msg, size_t msglen) {
  return ed_verify(pub, publen, sig, siglen, msg, msglen, 1);
}

typedef struct {
  size_t lo, hi;
  const uint8_t *pubs, *sigs, *msgs;
  size_t msglen;
  uint8_t* status;
} job_t;

static void* worker(void* p) {
  job_t* j = (job_t*)p;
  for (size_t i = j->lo; i < j->hi; i++)
    j->status[i] = (uint8_t)oracle_ed25519_verify(j->pubs + 32 * i, 32, j->sigs + 64 * i, 64,
                                                  j->msgs + j->msglen * i, j->msglen);
  return NULL;
}

void oracle_ed25519_verify_batch(size_t n, const uint8_t* pubs, const uint8_t* sigs,
                                 const uint8_t* msgs, size_t msglen, uint8_t* status, int nthreads) {
  pthread_once(&g_once, pthread_init);
  if (nthreads <= 1 || n < 64) {
    job_t j = {0, n, pubs, sigs, msgs, msglen, status};
    worker(&j);
    return;
  }
  pthread_t th[256];
  job_t jobs[256];
  if (nthreads > 256) nthreads = 256;
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (job_t){n * t / nthreads, n * (t + 1) / nthreads, pubs, sigs, msgs, msglen, status};
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* --- RFC 8032 keygen / sign (test-data generation) --- */
static void ge_scalarmult_base(ge_p3* r, const uint8_t k[32]) {
  ge_p3 B;
  ge_identity(r);
  /* B from table entry 0 is cached form; rebuild p3 by decoding the base point */
  uint8_t by[32];
  fe four, five, inv, fy;
  fe_from_u64(&four, 4); fe_from_u64(&five, 5); fe_invert(&inv, &five); fe_mul(&fy, &four, &inv);
  fe_tobytes(by, &fy);
  ge_decode_i2p(&B, by);
  ge_cached bc;
  ge_to_cached(&bc, &B);
  for (int i = 255; i >= 0; i--) {
    ge_dbl(r, r);
    if ((k[i >> 3] >> (i & 7)) & 1) ge_add(r, r, &bc);
  }
}

void oracle_ed25519_keypair(const uint8_t seed[32], uint8_t pub[32]) {
  pthread_once(&g_once, pthread_init);
  uint8_t h[64];
  oracle_sha512(seed, 32, h);
  h[0] &= 248; h[31] &= 63; h[31] |= 64;
  ge_p3 A;
  ge_scalarmult_base(&A, h);
  ge_tobytes(pub, &A);
}

static void sc_muladd(uint8_t s[32], const uint8_t a[32], const uint8_t b[32], const uint8_t c[32]) {
  /* s = (a*b + c) mod L, via 512-bit schoolbook then reduction */
  uint64_t aw[4], bw[4], cw[4], prod[9] = {0};
  for (int i = 0; i < 4; i++) {
    aw[i] = bw[i] = cw[i] = 0;
    for (int k = 7; k >= 0; k--) {
      aw[i] = (aw[i] << 8) | a[8 * i + k];
      bw[i] = (bw[i] << 8) | b[8 * i + k];
      cw[i] = (cw[i] << 8) | c[8 * i + k];
    }
  }
  for (int i = 0; i < 4; i++) {
    u128 carry = 0;
    for (int j = 0; j < 4; j++) {
      u128 t = (u128)aw[i] * bw[j] + prod[i + j] + carry;
      prod[i + j] = (uint64_t)t;
      carry = t >> 64;
    }
    prod[i + 4] += (uint64_t)carry;
  }
  u128 carry = 0;
  for (int i = 0; i < 9; i++) {
    u128 t = (u128)prod[i] + (i < 4 ? cw[i] : 0) + carry;
    prod[i] = (uint64_t)t;
    carry = t >> 64;
  }
  sc_reduce_words(prod, 9, s);
}

void oracle_ed25519_sign(const uint8_t seed[32], const uint8_t* msg, size_t msglen,
                         uint8_t pub[32], uint8_t sig[64]) {
  pthread_once(&g_once, pthread_init);
  uint8_t h[64], r64[64], r[32], hram64[64], hram[32];
  oracle_sha512(seed, 32, h);
  h[0] &= 248; h[31] &= 63; h[31] |= 64;
  ge_p3 A, R;
  ge_scalarmult_base(&A, h);
  ge_tobytes(pub, &A);
  uint8_t* buf = (uint8_t*)malloc(64 + msglen); /* holds prefix||M, then R||A||M */
  memcpy(buf, h + 32, 32);
  memcpy(buf + 32, msg, msglen);
  oracle_sha512(buf, 32 + msglen, r64);
  sc_reduce64(r, r64);
  ge_scalarmult_base(&R, r);
  ge_tobytes(sig, &R);
  memcpy(buf, sig, 32);
  memcpy(buf + 32, pub, 32);
  memcpy(buf + 64, msg, msglen);
  oracle_sha512(buf, 64 + msglen, hram64);
  free(buf);
  sc_reduce64(hram, hram64);
  sc_muladd(sig + 32, hram, h, r);
}
