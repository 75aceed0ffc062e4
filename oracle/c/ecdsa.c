/* ECDSA SHA256withECDSA with BouncyCastle 1.57 semantics — ORACLE (test infra only).
 *
 * C twin of oracle/bc_ecdsa.py (see its header for the step-by-step BC
 * 1.57 rules and the reference call sites: Crypto.kt:91-116 schemes,
 * :534-541 isValid -> JCA "SHA256withECDSA" -> BC DSABase/ECDSASigner).
 * Arithmetic: 4 x 64-bit limbs, Montgomery multiplication (generic modulus,
 * used for both p and n of both curves), Jacobian points, Shamir's trick.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } u256;
typedef struct {
  u256 m;      /* modulus */
  uint64_t m0; /* -m^-1 mod 2^64 */
  u256 r2;     /* 2^512 mod m */
  u256 one;    /* 2^256 mod m (Montgomery 1) */
} mod_t;

static int u256_cmp(const u256* a, const u256* b) {
  for (int i = 3; i >= 0; i--) {
    if (a->v[i] != b->v[i]) return a->v[i] > b->v[i] ? 1 : -1;
  }
  return 0;
}
static uint64_t u256_add(u256* r, const u256* a, const u256* b) {
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (u128)a->v[i] + b->v[i];
    r->v[i] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}
static uint64_t u256_sub(u256* r, const u256* a, const u256* b) {
  uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a->v[i] - b->v[i] - br;
    r->v[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  return br;
}
static int u256_iszero(const u256* a) { return !(a->v[0] | a->v[1] | a->v[2] | a->v[3]); }
static void u256_from_be(u256* r, const uint8_t b[32]) {
  for (int i = 0; i < 4; i++) {
    uint64_t x = 0;
    for (int k = 0; k < 8; k++) x = (x << 8) | b[(3 - i) * 8 + k];
    r->v[i] = x;
  }
}

static void mod_add(const mod_t* M, u256* r, const u256* a, const u256* b) {
  uint64_t c = u256_add(r, a, b);
  if (c || u256_cmp(r, &M->m) >= 0) u256_sub(r, r, &M->m);
}
static void mod_sub(const mod_t* M, u256* r, const u256* a, const u256* b) {
  if (u256_sub(r, a, b)) u256_add(r, r, &M->m);
}
/* Montgomery product a*b*2^-256 mod m (CIOS) */
static void mont_mul(const mod_t* M, u256* r, const u256* a, const u256* b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a->v[j] * b->v[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[4] = (uint64_t)c;
    t[5] = (uint64_t)(c >> 64);
    uint64_t q = t[0] * M->m0;
    c = (u128)q * M->m.v[0] + t[0];
    c >>= 64;
    for (int j = 1; j < 4; j++) {
      c += (u128)q * M->m.v[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[3] = (uint64_t)c;
    t[4] = t[5] + (uint64_t)(c >> 64);
  }
  u256 res = {{t[0], t[1], t[2], t[3]}};
  if (t[4] || u256_cmp(&res, &M->m) >= 0) u256_sub(&res, &res, &M->m);
  *r = res;
}
static void to_mont(const mod_t* M, u256* r, const u256* a) { mont_mul(M, r, a, &M->r2); }
static void from_mont(const mod_t* M, u256* r, const u256* a) {
  u256 one = {{1, 0, 0, 0}};
  mont_mul(M, r, a, &one);
}
/* a^e (Montgomery domain), e plain */
static void mont_pow(const mod_t* M, u256* r, const u256* a, const u256* e) {
  u256 acc = M->one;
  for (int i = 255; i >= 0; i--) {
    mont_mul(M, &acc, &acc, &acc);
    if ((e->v[i / 64] >> (i % 64)) & 1) mont_mul(M, &acc, &acc, a);
  }
  *r = acc;
}
static void mod_init(mod_t* M, const u256* m) {
  M->m = *m;
  uint64_t inv = 1; /* Newton: inv = m0^-1 mod 2^64 */
  for (int i = 0; i < 6; i++) inv *= 2 - m->v[0] * inv;
  M->m0 = (uint64_t)0 - inv;
  /* one = 2^256 mod m ; r2 = 2^512 mod m by repeated doubling */
  u256 x = {{1, 0, 0, 0}};
  for (int i = 0; i < 512; i++) {
    uint64_t c = u256_add(&x, &x, &x);
    if (c || u256_cmp(&x, m) >= 0) u256_sub(&x, &x, m);
    if (i == 255) M->one = x;
  }
  M->r2 = x;
}

typedef struct {
  mod_t P, N;
  u256 a, b;      /* Montgomery form (mod p) */
  u256 gx, gy;    /* Montgomery form */
  int a_is_m3;
} curve_t;

static curve_t CURVE_K1, CURVE_R1;
static pthread_once_t ec_once = PTHREAD_ONCE_INIT;

static void hex_to_u256(u256* r, const char* hex) {
  uint8_t b[32];
  for (int i = 0; i < 32; i++) {
    unsigned v;
    char t[3] = {hex[2 * i], hex[2 * i + 1], 0};
    v = (unsigned)strtoul(t, NULL, 16);
    b[i] = (uint8_t)v;
  }
  u256_from_be(r, b);
}

static void curve_init(curve_t* c, const char* p, const char* a, const char* b, const char* gx, const char* gy,
                       const char* n, int a_is_m3) {
  u256 t;
  hex_to_u256(&t, p);
  mod_init(&c->P, &t);
  hex_to_u256(&t, n);
  mod_init(&c->N, &t);
  hex_to_u256(&t, a); to_mont(&c->P, &c->a, &t);
  hex_to_u256(&t, b); to_mont(&c->P, &c->b, &t);
  hex_to_u256(&t, gx); to_mont(&c->P, &c->gx, &t);
  hex_to_u256(&t, gy); to_mont(&c->P, &c->gy, &t);
  c->a_is_m3 = a_is_m3;
}

static void ec_init(void) {
  curve_init(&CURVE_K1, "fffffffffffffffffffffffffffffffffffffffffffffffffffffffefffffc2f",
             "0000000000000000000000000000000000000000000000000000000000000000",
             "0000000000000000000000000000000000000000000000000000000000000007",
             "79be667ef9dcbbac55a06295ce870b07029bfcdb2dce28d959f2815b16f81798",
             "483ada7726a3c4655da4fbfc0e1108a8fd17b448a68554199c47d08ffb10d4b8",
             "fffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0364141", 0);
  curve_init(&CURVE_R1, "ffffffff00000001000000000000000000000000ffffffffffffffffffffffff",
             "ffffffff00000001000000000000000000000000fffffffffffffffffffffffc",
             "5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b",
             "6b17d1f2e12c4247f8bce6e563a440f277037d812deb33a0f4a13945d898c296",
             "4fe342e2fe1a7f9b8ee7eb4a7c0f9e162bce33576b315ececbb6406837bf51f5",
             "ffffffff00000000ffffffffffffffffbce6faada7179e84f3b9cac2fc632551", 1);
}

typedef struct { u256 X, Y, Z; int inf; } jac_t; /* Montgomery-form Jacobian */

static void jac_dbl(const curve_t* c, jac_t* r, const jac_t* p) {
  const mod_t* M = &c->P;
  if (p->inf || u256_iszero(&p->Y)) { r->inf = 1; return; }
  u256 xx, yy, yyyy, zz, s, m, t, x3, y3, z3;
  mont_mul(M, &xx, &p->X, &p->X);
  mont_mul(M, &yy, &p->Y, &p->Y);
  mont_mul(M, &yyyy, &yy, &yy);
  mont_mul(M, &zz, &p->Z, &p->Z);
  /* S = 4 X YY */
  mont_mul(M, &s, &p->X, &yy); mod_add(M, &s, &s, &s); mod_add(M, &s, &s, &s);
  /* M = 3 XX + a ZZ^2 */
  mod_add(M, &m, &xx, &xx); mod_add(M, &m, &m, &xx);
  mont_mul(M, &t, &zz, &zz); mont_mul(M, &t, &t, &c->a); mod_add(M, &m, &m, &t);
  /* X3 = M^2 - 2S */
  mont_mul(M, &x3, &m, &m); mod_sub(M, &x3, &x3, &s); mod_sub(M, &x3, &x3, &s);
  /* Y3 = M (S - X3) - 8 YYYY */
  mod_sub(M, &t, &s, &x3); mont_mul(M, &y3, &m, &t);
  mod_add(M, &t, &yyyy, &yyyy); mod_add(M, &t, &t, &t); mod_add(M, &t, &t, &t);
  mod_sub(M, &y3, &y3, &t);
  /* Z3 = 2 Y Z */
  mont_mul(M, &z3, &p->Y, &p->Z); mod_add(M, &z3, &z3, &z3);
  r->X = x3; r->Y = y3; r->Z = z3; r->inf = 0;
}

static void jac_add(const curve_t* c, jac_t* r, const jac_t* p, const jac_t* q) {
  const mod_t* M = &c->P;
  if (p->inf) { *r = *q; return; }
  if (q->inf) { *r = *p; return; }
  u256 z1z1, z2z2, u1, u2, s1, s2, h, rr, hh, hhh, v, t, x3, y3, z3;
  mont_mul(M, &z1z1, &p->Z, &p->Z);
  mont_mul(M, &z2z2, &q->Z, &q->Z);
  mont_mul(M, &u1, &p->X, &z2z2);
  mont_mul(M, &u2, &q->X, &z1z1);
  mont_mul(M, &s1, &p->Y, &q->Z); mont_mul(M, &s1, &s1, &z2z2);
  mont_mul(M, &s2, &q->Y, &p->Z); mont_mul(M, &s2, &s2, &z1z1);
  mod_sub(M, &h, &u2, &u1);
  mod_sub(M, &rr, &s2, &s1);
  if (u256_iszero(&h)) {
    if (u256_iszero(&rr)) { jac_dbl(c, r, p); return; }
    r->inf = 1;
    return;
  }
  mont_mul(M, &hh, &h, &h);
  mont_mul(M, &hhh, &hh, &h);
  mont_mul(M, &v, &u1, &hh);
  mont_mul(M, &x3, &rr, &rr); mod_sub(M, &x3, &x3, &hhh); mod_sub(M, &x3, &x3, &v); mod_sub(M, &x3, &x3, &v);
  mod_sub(M, &t, &v, &x3); mont_mul(M, &y3, &rr, &t);
  mont_mul(M, &t, &s1, &hhh); mod_sub(M, &y3, &y3, &t);
  mont_mul(M, &z3, &p->Z, &q->Z); mont_mul(M, &z3, &z3, &h);
  r->X = x3; r->Y = y3; r->Z = z3; r->inf = 0;
}

/* BC ECCurve.decodePoint with validation; returns 0 ok */
static int decode_point(const curve_t* c, jac_t* q, const uint8_t* enc, size_t len) {
  const mod_t* M = &c->P;
  u256 x, y, rhs, t;
  if (len == 65 && enc[0] == 4) {
    u256_from_be(&x, enc + 1);
    u256_from_be(&y, enc + 33);
    if (u256_cmp(&x, &M->m) >= 0 || u256_cmp(&y, &M->m) >= 0) return -1;
    to_mont(M, &x, &x); to_mont(M, &y, &y);
  } else if (len == 33 && (enc[0] == 2 || enc[0] == 3)) {
    u256_from_be(&x, enc + 1);
    if (u256_cmp(&x, &M->m) >= 0) return -1;
    to_mont(M, &x, &x);
    mont_mul(M, &rhs, &x, &x); mont_mul(M, &rhs, &rhs, &x);
    mont_mul(M, &t, &c->a, &x); mod_add(M, &rhs, &rhs, &t); mod_add(M, &rhs, &rhs, &c->b);
    /* y = rhs^((p+1)/4) */
    u256 e = M->m, one = {{1, 0, 0, 0}};
    u256_add(&e, &e, &one);
    for (int i = 0; i < 2; i++) { /* e >>= 1 twice */
      for (int k = 0; k < 3; k++) e.v[k] = (e.v[k] >> 1) | (e.v[k + 1] << 63);
      e.v[3] >>= 1;
    }
    mont_pow(M, &y, &rhs, &e);
    mont_mul(M, &t, &y, &y);
    if (u256_cmp(&t, &rhs) != 0) return -1;
    u256 yp;
    from_mont(M, &yp, &y);
    if ((yp.v[0] & 1) != (uint64_t)(enc[0] & 1)) mod_sub(M, &y, &(u256){{0, 0, 0, 0}}, &y);
    rhs = (u256){{0, 0, 0, 0}};
  } else {
    return -1;
  }
  /* on-curve check: y^2 == x^3 + a x + b */
  u256 lhs;
  mont_mul(M, &lhs, &y, &y);
  mont_mul(M, &rhs, &x, &x); mont_mul(M, &rhs, &rhs, &x);
  mont_mul(M, &t, &c->a, &x); mod_add(M, &rhs, &rhs, &t); mod_add(M, &rhs, &rhs, &c->b);
  if (u256_cmp(&lhs, &rhs) != 0) return -1;
  q->X = x; q->Y = y; q->Z = M->one; q->inf = 0;
  return 0;
}

/* BC StdDSAEncoder.decode: strict DER SEQUENCE{INTEGER r, INTEGER s}.
 * Returns 0 and sets r/s (magnitude in 32 bytes, neg flags, big flag if > 32
 * significant bytes) or -1 if malformed. */
typedef struct { u256 v; int neg; int big; } der_int_t;

static int der_len(const uint8_t* b, size_t n, size_t* i, size_t* out) {
  if (*i >= n) return -1;
  uint8_t l0 = b[(*i)++];
  if (l0 < 0x80) { *out = l0; return 0; }
  /* long form is never the DER encoding of a length < 128; longer lengths cannot
   * occur in a signature whose re-encoding could equal it with two 256-bit ints,
   * but we parse exactly and let the minimality test decide */
  size_t nb = l0 & 0x7f;
  if (nb == 0 || nb > 4 || *i + nb > n) return -1;
  size_t v = 0;
  for (size_t k = 0; k < nb; k++) v = (v << 8) | b[(*i)++];
  if (v < 0x80 || (nb > 1 && b[*i - nb] == 0)) return -1; /* non-minimal length */
  *out = v;
  return 0;
}

static int der_decode(const uint8_t* sig, size_t n, der_int_t out[2]) {
  size_t i = 0, len;
  if (n < 2 || sig[0] != 0x30) return -1;
  i = 1;
  if (der_len(sig, n, &i, &len) || i + len != n) return -1;
  int cnt = 0;
  while (i < n) {
    if (cnt == 2) return -1;
    if (sig[i++] != 0x02) return -1;
    size_t l;
    if (der_len(sig, n, &i, &l) || i + l > n || l == 0) return -1;
    const uint8_t* body = sig + i;
    if (l > 1 && ((body[0] == 0 && body[1] < 0x80) || (body[0] == 0xff && body[1] >= 0x80))) return -1;
    der_int_t* d = &out[cnt++];
    d->neg = body[0] >= 0x80;
    d->big = 0;
    memset(&d->v, 0, sizeof d->v);
    /* magnitude of positive values only (negatives are rejected by range anyway) */
    size_t start = 0;
    while (start < l && body[start] == 0) start++;
    if (l - start > 32) d->big = 1;
    else {
      uint8_t be[32] = {0};
      memcpy(be + 32 - (l - start), body + start, l - start);
      u256_from_be(&d->v, be);
    }
    i += l;
  }
  return cnt == 2 ? 0 : -1;
}

static int ec_verify(int scheme, const uint8_t* pub, size_t publen, const uint8_t* sig, size_t siglen,
                     const uint8_t* msg, size_t msglen, int is_valid) {
  pthread_once(&ec_once, ec_init);
  const curve_t* c = scheme == 2 ? &CURVE_K1 : scheme == 3 ? &CURVE_R1 : NULL;
  if (!c) return ORACLE_UNSUPPORTED;
  jac_t Q;
  if (decode_point(c, &Q, pub, publen)) return ORACLE_BAD_KEY;
  /* Crypto.doVerify require checks (Crypto.kt:475-476); Crypto.isValid (:534-541) has none */
  if (!is_valid && (siglen == 0 || msglen == 0)) return ORACLE_EMPTY;
  der_int_t rs[2];
  if (der_decode(sig, siglen, rs)) return ORACLE_MALFORMED_SIG;
  const mod_t* N = &c->N;
  for (int k = 0; k < 2; k++)
    if (rs[k].neg || rs[k].big || u256_iszero(&rs[k].v) || u256_cmp(&rs[k].v, &N->m) >= 0) return ORACLE_BAD_SIG;
  uint8_t h[32];
  oracle_sha256(msg, msglen, h);
  u256 e, w, u1, u2, t, sm, em, rm;
  u256_from_be(&e, h);
  if (u256_cmp(&e, &N->m) >= 0) u256_sub(&e, &e, &N->m);
  to_mont(N, &sm, &rs[1].v);
  u256 nm2 = N->m, two = {{2, 0, 0, 0}};
  u256_sub(&nm2, &nm2, &two);
  mont_pow(N, &w, &sm, &nm2); /* s^-1 (Montgomery) */
  to_mont(N, &em, &e);
  to_mont(N, &rm, &rs[0].v);
  mont_mul(N, &t, &em, &w); from_mont(N, &u1, &t);
  mont_mul(N, &t, &rm, &w); from_mont(N, &u2, &t);
  /* Shamir: P = u1 G + u2 Q */
  jac_t G = {c->gx, c->gy, c->P.one, 0}, GQ, R = {{{0}}, {{0}}, {{0}}, 1};
  jac_add(c, &GQ, &G, &Q);
  for (int i = 255; i >= 0; i--) {
    jac_dbl(c, &R, &R);
    int b1 = (u1.v[i / 64] >> (i % 64)) & 1, b2 = (u2.v[i / 64] >> (i % 64)) & 1;
    if (b1 && b2) jac_add(c, &R, &R, &GQ);
    else if (b1) jac_add(c, &R, &R, &G);
    else if (b2) jac_add(c, &R, &R, &Q);
  }
  if (R.inf) return ORACLE_BAD_SIG;
  /* x = X / Z^2 (mod p), then compare x mod n with r */
  const mod_t* M = &c->P;
  u256 zi, z2, x, pm2 = M->m;
  u256_sub(&pm2, &pm2, &two);
  mont_pow(M, &zi, &R.Z, &pm2);
  mont_mul(M, &z2, &zi, &zi);
  mont_mul(M, &x, &R.X, &z2);
  from_mont(M, &x, &x);
  if (u256_cmp(&x, &N->m) >= 0) u256_sub(&x, &x, &N->m);
  return u256_cmp(&x, &rs[0].v) == 0 ? ORACLE_OK : ORACLE_BAD_SIG;
}

int oracle_ecdsa_verify(int scheme, const uint8_t* pub, size_t publen, const uint8_t* sig, size_t siglen,
                        const uint8_t* msg, size_t msglen) {
  return ec_verify(scheme, pub, publen, sig, siglen, msg, msglen, 0);
}

int oracle_ecdsa_is_valid(int scheme, const uint8_t* pub, size_t publen, const uint8_t* sig, size_t siglen,
                          const uint8_t* msg, size_t msglen) {
  return ec_verify(scheme, pub, publen, sig, siglen, msg, msglen, 1);
}

typedef struct {
  size_t lo, hi;
  const uint8_t *scheme, *key, *sig, *msg;
  const uint64_t *key_off, *sig_off, *msg_off;
  uint8_t* status;
} ejob_t;

static void* eworker(void* p) {
  ejob_t* j = (ejob_t*)p;
  for (size_t i = j->lo; i < j->hi; i++)
    j->status[i] = (uint8_t)oracle_ecdsa_verify(j->scheme[i], j->key + j->key_off[i], j->key_off[i + 1] - j->key_off[i],
                                                j->sig + j->sig_off[i], j->sig_off[i + 1] - j->sig_off[i],
                                                j->msg + j->msg_off[i], j->msg_off[i + 1] - j->msg_off[i]);
  return NULL;
}

void oracle_ecdsa_verify_batch(size_t n, const uint8_t* scheme, const uint8_t* key, const uint64_t* key_off,
                               const uint8_t* sig, const uint64_t* sig_off, const uint8_t* msg,
                               const uint64_t* msg_off, uint8_t* status, int nthreads) {
  pthread_once(&ec_once, ec_init);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  ejob_t jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (ejob_t){n * t / nthreads, n * (t + 1) / nthreads, scheme, key, sig, msg, key_off, sig_off, msg_off,
                       status};
    pthread_create(&th[t], NULL, eworker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}
