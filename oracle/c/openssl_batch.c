/* OpenSSL 3 Ed25519 batch verifier: an INDEPENDENT CPU reference for the C1
 * baseline (bench.py --workload c1), not an oracle for parity: RFC 8032 as
 * implemented by OpenSSL rejects S >= L, which i2p 0.2.0 (the reference's
 * engine) accepts. Test/measurement infrastructure only; the product never
 * links it. Per tuple: EVP_PKEY_new_raw_public_key (key decode, as the JVM
 * decodes keys before Crypto.doVerify) + EVP_DigestVerify. */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

struct job {
  const uint8_t *keys, *sigs, *msgs;
  size_t msg_len, lo, hi;
  uint8_t* ok;
};

static void* run(void* p) {
  struct job* j = (struct job*)p;
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  for (size_t i = j->lo; i < j->hi; i++) {
    EVP_PKEY* k = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, NULL, j->keys + 32 * i, 32);
    int ok = 0;
    if (k) {
      EVP_MD_CTX_reset(ctx);
      ok = EVP_DigestVerifyInit(ctx, NULL, NULL, NULL, k) == 1 &&
           EVP_DigestVerify(ctx, j->sigs + 64 * i, 64, j->msgs + j->msg_len * i, j->msg_len) == 1;
      EVP_PKEY_free(k);
    }
    j->ok[i] = (uint8_t)ok;
  }
  EVP_MD_CTX_free(ctx);
  return NULL;
}

/* ok[i] = 1 iff OpenSSL accepts tuple i; returns 0, or -1 if threads fail */
int openssl_ed25519_verify_batch(size_t n, const uint8_t* keys, const uint8_t* sigs, const uint8_t* msgs,
                                 size_t msg_len, uint8_t* ok, int threads) {
  if (threads < 1) threads = 1;
  pthread_t* t = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  struct job* jobs = (struct job*)calloc((size_t)threads, sizeof(struct job));
  if (!t || !jobs) return -1;
  int rc = 0;
  for (int k = 0; k < threads; k++) {
    jobs[k] = (struct job){keys, sigs, msgs, msg_len, n * k / threads, n * (k + 1) / threads, ok};
    if (pthread_create(&t[k], NULL, run, &jobs[k])) rc = -1;
  }
  for (int k = 0; k < threads; k++) pthread_join(t[k], NULL);
  free(t);
  free(jobs);
  return rc;
}
