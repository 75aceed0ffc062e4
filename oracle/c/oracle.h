/* CPU restatement of the reference hot path — TEST INFRASTRUCTURE ONLY.
 *
 * ORACLE HEADER: everything under oracle/ is a checker. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle.so; the product (libcordahip.so) never links it and has no CPU
 * fallback.
 *
 * Restates:
 *   Crypto.doVerify/isValid EDDSA_ED25519_SHA512   Crypto.kt:472-483, :534-541
 *     -> i2p eddsa 0.2.0 EdDSAEngine.engineVerify (3P, not vendored)
 *   SecureHash.sha256 / hashConcat                 SecureHash.kt:24,36
 *   MerkleTree.getMerkleTree                       MerkleTree.kt:27-66
 *
 * Parity pinning: tests/golden/ed25519_vectors.json (expected statuses from
 * oracle/i2p_ed25519.py, valid path cross-checked against OpenSSL 3) and the
 * reference's structural Merkle tests (PartialMerkleTreeTest.kt:56-81).
 */
#ifndef CORDA_ORACLE_H
#define CORDA_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* lane statuses: identical to include/cordahip.h */
enum { ORACLE_OK = 0, ORACLE_BAD_SIG = 1, ORACLE_MALFORMED_SIG = 2, ORACLE_BAD_KEY = 3,
       ORACLE_UNSUPPORTED = 4, ORACLE_EMPTY = 5 };

void oracle_sha256(const uint8_t* m, size_t n, uint8_t out[32]);
void oracle_sha512(const uint8_t* m, size_t n, uint8_t out[64]);

/* i2p GroupElement.slide(): r[256] digits; returns 1 if the carry out of bit
 * 255 was dropped (digits then sum to a - 2^256). */
int oracle_slide(const uint8_t a[32], int8_t r[256]);

/* Per-lane status of Crypto.isValid(EDDSA_ED25519_SHA512, key, sig, msg). */
int oracle_ed25519_verify(const uint8_t* pub, size_t publen, const uint8_t* sig, size_t siglen,
                          const uint8_t* msg, size_t msglen);

/* Same lane under Crypto.isValid semantics (Crypto.kt:534-541): no emptiness
 * checks (an empty message is hashed; an empty signature fails the length check). */
int oracle_ed25519_is_valid(const uint8_t* pub, size_t publen, const uint8_t* sig, size_t siglen,
                            const uint8_t* msg, size_t msglen);

/* Dense batch: keys n*32, sigs n*64, msgs n*msglen; nthreads<=0 -> 1. */
void oracle_ed25519_verify_batch(size_t n, const uint8_t* pubs, const uint8_t* sigs,
                                 const uint8_t* msgs, size_t msglen, uint8_t* status,
                                 int nthreads);

/* RFC 8032 keygen/sign (test-data generation; mirrors Crypto.doSign). */
void oracle_ed25519_keypair(const uint8_t seed[32], uint8_t pub[32]);
void oracle_ed25519_sign(const uint8_t seed[32], const uint8_t* msg, size_t msglen,
                         uint8_t pub[32], uint8_t sig[64]);

/* MerkleTree.getMerkleTree(leaves).hash; returns -1 for 0 leaves
 * (MerkleTreeException, MerkleTree.kt:49-50). */
int oracle_merkle_root(const uint8_t* leaves, size_t nleaves, uint8_t root[32]);

/* Per-lane status of Crypto.isValid(ECDSA_SECP256K1_SHA256 (2) | ECDSA_SECP256R1_SHA256 (3),
 * SEC1 key, DER sig, msg) with BouncyCastle 1.57 semantics (oracle/bc_ecdsa.py). */
int oracle_ecdsa_verify(int scheme, const uint8_t* pub, size_t publen, const uint8_t* sig, size_t siglen,
                        const uint8_t* msg, size_t msglen);
int oracle_ecdsa_is_valid(int scheme, const uint8_t* pub, size_t publen, const uint8_t* sig, size_t siglen,
                          const uint8_t* msg, size_t msglen); /* Crypto.isValid semantics, as above */
void oracle_ecdsa_verify_batch(size_t n, const uint8_t* scheme, const uint8_t* key, const uint64_t* key_off,
                               const uint8_t* sig, const uint64_t* sig_off, const uint8_t* msg,
                               const uint64_t* msg_off, uint8_t* status, int nthreads);

/* WireTransaction.id from the serialised components (leaf preimages, CSR). */
int oracle_tx_id(const uint8_t* leaf_bytes, const uint64_t* leaf_off, size_t nleaves, uint8_t id[32]);
/* oracle_tx_id for each of ntx transactions (tx_leaf_off [ntx+1] into the leaf CSR),
 * on nthreads threads; status[t] 0, or 6 for no leaves */
void oracle_tx_id_batch(size_t ntx, const uint8_t* leaf_bytes, const uint64_t* leaf_off, const uint64_t* tx_leaf_off,
                        uint8_t* ids, uint8_t* status, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
