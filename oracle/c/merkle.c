/* MerkleTree.getMerkleTree restated — ORACLE (test infrastructure only).
 * core/src/main/kotlin/net/corda/core/crypto/MerkleTree.kt:27-66:
 *   padWithZeros (:33-41) to the next power of two with SecureHash.zeroHash
 *   (32 zero bytes, SecureHash.kt:41); buildMerkleTree (:48-66) pairs
 *   left.hash.hashConcat(right.hash) = SHA-256(left || right) (SecureHash.kt:24);
 *   empty list -> MerkleTreeException (:49-50); one leaf -> root = leaf. */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

int oracle_merkle_root(const uint8_t* leaves, size_t n, uint8_t root[32]) {
  if (n == 0) return -1;
  size_t m = 1;
  while (m < n) m <<= 1;
  uint8_t* lvl = (uint8_t*)calloc(m, 32);
  memcpy(lvl, leaves, n * 32);
  while (m > 1) {
    for (size_t i = 0; i < m / 2; i++) oracle_sha256(lvl + 64 * i, 64, lvl + 32 * i);
    m /= 2;
  }
  memcpy(root, lvl, 32);
  free(lvl);
  return 0;
}

/* WireTransaction.id (WireTransaction.kt:48,120): leaves are SHA-256 of the
 * serialised components (MerkleTransaction.kt:16-18,69), root per MerkleTree.kt.
 * leaf_off has nleaves+1 entries into leaf_bytes. Returns -1 for no leaves. */
int oracle_tx_id(const uint8_t* leaf_bytes, const uint64_t* leaf_off, size_t nleaves, uint8_t id[32]) {
  if (nleaves == 0) return -1;
  uint8_t* h = (uint8_t*)malloc(nleaves * 32);
  for (size_t i = 0; i < nleaves; i++)
    oracle_sha256(leaf_bytes + leaf_off[i], (size_t)(leaf_off[i + 1] - leaf_off[i]), h + 32 * i);
  int rc = oracle_merkle_root(h, nleaves, id);
  free(h);
  return rc;
}

/* oracle_tx_id over many transactions (the agreement sweeps' id checker):
 * tx t's leaves are [tx_leaf_off[t], tx_leaf_off[t+1]) of the leaf CSR;
 * status[t] = 0, or 6 (CORDAHIP_TX_NO_LEAVES) for a transaction without
 * leaves (MerkleTreeException, MerkleTree.kt:49-50), its id left zero. */
#include <pthread.h>

typedef struct {
  size_t lo, hi;
  const uint8_t* leaf_bytes;
  const uint64_t* leaf_off;
  const uint64_t* tx_leaf_off;
  uint8_t* ids;
  uint8_t* status;
} txid_job_t;

static void* txid_worker(void* p) {
  txid_job_t* j = (txid_job_t*)p;
  for (size_t t = j->lo; t < j->hi; t++) {
    const uint64_t a = j->tx_leaf_off[t], b = j->tx_leaf_off[t + 1];
    memset(j->ids + 32 * t, 0, 32);
    const int rc = oracle_tx_id(j->leaf_bytes, j->leaf_off + a, (size_t)(b - a), j->ids + 32 * t);
    j->status[t] = rc == 0 ? 0 : 6;
  }
  return NULL;
}

void oracle_tx_id_batch(size_t ntx, const uint8_t* leaf_bytes, const uint64_t* leaf_off, const uint64_t* tx_leaf_off,
                        uint8_t* ids, uint8_t* status, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  txid_job_t jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (txid_job_t){ntx * t / nthreads, ntx * (t + 1) / nthreads, leaf_bytes, leaf_off, tx_leaf_off, ids, status};
    pthread_create(&th[t], NULL, txid_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}
