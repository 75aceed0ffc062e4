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
