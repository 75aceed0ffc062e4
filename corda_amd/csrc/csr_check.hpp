// CSR validation at the C-ABI (ABI 4). Every offset array the host code indexes
// is checked before the host reads through it: offsets non-decreasing, the last
// one within the buffer length the caller declares, consecutive levels
// consistent (a transaction's leaves / items / signatures are ranges of the next
// level's arrays). A violation is CORDAHIP_ERR_INVALID_ARG, never a read outside
// the caller's buffers -- the reference turns bad input into an exception, not a
// crash (Crypto.kt:472-483, SignedTransaction.kt:37-39).
// The transaction-level batches are checked whole before any enqueue
// (check_txid_batch ...: a parallel pass over their offset arrays); the generic
// signature batch's per-lane offsets are checked in the classification pass
// that reads them anyway (pack_rows.hpp classify: a chunk with a bad lane is
// neither packed nor enqueued, the batch fails). No HIP here: tools/csr_fuzz.cpp
// runs this code and the per-lane classify/pack under ASan/UBSan on the CPU.
#pragma once
#include <stdint.h>

#include <atomic>

#include "../../include/cordahip.h"

namespace cordahip {
namespace rt {

// off[a..b] non-decreasing and off[b] <= limit. par(n, grain, fn(lo, hi)) runs
// fn over [0, n) in pieces (the context's host pool, or a serial loop).
template <class Par>
bool csr_ok(Par&& par, const uint64_t* off, uint64_t a, uint64_t b, uint64_t limit) {
  if (b < a || !off) return false;
  if (off[b] > limit) return false;
  std::atomic<bool> ok{true};
  par(b - a, 1u << 16, [&](uint64_t x, uint64_t y) {
    for (uint64_t i = a + x; i < a + y; i++)
      if (off[i] > off[i + 1]) {
        ok.store(false, std::memory_order_relaxed);
        return;
      }
  });
  return ok.load();
}

// the leaf level of a txid batch: tx_leaf_off[0..ntx] non-decreasing and within
// nleaves, and the leaves it spans inside leaf_bytes (leaf_off over them
// non-decreasing, the last <= leaf_bytes_len)
template <class Par>
bool check_txid_batch(Par&& par, const cordahip_txid_batch* b) {
  if (b->ntx == 0) return true;
  if (!b->tx_leaf_off || !b->leaf_off) return false;
  if (!csr_ok(par, b->tx_leaf_off, 0, b->ntx, b->nleaves)) return false;
  return csr_ok(par, b->leaf_off, b->tx_leaf_off[0], b->tx_leaf_off[b->ntx], b->leaf_bytes_len);
}

// the signature level of a signed-tx batch: tx_sig_off[0..ntx] non-decreasing and
// within nsig; key_off / sig_off over the signatures it spans inside key_bytes /
// sig_bytes (the per-lane classification checks them again as it reads them)
template <class Par>
bool check_sig_level(Par&& par, uint64_t ntx, const uint64_t* tx_sig_off, uint64_t nsig, const uint64_t* key_off,
                     uint64_t key_bytes, const uint64_t* sig_off, uint64_t sig_bytes) {
  if (ntx == 0) return true;
  if (!tx_sig_off || !csr_ok(par, tx_sig_off, 0, ntx, nsig)) return false;
  const uint64_t s0 = tx_sig_off[0], s1 = tx_sig_off[ntx];
  if (s0 == s1) return true;
  return csr_ok(par, key_off, s0, s1, key_bytes) && csr_ok(par, sig_off, s0, s1, sig_bytes);
}

// the item level of a component batch: tx_item_off[0..ntx] non-decreasing and
// within n_items (payload offsets are bounds-checked per item by the encoder)
template <class Par>
bool check_txcomp_batch(Par&& par, const cordahip_txcomp_batch* c) {
  if (c->ntx == 0) return true;
  return c->tx_item_off && csr_ok(par, c->tx_item_off, 0, c->ntx, c->n_items);
}

// a filtered-tx batch: the leaf level as in check_txid_batch, the token level
// tx_tok_off[0..ntx] non-decreasing and within ntok
template <class Par>
bool check_filtered_batch(Par&& par, const cordahip_filtered_tx_batch* b) {
  if (b->ntx == 0) return true;
  if (!b->tx_leaf_off || !b->leaf_off || !b->tx_tok_off) return false;
  if (!csr_ok(par, b->tx_leaf_off, 0, b->ntx, b->nleaves)) return false;
  if (!csr_ok(par, b->leaf_off, b->tx_leaf_off[0], b->tx_leaf_off[b->ntx], b->leaf_bytes_len)) return false;
  return csr_ok(par, b->tx_tok_off, 0, b->ntx, b->ntok);
}

}  // namespace rt
}  // namespace cordahip
