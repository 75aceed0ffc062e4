// Per-lane classification and row packing of generic signature batches
// (cordahip_sig_batch, the Crypto.isValid / doVerify batch of Crypto.kt:472-541):
// the host side of host_batch.cpp's pipelines, in a header of its own so that
// tools/pack_bench.cpp measures exactly this code on the CPU (the host budget
// of one process driving several GPUs). No HIP here.
//
// MV is the message view (runtime.hpp MsgView): len(i), ptr(i).
#pragma once
#include <stdint.h>

#include <cstring>

#include "../../include/cordahip.h"
#include "der.hpp"

namespace cordahip {
namespace rt {

// ---- the two sources of Ed25519 rows --------------------------------------------
// Ed25519 row of lane i of a cordahip_sig_batch (message length L): the
// Crypto.doVerify require()s and the engine's length check as the pre-status
template <class MV>
inline void pack_ed_row(const cordahip_sig_batch* b, const MV& mv, bool do_verify, uint64_t i, uint32_t L,
                        uint8_t* key, uint8_t* sig, uint8_t* msg, uint8_t* pre) {
  std::memcpy(key, b->key + b->key_off[i], 32);
  const uint64_t sl = b->sig_off[i + 1] - b->sig_off[i];
  uint8_t st = CORDAHIP_STATUS_OK;
  if (do_verify && (sl == 0 || L == 0)) st = CORDAHIP_STATUS_EMPTY;  // Crypto.kt:475-476
  else if (sl != 64) st = CORDAHIP_STATUS_MALFORMED_SIG;           // EdDSAEngine: signature length
  if (st == CORDAHIP_STATUS_OK) std::memcpy(sig, b->sig + b->sig_off[i], 64);
  else std::memset(sig, 0, 64);
  *pre = st;
  if (!msg) return;  // device-side message (MsgView::dev): gathered on the GPU
  if (L == 32) std::memcpy(msg, mv.ptr(i), 32);
  else if (L) std::memcpy(msg, mv.ptr(i), L);
}

// Lane classes of a generic batch: the per-lane checks that precede the
// engines (statuses decided here are written at once). kBadCsr: the lane's CSR
// ranges are not inside the batch's buffers (csr_check.hpp: the batch fails with
// CORDAHIP_ERR_INVALID_ARG before its chunk is packed).
enum : uint16_t { kDirect = 0, kEc = 1, kEdBase = 2, kBadCsr = 0xffff };

template <class MV>
inline uint16_t classify(const cordahip_sig_batch* b, const MV& mv, uint64_t i, uint64_t& mlen) {
  // the lane's ranges first, before any byte of it is read: non-decreasing and inside
  // the declared buffers (key_off[i + 1] <= key_bytes, ...; messages of a signed-tx
  // batch are its transactions' ids, checked with the transactions)
  const uint64_t k0 = b->key_off[i], k1 = b->key_off[i + 1], s0 = b->sig_off[i], s1 = b->sig_off[i + 1];
  mlen = 0;
  if (k1 < k0 || k1 > b->key_bytes || s1 < s0 || s1 > b->sig_bytes) return kBadCsr;
  if (!mv.tx_of && (mv.off[i + 1] < mv.off[i] || mv.off[i + 1] > b->msg_bytes)) return kBadCsr;
  const uint8_t sch = b->scheme[i];
  const uint64_t kl = k1 - k0;
  mlen = mv.len(i);
  if (sch == CORDAHIP_SCHEME_ECDSA_SECP256K1_SHA256 || sch == CORDAHIP_SCHEME_ECDSA_SECP256R1_SHA256) {
    if (kl != 33 && kl != 65) {
      b->status[i] = CORDAHIP_STATUS_BAD_KEY;  // ECCurve.decodePoint: invalid point encoding
      return kDirect;
    }
    return kEc;
  }
  if (sch != CORDAHIP_SCHEME_EDDSA_ED25519_SHA512) {
    b->status[i] = CORDAHIP_STATUS_UNSUPPORTED;  // Crypto.kt:474 require(isSupportedSignatureScheme)
    return kDirect;
  }
  if (kl != 32) {
    b->status[i] = CORDAHIP_STATUS_BAD_KEY;  // EdDSAPublicKeySpec: "public-key length is wrong"
    return kDirect;
  }
  return kEdBase;  // + the piece-local message-length group
}

// ECDSA slot packing of lane i into row r (messages CSR at *mo)
template <class MV>
inline void pack_ec_row(const cordahip_sig_batch* b, const MV& mv, bool do_verify, uint64_t i, uint64_t r, uint8_t* hsc, uint8_t* hk,
                        uint8_t* hkl, uint8_t* hs, uint8_t* hsl, uint8_t* hm, uint64_t* hmo, uint8_t* hp,
                        uint64_t& mo, uint32_t* hidx, uint64_t t0 = 0) {
  hsc[r] = b->scheme[i];
  const uint64_t kl = b->key_off[i + 1] - b->key_off[i];  // 33 or 65 (classified)
  std::memcpy(hk + r * 65, b->key + b->key_off[i], kl);
  std::memset(hk + r * 65 + kl, 0, 65 - kl);
  hkl[r] = (uint8_t)kl;
  const uint64_t sl = b->sig_off[i + 1] - b->sig_off[i];
  const uint64_t ml = mv.len(i);
  uint8_t pre = CORDAHIP_STATUS_OK;
  if (sl <= 72) {
    std::memcpy(hs + r * 72, b->sig + b->sig_off[i], sl);
    std::memset(hs + r * 72 + sl, 0, 72 - sl);
    hsl[r] = (uint8_t)sl;
  } else {
    // longer than the slot: no r, s < n fits, so the DER rules alone decide (BC:
    // well-formed -> false, else SignatureException); the kernel still decodes
    // the key first, so key errors keep precedence
    DerInt dr, ds;
    pre = (ml == 0 && do_verify) ? CORDAHIP_STATUS_EMPTY
          : der_decode_sig(b->sig + b->sig_off[i], (uint32_t)std::min<uint64_t>(sl, 0xffffffffu), dr, ds)
              ? CORDAHIP_STATUS_BAD_SIG
              : CORDAHIP_STATUS_MALFORMED_SIG;
    std::memset(hs + r * 72, 0, 72);
    hsl[r] = 72;
  }
  hp[r] = pre;
  hmo[r] = mo;
  if (hidx) hidx[r] = (uint32_t)(mv.tx_of[i] - t0);  // the row is gathered on the device
  else std::memcpy(hm + mo, mv.ptr(i), ml);
  mo += ml;
}

}  // namespace rt
}  // namespace cordahip
