// Host batches: the generic CSR signature batch (cordahip_sig_verify /
// cordahip_sig_submit -- the Crypto.isValid / Crypto.doVerify boundary,
// Crypto.kt:472-483,534-541, one call per BATCH instead of one JCA call per
// signature at Crypto.kt:537-540) and dense Ed25519 rows in host memory
// (cordahip_ed25519_verify_host).
//
// Shape, MI355X-first:
//  1. classify every lane on the host pool (parallel counting sort, no per-lane
//     map): direct statuses (UNSUPPORTED, key-length BAD_KEY), one lane list per
//     Ed25519 message length, one ECDSA lane list (both curves: the kernels
//     partition by curve on the device);
//  2. shard every list over the context devices (cordahip_shard_range: contiguous,
//     64-aligned); per device, the Ed25519 and ECDSA sections run at once, each a
//     pipeline over kPackStages stages: the host pool packs chunk k into a stage's
//     pinned buffers (dense rows / 65- and 72-byte slots, 16-B aligned) while the
//     GPU verifies chunks k-1, k-2 and PCIe carries their inputs and statuses;
//     when a stage comes round again its statuses are scattered back to the
//     caller's lanes. H2D on the device's copy stream, each section's kernels and
//     status D2H on its own stream (ECDSA at high priority), as in the C5 drain;
//  3. verdict words from the statuses.
// The caller's buffers may be pageable: every PCIe transfer is from/to pinned
// staging. Per-lane rules are those of the reference call chain (see
// include/cordahip.h): key length before scheme engine checks before DER/length
// before the math.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <future>

#include "der.hpp"
#include "runtime.hpp"
#include "status.hpp"

namespace cordahip {
namespace rt {
namespace {

// lanes per chunk: Ed25519 rows 2^22 (launches of 2^22 lose ~1% to grid tails
// against one 2^24 launch, C2 measured), ECDSA slots 2^21
constexpr uint64_t kEdChunk = 1ull << 22;
constexpr uint64_t kEcChunk = 1ull << 21;
constexpr uint64_t kGrain = 1ull << 14;  // lanes per packing piece

uint64_t chunk_lanes(const char* env, uint64_t dflt) {
  const uint64_t v = env_lanes(env, 0);
  return v ? v : dflt;
}

// A contiguous slice [lo, hi) of a lane list (lanes == nullptr: the identity)
struct Unit {
  const uint64_t* lanes = nullptr;
  uint64_t lo = 0, hi = 0;
  uint32_t mlen = 0;  // Ed25519 units: the message length of every lane
};

// Chunks [a, b) of the units' lanes: the section's first chunks ramp up
// (chunk/16, chunk/4, then chunk) so the GPU starts after a short first pack
// and copy instead of a whole chunk's.
struct Chunk {
  uint32_t unit;
  uint64_t a, b;
};
std::vector<Chunk> make_chunks(const std::vector<Unit>& units, uint64_t chunk) {
  std::vector<Chunk> out;
  int k = 0;
  for (uint32_t u = 0; u < units.size(); u++)
    for (uint64_t a = units[u].lo; a < units[u].hi; k++) {
      const uint64_t sz = std::max<uint64_t>(64, k == 0 ? chunk / 16 : k == 1 ? chunk / 4 : chunk);
      const uint64_t b = std::min(units[u].hi, a + sz);
      out.push_back({u, a, b});
      a = b;
    }
  return out;
}

// ---- the two sources of Ed25519 rows --------------------------------------------
struct CsrEdSource {  // lanes of a cordahip_sig_batch
  const cordahip_sig_batch* b;
  bool do_verify;
  void pack(const Unit& u, uint64_t a, uint64_t b0, uint64_t b1, uint8_t* keys, uint8_t* sigs, uint8_t* msgs,
            uint8_t* pre) const {
    const uint32_t L = u.mlen;
    for (uint64_t p = b0; p < b1; p++) {
      const uint64_t i = u.lanes[p], r = p - a;
      std::memcpy(keys + r * 32, b->key + b->key_off[i], 32);
      const uint64_t sl = b->sig_off[i + 1] - b->sig_off[i];
      uint8_t st = CORDAHIP_STATUS_OK;
      if (do_verify && (sl == 0 || L == 0)) st = CORDAHIP_STATUS_EMPTY;  // Crypto.kt:475-476
      else if (sl != 64) st = CORDAHIP_STATUS_MALFORMED_SIG;           // EdDSAEngine: signature length
      if (st == CORDAHIP_STATUS_OK) std::memcpy(sigs + r * 64, b->sig + b->sig_off[i], 64);
      else std::memset(sigs + r * 64, 0, 64);
      pre[r] = st;
      if (L == 32) std::memcpy(msgs + r * 32, b->msg + b->msg_off[i], 32);
      else if (L) std::memcpy(msgs + r * (uint64_t)L, b->msg + b->msg_off[i], L);
    }
  }
  void scatter(const Unit& u, uint64_t a, uint64_t b0, uint64_t b1, const uint8_t* st) const {
    for (uint64_t p = b0; p < b1; p++) b->status[u.lanes[p]] = st[p - a];
  }
};

struct DenseEdSource {  // cordahip_ed25519_verify_host rows
  const uint8_t *keys, *sigs, *msgs;
  uint8_t* status;
  void pack(const Unit& u, uint64_t a, uint64_t b0, uint64_t b1, uint8_t* k, uint8_t* s, uint8_t* m,
            uint8_t* pre) const {
    const uint64_t r = b0 - a, c = b1 - b0, L = u.mlen;
    std::memcpy(k + r * 32, keys + b0 * 32, c * 32);
    std::memcpy(s + r * 64, sigs + b0 * 64, c * 64);
    if (L) std::memcpy(m + r * L, msgs + b0 * L, c * L);
    std::memset(pre + r, 0, c);
  }
  void scatter(const Unit&, uint64_t a, uint64_t b0, uint64_t b1, const uint8_t* st) const {
    std::memcpy(status + b0, st + (b0 - a), b1 - b0);
  }
};

hipError_t ensure_events(PackStage* set) {
  for (int k = 0; k < kPackStages; k++)
    for (hipEvent_t* pe : {&set[k].copied, &set[k].done})
      if (!*pe && hipEventCreateWithFlags(pe, hipEventDisableTiming) != hipSuccess) return hipErrorUnknown;
  return hipSuccess;
}

// Ed25519 section of one device: stage buffers h/d[0] keys, [1] sigs, [2] msgs,
// [3] pre-status, [4] status.
template <class Src>
int ed_pipeline(cordahip_ctx* ctx, Device& d, const std::vector<Unit>& units, const Src& src, uint32_t flags) {
  const std::vector<Chunk> chunks = make_chunks(units, chunk_lanes("CORDAHIP_HOST_CHUNK", kEdChunk));
  if (chunks.empty()) return CORDAHIP_SUCCESS;
  std::lock_guard<std::mutex> g(d.ped_mu);
  if (hipSetDevice(d.id) != hipSuccess || ensure_streams(d) != hipSuccess || ensure_events(d.ped) != hipSuccess)
    return CORDAHIP_ERR_HIP;
  HostPool& pool = *ctx->host;
  auto finish = [&](PackStage& st) -> hipError_t {  // wait for a stage's chunk, scatter its statuses
    if (!st.pending) return hipSuccess;
    st.pending = false;
    hipError_t e = hipEventSynchronize(st.done);
    if (e != hipSuccess) return e;
    const Unit& u = units[st.tag0];
    const uint8_t* sts = st.h[4].as<uint8_t>();
    pool.parallel_for(st.tag2 - st.tag1, kGrain * 4, [&](uint64_t x, uint64_t y) {
      src.scatter(u, st.tag1, st.tag1 + x, st.tag1 + y, sts);
    });
    return hipSuccess;
  };
  hipError_t e = hipSuccess;
  int rc = CORDAHIP_SUCCESS;
  for (size_t k = 0; k < chunks.size() && e == hipSuccess && rc == CORDAHIP_SUCCESS; k++) {
    PackStage& st = d.ped[k % kPackStages];
    e = finish(st);
    if (e != hipSuccess) break;
    const Chunk& c = chunks[k];
    const Unit& u = units[c.unit];
    const uint64_t m = c.b - c.a, L = u.mlen;
    const size_t sz[5] = {m * 32, m * 64, std::max<uint64_t>(m * L, 16), m, m};
    for (int q = 0; q < 5; q++)
      if (st.h[q].ensure(sz[q]) != hipSuccess || st.d[q].ensure(sz[q]) != hipSuccess) rc = CORDAHIP_ERR_OUT_OF_MEMORY;
    if (rc != CORDAHIP_SUCCESS) break;
    uint8_t *hk = st.h[0].as<uint8_t>(), *hs = st.h[1].as<uint8_t>(), *hm = st.h[2].as<uint8_t>(),
            *hp = st.h[3].as<uint8_t>();
    pool.parallel_for(m, kGrain, [&](uint64_t x, uint64_t y) { src.pack(u, c.a, c.a + x, c.a + y, hk, hs, hm, hp); });
    for (int q = 0; q < 4; q++)
      if (q != 2 || L) e = e ? e : hipMemcpyAsync(st.d[q].p, st.h[q].p, q == 2 ? m * L : sz[q], hipMemcpyHostToDevice, d.s_copy);
    e = e ? e : hipEventRecord(st.copied, d.s_copy);
    e = e ? e : hipStreamWaitEvent(d.s_ed, st.copied, 0);
    e = e ? e
          : ed_verify_enqueue(d, st.d[0].as<uint8_t>(), st.d[1].as<uint8_t>(), st.d[2].as<uint8_t>(), (uint32_t)L, m,
                              st.d[3].as<uint8_t>(), st.d[4].as<uint8_t>(), nullptr, flags, d.s_ed);
    e = e ? e : hipMemcpyAsync(st.h[4].p, st.d[4].p, m, hipMemcpyDeviceToHost, d.s_ed);
    e = e ? e : hipEventRecord(st.done, d.s_ed);
    if (e == hipSuccess) {
      st.pending = true;
      st.tag0 = c.unit;
      st.tag1 = c.a;
      st.tag2 = c.b;
    }
  }
  // drain every stage even after an error, so no queued work outlives the call
  for (int k = 0; k < kPackStages; k++) {
    if (e == hipSuccess && rc == CORDAHIP_SUCCESS) e = finish(d.ped[k]);
    d.ped[k].pending = false;
  }
  const hipError_t e1 = hipStreamSynchronize(d.s_copy), e2 = hipStreamSynchronize(d.s_ed);
  if (rc != CORDAHIP_SUCCESS) return rc;
  return (e || e1 || e2) ? CORDAHIP_ERR_HIP : CORDAHIP_SUCCESS;
}

// ECDSA section of one device (lanes of a cordahip_sig_batch): slot layout of
// the K2 kernels. Stage buffers h/d[0] scheme, [1] keys (65-B slots), [2]
// key_len, [3] sigs (72-B slots), [4] sig_len, [5] msgs (CSR bytes), [6]
// msg_off (chunk-relative), [7] pre-status, [8] status.
int ec_pipeline(cordahip_ctx* ctx, Device& d, const Unit& unit, const cordahip_sig_batch* b) {
  const std::vector<Unit> units{unit};
  const std::vector<Chunk> chunks = make_chunks(units, chunk_lanes("CORDAHIP_HOST_EC_CHUNK", kEcChunk));
  if (chunks.empty()) return CORDAHIP_SUCCESS;
  const bool do_verify = !(b->flags & CORDAHIP_FLAG_IS_VALID);
  std::lock_guard<std::mutex> g(d.pec_mu);
  if (hipSetDevice(d.id) != hipSuccess || ensure_streams(d) != hipSuccess || ensure_events(d.pec) != hipSuccess)
    return CORDAHIP_ERR_HIP;
  HostPool& pool = *ctx->host;
  const uint64_t* lanes = unit.lanes;
  auto finish = [&](PackStage& st) -> hipError_t {
    if (!st.pending) return hipSuccess;
    st.pending = false;
    hipError_t e = hipEventSynchronize(st.done);
    if (e != hipSuccess) return e;
    const uint8_t* sts = st.h[8].as<uint8_t>();
    const uint64_t a = st.tag1;
    pool.parallel_for(st.tag2 - a, kGrain * 4, [&](uint64_t x, uint64_t y) {
      for (uint64_t p = a + x; p < a + y; p++) b->status[lanes[p]] = sts[p - a];
    });
    return hipSuccess;
  };
  hipError_t e = hipSuccess;
  int rc = CORDAHIP_SUCCESS;
  std::vector<uint64_t> piece_bytes;
  for (size_t k = 0; k < chunks.size() && e == hipSuccess && rc == CORDAHIP_SUCCESS; k++) {
    PackStage& st = d.pec[k % kPackStages];
    e = finish(st);
    if (e != hipSuccess) break;
    const Chunk& c = chunks[k];
    const uint64_t m = c.b - c.a;
    // message bytes per piece (fixed pieces), then their prefix: each piece
    // packs its messages at its own offset
    const uint64_t npiece = (m + kGrain - 1) / kGrain;
    piece_bytes.assign(npiece + 1, 0);
    pool.parallel_for(npiece, 1, [&](uint64_t x, uint64_t y) {
      for (uint64_t q = x; q < y; q++) {
        uint64_t t = 0;
        for (uint64_t p = c.a + q * kGrain; p < std::min(c.b, c.a + (q + 1) * kGrain); p++)
          t += b->msg_off[lanes[p] + 1] - b->msg_off[lanes[p]];
        piece_bytes[q + 1] = t;
      }
    });
    for (uint64_t q = 0; q < npiece; q++) piece_bytes[q + 1] += piece_bytes[q];
    const uint64_t mbytes = piece_bytes[npiece];
    const size_t sz[9] = {m, m * 65, m, m * 72, m, std::max<uint64_t>(mbytes, 16), (m + 1) * 8, m, m};
    for (int q = 0; q < 9; q++)
      if (st.h[q].ensure(sz[q]) != hipSuccess || st.d[q].ensure(sz[q]) != hipSuccess) rc = CORDAHIP_ERR_OUT_OF_MEMORY;
    if (rc != CORDAHIP_SUCCESS) break;
    uint8_t *hsc = st.h[0].as<uint8_t>(), *hk = st.h[1].as<uint8_t>(), *hkl = st.h[2].as<uint8_t>(),
            *hs = st.h[3].as<uint8_t>(), *hsl = st.h[4].as<uint8_t>(), *hm = st.h[5].as<uint8_t>(),
            *hp = st.h[7].as<uint8_t>();
    uint64_t* hmo = st.h[6].as<uint64_t>();
    pool.parallel_for(npiece, 1, [&](uint64_t x, uint64_t y) {
      for (uint64_t q = x; q < y; q++) {
        uint64_t mo = piece_bytes[q];
        for (uint64_t p = c.a + q * kGrain; p < std::min(c.b, c.a + (q + 1) * kGrain); p++) {
          const uint64_t i = lanes[p], r = p - c.a;
          hsc[r] = b->scheme[i];
          const uint64_t kl = b->key_off[i + 1] - b->key_off[i];  // 33 or 65 (classified)
          std::memcpy(hk + r * 65, b->key + b->key_off[i], kl);
          std::memset(hk + r * 65 + kl, 0, 65 - kl);
          hkl[r] = (uint8_t)kl;
          const uint64_t sl = b->sig_off[i + 1] - b->sig_off[i];
          const uint64_t ml = b->msg_off[i + 1] - b->msg_off[i];
          uint8_t pre = CORDAHIP_STATUS_OK;
          if (sl <= 72) {
            std::memcpy(hs + r * 72, b->sig + b->sig_off[i], sl);
            std::memset(hs + r * 72 + sl, 0, 72 - sl);
            hsl[r] = (uint8_t)sl;
          } else {
            // longer than the slot: no r, s < n fits, so the DER rules alone
            // decide (BC: well-formed -> false, else SignatureException); the
            // kernel still decodes the key first, so key errors keep precedence
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
          std::memcpy(hm + mo, b->msg + b->msg_off[i], ml);
          mo += ml;
        }
      }
    });
    hmo[m] = mbytes;
    const size_t bytes[8] = {m, m * 65, m, m * 72, m, mbytes, (m + 1) * 8, m};
    for (int q = 0; q < 8; q++)
      if (bytes[q]) e = e ? e : hipMemcpyAsync(st.d[q].p, st.h[q].p, bytes[q], hipMemcpyHostToDevice, d.s_copy);
    e = e ? e : hipEventRecord(st.copied, d.s_copy);
    e = e ? e : hipStreamWaitEvent(d.s_ec, st.copied, 0);
    if (e == hipSuccess) {
      std::lock_guard<std::mutex> ge(d.ec_mu);
      e = ec_verify_enqueue(d, st.d[0].as<uint8_t>(), st.d[1].as<uint8_t>(), st.d[2].as<uint8_t>(),
                            st.d[3].as<uint8_t>(), st.d[4].as<uint8_t>(), st.d[5].as<uint8_t>(),
                            st.d[6].as<uint64_t>(), 0, m, st.d[7].as<uint8_t>(), st.d[8].as<uint8_t>(), nullptr,
                            b->flags, d.s_ec);
    }
    e = e ? e : hipMemcpyAsync(st.h[8].p, st.d[8].p, m, hipMemcpyDeviceToHost, d.s_ec);
    e = e ? e : hipEventRecord(st.done, d.s_ec);
    if (e == hipSuccess) {
      st.pending = true;
      st.tag1 = c.a;
      st.tag2 = c.b;
    }
  }
  for (int k = 0; k < kPackStages; k++) {
    if (e == hipSuccess && rc == CORDAHIP_SUCCESS) e = finish(d.pec[k]);
    d.pec[k].pending = false;
  }
  const hipError_t e1 = hipStreamSynchronize(d.s_copy), e2 = hipStreamSynchronize(d.s_ec);
  if (rc != CORDAHIP_SUCCESS) return rc;
  return (e || e1 || e2) ? CORDAHIP_ERR_HIP : CORDAHIP_SUCCESS;
}

// Lane classes of a generic batch.
enum : uint8_t { kDirect = 0, kEd = 1, kEc = 2 };

inline uint8_t classify(const cordahip_sig_batch* b, uint64_t i, uint64_t& mlen) {
  const uint8_t sch = b->scheme[i];
  const uint64_t kl = b->key_off[i + 1] - b->key_off[i];
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
  mlen = b->msg_off[i + 1] - b->msg_off[i];
  return kEd;
}

}  // namespace

void verdict_from_status(cordahip_ctx* ctx, const uint8_t* status, uint64_t n, uint64_t* verdict) {
  ctx->host->parallel_for((n + 63) / 64, 1024, [&](uint64_t w0, uint64_t w1) {
    for (uint64_t w = w0; w < w1; w++) {
      uint64_t m = 0;
      for (uint64_t b = 0; b < 64 && w * 64 + b < n; b++)
        if (status[w * 64 + b] == CORDAHIP_STATUS_OK) m |= 1ull << b;
      verdict[w] = m;
    }
  });
}

int sig_verify_impl(cordahip_ctx* ctx, const cordahip_sig_batch* b) {
  const uint64_t n = b->n;
  if (n == 0) return CORDAHIP_SUCCESS;
  if (!b->scheme || !b->key || !b->key_off || !b->sig || !b->sig_off || !b->msg || !b->msg_off || !b->status ||
      (b->flags & ~CORDAHIP_FLAG_IS_VALID))
    return CORDAHIP_ERR_INVALID_ARG;
  HostPool& pool = *ctx->host;
  // 1. classification: fixed pieces, two passes (count, then place) = a stable
  // counting sort of the lanes into one list per Ed25519 message length + ECDSA
  const uint64_t piece = std::max<uint64_t>(kGrain, (n + 8 * pool.threads() - 1) / (8 * pool.threads()));
  const uint64_t npiece = (n + piece - 1) / piece;
  struct PieceCount {
    std::vector<std::pair<uint64_t, uint64_t>> ed;  // (message length, lanes)
    uint64_t ec = 0;
    bool too_long = false;
  };
  std::vector<PieceCount> pc(npiece);
  pool.parallel_for(npiece, 1, [&](uint64_t x, uint64_t y) {
    for (uint64_t q = x; q < y; q++) {
      PieceCount& c = pc[q];
      for (uint64_t i = q * piece; i < std::min(n, (q + 1) * piece); i++) {
        uint64_t mlen = 0;
        const uint8_t cls = classify(b, i, mlen);
        if (cls == kEc) {
          c.ec++;
        } else if (cls == kEd) {
          if (mlen > 0xffffffffull) c.too_long = true;
          size_t k = 0;
          while (k < c.ed.size() && c.ed[k].first != mlen) k++;
          if (k == c.ed.size()) c.ed.push_back({mlen, 0});
          c.ed[k].second++;
        }
      }
    }
  });
  std::vector<uint64_t> lens;
  uint64_t n_ec = 0;
  for (const PieceCount& c : pc) {
    if (c.too_long) return CORDAHIP_ERR_INVALID_ARG;
    for (const auto& kv : c.ed) lens.push_back(kv.first);
    n_ec += c.ec;
  }
  std::sort(lens.begin(), lens.end());
  lens.erase(std::unique(lens.begin(), lens.end()), lens.end());
  const size_t ng = lens.size();
  // start[g][q]: where piece q's lanes of group g go; group ng = ECDSA
  std::vector<std::vector<uint64_t>> start(ng + 1, std::vector<uint64_t>(npiece + 1, 0));
  for (uint64_t q = 0; q < npiece; q++) {
    for (size_t g = 0; g < ng; g++) {
      uint64_t cnt = 0;
      for (const auto& kv : pc[q].ed)
        if (kv.first == lens[g]) cnt = kv.second;
      start[g][q + 1] = start[g][q] + cnt;
    }
    start[ng][q + 1] = start[ng][q] + pc[q].ec;
  }
  std::vector<std::vector<uint64_t>> lists(ng + 1);
  for (size_t g = 0; g <= ng; g++) lists[g].resize(start[g][npiece]);
  pool.parallel_for(npiece, 1, [&](uint64_t x, uint64_t y) {
    std::vector<uint64_t> pos(ng + 1);
    for (uint64_t q = x; q < y; q++) {
      for (size_t g = 0; g <= ng; g++) pos[g] = start[g][q];
      for (uint64_t i = q * piece; i < std::min(n, (q + 1) * piece); i++) {
        uint64_t mlen = 0;
        const uint8_t cls = classify(b, i, mlen);
        if (cls == kEc) {
          lists[ng][pos[ng]++] = i;
        } else if (cls == kEd) {
          const size_t g = std::lower_bound(lens.begin(), lens.end(), mlen) - lens.begin();
          lists[g][pos[g]++] = i;
        }
      }
    }
  });
  (void)n_ec;
  // 2. per device: its shard of every list; Ed25519 and ECDSA sections at once
  const bool do_verify = !(b->flags & CORDAHIP_FLAG_IS_VALID);
  const CsrEdSource src{b, do_verify};
  const uint64_t nd = ctx->devs.size();
  std::vector<std::future<int>> fs;
  for (uint64_t di = 0; di < nd; di++) {
    std::vector<Unit> eu;
    for (size_t g = 0; g < ng; g++) {
      Unit u;
      u.lanes = lists[g].data();
      shard_range(lists[g].size(), nd, di, 64, u.lo, u.hi);
      u.mlen = (uint32_t)lens[g];
      if (u.lo < u.hi) eu.push_back(u);
    }
    Unit cu;
    cu.lanes = lists[ng].data();
    shard_range(lists[ng].size(), nd, di, 64, cu.lo, cu.hi);
    Device* d = ctx->devs[di].get();
    if (cu.lo < cu.hi) fs.push_back(std::async(std::launch::async, [=] { return ec_pipeline(ctx, *d, cu, b); }));
    if (!eu.empty())
      fs.push_back(std::async(std::launch::async,
                              [=, &src] { return ed_pipeline(ctx, *d, eu, src, b->flags); }));
  }
  int rc = CORDAHIP_SUCCESS;
  for (auto& f : fs) {
    const int r = f.get();
    if (r != CORDAHIP_SUCCESS && rc == CORDAHIP_SUCCESS) rc = r;
  }
  if (rc != CORDAHIP_SUCCESS) return rc;
  // 3. verdict words
  if (b->verdict) verdict_from_status(ctx, b->status, n, b->verdict);
  return CORDAHIP_SUCCESS;
}

int ed25519_dense_host(cordahip_ctx* ctx, const uint8_t* keys, const uint8_t* sigs, const uint8_t* msgs,
                       uint32_t msg_len, uint64_t n, uint8_t* status, uint64_t* verdict) {
  if (n == 0) return CORDAHIP_SUCCESS;
  const DenseEdSource src{keys, sigs, msgs, status};
  // contiguous 64-aligned shards: no cross-device dependency
  const int rc = for_shards(ctx->devs, n, 64, [&](Device& d, uint64_t lo, uint64_t hi) {
    Unit u;
    u.lo = lo;
    u.hi = hi;
    u.mlen = msg_len;
    return ed_pipeline(ctx, d, std::vector<Unit>{u}, src, 0u);
  });
  if (rc == CORDAHIP_SUCCESS && verdict) verdict_from_status(ctx, status, n, verdict);
  return rc;
}

}  // namespace rt
}  // namespace cordahip
