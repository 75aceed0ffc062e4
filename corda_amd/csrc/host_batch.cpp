// Host batches: the generic CSR signature batch (cordahip_sig_verify /
// cordahip_sig_submit -- the Crypto.isValid / Crypto.doVerify boundary,
// Crypto.kt:472-483,534-541, one call per BATCH instead of one JCA call per
// signature at Crypto.kt:537-540) and dense Ed25519 rows in host memory
// (cordahip_ed25519_verify_host).
//
// Shape, MI355X-first: the batch is split into contiguous 64-aligned input
// shards, one per context device (cordahip_shard_range); each device streams
// its shard in chunks through kPackStages stages. Per chunk the host pool
// classifies every lane (the checks that precede the engines, written as
// statuses at once; Ed25519 lanes grouped by message length; ECDSA lanes, both
// curves: the kernels partition by curve on the device) and packs it straight
// into its row of the stage's pinned buffers (dense 32/64-byte rows, 65/72-byte
// ECDSA slots, CSR messages), while the GPU verifies the previous chunks and
// PCIe carries their inputs and statuses. H2D on the device's copy stream, the
// Ed25519 launches and the ECDSA launch on their own streams (beside each
// other, ECDSA at high priority) as in the C5 drain; when a stage comes round
// again its statuses go back to the caller's lanes. Verdict words last.
// The caller's buffers may be pageable: every PCIe transfer is from/to pinned
// staging. Per-lane rules are those of the reference call chain (see
// include/cordahip.h): key length before scheme engine checks before DER/length
// before the math.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <unordered_map>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>

#include "der.hpp"
#include "pack_rows.hpp"
#include "runtime.hpp"
#include "status.hpp"

namespace cordahip {
namespace rt {
namespace {

// lanes per chunk after the ramp (chunk/16, chunk/4, chunk): 2^22. The host
// packs ~6x (Ed25519) / ~3.5x (ECDSA) faster than the GPU verifies, and PCIe
// carries ~3x the GPU's rate (profiles/r03_trace_*_host.txt, CORDAHIP_TRACE),
// so a x4 ramp keeps the GPU fed from a short first pack. 2^23-lane chunks
// measured worse (c2h 87.6 vs 92.7 M/s, profiles/r03_bench_c2h_chunk23.json):
// the 1.1 GB H2D of the first big chunk can no longer hide behind the 2^21-lane
// chunk before it. Pinned staging: ~0.55 GB per stage for Ed25519 rows, ~0.75
// GB for ECDSA slots (grow-only, 3 stages).
constexpr uint64_t kEdChunk = 1ull << 22;
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

// Chunks [a, b) of the units' lanes: the first chunk is chunk/16 lanes so the
// GPU starts after a short first pack and copy, and each next one is up to 4x
// the previous, to at most 4 x chunk (2^18, 2^20, 2^22, 2^24 by default): the
// host packs a chunk (copy groups overlapping PCIe) ~4x faster than the GPU
// verifies the one before it, and fewer, larger launches pay fewer end-of-grid
// tails (C2 through cordahip_sig_verify ran 6 launch pairs of 2^18..2^22 lanes
// at 158.6 ms of kernels per 2^24 lanes against 153 for one launch pair,
// profiles/r04_b trace).
struct Chunk {
  uint32_t unit;
  uint64_t a, b;
};
std::vector<Chunk> make_chunks(const std::vector<Unit>& units, uint64_t chunk) {
  std::vector<Chunk> out;
  // chunk/16, chunk/4, then chunk lanes: `chunk` (CORDAHIP_HOST_CHUNK) is the
  // largest chunk, which sizes the pinned stages and the workspace slots
  const uint64_t top = std::max<uint64_t>(64, chunk / 64 * 64);
  uint64_t sz = std::max<uint64_t>(64, chunk / 16 / 64 * 64);  // multiples of 64: chunks start word-aligned
  for (uint32_t u = 0; u < units.size(); u++)
    for (uint64_t a = units[u].lo; a < units[u].hi;) {
      const uint64_t b = std::min(units[u].hi, a + sz);
      out.push_back({u, a, b});
      a = b;
      sz = std::min<uint64_t>(top, 4 * sz);
    }
  return out;
}

// ---- dense Ed25519 rows in host memory -------------------------------------------
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
  const NodeBind nb(d);  // packing and the pinned stages' first touch on the GPU's NUMA node
  const Activity act(d);
  if (hipSetDevice(d.id) != hipSuccess || ensure_streams(d) != hipSuccess || ensure_events(d.ped) != hipSuccess)
    return CORDAHIP_ERR_HIP;
  HostPool& pool = pool_of(ctx, d);
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

// Per-piece results of the classification pass of one chunk.
struct PieceInfo {
  std::vector<std::pair<uint64_t, uint64_t>> ed;  // (message length, lanes), piece-local group order
  std::vector<uint32_t> ed_global;               // piece-local group -> chunk group
  uint64_t ec = 0, ec_bytes = 0;                 // ECDSA lanes and their message bytes
  bool too_long = false;
  bool bad_csr = false;                          // a lane's CSR ranges outside the batch's buffers
};

// One device's input shard [lo, hi) of a generic batch, streamed in chunks
// through kPackStages BatchStages (signed-tx signature chunks: kTxStages). Per chunk, on the host pool: (1) classify
// every lane (direct statuses written now; Ed25519 lanes grouped by message
// length; ECDSA lanes) into per-lane class codes and per-piece counts, (2) pack
// every lane straight into its row: Ed25519 rows group after group (each
// group's messages at a 16-B aligned offset, one kernel launch per group),
// ECDSA rows in lane order with CSR messages. Then H2D on the copy stream, the
// Ed25519 launches on s_ed and the ECDSA launch on s_ec (beside each other),
// status D2H on each section's stream. Classification and packing of chunk k
// run while the GPU verifies chunks k-1 and k-2; a stage's statuses go back to
// the caller's lanes when the stage comes round again.
int sig_pipeline(cordahip_ctx* ctx, Device& d, TxSet& set, const cordahip_sig_batch* b, const MsgView& mv,
                 uint64_t lo, uint64_t hi) {
  if (lo >= hi) return CORDAHIP_SUCCESS;
  std::vector<Unit> units(1);
  units[0].lo = lo;
  units[0].hi = hi;
  std::vector<Chunk> chunks;
  const DeviceIds* dev = mv.dev;
  if (dev && !dev->chunk_bound.empty()) {  // signed-tx batches: chunk boundaries at id-slice boundaries
    for (size_t j = 0; j + 1 < dev->chunk_bound.size(); j++) {
      const uint64_t x = std::max(lo, dev->chunk_bound[j]), y = std::min(hi, dev->chunk_bound[j + 1]);
      if (x < y) chunks.push_back({0, x, y});
    }
  } else {
    chunks = make_chunks(units, mv.chunk ? mv.chunk : chunk_lanes("CORDAHIP_HOST_CHUNK", kEdChunk));
  }
  const bool do_verify = !(b->flags & CORDAHIP_FLAG_IS_VALID);
  const NodeBind nb(d);  // packing and the pinned stages' first touch on the GPU's NUMA node
  const Activity act(d);
  if (hipSetDevice(d.id) != hipSuccess || ensure_streams(d) != hipSuccess) return CORDAHIP_ERR_HIP;
  for (BatchStage& st : set.pb)
    for (hipEvent_t* pe : {&st.copied, &st.ed_done, &st.ec_done})
      if (!*pe && hipEventCreateWithFlags(pe, hipEventDisableTiming) != hipSuccess) return CORDAHIP_ERR_HIP;
  HostPool& pool = pool_of(ctx, d);
  // Chunks whose rows are the lanes in order (one message length, Ed25519 only:
  // the common JVM batch) skip the host scatter: a kernel stores the statuses
  // straight into the caller's status array and the wave-ballot verdict words
  // into its verdict array through their device mapping -- when those are
  // pinned; the last, largest chunk's scatter was the exposed tail of the call.
  uint8_t* dst_status = nullptr;
  uint64_t* dst_verdict = nullptr;
  if (!dev) {
    dst_status = static_cast<uint8_t*>(host_mapped(b->status));
    dst_verdict = b->verdict ? static_cast<uint64_t*>(host_mapped(b->verdict)) : nullptr;
  }
  const bool out_pinned = dst_status && (!b->verdict || dst_verdict);
  auto finish = [&](BatchStage& st) -> hipError_t {  // wait for the stage's chunk, scatter its statuses
    if (!st.pending) return hipSuccess;
    st.pending = false;
    hipError_t e = blocked("chunk verified", [&] { return hipEventSynchronize(st.ed_done); });
    e = e ? e : hipEventSynchronize(st.ec_done);
    if (e != hipSuccess) return e;
    if (st.direct) return hipSuccess;  // statuses and verdict words are already in the caller's arrays
    const uint8_t *se = st.h[4].as<uint8_t>(), *sc = st.h[13].as<uint8_t>();
    const uint64_t ne = st.ed_lanes.size(), nc = st.ec_lanes.size();
    pool.parallel_for(ne + nc, kGrain * 4, [&](uint64_t x, uint64_t y) {
      for (uint64_t r = x; r < y; r++) {
        if (r < ne) b->status[st.ed_lanes[r]] = se[r];
        else b->status[st.ec_lanes[r - ne]] = sc[r - ne];
      }
    });
    // the chunk's verdict words now (its lanes' statuses are final: the direct
    // ones were written at classification), overlapped with later chunks' GPU
    // work; chunks start 64-aligned (shard starts and chunk sizes are)
    if (dev && dev->done && (e = dev->done(st.a, st.b)) != hipSuccess) return e;
    if (b->verdict)
      pool.parallel_for((st.b - st.a + 63) / 64, 1024, [&](uint64_t x, uint64_t y) {
        for (uint64_t w = st.a / 64 + x; w < st.a / 64 + y; w++) {
          uint64_t v = 0;
          for (uint64_t l = 0; l < 64 && w * 64 + l < st.b; l++)
            if (b->status[w * 64 + l] == CORDAHIP_STATUS_OK) v |= 1ull << l;
          b->verdict[w] = v;
        }
      });
    return hipSuccess;
  };
  std::vector<uint16_t> cls;
  std::vector<PieceInfo> pieces;
  std::vector<uint64_t> lens, grow, gmsg, ec_row0, ec_mo0;  // chunk groups: length, first row, message offset
  std::vector<std::vector<uint64_t>> prow;                   // [piece][group]: the piece's first row in the group
  hipError_t e = hipSuccess;
  int rc = CORDAHIP_SUCCESS;
  const double t_start = tracing() ? now_ms() : 0;
  const int nst = dev ? kTxStages : kPackStages;  // signed-tx chunks: more of them in flight
  static const bool ec_alt = !(getenv("CORDAHIP_EC_ALTERNATE") && getenv("CORDAHIP_EC_ALTERNATE")[0] == '0');
  const bool ec_alone = ec_alt && d.active.load() <= 1;  // no other call on the device as this one starts
  for (size_t k = 0; k < chunks.size() && e == hipSuccess && rc == CORDAHIP_SUCCESS; k++) {
    BatchStage& st = set.pb[k % nst];
    const double t0 = tracing() ? now_ms() : 0;
    e = finish(st);
    if (e != hipSuccess) break;
    const double t1 = tracing() ? now_ms() : 0;
    const uint64_t a = chunks[k].a, m = chunks[k].b - a;
    if (dev && dev->advance && (e = dev->advance(a + m, false)) != hipSuccess) break;
    const double t1b = tracing() ? now_ms() : 0;
    const uint64_t np = (m + kGrain - 1) / kGrain;
    cls.resize(m);
    pieces.resize(np);
    // (1) classify
    pool.parallel_for(np, 1, [&](uint64_t x, uint64_t y) {
      for (uint64_t q = x; q < y; q++) {
        PieceInfo& P = pieces[q];
        P.ed.clear();
        P.ec = P.ec_bytes = 0;
        P.too_long = P.bad_csr = false;
        // length -> group: the previous lane's group first (batches are mostly
        // one message length), a hash map once a piece has many lengths, so a
        // batch of adversarially varied lengths stays linear
        std::unordered_map<uint64_t, uint32_t> gidx;
        size_t last = 0;
        for (uint64_t r = q * kGrain; r < std::min(m, (q + 1) * kGrain); r++) {
          uint64_t mlen = 0;
          uint16_t c = classify(b, mv, a + r, mlen);
          if (c == kBadCsr) {
            P.bad_csr = true;
            c = kDirect;  // not packed: the chunk is not enqueued
          } else if (c == kEc) {
            P.ec++;
            P.ec_bytes += mlen;
          } else if (c == kEdBase) {
            if (mlen > 0xffffffffull) P.too_long = true;
            size_t j = last;
            if (j >= P.ed.size() || P.ed[j].first != mlen) {
              if (P.ed.size() <= 8) {
                j = 0;
                while (j < P.ed.size() && P.ed[j].first != mlen) j++;
              } else {
                if (gidx.empty())
                  for (size_t u = 0; u < P.ed.size(); u++) gidx.emplace(P.ed[u].first, (uint32_t)u);
                auto it = gidx.find(mlen);
                j = it == gidx.end() ? P.ed.size() : it->second;
              }
              if (j == P.ed.size()) {
                P.ed.push_back({mlen, 0});
                if (!gidx.empty()) gidx.emplace(mlen, (uint32_t)j);
              }
            }
            last = j;
            P.ed[j].second++;
            c = (uint16_t)(kEdBase + j);
          }
          cls[r] = c;
        }
      }
    });
    const double t2 = tracing() ? now_ms() : 0;
    // (2) chunk layout: groups by length, rows and message offsets per piece
    lens.clear();
    for (const PieceInfo& P : pieces) {
      if (P.too_long || P.bad_csr) rc = CORDAHIP_ERR_INVALID_ARG;
      for (const auto& kv : P.ed) lens.push_back(kv.first);
    }
    if (rc != CORDAHIP_SUCCESS) break;
    std::sort(lens.begin(), lens.end());
    lens.erase(std::unique(lens.begin(), lens.end()), lens.end());
    const size_t ng = lens.size();
    prow.assign(np, std::vector<uint64_t>(ng, 0));
    grow.assign(ng + 1, 0);
    gmsg.assign(ng + 1, 0);
    for (uint64_t q = 0; q < np; q++) {
      PieceInfo& P = pieces[q];
      P.ed_global.resize(P.ed.size());
      for (size_t j = 0; j < P.ed.size(); j++)
        P.ed_global[j] = (uint32_t)(std::lower_bound(lens.begin(), lens.end(), P.ed[j].first) - lens.begin());
    }
    // rows of group gi, piece by piece: prow[q][gi] = lanes of group gi in
    // pieces < q (then offset by the group's first row); O(pieces x groups)
    for (uint64_t q = 0; q + 1 < np; q++)
      for (size_t j = 0; j < pieces[q].ed.size(); j++) prow[q + 1][pieces[q].ed_global[j]] = pieces[q].ed[j].second;
    for (size_t gi = 0; gi < ng; gi++) {
      uint64_t r = grow[gi];
      for (uint64_t q = 0; q < np; q++) {
        r += prow[q][gi];  // lanes of piece q - 1
        prow[q][gi] = r;
      }
      for (size_t j = 0; j < pieces[np - 1].ed.size(); j++)
        if (pieces[np - 1].ed_global[j] == gi) r += pieces[np - 1].ed[j].second;
      grow[gi + 1] = r;
      gmsg[gi + 1] = (gmsg[gi] + (r - grow[gi]) * lens[gi] + 15) / 16 * 16;
    }
    ec_row0.assign(np + 1, 0);
    ec_mo0.assign(np + 1, 0);
    for (uint64_t q = 0; q < np; q++) {
      ec_row0[q + 1] = ec_row0[q] + pieces[q].ec;
      ec_mo0[q + 1] = ec_mo0[q] + pieces[q].ec_bytes;
    }
    const uint64_t ne = grow[ng], nc = ec_row0[np], mb = ec_mo0[np];
    const size_t sz[14] = {ne * 32, ne * 64, std::max<uint64_t>(gmsg[ng], 16), ne, ne,
                           nc, nc * 65, nc, nc * 72, nc, std::max<uint64_t>(mb, 16), (nc + 1) * 8, nc, nc};
    for (int q = 0; q < 14; q++) {
      const bool host = !(dev && (q == 2 || q == 10));  // device-id messages have no host rows
      if (sz[q] && ((host && st.h[q].ensure(sz[q]) != hipSuccess) || st.d[q].ensure(sz[q]) != hipSuccess))
        rc = CORDAHIP_ERR_OUT_OF_MEMORY;
    }
    if (dev)
      for (int q = 0; q < 2; q++) {
        const uint64_t rows = std::max<uint64_t>(q ? nc : ne, 1);
        if (st.hidx[q].ensure(rows * 4) != hipSuccess || st.didx[q].ensure(rows * 4) != hipSuccess)
          rc = CORDAHIP_ERR_OUT_OF_MEMORY;
      }
    if (rc != CORDAHIP_SUCCESS) break;
    st.ed_lanes.resize(ne);
    st.ec_lanes.resize(nc);
    if (nc) st.h[11].as<uint64_t>()[nc] = mb;
    // (3) pack every lane into its row, in copy groups of pieces, each group's
    // rows going H2D as soon as they are packed: the rows of a length group are
    // allocated piece by piece, so a range of pieces is a row range in every
    // group (and in the ECDSA section), and PCIe carries group g while the pool
    // packs group g + 1 -- a chunk's inputs land ~one copy group after its pack
    // instead of a whole pack plus a whole copy later
    const uint64_t ncg = std::min<uint64_t>(np, m >= (1u << 20) ? 8 : 1);
    const double t3 = tracing() ? now_ms() : 0;
    auto h2d = [&](int q, uint64_t off, uint64_t bytes) {
      if (bytes) e = e ? e : hipMemcpyAsync(st.d[q].as<uint8_t>() + off, st.h[q].as<uint8_t>() + off, bytes,
                                            hipMemcpyHostToDevice, d.s_copy);
    };
    for (uint64_t cg = 0; cg < ncg && e == hipSuccess; cg++) {
      const uint64_t q0 = np * cg / ncg, q1 = np * (cg + 1) / ncg;
      pool.parallel_for(q1 - q0, 1, [&](uint64_t x, uint64_t y) {
        std::vector<uint64_t> row;
        for (uint64_t q = q0 + x; q < q0 + y; q++) {
          const PieceInfo& P = pieces[q];
          row.assign(P.ed.size(), 0);
          for (size_t j = 0; j < P.ed.size(); j++) row[j] = prow[q][P.ed_global[j]];
          uint64_t er = ec_row0[q], mo = ec_mo0[q];
          for (uint64_t r = q * kGrain; r < std::min(m, (q + 1) * kGrain); r++) {
            const uint16_t c = cls[r];
            const uint64_t i = a + r;
            if (c == kEc) {
              st.ec_lanes[er] = i;
              pack_ec_row(b, mv, do_verify, i, er, st.h[5].as<uint8_t>(), st.h[6].as<uint8_t>(),
                          st.h[7].as<uint8_t>(), st.h[8].as<uint8_t>(), st.h[9].as<uint8_t>(), st.h[10].as<uint8_t>(),
                          st.h[11].as<uint64_t>(), st.h[12].as<uint8_t>(), mo,
                          dev ? st.hidx[1].as<uint32_t>() : nullptr, dev ? dev->t0 : 0);
              er++;
            } else if (c >= kEdBase) {
              const size_t j = c - kEdBase, gi = P.ed_global[j];
              const uint64_t rr = row[j]++;
              st.ed_lanes[rr] = i;
              // group gi's messages start at gmsg[gi]; device-id messages: all 32
              // bytes, one group, row rr's message at rr * 32 once gathered
              if (dev) st.hidx[0].as<uint32_t>()[rr] = (uint32_t)(mv.tx_of[i] - dev->t0);
              pack_ed_row(b, mv, do_verify, i, (uint32_t)lens[gi], st.h[0].as<uint8_t>() + rr * 32,
                          st.h[1].as<uint8_t>() + rr * 64,
                          dev ? nullptr : st.h[2].as<uint8_t>() + gmsg[gi] + (rr - grow[gi]) * lens[gi],
                          st.h[3].as<uint8_t>() + rr);
            }
          }
        }
      });
      // this copy group's rows: [prow[q0][g], prow[q1][g]) of each Ed25519 group,
      // [ec_row0[q0], ec_row0[q1]) of the ECDSA section
      for (size_t gi = 0; gi < ng; gi++) {
        const uint64_t r0 = prow[q0][gi], r1 = q1 < np ? prow[q1][gi] : grow[gi + 1];
        h2d(0, r0 * 32, (r1 - r0) * 32);
        h2d(1, r0 * 64, (r1 - r0) * 64);
        h2d(3, r0, r1 - r0);
        if (dev) {
          if (r1 > r0)
            e = e ? e : hipMemcpyAsync(st.didx[0].as<uint32_t>() + r0, st.hidx[0].as<uint32_t>() + r0, (r1 - r0) * 4,
                                       hipMemcpyHostToDevice, d.s_copy);
        } else {
          h2d(2, gmsg[gi] + (r0 - grow[gi]) * lens[gi], (r1 - r0) * lens[gi]);
        }
      }
      const uint64_t c0 = ec_row0[q0], c1 = ec_row0[q1];
      h2d(5, c0, c1 - c0);
      h2d(6, c0 * 65, (c1 - c0) * 65);
      h2d(7, c0, c1 - c0);
      h2d(8, c0 * 72, (c1 - c0) * 72);
      h2d(9, c0, c1 - c0);
      h2d(11, c0 * 8, (c1 - c0 + (q1 == np && nc ? 1 : 0)) * 8);  // the last group carries off[nc]
      h2d(12, c0, c1 - c0);
      if (dev) {
        if (c1 > c0)
          e = e ? e : hipMemcpyAsync(st.didx[1].as<uint32_t>() + c0, st.hidx[1].as<uint32_t>() + c0, (c1 - c0) * 4,
                                     hipMemcpyHostToDevice, d.s_copy);
      } else {
        h2d(10, ec_mo0[q0], ec_mo0[q1] - ec_mo0[q0]);
      }
    }
    const double t3b = tracing() ? now_ms() : 0;
    if (dev && dev->advance) e = e ? e : dev->advance(a + m, true);
    const double t3c = tracing() ? now_ms() : 0;
    // (4) launches
    // consecutive chunks alternate between s_ed / s_ed2 and the two Ed25519
    // workspace slots: chunk k + 1's kernels overlap chunk k's end-of-grid tail
    const int slot = (int)(d.ed_turn.fetch_add(1) & 1);  // alternating across calls too
    hipStream_t es = slot ? d.s_ed2 : d.s_ed;
    e = e ? e : hipEventRecord(st.copied, d.s_copy);
    e = e ? e : hipStreamWaitEvent(es, st.copied, 0);
    // device-id messages: each section's stream waits for the id slice holding
    // the chunk's last transaction, then gathers its rows from the ids in HBM
    const hipEvent_t ids_ready = dev ? dev->wait_for(mv.tx_of[a + m - 1]) : nullptr;
    // one length group (the ids): the keys' half of the prep is enqueued first and the
    // wait for the ids + the gather after it, so key / R decoding and their tables
    // do not wait for the chunk's id slice
    const bool split = dev && dev->split_prep && ne && ng == 1;
    const std::function<hipError_t()> gather_ids = [&]() -> hipError_t {
      hipError_t x = hipStreamWaitEvent(es, ids_ready, 0);
      return x ? x : launch_gather_rows32(dev->txid, st.didx[0].as<uint32_t>(), ne, st.d[2].as<uint8_t>(), es);
    };
    if (dev && ne && !split) e = e ? e : gather_ids();
    st.direct = out_pinned && ng == 1 && ne == m && nc == 0 && a % 64 == 0;
    const uint64_t words = (m + 63) / 64;
    if (st.direct && b->verdict && st.dverdict.ensure(words * 8) != hipSuccess) st.direct = false;
    for (size_t gi = 0; gi < ng && e == hipSuccess; gi++) {
      const uint64_t r0 = grow[gi], cnt = grow[gi + 1] - r0;
      if (cnt)
        e = ed_verify_enqueue(d, st.d[0].as<uint8_t>() + r0 * 32, st.d[1].as<uint8_t>() + r0 * 64,
                              st.d[2].as<uint8_t>() + gmsg[gi], (uint32_t)lens[gi], cnt, st.d[3].as<uint8_t>() + r0,
                              st.d[4].as<uint8_t>() + r0,
                              st.direct && b->verdict ? st.dverdict.as<unsigned long long>() : nullptr, b->flags,
                              es, slot, split ? &gather_ids : nullptr);
    }
    if (st.direct) {
      e = e ? e : launch_store_to_host(st.d[4].p, dst_status + a, m, es);
      if (b->verdict) e = e ? e : launch_store_to_host(st.dverdict.p, dst_verdict + a / 64, words * 8, es);
    } else if (ne) {
      e = e ? e : launch_store_to_host(st.d[4].p, st.h[4].p, ne, es);
    }
    e = e ? e : hipEventRecord(st.ed_done, es);
    // ECDSA sections: a generic batch alone on the device alternates its chunks
    // between s_ec with workspace slot 0 and s_ec2 (the id-copy stream, idle in
    // generic batches) with slot 1, so chunk k + 1's partition, prep and batch
    // inversion run beside chunk k's ladders instead of after them; a call that
    // starts beside another keeps s_ec and slot 0. c3h +1.2-1.4% at one call in
    // flight, +1.3% at two (CORDAHIP_EC_ALTERNATE=0 turns it off;
    // profiles/r06_ec_slots_ab/summary.json)
    const int ecs = nc && ec_alone && !dev ? (int)(d.ec_turn.fetch_add(1) & 1) : 0;
    hipStream_t xs = ecs && d.s_ec2 ? d.s_ec2 : d.s_ec;
    e = e ? e : hipStreamWaitEvent(xs, st.copied, 0);
    if (dev && nc) {
      e = e ? e : hipStreamWaitEvent(xs, ids_ready, 0);
      e = e ? e : launch_gather_rows32(dev->txid, st.didx[1].as<uint32_t>(), nc, st.d[10].as<uint8_t>(), xs);
    }
    if (nc && e == hipSuccess) {
      std::lock_guard<std::mutex> ge(d.ec_mu[ecs]);
      e = ec_verify_enqueue(d, st.d[5].as<uint8_t>(), st.d[6].as<uint8_t>(), st.d[7].as<uint8_t>(),
                            st.d[8].as<uint8_t>(), st.d[9].as<uint8_t>(), st.d[10].as<uint8_t>(),
                            st.d[11].as<uint64_t>(), 0, nc, st.d[12].as<uint8_t>(), st.d[13].as<uint8_t>(), nullptr,
                            b->flags, xs, ecs);
    }
    if (nc) e = e ? e : launch_store_to_host(st.d[13].p, st.h[13].p, nc, xs);
    e = e ? e : hipEventRecord(st.ec_done, xs);
    if (e == hipSuccess) {
      st.pending = true;
      st.a = a;
      st.b = a + m;
    }
    if (tracing())
      fprintf(stderr, "[cordahip] dev %d chunk %zu: %llu lanes (%llu ed, %llu ec) at %.1f ms: wait %.2f ids-ahead %.2f "
                      "classify %.2f layout %.2f pack+copy %.2f ids-after %.2f launch %.2f ms\n", d.id, k,
              (unsigned long long)m, (unsigned long long)ne, (unsigned long long)nc, t0 - t_start, t1 - t0,
              t1b - t1, t2 - t1b, t3 - t2, t3b - t3, t3c - t3b, now_ms() - t3c);
  }
  // every chunk is enqueued: the caller's hook (the signed-tx path hands its
  // enqueue token on; the stages below are this call's own)
  if (dev && dev->enqueued && e == hipSuccess && rc == CORDAHIP_SUCCESS) e = dev->enqueued();
  // drain every stage: each stage's events follow its chunk's last work on every
  // stream it used, so waiting for them (not for the shared streams, which may
  // already carry the next call's work) drains this call. After an error the
  // streams themselves are drained, so no queued work outlives the call.
  for (int k = 0; k < nst; k++) {
    if (e == hipSuccess && rc == CORDAHIP_SUCCESS) e = finish(set.pb[k]);
    set.pb[k].pending = false;
  }
  if (e != hipSuccess || rc != CORDAHIP_SUCCESS) {
    for (hipStream_t x : {d.s_copy, d.s_ed, d.s_ed2, d.s_ec, d.s_ec2})  // s_ec2: the id-copy stream
      if (x) (void)hipStreamSynchronize(x);
    for (BatchStage& st : set.pb)
      for (hipEvent_t ev : {st.copied, st.ed_done, st.ec_done}) (void)hipEventSynchronize(ev);
  }
  if (tracing()) fprintf(stderr, "[cordahip] dev %d: shard done at %.1f ms\n", d.id, now_ms() - t_start);
  if (rc != CORDAHIP_SUCCESS) return rc;
  return e ? CORDAHIP_ERR_HIP : CORDAHIP_SUCCESS;
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

int sig_verify_msgs(cordahip_ctx* ctx, const cordahip_sig_batch* b, const MsgView& mv) {
  const uint64_t n = b->n;
  if (n == 0) return CORDAHIP_SUCCESS;
  // contiguous 64-aligned input shards, one pipeline per device
  const int rc = for_shards(ctx->devs, n, 64, [&](Device& d, uint64_t lo, uint64_t hi) {
    SetLease lease(d);
    if (hipSetDevice(d.id) != hipSuccess || hipEventSynchronize(lease.get().tx_ev) != hipSuccess)
      return (int)CORDAHIP_ERR_HIP;
    return sig_pipeline(ctx, d, lease.get(), b, mv, lo, hi);
  });
  if (rc != CORDAHIP_SUCCESS) return rc;
  // verdict words: built per chunk by the pipelines (sig_pipeline's finish)
  return CORDAHIP_SUCCESS;
}

int sig_verify_range(cordahip_ctx* ctx, Device& d, TxSet& set, const cordahip_sig_batch* b, const MsgView& mv,
                     uint64_t lo, uint64_t hi) {
  return sig_pipeline(ctx, d, set, b, mv, lo, hi);
}

int sig_verify_impl(cordahip_ctx* ctx, const cordahip_sig_batch* b) {
  if (b->n == 0) return CORDAHIP_SUCCESS;
  if (!b->scheme || !b->key || !b->key_off || !b->sig || !b->sig_off || !b->msg || !b->msg_off || !b->status ||
      (b->flags & ~CORDAHIP_FLAG_IS_VALID))
    return CORDAHIP_ERR_INVALID_ARG;
  // every lane's ranges are checked as its chunk is classified (pack_rows.hpp classify)
  return sig_verify_msgs(ctx, b, MsgView{b->msg, b->msg_off, nullptr});
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
