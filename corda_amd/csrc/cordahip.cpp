// libcordahip.so host runtime: contexts, devices, streams, pinned memory,
// batch partitioning and the C-ABI of include/cordahip.h.
//
// MI355X-first shape: one context drives the devices named by its mask; a
// host batch is split into contiguous 64-aligned shards, one per device
// (Ed25519 and ECDSA lanes alike; transactions whole), and each shard streams
// through HIP streams in fixed chunks (H2D of chunk k+1 overlaps the kernel of
// chunk k). Device buffers are grow-only per device and reused across calls;
// every buffer shared between streams is fenced by an event (the next user's
// stream waits on the last user's completion). Tickets run on a per-context
// worker pool. The fixed-base tables are built once per device at init by a
// kernel. There is no CPU verification fallback: a HIP failure is returned to
// the caller as CORDAHIP_ERR_HIP. The generic CSR signature batch lives in
// host_batch.cpp; the shared runtime types in runtime.hpp.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "csr_check.hpp"
#include "der.hpp"
#include "kryo_core.hpp"
#include "runtime.hpp"
#include "status.hpp"

using namespace cordahip;
using namespace cordahip::rt;

namespace cordahip {
namespace rt {

// ---- host fork-join pool -----------------------------------------------------
HostPool::HostPool(int nthreads, const std::vector<int>& cpus) {
  for (int i = 1; i < nthreads; i++) {
    threads_.emplace_back([this] { worker(); });
    if (!cpus.empty()) {  // the device's node: its rows are packed next to its GPU
      cpu_set_t cs;
      CPU_ZERO(&cs);
      for (int c : cpus)
        if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &cs);
      (void)pthread_setaffinity_np(threads_.back().native_handle(), sizeof(cs), &cs);
    }
  }
}

NodeBind::NodeBind(const Device& d) {
  if (d.place.cpus.empty()) return;
  cpu_set_t old, cs;
  if (pthread_getaffinity_np(pthread_self(), sizeof(old), &old) != 0) return;
  CPU_ZERO(&cs);
  for (int c : d.place.cpus)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &cs);
  if (CPU_EQUAL(&cs, &old) || pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs) != 0) return;
  saved_.assign(reinterpret_cast<unsigned char*>(&old), reinterpret_cast<unsigned char*>(&old) + sizeof(old));
  bound_ = true;
}

NodeBind::~NodeBind() {
  if (bound_) (void)pthread_setaffinity_np(pthread_self(), sizeof(cpu_set_t), reinterpret_cast<cpu_set_t*>(saved_.data()));
}

HostPool& pool_of(cordahip_ctx* ctx, Device& d) { return d.pool ? *d.pool : *ctx->host; }

MemAcct& mem_acct(int dev) {
  static MemAcct acct[kMaxHipDevices];
  return acct[dev >= 0 && dev < kMaxHipDevices ? dev : 0];
}

HostPool::~HostPool() {
  {
    std::lock_guard<std::mutex> g(m_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

void HostPool::run_pieces(Job& j) {
  for (;;) {
    const uint64_t k = j.next.fetch_add(1);
    if (k >= j.npieces) return;
    const uint64_t lo = k * j.piece, hi = std::min(j.n, lo + j.piece);
    (*j.fn)(lo, hi);
    if (j.done.fetch_add(1) + 1 == j.npieces) {
      std::lock_guard<std::mutex> g(j.m);
      j.cv.notify_all();
    }
  }
}

void HostPool::worker() {
  for (;;) {
    std::shared_ptr<Job> j;
    {
      std::unique_lock<std::mutex> g(m_);
      for (;;) {
        while (!q_.empty() && q_.front()->next.load() >= q_.front()->npieces) q_.pop_front();  // exhausted
        if (!q_.empty()) {
          j = q_.front();
          break;
        }
        if (stop_) return;
        cv_.wait(g);
      }
    }
    run_pieces(*j);
  }
}

void HostPool::parallel_for(uint64_t n, uint64_t grain, const std::function<void(uint64_t, uint64_t)>& fn) {
  if (n == 0) return;
  grain = std::max<uint64_t>(grain, 1);
  const uint64_t want = std::max<uint64_t>(1, std::min<uint64_t>((n + grain - 1) / grain, 4 * (uint64_t)threads()));
  if (want == 1 || threads_.empty()) {
    fn(0, n);
    return;
  }
  auto j = std::make_shared<Job>();
  j->fn = &fn;
  j->n = n;
  j->piece = (n + want - 1) / want;
  j->npieces = (n + j->piece - 1) / j->piece;
  {
    std::lock_guard<std::mutex> g(m_);
    q_.push_back(j);
  }
  cv_.notify_all();
  run_pieces(*j);
  {
    std::unique_lock<std::mutex> g(j->m);
    j->cv.wait(g, [&] { return j->done.load() == j->npieces; });
  }
  std::lock_guard<std::mutex> g(m_);  // drop it if no worker got to pop it
  for (auto it = q_.begin(); it != q_.end(); ++it)
    if (*it == j) {
      q_.erase(it);
      break;
    }
}

// ---- ticket pool ---------------------------------------------------------------
WorkerPool::WorkerPool(int nthreads) {
  for (int i = 0; i < nthreads; i++) threads_.emplace_back([this] { run(); });
}

WorkerPool::~WorkerPool() {
  {
    std::lock_guard<std::mutex> g(m_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

void WorkerPool::push(std::shared_ptr<JobState> st, std::function<int()> fn) {
  {
    std::lock_guard<std::mutex> g(m_);
    q_.emplace_back(std::move(st), std::move(fn));
  }
  cv_.notify_one();
}

void WorkerPool::run() {
  for (;;) {
    std::pair<std::shared_ptr<JobState>, std::function<int()>> job;
    {
      std::unique_lock<std::mutex> g(m_);
      cv_.wait(g, [this] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stop_ and drained: queued jobs always run
      job = std::move(q_.front());
      q_.pop_front();
    }
    int rc;
    try {
      rc = job.second();
    } catch (...) {
      rc = CORDAHIP_ERR_OUT_OF_MEMORY;  // std::bad_alloc from host staging vectors
    }
    {
      std::lock_guard<std::mutex> g(job.first->m);
      job.first->rc = rc;
      job.first->done = true;
    }
    job.first->cv.notify_all();
  }
}

int hip_err(hipError_t e) { return e == hipSuccess ? CORDAHIP_SUCCESS : CORDAHIP_ERR_HIP; }

hipError_t ensure_streams(Device& d) {
  std::lock_guard<std::mutex> g(d.streams_mu);
  if (d.s_copy) return hipSuccess;
  // Every pipeline stream needs a hardware queue of its own: streams sharing a
  // queue serialise, and a copy enqueued early (the tx-id slices' leaf bytes,
  // a C5 chunk waiting for its stage) then holds back every later kernel of the
  // other stream. HIP hands out pool queues (GPU_MAX_HW_QUEUES, 4 on the box)
  // round-robin over every stream of the process, so a 4th pipeline stream
  // shared one with s_ed or s_copy depending on creation order (c4h 45.1 M
  // sigs/s, or C5 84.6 instead of 95.8 M/s: profiles/r03_stream_queues.json). A
  // stream created with a CU mask (here: all CUs) gets a dedicated queue; the
  // ECDSA stream keeps the higher priority, which also gives it a queue of its
  // own (at normal priority it shared s_ed's and the two sections ran back to back).
  int lo = 0, hi = 0, ncu = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
  e = e ? e : hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, d.id);
  std::vector<uint32_t> all((std::max(ncu, 1) + 31) / 32, 0xffffffffu);
  auto dedicated = [&](hipStream_t* st) { return hipExtStreamCreateWithCUMask(st, (uint32_t)all.size(), all.data()); };
  hipStream_t c = nullptr, x = nullptr, y = nullptr, z = nullptr, x2 = nullptr;
  e = e ? e : dedicated(&c);
  e = e ? e : dedicated(&x);
  e = e ? e : hipStreamCreateWithPriority(&y, hipStreamNonBlocking, hi);
  e = e ? e : dedicated(&z);
  e = e ? e : dedicated(&x2);
  if (e != hipSuccess) {
    for (hipStream_t s : {c, x, y, z, x2})
      if (s) (void)hipStreamDestroy(s);
    return e;
  }
  d.s_ed = x;
  d.s_ed2 = x2;
  d.s_ec = y;
  // generic batches' alternate ECDSA chunks run on the id-copy stream, idle in those
  // batches (no sixth hardware queue)
  d.s_ec2 = z;
  d.s_idcopy = z;
  d.s_copy = c;
  return hipSuccess;
}

// Launch-pair sizes of the split kernels = the largest workspace per device.
// Bigger launches pay fewer end-of-grid tails (C2, measured: 2^18 91.5, 2^20
// 93.2, 2^22 96.4, 2^24 97.2 M verifs/s): a 2^24-lane batch runs as ONE
// prep/ladder pair over 54 GB of HBM (19% of the MI355X's 288 GB). Smaller
// batches allocate only what they use (grow-only, from 2^18 lanes up).
constexpr uint64_t kEdWsLanes = 1ull << 24;  // x 3,200 B = 54 GB of Ed25519 workspace at most
constexpr uint64_t kEcWsSlots = 1ull << 24;  // x 1,120 B = 18.8 GB of ECDSA workspace at most
constexpr uint64_t kWsMinLanes = 1ull << 18;

// Workspace-size overrides (multiples of 64): tests use them to force the
// multi-chunk paths (several prep/ladder launch sets per batch) at small sizes.
uint64_t env_lanes(const char* name, uint64_t dflt) {
  const char* v = getenv(name);
  const uint64_t x = v ? strtoull(v, nullptr, 10) : 0;
  return x >= 64 ? x / 64 * 64 : dflt;
}

// a zeroed 64-byte host-mapped buffer (the encoder's usage reports)
hipError_t usage_buffer(uint32_t*& h, uint32_t*& dp) {
  if (h) return hipSuccess;
  void* hp = nullptr;
  void* dv = nullptr;
  if (hipHostMalloc(&hp, 64, hipHostMallocMapped) != hipSuccess) return hipErrorOutOfMemory;
  if (hipHostGetDevicePointer(&dv, hp, 0) != hipSuccess) {
    (void)hipHostFree(hp);
    return hipErrorUnknown;
  }
  std::memset(hp, 0, 64);
  h = static_cast<uint32_t*>(hp);
  dp = static_cast<uint32_t*>(dv);
  return hipSuccess;
}

// The Kryo encoder's persistent state ready for a call on stream s (kryo_mu
// held, d.kryo_fixed allocated): zeroed when freshly allocated; cleared when the
// usage a call reported passes half the table or nearly fills the template
// arena (recurring shapes then rebuild once). The reports are snapshots of
// counters that only grow between clears, so the largest one is the latest; a
// report may lag by the calls still running (cordahip_kryo_encode_device's is
// read without waiting for its stream): the table then clears one call later,
// and until then new shapes take the direct encoder -- slower, never wrong.
hipError_t kryo_state_ready(Device& d, hipStream_t s) {
  if (hipError_t e = usage_buffer(d.kryo_usage, d.kryo_usage_dev)) return e;
  uint32_t templates = 0, slots = 0;
  for (const uint32_t* p : {(const uint32_t*)d.kryo_usage, (const uint32_t*)d.set[0].kryo_usage,
                            (const uint32_t*)d.set[1].kryo_usage})
    if (p) {
      const volatile uint32_t* u = p;
      templates = std::max<uint32_t>(templates, (uint32_t)u[0]);
      slots = std::max<uint32_t>(slots, (uint32_t)u[1]);
    }
  if (d.kryo_fresh || templates > kryo_clear_threshold_templates() || slots > kryo_clear_threshold_slots()) {
    d.kryo_fresh = false;
    d.kryo_templates_ok = false;  // an empty table: the next component batch builds its shapes
    d.kryo_gen++;                 // a call that started before the clear does not vouch for the new table
    for (uint32_t* p : {d.kryo_usage, d.set[0].kryo_usage, d.set[1].kryo_usage})
      if (p) p[0] = p[1] = 0;
    return kryo_clear(d.kryo_fixed.as<uint8_t>(), s);
  }
  return hipSuccess;
}
// after a call's encoder launches: its usage counters to the host-mapped copy of
// its set (nullptr: cordahip_kryo_encode_device's own)
hipError_t kryo_usage_report(Device& d, TxSet* set, hipStream_t s) {
  return launch_store_to_host(kryo_usage_src(d.kryo_fixed.as<uint8_t>()),
                              set ? set->kryo_usage_dev : d.kryo_usage_dev, kKryoUsageBytes, s);
}
// grows kryo_fixed if needed (once: its size is fixed), marking it fresh
hipError_t kryo_fixed_ensure(Device& d) {
  if (d.kryo_fixed.cap >= kryo_fixed_scratch_bytes()) return hipSuccess;
  d.kryo_fresh = true;
  return d.kryo_fixed.ensure(kryo_fixed_scratch_bytes());
}

// Enqueue ECDSA verification of n slot-layout lanes on stream s (device current,
// d.ec_mu[slot] held): the slot's work buffers are reused only after their previous
// user's kernels (on whatever stream) have finished.
hipError_t ec_verify_enqueue(Device& d, const uint8_t* scheme, const uint8_t* keys, const uint8_t* key_len,
                             const uint8_t* sigs, const uint8_t* sig_len, const uint8_t* msgs, const uint64_t* msg_off,
                             uint32_t msg_len, uint64_t n, const uint8_t* pre, uint8_t* status,
                             unsigned long long* verdict, uint32_t flags, hipStream_t s, int slot) {
  EcWork& w = d.ec[slot];
  // the budget's ECDSA share (cordahip_init); slot 1 serves the host pipelines'
  // alternate chunks and holds at most half of slot 0
  const uint64_t ws_slots = slot ? std::max<uint64_t>(64, d.ec_ws_slots / 2 / 64 * 64) : d.ec_ws_slots;
  const uint64_t slots = std::min<uint64_t>(ws_slots, (std::max<uint64_t>(n, 1) + 63) / 64 * 64);
  if (w.ws.cap < slots * ecdsa_ws_slot_bytes() || w.perm.cap < std::max<uint64_t>(n, 1) * 4) {
    hipError_t e = w.ev ? hipEventSynchronize(w.ev) : hipSuccess;  // a smaller buffer may still be in use
    if (e != hipSuccess) return e;
    if (w.ws.ensure(std::max<uint64_t>(slots, std::min<uint64_t>(ws_slots, kWsMinLanes)) * ecdsa_ws_slot_bytes()) ||
        w.perm.ensure(std::max<uint64_t>(n, 1) * 4))
      return hipErrorOutOfMemory;
  }
  if (w.counters.ensure(64)) return hipErrorOutOfMemory;
  if (!w.ev && hipEventCreateWithFlags(&w.ev, hipEventDisableTiming) != hipSuccess) return hipErrorUnknown;
  hipError_t e = hipStreamWaitEvent(s, w.ev, 0);
  e = e ? e
        : launch_ecdsa_verify(scheme, keys, key_len, sigs, sig_len, msgs, msg_off, msg_len, n, d.gtab_k1, d.gtab_r1,
                              pre, status, verdict, w.counters.as<unsigned int>(), w.perm.as<unsigned int>(),
                              w.ws.as<uint32_t>(), w.ws.cap / ecdsa_ws_slot_bytes() / 64 * 64, flags, s);
  e = e ? e : hipEventRecord(w.ev, s);
  return e;
}

// Enqueue Ed25519 verification of n dense lanes on stream s (device already current).
hipError_t ed_verify_enqueue(Device& d, const uint8_t* keys, const uint8_t* sigs, const uint8_t* msgs,
                             uint32_t msg_len, uint64_t n, const uint8_t* pre, uint8_t* status,
                             unsigned long long* verdict, uint32_t flags, hipStream_t s, int slot,
                             const std::function<hipError_t()>* before_msgs) {
  std::lock_guard<std::mutex> g(d.ed_mu[slot]);
  DevBuf& ws = d.ed_ws[slot];
  hipEvent_t& ev = d.ed_ev[slot];
  // the budget's Ed25519 shares (cordahip_init, device_budget): slot 1 only serves the
  // alternating chunks of the pipelines (host batches, streams, signed-tx chunks) and
  // holds at most half of slot 0. The launch loops over whatever the workspace holds,
  // so a smaller one only costs extra launch pairs.
  const uint64_t cap_lanes = d.ed_ws_lanes[slot ? 1 : 0];
  const uint64_t lanes = std::min<uint64_t>(cap_lanes, (std::max<uint64_t>(n, 1) + 63) / 64 * 64);
  const uint64_t lane_bytes = ed25519_ws_lane_bytes();
  if (ws.cap < lanes * lane_bytes) {
    // a smaller buffer may still be in use by an earlier stream
    hipError_t e = ev ? hipEventSynchronize(ev) : hipSuccess;
    if (e != hipSuccess) return e;
    uint64_t want = std::max<uint64_t>(lanes, std::min<uint64_t>(cap_lanes, kWsMinLanes));
    const uint64_t had = ws.cap / lane_bytes / 64 * 64;  // ensure() frees it before allocating
    e = ws.ensure(want * lane_bytes);
    // HBM shared with other work: halve the request until it fits (at least
    // what the slot held before, or one wave's lanes) instead of failing the call
    while (e == hipErrorOutOfMemory && want > std::max<uint64_t>(64, had)) {
      (void)hipGetLastError();
      want = std::max<uint64_t>(std::max<uint64_t>(64, had), want / 2 / 64 * 64);
      e = ws.ensure(want * lane_bytes);
    }
    if (e != hipSuccess) return e;
  }
  if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return hipErrorUnknown;
  hipError_t e = hipStreamWaitEvent(s, ev, 0);
  e = e ? e
        : launch_ed25519_verify(keys, sigs, msgs, msg_len, n, d.btab, pre, status, verdict, ws.as<uint32_t>(),
                                ws.cap / ed25519_ws_lane_bytes() / 64 * 64, flags, s, before_msgs);
  e = e ? e : hipEventRecord(ev, s);
  return e;
}

// The Ed25519 section of a device signed-tx call (32-byte messages in HBM, on the
// caller's stream s): chunks of CORDAHIP_DEVICE_ED_CHUNK signatures (default
// 98,304 = 0.75 of a ladder round of 2 waves x 1,024 SIMDs x 64 lanes; 0: one
// launch pair) alternate between s with workspace slot 0 and the device's s_ed2
// with slot 1, the short remainder first. Every ladder wave takes about the same
// time, so one launch over C4's 2.5 M signatures (19.07 rounds) ran 20 rounds, its
// last with 7% of the CUs; alternating chunks let chunk k + 1's prep fill chunk k's
// ladder tail, as the host pipelines do. Two streams hold two chunks, so a chunk
// below half a round leaves CUs idle (2^15: C4 64.7 M sig/s). One box
// (profiles/r06_device_ed_chunk_ab/): C4 93.4-94.5 with one launch pair, 95.1-96.4
// at 2^17, 95.8-96.7 at 2^16, 97.0-97.7 at 98,304; C4 --device-encode 87.1-87.2,
// 88.7-89.2, 89.3-89.4, 89.2-89.2.
hipError_t ed_verify_device_chunks(Device& d, TxSet& S, const uint8_t* keys, const uint8_t* sigs, const uint8_t* msgs,
                                   uint64_t n, uint8_t* status, hipStream_t s) {
  static const uint64_t chunk = [] {
    const char* v = getenv("CORDAHIP_DEVICE_ED_CHUNK");
    return v ? (uint64_t)strtoull(v, nullptr, 10) / 64 * 64 : (uint64_t)98304;
  }();
  if (!chunk || n <= chunk || !d.s_ed2)
    return ed_verify_enqueue(d, keys, sigs, msgs, 32, n, nullptr, status, nullptr, 0u, s, 0, nullptr);
  hipError_t e = hipEventRecord(S.ed_fork, s);
  e = e ? e : hipStreamWaitEvent(d.s_ed2, S.ed_fork, 0);
  const uint64_t r = n % chunk;
  uint64_t lo = 0;
  for (int k = 0; lo < n && e == hipSuccess; k++) {
    const uint64_t hi = lo + (k == 0 && r ? r : chunk);
    e = ed_verify_enqueue(d, keys + lo * 32, sigs + lo * 64, msgs + lo * 32, 32, hi - lo, nullptr, status + lo,
                          nullptr, 0u, k % 2 ? d.s_ed2 : s, k % 2, nullptr);
    lo = hi;
  }
  e = e ? e : hipEventRecord(S.ed_join, d.s_ed2);
  return e ? e : hipStreamWaitEvent(s, S.ed_join, 0);
}

// CORDAHIP_DEVICE_MEM_BUDGET (bytes, K/M/G suffixes; default 128 GiB, at most 90%
// of the device): the workspaces it sizes -- Ed25519 slot 0 45% of it, slot 1 20%
// (and half of slot 0 at most), ECDSA 15% -- each also capped by its r05 maximum
// (2^24 lanes / slots, CORDAHIP_ED25519_WS_LANES / CORDAHIP_ECDSA_WS_SLOTS). The
// default therefore keeps C2's single 2^24-lane launch pair (53.7 GB) and the
// r05 peak: 53.7 + 26.8 + 18.8 GB of workspaces. The other buffers follow the
// batches (the id and signature stages, component slices, C5's stages) and are
// not split. A smaller budget costs extra launch pairs, never a failed batch.
uint64_t parse_bytes(const char* v, uint64_t dflt) {
  if (!v || !*v) return dflt;
  char* end = nullptr;
  const double x = strtod(v, &end);
  if (end == v || x <= 0) return dflt;
  const char u = end ? (char)toupper((unsigned char)*end) : 0;
  const double m = u == 'K' ? 1024.0 : u == 'M' ? 1048576.0 : u == 'G' ? 1073741824.0 : 1.0;
  return (uint64_t)(x * m);
}

void device_budget(Device& d) {  // device current
  uint64_t b = parse_bytes(getenv("CORDAHIP_DEVICE_MEM_BUDGET"), 128ull << 30);
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) == hipSuccess && tot) b = std::min<uint64_t>(b, (uint64_t)tot / 10 * 9);
  d.mem_budget = b;
  auto lanes = [](uint64_t bytes, uint64_t per) { return std::max<uint64_t>(64, bytes / per / 64 * 64); };
  const uint64_t lb = ed25519_ws_lane_bytes(), sb = ecdsa_ws_slot_bytes();
  d.ed_ws_lanes[0] = std::min(env_lanes("CORDAHIP_ED25519_WS_LANES", kEdWsLanes), lanes(b / 100 * 45, lb));
  d.ed_ws_lanes[1] = std::min(std::max<uint64_t>(64, d.ed_ws_lanes[0] / 2 / 64 * 64), lanes(b / 5, lb));
  d.ec_ws_slots = std::min(env_lanes("CORDAHIP_ECDSA_WS_SLOTS", kEcWsSlots), lanes(b / 100 * 15, sb));
}

// Free an idle device's grow-only buffers (the idle release, cordahip_trim): both
// buffer sets and every lock that guards a buffer, in an order every path keeps
// (sets, then kryo_mu, stream_mu, ped_mu, ed_mu, ec_mu, each slot in order); the events that fence
// device-path users (kernels on caller streams) synchronised first. The fixed
// tables and the encoder's shape table stay (derived data, 18 MB).
void trim_device(Device& d) {
  SetLease l0(d, 0, true), l1(d, 1, true);
  std::lock_guard<std::mutex> gk(d.kryo_mu), gs(d.stream_mu), gp(d.ped_mu), ge0(d.ed_mu[0]), ge1(d.ed_mu[1]),
      gc0(d.ec_mu[0]), gc1(d.ec_mu[1]);
  if (hipSetDevice(d.id) != hipSuccess) return;
  for (hipEvent_t ev : {d.ed_ev[0], d.ed_ev[1], d.ec[0].ev, d.ec[1].ev, d.kryo_ev, d.set[0].tx_ev, d.set[1].tx_ev})
    if (ev) (void)hipEventSynchronize(ev);
  for (auto& w : d.ed_ws) w.release();
  for (EcWork& w : d.ec) {
    w.ws.release();
    w.perm.release();
  }
  for (TxSet& S : d.set) {
    TxWork& w = S.tx;
    for (DevBuf* b : {&w.leaf_bytes, &w.leaf_off, &w.tx_leaf_off, &w.hashes, &w.txid, &w.tx_status, &w.tx_sig_off,
                      &w.msgs, &w.comp_items, &w.payload, &w.comp_status, &w.tok, &w.tok_hash, &w.tx_tok_off, &w.root,
                      &w.stack})
      b->release();
    for (BatchStage& st : S.pb) {
      for (hipEvent_t ev : {st.copied, st.ed_done, st.ec_done})
        if (ev) (void)hipEventSynchronize(ev);
      for (auto& b : st.h) b.release();
      for (auto& b : st.d) b.release();
      for (auto& b : st.hidx) b.release();
      for (auto& b : st.didx) b.release();
      st.dverdict.release();
    }
  }
  for (auto& st : d.sstage)
    for (DevBuf* b : {&st.ed_keys, &st.ed_sigs, &st.ed_msgs, &st.ed_status, &st.ec_scheme, &st.ec_keys,
                      &st.ec_key_len, &st.ec_sigs, &st.ec_sig_len, &st.ec_msgs, &st.ec_status})
      b->release();
  for (PackStage& st : d.ped) {
    for (auto& b : st.h) b.release();
    for (auto& b : st.d) b.release();
  }
  for (DevBuf* b : {&d.kryo_sizes, &d.kryo_temp, &d.kryo_ws, &d.kryo_items}) b->release();
  if (tracing()) fprintf(stderr, "[cordahip] dev %d: idle buffers released\n", d.id);
}

// the in-process partition rule (cordahip_shard_range)
void shard_range(uint64_t n, uint64_t nshards, uint64_t shard, uint64_t align, uint64_t& lo, uint64_t& hi) {
  if (nshards == 0 || shard >= nshards) {
    lo = hi = n;
    return;
  }
  align = align ? align : 1;
  const uint64_t per = ((n + nshards - 1) / nshards + align - 1) / align * align;
  lo = std::min(n, shard * per);
  hi = std::min(n, lo + per);
}

}  // namespace rt
}  // namespace cordahip

namespace {

std::atomic<uint64_t> g_device_uid{1};

// the context's host pool as csr_check.hpp's parallel runner
struct PoolPar {
  HostPool& pool;
  template <class F>
  void operator()(uint64_t n, uint64_t grain, F&& fn) const {
    pool.parallel_for(n, grain, std::function<void(uint64_t, uint64_t)>(fn));
  }
};

// device uid -> (ring slot, generation) of this thread's most recent timed call
thread_local std::unordered_map<uint64_t, std::pair<int, uint64_t>> tl_last_call;

uint64_t submit_job(cordahip_ctx* ctx, std::function<int()> fn) {
  auto st = std::make_shared<JobState>();
  uint64_t t;
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    t = ctx->next_ticket++;
    ctx->jobs.emplace(t, st);
  }
  ctx->pool->push(st, std::move(fn));
  return t;
}

// timing slot for one *_device call (records `a` now on stream s); the slot's
// generation is the call's sequence number, so a reader whose slot was reused
// by a later call (more than kTimingRing calls in between) can tell
TimedCall* timed_begin(Device& d, hipStream_t s) {
  std::lock_guard<std::mutex> g(d.tmu);
  const uint64_t seq = ++d.ring_next;
  const int idx = (int)(seq % kTimingRing);
  TimedCall* tc = &d.ring[idx];
  tc->gen = seq;
  if (hipEventRecord(tc->a, s) != hipSuccess) return nullptr;
  tl_last_call[d.uid] = {idx, seq};
  return tc;
}

// A leased set's buffers for a host tx path: the last device-path user of the
// set may still be running kernels on its own stream.
int tx_acquire_host(Device& d, TxSet& set) {
  if (hipSetDevice(d.id) != hipSuccess) return CORDAHIP_ERR_HIP;
  if (hipEventSynchronize(set.tx_ev) != hipSuccess) return CORDAHIP_ERR_HIP;
  return CORDAHIP_SUCCESS;
}

// Transaction ids for txs [t0, t1) on one device. The caller's offset arrays go
// to the device as they are (absolute offsets, no host rebasing pass): the
// kernels get base pointers shifted by the shard's first byte / first leaf.
int tx_ids_shard(cordahip_ctx* ctx, Device& d, const cordahip_txid_batch* b, uint64_t t0, uint64_t t1) {
  (void)ctx;
  SetLease lease(d);
  TxSet& S = lease.get();
  const NodeBind nb(d);
  const Activity act(d);
  if (int rc = tx_acquire_host(d, S)) return rc;
  const uint64_t ntx = t1 - t0;
  const uint64_t l0 = b->tx_leaf_off[t0], l1 = b->tx_leaf_off[t1];
  const uint64_t nleaves = l1 - l0;
  const uint64_t b0 = b->leaf_off[l0], b1 = b->leaf_off[l1];
  TxWork& w = S.tx;
  if (w.leaf_bytes.ensure(std::max<uint64_t>(b1 - b0, 16)) || w.leaf_off.ensure((nleaves + 1) * 8) ||
      w.tx_leaf_off.ensure((ntx + 1) * 8) || w.hashes.ensure(std::max<uint64_t>(nleaves, 1) * 32) ||
      w.txid.ensure(ntx * 32) || w.tx_status.ensure(ntx))
    return CORDAHIP_ERR_OUT_OF_MEMORY;
  hipStream_t s = d.stream;
  hipError_t e = hipSuccess;
  if (b1 > b0) e = hipMemcpyAsync(w.leaf_bytes.p, b->leaf_bytes + b0, b1 - b0, hipMemcpyHostToDevice, s);
  e = e ? e : hipMemcpyAsync(w.leaf_off.p, b->leaf_off + l0, (nleaves + 1) * 8, hipMemcpyHostToDevice, s);
  e = e ? e : hipMemcpyAsync(w.tx_leaf_off.p, b->tx_leaf_off + t0, (ntx + 1) * 8, hipMemcpyHostToDevice, s);
  // leaf i's bytes at leaf_bytes + (leaf_off[l0 + i] - b0); tx t's hashes at hashes + (tx_leaf_off[t] - l0) * 8
  const uint8_t* bytes_base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(w.leaf_bytes.p) - b0);
  uint32_t* hash_base = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(w.hashes.p) - l0 * 32);
  e = e ? e : launch_sha256_leaves(bytes_base, w.leaf_off.as<uint64_t>(), nleaves, w.hashes.as<uint32_t>(), s);
  e = e ? e : launch_merkle_root(hash_base, w.tx_leaf_off.as<uint64_t>(), ntx, w.txid.as<uint8_t>(),
                                 w.tx_status.as<uint8_t>(), s);
  e = e ? e : hipMemcpyAsync(b->txid + t0 * 32, w.txid.p, ntx * 32, hipMemcpyDeviceToHost, s);
  e = e ? e : hipMemcpyAsync(b->tx_status + t0, w.tx_status.p, ntx, hipMemcpyDeviceToHost, s);
  e = e ? e : hipEventRecord(S.tx_ev, s);
  e = e ? e : hipEventSynchronize(S.tx_ev);
  if (e != hipSuccess) (void)hipStreamSynchronize(s);
  return hip_err(e);
}

int tx_ids_impl(cordahip_ctx* ctx, const cordahip_txid_batch* b) {
  if (b->ntx && (!b->leaf_off || !b->tx_leaf_off || !b->txid || !b->tx_status || !b->leaf_bytes))
    return CORDAHIP_ERR_INVALID_ARG;
  if (b->ntx == 0) return CORDAHIP_SUCCESS;
  if (!check_txid_batch(PoolPar{*ctx->host}, b)) return CORDAHIP_ERR_INVALID_ARG;  // before any enqueue
  // contiguous tx shards: a transaction's tree stays on one device
  return for_shards(ctx->devs, b->ntx, 1,
                    [&](Device& d, uint64_t t0, uint64_t t1) { return tx_ids_shard(ctx, d, b, t0, t1); });
}

// The tx ids of one device's shard, in slices on the device's context stream
// (the set S leased, its previous users finished): slice j's leaf bytes and
// offsets go H2D into their region of whole-shard buffers (offset arrays
// unchanged, shifted base pointers) on d.s_idcopy, followed by cev[j]; its
// SHA-256 and Merkle kernels run on the context stream behind cev[j], then
// kev[j] marks its ids in HBM, its ids and statuses come back, and ev[j] marks
// them on the host. tx_ids_prepare sizes the buffers once; tx_ids_enqueue
// enqueues slices [j0, j1) (the signed-tx path releases them a few at a time,
// interleaved with the signature chunks' copies, because H2D copies of all
// streams leave through the DMA engine in submission order).
// Leaf bytes one component may need (kryo_core.hpp): the kind's constant text
// (class and field names, framing; < 2 KB for a cash state) plus at most 4
// bytes per payload byte (a cash state writes the owner's key and name up to 3
// times; a string 3 bytes per UTF-16 unit). A leaf beyond its slice's bound
// would be reported, not written (CORDAHIP_TX_BAD_COMPONENT);
// tests/test_kryo_template.py checks the bound on every test item.
uint64_t comp_leaf_bound(uint64_t payload_bytes) { return 4096 + 4 * payload_bytes; }
uint64_t comp_payload_bytes(const cordahip_kryo_item& it) {
  return (it.kind == CORDAHIP_KRYO_STRING || it.kind == CORDAHIP_KRYO_KOTLIN_OBJECT) ? 2 * it.len : it.len;
}

// Component-level batches (cordahip_txcomp_batch): per id slice, how far the
// payload must reach, the leaf buffer it needs, and its items per tx.
// The payload crosses PCIe as two windows: the low one [0, low_end) -- the
// payloads below `split`, in practice those every transaction shares (the
// notary Party, TransactionType), written first -- once with the first slice,
// and the high one [high_min, pay_end[j]) growing slice by slice. Any split
// covers every item (an item lies below it or not); taking it at the shard's
// first transaction's last payload makes the high window start at this shard's
// own payloads, so a device of a multi-device context no longer copies the
// earlier shards' payloads (r05 copied [0, pay_end) on every device).
struct CompPlan {
  const cordahip_txcomp_batch* c = nullptr;
  std::vector<uint64_t> pay_end;  // high-window bytes slices 0..j reference (running max)
  std::vector<uint32_t> group;    // items per transaction when uniform in the slice (the encoder's hint), else 1
  uint64_t slice_cap = 16;        // leaf bytes of the largest piece's bound (the full chain's one leaf buffer)
  std::vector<std::vector<uint64_t>> cuts;  // per slice: the transactions that start a new piece of the full chain
  uint64_t max_items = 0;
  uint64_t split = 0;             // items at offsets below it are the low window's
  uint64_t low_end = 0;           // the low window [0, low_end)
  uint64_t high_min = UINT64_MAX; // the high window's first byte
  uint64_t copied = 0;            // high window enqueued up to here (from high_min)
  bool low_copied = false;
  bool templates_only = false;    // the steady-state encoder chain (misses redo the call)
  static constexpr uint64_t kDirectWriters = 1u << 13;  // the direct encoder's writers (rarely any work)
};

hipError_t tx_ids_prepare(cordahip_ctx* ctx, Device& d, TxSet& S, int set_idx, const cordahip_txid_batch* b,
                          const std::vector<uint64_t>& bound, CompPlan* cp) {
  const uint64_t t0 = bound.front(), t1 = bound.back(), ntx = t1 - t0;
  const uint64_t l0 = b->tx_leaf_off[t0], l1 = b->tx_leaf_off[t1], nleaves = l1 - l0;
  TxWork& w = S.tx;
  uint64_t leaf_buf = 0;
  if (cp) {
    const cordahip_txcomp_batch* c = cp->c;
    const size_t ns = bound.size() - 1;
    cp->pay_end.assign(ns, 0);
    cp->group.assign(ns, 1);
    cp->cuts.assign(ns, {});
    // the full chain's leaf buffer: a tenth of the device budget at most (the budget's
    // share for component slices; C4's 2^17-signature slices bound ~1.4 GB, far below
    // the default's 13.7 GB); a slice whose bound exceeds it is encoded and hashed in
    // pieces of whole transactions, one after another through the one buffer
    const uint64_t piece_cap = std::max<uint64_t>(d.mem_budget / 10, 1u << 20);
    std::vector<uint64_t> cap(ns, 0), low(ns, 0), hmin(ns, UINT64_MAX);
    auto fits = [&](const cordahip_kryo_item& it, uint64_t& off, uint64_t& nb) {
      off = (uint64_t)(uintptr_t)it.data;
      nb = comp_payload_bytes(it);
      return off <= c->payload_len && nb <= c->payload_len - off;
    };
    cp->split = 0;  // the shard's first transaction's last payload (its own, past the shared ones)
    for (uint64_t i = c->tx_item_off[t0]; i < c->tx_item_off[t0 + 1]; i++) {
      uint64_t off, nb;
      if (fits(c->items[i], off, nb) && nb) cp->split = std::max(cp->split, off);
    }
    pool_of(ctx, d).parallel_for(ns, 1, [&](uint64_t x, uint64_t y) {
      for (uint64_t j = x; j < y; j++) {
        const uint64_t ts0 = bound[j], ts1 = bound[j + 1];
        const uint64_t g = ts1 > ts0 ? c->tx_item_off[ts0 + 1] - c->tx_item_off[ts0] : 1;
        bool uniform = g > 0;
        uint64_t end = 0, bd = 0, lo_end = 0, hi_min = UINT64_MAX, piece_max = 0;
        for (uint64_t t = ts0; t < ts1; t++) {
          uniform = uniform && c->tx_item_off[t + 1] - c->tx_item_off[t] == g;
          const uint64_t bd_tx = bd;
          for (uint64_t i = c->tx_item_off[t]; i < c->tx_item_off[t + 1]; i++) {
            const cordahip_kryo_item& it = c->items[i];
            uint64_t off, nb;
            const bool ok = fits(it, off, nb);
            if (it.kind != CORDAHIP_KRYO_RAW && nb == 0) {
              bd += comp_leaf_bound(0);
              continue;
            }
            if (ok) {
              if (off < cp->split) {
                lo_end = std::max(lo_end, off + nb);
              } else {
                hi_min = std::min(hi_min, off);
                end = std::max(end, off + nb);
              }
            }
            bd += comp_leaf_bound(ok ? nb : 0);
          }
          if (bd > piece_cap && bd_tx > 0 && t > ts0) {  // t starts a new piece
            cp->cuts[j].push_back(t);
            piece_max = std::max(piece_max, bd_tx);
            bd -= bd_tx;
          }
        }
        cp->pay_end[j] = end;
        low[j] = lo_end;
        hmin[j] = hi_min;
        cp->group[j] = uniform && g <= 64 ? (uint32_t)g : 1;
        cap[j] = std::max(piece_max, bd);
      }
    });
    cp->low_end = 0;
    cp->high_min = UINT64_MAX;
    for (size_t j = 0; j < ns; j++) {
      cp->low_end = std::max(cp->low_end, low[j]);
      cp->high_min = std::min(cp->high_min, hmin[j]);
    }
    if (cp->high_min == UINT64_MAX) cp->high_min = 0;
    for (size_t j = 0; j < ns; j++) {
      if (j) cp->pay_end[j] = std::max(cp->pay_end[j], cp->pay_end[j - 1]);
      cp->slice_cap = std::max(cp->slice_cap, cap[j]);
      cp->max_items = std::max(cp->max_items, b->tx_leaf_off[bound[j + 1]] - b->tx_leaf_off[bound[j]]);
    }
    cp->copied = cp->high_min;
    cp->low_copied = false;
    // the templates-only chain hashes the leaves from their templates: no leaf buffers
    // (the full chain's leaf buffer is bounded at 4 KB + 4 B per payload byte per
    // component of its largest piece: ~1.4 GB for C4's 2^17-signature slices)
    cp->templates_only = cp->templates_only && d.kryo_templates_ok;
    if (w.comp_items.ensure(std::max<uint64_t>(nleaves, 1) * sizeof(cordahip_kryo_item)) ||
        w.payload.ensure(std::max<uint64_t>(std::max(ns ? cp->pay_end.back() : 0, cp->low_end), 16)) ||
        w.comp_status.ensure(std::max<uint64_t>(nleaves, 1)))
      return hipErrorOutOfMemory;
    // the encoder's scratch (d.kryo_*, kryo_mu held by the caller) for the largest slice
    const uint64_t n = cp->max_items;
    size_t temp_bytes = 0;
    if (hipError_t e = kryo_scan_bytes(temp_bytes, n + 1, d.stream)) return e;
    if (d.kryo_sizes.cap < (n + 1) * 8 || d.kryo_temp.cap < temp_bytes || d.kryo_items.cap < n * 8 + 8 ||
        d.kryo_ws.cap < kryo_direct_ws_bytes(CompPlan::kDirectWriters) || d.kryo_fixed.cap < kryo_fixed_scratch_bytes()) {
      if (d.kryo_ev && hipEventSynchronize(d.kryo_ev) != hipSuccess) return hipErrorUnknown;
      if (d.kryo_sizes.ensure((n + 1) * 8) || d.kryo_temp.ensure(std::max<size_t>(temp_bytes, 16)) ||
          d.kryo_items.ensure(n * 8 + 8) || d.kryo_ws.ensure(kryo_direct_ws_bytes(CompPlan::kDirectWriters)) ||
          kryo_fixed_ensure(d))
        return hipErrorOutOfMemory;
    }
    if (hipError_t e = usage_buffer(S.kryo_usage, S.kryo_usage_dev)) return e;
    if (hipError_t e = kryo_state_ready(d, d.stream)) return e;
    if (hipError_t e = kryo_reset_misses(d.kryo_fixed.as<uint8_t>(), (uint32_t)set_idx, d.stream)) return e;
    cp->templates_only = cp->templates_only && d.kryo_templates_ok;  // kryo_state_ready may have cleared the table
    // sized after that: a cleared table runs the full chain, which writes leaves
    leaf_buf = cp->templates_only ? 0 : cp->slice_cap;
    if (tracing())
      fprintf(stderr, "[cordahip] dev %d set %d component call: %s chain (templates %u, slots %u in use)\n", d.id,
              set_idx, cp->templates_only ? "templates-only" : "full encoder", S.kryo_usage[0], S.kryo_usage[1]);
  } else {
    leaf_buf = b->leaf_off[l1] - b->leaf_off[l0];
  }
  if (w.leaf_bytes.ensure(std::max<uint64_t>(leaf_buf, 16)) || w.leaf_off.ensure((nleaves + 1) * 8) ||
      w.tx_leaf_off.ensure((ntx + 1) * 8) || w.hashes.ensure(std::max<uint64_t>(nleaves, 1) * 32) ||
      w.txid.ensure(std::max<uint64_t>(ntx, 1) * 32) || w.tx_status.ensure(std::max<uint64_t>(ntx, 1)))
    return hipErrorOutOfMemory;
  return hipSuccess;
}

hipError_t tx_ids_enqueue(Device& d, TxSet& S, int set_idx, const cordahip_txid_batch* b,
                          const std::vector<uint64_t>& bound, size_t j0, size_t j1, std::vector<hipEvent_t>& ev,
                          std::vector<hipEvent_t>& cev, std::vector<hipEvent_t>& kev, uint8_t* map_txid,
                          uint8_t* map_status, CompPlan* cp) {
  const uint64_t t0 = bound.front();
  const uint64_t l0 = b->tx_leaf_off[t0], b0 = cp ? 0 : b->leaf_off[l0];
  TxWork& w = S.tx;
  hipStream_t s = d.stream, sc = d.s_idcopy ? d.s_idcopy : d.stream;
  const hipMemcpyKind h2d = hipMemcpyHostToDevice, d2h = hipMemcpyDeviceToHost;
  const uint8_t* bytes_base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(w.leaf_bytes.p) - b0);
  uint32_t* hash_base = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(w.hashes.p) - l0 * 32);
  hipError_t e = hipSuccess;
  for (size_t j = j0; j < j1 && e == hipSuccess; j++) {
    const uint64_t ts0 = bound[j], ts1 = bound[j + 1];
    const uint64_t ls0 = b->tx_leaf_off[ts0], ls1 = b->tx_leaf_off[ts1];
    if (!cp) {
      const uint64_t bs0 = b->leaf_off[ls0], bs1 = b->leaf_off[ls1];
      if (bs1 > bs0)
        e = blocked("leaf-bytes H2D", [&] {
          return hipMemcpyAsync(w.leaf_bytes.as<uint8_t>() + (bs0 - b0), b->leaf_bytes + bs0, bs1 - bs0, h2d, sc);
        });
      e = e ? e : hipMemcpyAsync(w.leaf_off.as<uint64_t>() + (ls0 - l0), b->leaf_off + ls0, (ls1 - ls0 + 1) * 8, h2d, sc);
    } else {
      // the slice's components, and the payload prefix they reach
      const cordahip_txcomp_batch* c = cp->c;
      if (ls1 > ls0)
        e = hipMemcpyAsync(w.comp_items.as<cordahip_kryo_item>() + (ls0 - l0), c->items + ls0,
                           (ls1 - ls0) * sizeof(cordahip_kryo_item), h2d, sc);
      if (e == hipSuccess && !cp->low_copied) {  // the low window, once (the shared payloads)
        cp->low_copied = true;
        if (cp->low_end)
          e = hipMemcpyAsync(w.payload.as<uint8_t>(), c->payload, cp->low_end, h2d, sc);
      }
      if (e == hipSuccess && cp->pay_end[j] > cp->copied) {  // the high window grows with the slices
        e = blocked("payload H2D", [&] {
          return hipMemcpyAsync(w.payload.as<uint8_t>() + cp->copied, c->payload + cp->copied,
                                cp->pay_end[j] - cp->copied, h2d, sc);
        });
        cp->copied = cp->pay_end[j];
      }
    }
    e = e ? e : hipMemcpyAsync(w.tx_leaf_off.as<uint64_t>() + (ts0 - t0), b->tx_leaf_off + ts0, (ts1 - ts0 + 1) * 8, h2d, sc);
    e = e ? e : hipEventRecord(cev[j], sc);
    e = e ? e : hipStreamWaitEvent(s, cev[j], 0);
    if (cp && cp->templates_only) {
      // steady state: shapes, then every leaf's SHA-256 straight from its template
      // (no leaf bytes in HBM)
      uint32_t* slots = d.kryo_items.as<uint32_t>();
      const uint64_t n = ls1 - ls0;
      const cordahip_kryo_item* it = w.comp_items.as<cordahip_kryo_item>() + (ls0 - l0);
      uint8_t* cst = w.comp_status.as<uint8_t>() + (ls0 - l0);
      // shapes and hashes in one launch per slice (the shape pass inside kryo_hash's
      // template-grouped blocks): c4h --components at two calls in flight 88.7-90.1 ->
      // 91.3-92.1 M sig/s, alternating on one box (profiles/r06_kryo_fused_ab/);
      // CORDAHIP_KRYO_FUSED=0: the two launches
      static const bool fused = !(getenv("CORDAHIP_KRYO_FUSED") && getenv("CORDAHIP_KRYO_FUSED")[0] == '0');
      if (fused) {
        e = e ? e : launch_kryo_shape_hash(it, w.payload.as<uint8_t>(), cp->c->payload_len, n, cp->group[j],
                                           d.kryo_fixed.as<uint8_t>(), cst, w.hashes.as<uint32_t>() + (ls0 - l0) * 8,
                                           s, (uint32_t)set_idx);
      } else {
        e = e ? e : launch_kryo_shape(it, w.payload.as<uint8_t>(), cp->c->payload_len, n, cp->group[j],
                                      d.kryo_fixed.as<uint8_t>(), slots, slots + n, d.kryo_sizes.as<uint64_t>(), cst, s,
                                      true, (uint32_t)set_idx);
        e = e ? e : launch_kryo_hash(it, w.payload.as<uint8_t>(), cp->c->payload_len, n, cp->group[j],
                                     d.kryo_fixed.as<uint8_t>(), slots, d.kryo_sizes.as<uint64_t>(), cst,
                                     w.hashes.as<uint32_t>() + (ls0 - l0) * 8, s);
      }
    } else if (cp) {
      // the slice's leaves on the GPU (the template encoder) into the leaf buffer,
      // offsets relative to it, then their SHA-256; piece by piece (whole
      // transactions) when the slice's bound exceeds the buffer. Every piece runs
      // on s, so the next piece's writes follow the previous piece's hashing.
      uint8_t* sb = w.leaf_bytes.as<uint8_t>();
      uint32_t* slots = d.kryo_items.as<uint32_t>();
      uint64_t pa = ts0;
      for (size_t k = 0; k <= cp->cuts[j].size() && e == hipSuccess; k++) {
        const uint64_t pb = k < cp->cuts[j].size() ? cp->cuts[j][k] : ts1;
        const uint64_t is0 = b->tx_leaf_off[pa], n = b->tx_leaf_off[pb] - is0;
        pa = pb;
        if (!n) continue;
        e = launch_kryo_encode(w.comp_items.as<cordahip_kryo_item>() + (is0 - l0), w.payload.as<uint8_t>(),
                               cp->c->payload_len, n, cp->group[j], d.kryo_fixed.as<uint8_t>(), slots, slots + n,
                               d.kryo_sizes.as<uint64_t>(), w.leaf_off.as<uint64_t>() + (is0 - l0), sb, cp->slice_cap,
                               w.comp_status.as<uint8_t>() + (is0 - l0), d.kryo_ws.as<uint8_t>(),
                               CompPlan::kDirectWriters, d.kryo_temp.p, d.kryo_temp.cap, s, cp->templates_only,
                               (uint32_t)set_idx);
        e = e ? e : launch_sha256_leaves(sb, w.leaf_off.as<uint64_t>() + (is0 - l0), n,
                                         w.hashes.as<uint32_t>() + (is0 - l0) * 8, s);
      }
    } else {
      e = e ? e : blocked("sha256_leaves launch", [&] {
        return launch_sha256_leaves(bytes_base, w.leaf_off.as<uint64_t>() + (ls0 - l0), ls1 - ls0,
                                    w.hashes.as<uint32_t>() + (ls0 - l0) * 8, s);
      });
    }
    // the ids, and in the same launch: a component the encoder rejected (no id for its
    // transaction, CORDAHIP_TX_BAD_COMPONENT) and the stores into pinned caller arrays
    // through their device mapping (three launches per slice before r05)
    const uint8_t* st_base =
        cp ? reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(w.comp_status.p) - l0) : nullptr;
    const bool mapped = ts1 > ts0 && map_txid && map_status;
    e = e ? e : launch_merkle_root(hash_base, w.tx_leaf_off.as<uint64_t>() + (ts0 - t0), ts1 - ts0,
                                   w.txid.as<uint8_t>() + (ts0 - t0) * 32, w.tx_status.as<uint8_t>() + (ts0 - t0), s,
                                   st_base, mapped ? map_txid + ts0 * 32 : nullptr, mapped ? map_status + ts0 : nullptr);
    e = e ? e : hipEventRecord(kev[j], s);  // the slice's ids are in HBM: its signatures may gather them
    if (mapped) {
      // stored by merkle_root
    } else if (ts1 > ts0) {
      e = e ? e : blocked("ids D2H", [&] {
        return hipMemcpyAsync(b->txid + ts0 * 32, w.txid.as<uint8_t>() + (ts0 - t0) * 32, (ts1 - ts0) * 32, d2h, s);
      });
      e = e ? e : blocked("id status D2H", [&] {
        return hipMemcpyAsync(b->tx_status + ts0, w.tx_status.as<uint8_t>() + (ts0 - t0), ts1 - ts0, d2h, s);
      });
    }
    e = e ? e : hipEventRecord(ev[j], s);
  }
  if (e == hipSuccess && j1 + 1 == bound.size()) {
    // the last slice: the encoder's usage report, then the fences of the set's
    // buffers (S.tx_ev: the call's drain waits on it) and of the encoder's
    // scratch (d.kryo_*)
    if (cp) e = kryo_usage_report(d, &S, s);
    e = e ? e : hipEventRecord(S.tx_ev, s);
    if (cp && e == hipSuccess) {
      if (!d.kryo_ev) e = e ? e : hipEventCreateWithFlags(&d.kryo_ev, hipEventDisableTiming);
      e = e ? e : hipEventRecord(d.kryo_ev, s);
    }
  }
  return e;
}

// The per-transaction verdict of txs [t0, t1) from their id statuses and
// signature statuses (SignedTransaction.verifySignaturesExcept -> the first
// signature that fails, SignedTransaction.kt:95-100): first_bad_sig, and the
// tx status becomes that signature's status.
void reduce_txs(HostPool& pool, const cordahip_signed_tx_batch* b, uint64_t t0, uint64_t t1) {
  if (t0 >= t1) return;
  pool.parallel_for(t1 - t0, 4096, [&](uint64_t x, uint64_t y) {
    for (uint64_t t = t0 + x; t < t0 + y; t++) {
      const uint64_t lo = b->tx_sig_off[t], hi = b->tx_sig_off[t + 1];
      b->first_bad_sig[t] = -1;
      if (lo == hi) {  // require(sigs.isNotEmpty()) in the constructor (SignedTransaction.kt:37-39) precedes tx.id
        b->tx.tx_status[t] = CORDAHIP_TX_NO_SIGNATURES;
        continue;
      }
      if (b->tx.tx_status[t] != CORDAHIP_STATUS_OK) {  // tx.id threw before any signature was checked
        for (uint64_t s = lo; s < hi; s++) b->sig_status[s] = b->tx.tx_status[t];
        continue;
      }
      for (uint64_t s = lo; s < hi; s++)
        if (b->sig_status[s] != CORDAHIP_STATUS_OK) {
          b->first_bad_sig[t] = (int64_t)(s - lo);
          b->tx.tx_status[t] = b->sig_status[s];
          break;
        }
    }
  });
}

// SignedTransaction.checkSignaturesAreValid over the batch: tx ids (K3/K4),
// every signature over its tx's id (the generic signature pipeline), then the
// per-tx first failing signature. Each device takes a contiguous shard of the
// transactions AND their signatures (a transaction's leaves and signatures stay
// on one GPU). Its ids are computed in slices (tx_ids_enqueue: slice
// j + 1's leaf bytes cross PCIe on their own stream while slice j hashes), each
// slice marking an event when its ids are in HBM. The signature pipeline runs
// over the shard's signatures in chunks of one or more whole slices: it packs
// and copies keys and signatures without waiting for any id -- they do not
// depend on the ids -- plus each row's id index, and the GPU gathers the message
// rows from the ids in HBM after the slice's event (gather_rows32). Slices are
// released just ahead of the chunk that needs them and `lookahead` more after
// its copies (DeviceIds::advance), so the DMA engine, which serves H2D copies in
// submission order, interleaves leaf bytes and signature chunks. The ids go to
// the caller (txid) on the side; no signature waits for an id to reach the
// host. (r03 waited for each slice's ids on the host and copied them back as
// messages: the GPU sat idle ~5 ms per C4 step until the first signatures were
// packed.)
// Consecutive calls on one device overlap (r06): a call holds one of the
// device's two buffer sets (SetLease: ids, leaf / component buffers, the
// signature stages) from start to finish, but the device's enqueue token
// (tx_order_mu) -- and, for component batches, the encoder's scratch lock
// (kryo_mu) -- only until its last signature chunk and id slice are enqueued.
// The next call then packs and enqueues its first slices and chunks while this
// one drains (its last chunks' ladders, the statuses, the per-tx reduce), so
// the GPU no longer idles through each call's fill (the first slice's leaf
// bytes and pack) and drain. Work reaches the shared streams in call order; a
// call's drain waits on its own events, never on the streams.
constexpr int kRedoFull = -1000;  // a templates-only component call missed: run it again with the full encoder

int signed_tx_device_once(cordahip_ctx* ctx, Device& d, const cordahip_signed_tx_batch* b, uint64_t* tx_of,
                          uint64_t lo, uint64_t hi, uint64_t slices, const cordahip_txcomp_batch* comps,
                          bool templates_only) {
  SetLease lease(d);  // S.tx (the ids) and S.pb stay ours until every gather has run
  TxSet& S = lease.get();
  const int set_idx = lease.index();
  const NodeBind nb(d);  // this thread packs and first-touches on the GPU's NUMA node
  const Activity act(d);
  std::unique_lock<std::mutex> tok(d.tx_order_mu);
  // component batches also enqueue on the GPU encoder's shared scratch (d.kryo_*)
  std::unique_lock<std::mutex> gk(d.kryo_mu, std::defer_lock);
  CompPlan plan, *cp = nullptr;
  uint64_t gen = 0;
  if (comps) {
    gk.lock();
    plan.c = comps;
    plan.templates_only = templates_only;
    cp = &plan;
  }
  int r = tx_acquire_host(d, S);
  if (r == CORDAHIP_SUCCESS && ensure_streams(d) != hipSuccess) r = CORDAHIP_ERR_HIP;
  if (r == CORDAHIP_SUCCESS && cp && d.kryo_ev && hipStreamWaitEvent(d.stream, d.kryo_ev, 0) != hipSuccess)
    r = CORDAHIP_ERR_HIP;  // an earlier cordahip_kryo_encode_device still using the scratch
  if (r != CORDAHIP_SUCCESS) return r;
  DeviceIds di;
  const uint64_t s0 = b->tx_sig_off[lo], s1 = b->tx_sig_off[hi];
  // signature chunks of whole full-occupancy rounds of the Ed25519 ladder
  // (2^17 lanes: 2 waves x 1,024 SIMDs x 64), each waiting on device for the
  // slice that holds its last transaction. r04 ran half rounds (2^16: the GPU
  // starts after the leaf bytes of fewer transactions, and two Ed25519 streams
  // keep two chunks in flight so one chunk's tail overlaps the next). Since the
  // id kernels run at raised wave priority (tx.hip g_id_prio) a slice's ids no
  // longer trail the ladders, and whole rounds win: interleaved on one corpus,
  // c4h 84.1 against 81.6 M sig/s, c4h --components 75.0 against 72.3; 2^18:
  // 70.3 (profiles/r05_c4h_chunk_ab/).
  uint64_t chunk = 1u << 17;
  if (const char* v = getenv("CORDAHIP_TX_SIG_CHUNK")) chunk = std::max<uint64_t>(1, strtoull(v, nullptr, 10));
  // chunks double from `chunk` up to CORDAHIP_TX_SIG_CHUNK_MAX (default: chunk,
  // constant chunks; 2^16 doubling to 2^17 ran 83.9 against 84.1 M/s, r05)
  uint64_t chunk_max = chunk;
  if (const char* v = getenv("CORDAHIP_TX_SIG_CHUNK_MAX")) chunk_max = std::max<uint64_t>(chunk, strtoull(v, nullptr, 10));
  for (uint64_t x = s0, c = chunk; x < s1; x += c, c = std::min(chunk_max, 2 * c)) di.chunk_bound.push_back(x);
  di.chunk_bound.push_back(s1);
  if (slices == 0 && s1 > s0) {
    // default: the id slices follow the chunks -- slice k ends with chunk k's
    // last transaction, so chunk k waits for exactly its own ids, and the first
    // slice's leaf bytes (what the GPU waits for before its first ladder) are
    // one round's worth, not a sixteenth of the shard (r04_n trace: 1.1 ms of
    // PCIe before the first kernel)
    di.tx_bound.push_back(lo);
    for (size_t c = 1; c + 1 < di.chunk_bound.size(); c++) {
      // one past the transaction holding the chunk's last signature (tx_of is
      // not filled yet: it is built while slice 0 crosses PCIe)
      const uint64_t t = (uint64_t)(std::upper_bound(b->tx_sig_off + lo, b->tx_sig_off + hi + 1,
                                                     di.chunk_bound[c] - 1) - b->tx_sig_off);
      if (t > di.tx_bound.back() && t < hi) di.tx_bound.push_back(t);
    }
    di.tx_bound.push_back(hi);
    slices = di.tx_bound.size() - 1;
  } else {  // CORDAHIP_TX_SLICES, or no signatures: uniform slices
    slices = std::max<uint64_t>(1, std::min<uint64_t>(slices ? slices : 1, hi - lo));
    for (uint64_t q = 0; q <= slices; q++) di.tx_bound.push_back(lo + (hi - lo) * q / slices);
  }
  std::vector<hipEvent_t> ev(slices, nullptr), cev(slices, nullptr);
  di.ready.assign(slices, nullptr);
  struct Events {  // destroyed on every exit
    std::vector<hipEvent_t>* v[3];
    ~Events() {
      for (auto* x : v)
        for (hipEvent_t e : *x)
          if (e) (void)hipEventDestroy(e);
    }
  } events{{&ev, &cev, &di.ready}};
  for (auto* v : {&ev, &cev, &di.ready})
    for (auto& e : *v)
      if (r == CORDAHIP_SUCCESS && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) r = CORDAHIP_ERR_HIP;
  // slices go out a few ahead of the signature chunk that needs them (the
  // chunk's own H2D follows them through the DMA engine in submission order):
  // with every slice enqueued first, r04's first signature copies waited ~20 ms
  // behind all of C4's 1.05 GB of leaf bytes
  size_t issued = 0;
  uint8_t* map_txid = static_cast<uint8_t*>(host_mapped(b->tx.txid));
  uint8_t* map_status = static_cast<uint8_t*>(host_mapped(b->tx.tx_status));
  uint64_t lookahead = 1;  // r04_o: 1 slice ahead 73.6 M/s, 2 ahead 73.1
  if (const char* v = getenv("CORDAHIP_TX_SLICE_AHEAD")) lookahead = strtoull(v, nullptr, 10);
  auto issue_through = [&](size_t j) -> hipError_t {  // enqueue slices [issued, j]
    const size_t j1 = std::min<size_t>(slices, j + 1);
    hipError_t e = hipSuccess;
    if (j1 > issued)
      e = tx_ids_enqueue(d, S, set_idx, &b->tx, di.tx_bound, issued, j1, ev, cev, di.ready, map_txid, map_status, cp);
    issued = std::max(issued, j1);
    return e;
  };
  // the end of this call's enqueues: the slices no signature asked for
  // (transactions without signatures at the end), then the token and the
  // encoder's scratch go to the next call (idempotent: called by the pipeline
  // once its last chunk is enqueued, and after it)
  bool handed_on = false;
  auto hand_on = [&]() -> hipError_t {
    if (handed_on) return hipSuccess;
    handed_on = true;
    const hipError_t e = issue_through(slices);
    if (gk.owns_lock()) gk.unlock();
    if (tok.owns_lock()) tok.unlock();
    return e;
  };
  if (r == CORDAHIP_SUCCESS && tx_ids_prepare(ctx, d, S, set_idx, &b->tx, di.tx_bound, cp) != hipSuccess)
    r = CORDAHIP_ERR_OUT_OF_MEMORY;
  if (cp) gen = d.kryo_gen;  // after a clear in prepare: this call builds the new table's shapes
  if (r == CORDAHIP_SUCCESS && issue_through(0) != hipSuccess) r = CORDAHIP_ERR_HIP;
  // each signature signs its transaction's id (SignedTransaction.kt:98): the
  // pipeline finds it through tx_of, filled chunk by chunk just ahead of its use
  // (fill_to, from di.advance) -- built whole before the first chunk it held the
  // first pack ~0.5 ms (r05 host trace: C4's 2.5 M signatures)
  uint64_t filled = s0;  // tx_of holds signatures [s0, filled)
  auto fill_to = [&](uint64_t s_end) {
    s_end = std::min(s_end, s1);
    if (s_end <= filled) return;
    const uint64_t* so = b->tx_sig_off;
    const uint64_t ta = (uint64_t)(std::upper_bound(so + lo, so + hi + 1, filled) - so) - 1;
    const uint64_t tb = (uint64_t)(std::upper_bound(so + lo, so + hi + 1, s_end - 1) - so);
    const uint64_t f0 = filled;
    pool_of(ctx, d).parallel_for(tb - ta, 4096, [&](uint64_t x, uint64_t y) {
      for (uint64_t t = ta + x; t < ta + y; t++)
        for (uint64_t q = std::max(so[t], f0); q < std::min(so[t + 1], s_end); q++) tx_of[q] = t;
    });
    filled = s_end;
  };
  std::vector<std::pair<uint64_t, uint64_t>> reduced;  // tx ranges the chunks reduced
  if (r == CORDAHIP_SUCCESS && s1 > s0) {
    di.txid = S.tx.txid.as<uint8_t>();
    di.t0 = lo;
    // CORDAHIP_TX_SPLIT_PREP (A/B): 0 fused prep everywhere, 1 split for component batches
    // too; default split for leaf batches only (r05, profiles/r05_prep_split_ab/)
    static const int split_env = getenv("CORDAHIP_TX_SPLIT_PREP") ? atoi(getenv("CORDAHIP_TX_SPLIT_PREP")) : -1;
    di.split_prep = split_env < 0 ? cp == nullptr : split_env > 0;
    // before a chunk's copies: the slices it needs; after them: `lookahead` more,
    // so PCIe carries leaf bytes while the GPU verifies the chunk
    di.advance = [&](uint64_t sig_end, bool after) {
      // after: the slices of the next `lookahead` chunks' signatures
      const uint64_t e = after ? std::min(s1, sig_end + lookahead * chunk_max) : sig_end;
      fill_to(e);
      const uint64_t tx = tx_of[e - 1];
      const size_t j = (size_t)(std::upper_bound(di.tx_bound.begin(), di.tx_bound.end(), tx) - di.tx_bound.begin()) - 1;
      return issue_through(j);
    };
    di.enqueued = hand_on;
    // each finished chunk reduces the transactions whose signatures it holds
    // entirely (once their ids are on the host), overlapped with later chunks'
    // GPU work: the whole-batch pass after the drain was ~0.55 ms of a 32 ms
    // C4 call with the GPU idle; edge transactions are reduced after the drain
    di.done = [&](uint64_t a, uint64_t e) -> hipError_t {
      uint64_t t0 = tx_of[a], t1 = tx_of[e - 1];
      if (b->tx_sig_off[t0] != a) t0++;       // starts in an earlier chunk
      if (b->tx_sig_off[t1 + 1] == e) t1++;   // ends here: included
      if (t0 >= t1) return hipSuccess;
      const size_t j0 = (size_t)(std::upper_bound(di.tx_bound.begin(), di.tx_bound.end(), t0) - di.tx_bound.begin()) - 1;
      const size_t j1 = (size_t)(std::upper_bound(di.tx_bound.begin(), di.tx_bound.end(), t1 - 1) - di.tx_bound.begin());
      for (size_t j = j0; j < j1; j++) {  // their slices' ids and statuses are back (issued: the chunk needed them)
        if (j >= issued) return hipErrorInvalidValue;
        if (hipError_t x = blocked("ids on the host", [&] { return hipEventSynchronize(ev[j]); })) return x;
      }
      const double tr = tracing() ? now_ms() : 0;
      reduce_txs(pool_of(ctx, d), b, t0, t1);
      if (tracing() && now_ms() - tr > 1.0) fprintf(stderr, "[cordahip] reduce of %llu txs %.2f ms\n",
                                                    (unsigned long long)(t1 - t0), now_ms() - tr);
      reduced.push_back({t0, t1});
      return hipSuccess;
    };
    MsgView mv{b->tx.txid, nullptr, tx_of};
    mv.dev = &di;
    // checkSignaturesAreValid -> sig.verify -> Crypto.doVerify: doVerify semantics
    cordahip_sig_batch sb{b->tx_sig_off[b->tx.ntx], b->scheme, b->key, b->key_off, b->sig, b->sig_off, b->tx.txid,
                          nullptr, b->sig_status, nullptr, 0u, b->key_bytes, b->sig_bytes, 0};
    try {
      r = sig_verify_range(ctx, d, S, &sb, mv, s0, s1);
    } catch (const std::bad_alloc&) {
      r = CORDAHIP_ERR_OUT_OF_MEMORY;
    } catch (...) {
      r = CORDAHIP_ERR_HIP;
    }
  }
  const double tr0 = tracing() ? now_ms() : 0;
  // slices no signature asked for; the token goes on (if the pipeline did not hand
  // it on; after an error nothing more is enqueued)
  if (r == CORDAHIP_SUCCESS) {
    if (hand_on() != hipSuccess) r = CORDAHIP_ERR_HIP;
  } else {
    handed_on = true;
    if (gk.owns_lock()) gk.unlock();
    if (tok.owns_lock()) tok.unlock();
  }
  // every slice writes the caller's txid / tx_status: drain before returning,
  // errors included. S.tx_ev follows the last slice (and the encoder's usage
  // report) on the id stream, after every earlier slice; the id copies on
  // s_idcopy precede their slices' kernels. After an error the streams
  // themselves are drained.
  hipError_t e1 = hipSuccess;
  if (r == CORDAHIP_SUCCESS) e1 = hipEventSynchronize(S.tx_ev);
  if (r != CORDAHIP_SUCCESS || e1 != hipSuccess) {
    (void)hipStreamSynchronize(d.s_idcopy ? d.s_idcopy : d.stream);
    (void)hipStreamSynchronize(d.stream);
  }
  const double tr1 = tracing() ? now_ms() : 0;
  if (r == CORDAHIP_SUCCESS && e1 != hipSuccess) r = CORDAHIP_ERR_HIP;
  if (r != CORDAHIP_SUCCESS) return r;
  if (cp) {
    // the encoder's misses in this call (this set's counter, reported after its last
    // slice, drained above): a templates-only call with any is void; a full call
    // without any lets the next call on this device take the templates-only chain
    const uint32_t misses = static_cast<const volatile uint32_t*>(S.kryo_usage)[2 + set_idx];
    if (tracing()) fprintf(stderr, "[cordahip] dev %d set %d component call: %u encoder misses\n", d.id, set_idx, misses);
    std::lock_guard<std::mutex> g(d.kryo_mu);
    if (cp->templates_only && misses) {
      d.kryo_templates_ok = false;
      return kRedoFull;
    }
    if (d.kryo_gen == gen) d.kryo_templates_ok = misses == 0;
  }
  // the transactions no chunk reduced: chunk-edge ones, those without signatures
  std::sort(reduced.begin(), reduced.end());
  uint64_t t = lo;
  for (const auto& rg : reduced) {
    reduce_txs(pool_of(ctx, d), b, t, rg.first);
    t = std::max(t, rg.second);
  }
  reduce_txs(pool_of(ctx, d), b, t, hi);
  if (tracing())
    fprintf(stderr, "[cordahip] dev %d signed tx tail: id streams drained %.2f ms, edge reduce %.2f ms\n", d.id,
            tr1 - tr0, now_ms() - tr1);
  return r;
}

// A component batch runs the encoder's templates-only chain when the device's
// last component batch needed no new template and no direct encoder
// (Device::kryo_templates_ok): per id slice, the shape pass and the leaf hashes
// straight from the templates (kryo_hash: no leaf bytes), without the build /
// size / direct-write kernels whose empty launches sat on each slice's critical
// path. An item that would need them is a miss; the call
// then runs again with the full chain (its results overwrite every output).
// CORDAHIP_KRYO_TEMPLATES_ONLY=0 always runs the full chain.
int signed_tx_device(cordahip_ctx* ctx, Device& d, const cordahip_signed_tx_batch* b, uint64_t* tx_of, uint64_t lo,
                     uint64_t hi, uint64_t slices, const cordahip_txcomp_batch* comps) {
  static const bool spec = [] {
    const char* v = getenv("CORDAHIP_KRYO_TEMPLATES_ONLY");
    return !(v && v[0] == '0');
  }();
  const int r = signed_tx_device_once(ctx, d, b, tx_of, lo, hi, slices, comps, comps && spec);
  if (r == kRedoFull && tracing())
    fprintf(stderr, "[cordahip] dev %d component call: templates-only chain missed, redone with the full encoder\n",
            d.id);
  return r == kRedoFull ? signed_tx_device_once(ctx, d, b, tx_of, lo, hi, slices, comps, false) : r;
}

int signed_tx_impl(cordahip_ctx* ctx, const cordahip_signed_tx_batch* b, const cordahip_txcomp_batch* comps = nullptr) {
  const uint64_t ntx = b->tx.ntx;
  if (ntx == 0) return CORDAHIP_SUCCESS;
  if (!b->tx_sig_off || !b->first_bad_sig || !b->sig_status) return CORDAHIP_ERR_INVALID_ARG;
  if (comps) {  // components instead of leaves (b->tx.tx_leaf_off = comps->tx_item_off)
    if (!comps->tx_item_off || !comps->txid || !comps->tx_status || (comps->tx_item_off[ntx] && !comps->items) ||
        (comps->payload_len && !comps->payload))
      return CORDAHIP_ERR_INVALID_ARG;
  } else if (!b->tx.leaf_off || !b->tx.tx_leaf_off || !b->tx.txid || !b->tx.tx_status || !b->tx.leaf_bytes) {
    return CORDAHIP_ERR_INVALID_ARG;
  }
  // the CSR levels (csr_check.hpp), whole, before any enqueue: the leaves or the
  // items, then the signatures
  const PoolPar par{*ctx->host};
  if (comps ? !check_txcomp_batch(par, comps) : !check_txid_batch(par, &b->tx)) return CORDAHIP_ERR_INVALID_ARG;
  if (!check_sig_level(par, ntx, b->tx_sig_off, b->nsig, b->key_off, b->key_bytes, b->sig_off, b->sig_bytes))
    return CORDAHIP_ERR_INVALID_ARG;
  const uint64_t nsig = b->tx_sig_off[ntx];
  if (nsig && (!b->scheme || !b->key || !b->key_off || !b->sig || !b->sig_off)) return CORDAHIP_ERR_INVALID_ARG;
  const double t0 = tracing() ? now_ms() : 0;
  // signature -> transaction (tx_of), each device filling its shard's part
  // (signed_tx_device); the buffer comes from the context's cache and goes
  // back to it on every exit
  struct TxOf {
    cordahip_ctx* ctx;
    std::unique_ptr<uint64_t[]> p;
    uint64_t cap = 0;
    TxOf(cordahip_ctx* c, uint64_t n) : ctx(c) {
      std::lock_guard<std::mutex> g(ctx->txof_mu);
      auto& f = ctx->txof_free;
      for (size_t i = 0; i < f.size(); i++)
        if (f[i].second >= n) {
          p = std::move(f[i].first);
          cap = f[i].second;
          f.erase(f.begin() + (long)i);
          return;
        }
    }
    ~TxOf() {
      if (!p) return;
      std::lock_guard<std::mutex> g(ctx->txof_mu);
      auto& f = ctx->txof_free;
      if (f.size() < cordahip_ctx::kTxOfCache) f.emplace_back(std::move(p), cap);
    }
  } buf(ctx, nsig);
  if (!buf.p && nsig) {
    buf.p.reset(new uint64_t[nsig]);
    buf.cap = nsig;
  }
  uint64_t* tx_of = buf.p.get();
  const double t_of = tracing() ? now_ms() : 0;
  // per device: its contiguous tx shard in slices (CORDAHIP_TX_SLICES; default:
  // one slice per signature chunk) and, chunk by
  // chunk and after the drain, the per-transaction reduce (reduce_txs)
  uint64_t slices = 0;
  if (const char* v = getenv("CORDAHIP_TX_SLICES")) slices = std::max<uint64_t>(1, strtoull(v, nullptr, 10));
  const int rc = for_shards(ctx->devs, ntx, 1, [&](Device& d, uint64_t lo, uint64_t hi) {
    return signed_tx_device(ctx, d, b, tx_of, lo, hi, slices, comps);
  });
  const double t_ids = tracing() ? now_ms() : 0;
  if (rc != CORDAHIP_SUCCESS) return rc;
  if (tracing())
    fprintf(stderr, "[cordahip] signed tx batch: %llu txs, %llu sigs, %llu id slices per device: tx_of %.2f ms, "
            "ids, signatures and reduce done at %.2f ms\n", (unsigned long long)ntx, (unsigned long long)nsig,
            (unsigned long long)slices, t_of - t0, t_ids - t0);  // slices 0: the per-device default
  return CORDAHIP_SUCCESS;
}

// cordahip_signed_txcomp_batch as the leaf-batch descriptor the pipeline reads
// (no leaf bytes: the slices encode them on the device), plus the components
int signed_txcomp_impl(cordahip_ctx* ctx, const cordahip_signed_txcomp_batch* cb) {
  cordahip_signed_tx_batch b{};
  b.tx.ntx = cb->tx.ntx;
  b.tx.tx_leaf_off = cb->tx.tx_item_off;  // one leaf per component
  b.tx.txid = cb->tx.txid;
  b.tx.tx_status = cb->tx.tx_status;
  b.tx_sig_off = cb->tx_sig_off;
  b.scheme = cb->scheme;
  b.key = cb->key;
  b.key_off = cb->key_off;
  b.sig = cb->sig;
  b.sig_off = cb->sig_off;
  b.sig_status = cb->sig_status;
  b.first_bad_sig = cb->first_bad_sig;
  b.nsig = cb->nsig;
  b.key_bytes = cb->key_bytes;
  b.sig_bytes = cb->sig_bytes;
  return signed_tx_impl(ctx, &b, &cb->tx);
}

// C5: one device's contiguous shard of both sections, [e0, e1) Ed25519 and
// [c0, c1) ECDSA lanes, streamed in chunks through kStreamStages buffer sets.
// The host enqueues every chunk at once; events do the ordering: a chunk's H2D
// (on s_copy, so PCIe serves the chunks in order and the first one arrives at
// full rate) waits until its stage's previous chunk has finished with the
// buffers; each section's kernels wait for that section's copies. While one
// chunk computes, the next chunks' inputs and the previous chunk's statuses
// cross PCIe, and a chunk's ECDSA kernels (small, the batch inversion
// latency-bound) run beside its Ed25519 ladder on their own stream.
int stream_shard(Device& d, const cordahip_stream_batch* b, uint64_t e0, uint64_t e1, uint64_t c0, uint64_t c1) {
  std::lock_guard<std::mutex> g(d.stream_mu);
  const NodeBind nb(d);
  const Activity act(d);
  if (hipSetDevice(d.id) != hipSuccess) return CORDAHIP_ERR_HIP;
  const uint64_t ne = e1 - e0, nc = c1 - c0;
  uint64_t chunk = kStreamChunk;  // CORDAHIP_STREAM_CHUNK: smaller chunks for tests of the pipeline itself
  if (const char* v = getenv("CORDAHIP_STREAM_CHUNK")) chunk = std::max<uint64_t>(64, strtoull(v, nullptr, 10));
  // Chunk boundaries over the combined lane count T = ne + nc, each section cut
  // at the same fraction of its length (64-aligned). The first chunks ramp up
  // (chunk/16, chunk/4, then chunk): the GPU starts after a short first copy
  // instead of a full chunk's H2D (~1.2 GB for C5), and PCIe (~4x faster than
  // the kernels per lane) stays ahead while the sizes grow.
  const uint64_t T = ne + nc;
  std::vector<uint64_t> bound(1, 0);  // cumulative combined lanes at chunk ends
  for (int k = 0; bound.back() < T; k++) {
    const uint64_t sz = std::max<uint64_t>(64, k == 0 ? chunk / 16 : k == 1 ? chunk / 4 : chunk);
    bound.push_back(std::min(T, bound.back() + sz));
  }
  const uint64_t nchunks = std::max<size_t>(1, bound.size() - 1);
  auto cut = [&](uint64_t n, uint64_t k) -> uint64_t {  // section offset at the end of chunk k-1
    if (k >= nchunks) return n;
    const uint64_t v = (uint64_t)((__uint128_t)n * bound[k] / (T ? T : 1));
    return std::min(n, v / 64 * 64);
  };
  uint64_t ce = 0, cc = 0;  // largest per-chunk section sizes: the stage buffers
  for (uint64_t k = 0; k < nchunks; k++) {
    ce = std::max(ce, cut(ne, k + 1) - cut(ne, k));
    cc = std::max(cc, cut(nc, k + 1) - cut(nc, k));
  }
  const uint64_t eml = b->ed_msg_len, cml = b->ec_msg_len;
  if (ensure_streams(d) != hipSuccess) return CORDAHIP_ERR_HIP;
  for (StreamStage& st : d.sstage) {
    for (hipEvent_t* pe : {&st.ed_copied, &st.ec_copied, &st.ed_done, &st.ec_done})
      if (!*pe && hipEventCreateWithFlags(pe, hipEventDisableTiming) != hipSuccess) return CORDAHIP_ERR_HIP;
    // a grow replaces buffers: the previous call's work on them is finished
    // (every call synchronises its streams before returning)
    if ((ce && (st.ed_keys.ensure(ce * 32) || st.ed_sigs.ensure(ce * 64) ||
                st.ed_msgs.ensure(std::max<uint64_t>(ce * eml, 16)) || st.ed_status.ensure(ce))) ||
        (cc && (st.ec_scheme.ensure(cc) || st.ec_keys.ensure(cc * 65) || st.ec_key_len.ensure(cc) ||
                st.ec_sigs.ensure(cc * 72) || st.ec_sig_len.ensure(cc) ||
                st.ec_msgs.ensure(std::max<uint64_t>(cc * cml, 16)) || st.ec_status.ensure(cc))))
      return CORDAHIP_ERR_OUT_OF_MEMORY;
  }
  const hipMemcpyKind h2d = hipMemcpyHostToDevice, d2h = hipMemcpyDeviceToHost;
  hipStream_t cs = d.s_copy, xs = d.s_ec;
  // statuses reach pinned caller arrays by kernel stores (a D2H copy queued
  // behind busy compute streams can hold the enqueuing thread for milliseconds,
  // delaying the next chunks' H2D: profiles/r04_q); pageable ones by copies
  uint8_t* map_ed = static_cast<uint8_t*>(host_mapped(b->ed_status));
  uint8_t* map_ec = static_cast<uint8_t*>(host_mapped(b->ec_status));
  hipError_t e = hipSuccess;
  for (uint64_t k = 0; k < nchunks && e == hipSuccess; k++) {
    StreamStage& st = d.sstage[k % kStreamStages];
    // consecutive chunks alternate between s_ed / s_ed2 and the two Ed25519
    // workspace slots: chunk k + 1's prep fills the CUs chunk k's ladder tail
    // leaves idle
    const int slot = (int)(k & 1);
    hipStream_t es = slot ? d.s_ed2 : d.s_ed;
    const uint64_t a = e0 + cut(ne, k), ma = cut(ne, k + 1) - cut(ne, k);
    const uint64_t c = c0 + cut(nc, k), mc = cut(nc, k + 1) - cut(nc, k);
    if (k >= (uint64_t)kStreamStages) {  // the stage's buffers: chunk k-3 must be done with them
      e = hipStreamWaitEvent(cs, st.ed_done, 0);
      e = e ? e : hipStreamWaitEvent(cs, st.ec_done, 0);
    }
    if (ma) {
      e = e ? e : hipMemcpyAsync(st.ed_keys.p, b->ed_keys + a * 32, ma * 32, h2d, cs);
      e = e ? e : hipMemcpyAsync(st.ed_sigs.p, b->ed_sigs + a * 64, ma * 64, h2d, cs);
      if (eml) e = e ? e : hipMemcpyAsync(st.ed_msgs.p, b->ed_msgs + a * eml, ma * eml, h2d, cs);
    }
    e = e ? e : hipEventRecord(st.ed_copied, cs);
    if (mc) {
      e = e ? e : hipMemcpyAsync(st.ec_scheme.p, b->ec_scheme + c, mc, h2d, cs);
      e = e ? e : hipMemcpyAsync(st.ec_keys.p, b->ec_keys + c * 65, mc * 65, h2d, cs);
      e = e ? e : hipMemcpyAsync(st.ec_key_len.p, b->ec_key_len + c, mc, h2d, cs);
      e = e ? e : hipMemcpyAsync(st.ec_sigs.p, b->ec_sigs + c * 72, mc * 72, h2d, cs);
      e = e ? e : hipMemcpyAsync(st.ec_sig_len.p, b->ec_sig_len + c, mc, h2d, cs);
      if (cml) e = e ? e : hipMemcpyAsync(st.ec_msgs.p, b->ec_msgs + c * cml, mc * cml, h2d, cs);
    }
    e = e ? e : hipEventRecord(st.ec_copied, cs);
    e = e ? e : hipStreamWaitEvent(es, st.ed_copied, 0);
    if (ma)
      e = e ? e
            : ed_verify_enqueue(d, st.ed_keys.as<uint8_t>(), st.ed_sigs.as<uint8_t>(), st.ed_msgs.as<uint8_t>(),
                                (uint32_t)eml, ma, nullptr, st.ed_status.as<uint8_t>(), nullptr, 0u, es, slot);
    if (ma && map_ed) e = e ? e : launch_store_to_host(st.ed_status.p, map_ed + a, ma, es);
    else if (ma) e = e ? e : hipMemcpyAsync(b->ed_status + a, st.ed_status.p, ma, d2h, es);
    e = e ? e : hipEventRecord(st.ed_done, es);
    e = e ? e : hipStreamWaitEvent(xs, st.ec_copied, 0);
    if (mc && e == hipSuccess) {
      std::lock_guard<std::mutex> ge(d.ec_mu[0]);
      e = ec_verify_enqueue(d, st.ec_scheme.as<uint8_t>(), st.ec_keys.as<uint8_t>(), st.ec_key_len.as<uint8_t>(),
                            st.ec_sigs.as<uint8_t>(), st.ec_sig_len.as<uint8_t>(), st.ec_msgs.as<uint8_t>(), nullptr,
                            (uint32_t)cml, mc, nullptr, st.ec_status.as<uint8_t>(), nullptr, 0u, xs);
    }
    if (mc && map_ec) e = e ? e : launch_store_to_host(st.ec_status.p, map_ec + c, mc, xs);
    else if (mc) e = e ? e : hipMemcpyAsync(b->ec_status + c, st.ec_status.p, mc, d2h, xs);
    e = e ? e : hipEventRecord(st.ec_done, xs);
  }
  // drain all four streams even after an error, so no queued work outlives the call
  const hipError_t e1s = hipStreamSynchronize(cs), e2s = hipStreamSynchronize(d.s_ed),
                   e2b = hipStreamSynchronize(d.s_ed2), e3s = hipStreamSynchronize(xs);
  if (e != hipSuccess || e1s != hipSuccess || e2s != hipSuccess || e2b != hipSuccess || e3s != hipSuccess)
    return CORDAHIP_ERR_HIP;
  return CORDAHIP_SUCCESS;
}

int stream_verify_impl(cordahip_ctx* ctx, const cordahip_stream_batch* b) {
  if ((b->n_ed && (!b->ed_keys || !b->ed_sigs || !b->ed_status || (b->ed_msg_len && !b->ed_msgs))) ||
      (b->n_ec && (!b->ec_scheme || !b->ec_keys || !b->ec_key_len || !b->ec_sigs || !b->ec_sig_len ||
                   !b->ec_status || (b->ec_msg_len && !b->ec_msgs))))
    return CORDAHIP_ERR_INVALID_ARG;
  const uint64_t nd = ctx->devs.size();
  std::vector<std::future<int>> fs;
  for (uint64_t i = 0; i < nd; i++) {
    uint64_t e0, e1, c0, c1;
    shard_range(b->n_ed, nd, i, 64, e0, e1);
    shard_range(b->n_ec, nd, i, 64, c0, c1);
    if (e0 >= e1 && c0 >= c1) continue;
    Device* d = ctx->devs[i].get();
    fs.push_back(std::async(std::launch::async, [=] { return stream_shard(*d, b, e0, e1, c0, c1); }));
  }
  int rc = CORDAHIP_SUCCESS;
  for (auto& f : fs) {
    const int r = f.get();
    if (r != CORDAHIP_SUCCESS && rc == CORDAHIP_SUCCESS) rc = r;
  }
  return rc;
}

// FilteredTransaction.verify for txs [t0, t1) on one device: K3 hashes the
// filtered leaves, K6 evaluates each partial tree and compares.
int filtered_tx_shard(Device& d, const cordahip_filtered_tx_batch* b, uint64_t t0, uint64_t t1) {
  SetLease lease(d);
  TxSet& S = lease.get();
  const NodeBind nb(d);
  const Activity act(d);
  if (int rc = tx_acquire_host(d, S)) return rc;
  const uint64_t ntx = t1 - t0;
  const uint64_t l0 = b->tx_leaf_off[t0], l1 = b->tx_leaf_off[t1], nleaves = l1 - l0;
  const uint64_t b0 = nleaves ? b->leaf_off[l0] : 0, b1 = nleaves ? b->leaf_off[l1] : 0;
  const uint64_t k0 = b->tx_tok_off[t0], k1 = b->tx_tok_off[t1], ntok = k1 - k0;
  std::vector<uint64_t> loff(nleaves + 1), toff(ntx + 1), koff(ntx + 1);
  for (uint64_t i = 0; i <= nleaves; i++) loff[i] = nleaves ? b->leaf_off[l0 + i] - b0 : 0;
  for (uint64_t i = 0; i <= ntx; i++) {
    toff[i] = b->tx_leaf_off[t0 + i] - l0;
    koff[i] = b->tx_tok_off[t0 + i] - k0;
  }
  TxWork& w = S.tx;
  if (w.leaf_bytes.ensure(std::max<uint64_t>(b1 - b0, 16)) || w.leaf_off.ensure((nleaves + 1) * 8) ||
      w.tx_leaf_off.ensure((ntx + 1) * 8) || w.hashes.ensure(std::max<uint64_t>(nleaves, 1) * 32) ||
      w.tok.ensure(std::max<uint64_t>(ntok, 1)) || w.tok_hash.ensure(std::max<uint64_t>(ntok, 1) * 32) ||
      w.tx_tok_off.ensure((ntx + 1) * 8) || w.root.ensure(ntx * 32) ||
      w.stack.ensure(std::max<uint64_t>(ntok, 1) * 32) || w.tx_status.ensure(ntx))
    return CORDAHIP_ERR_OUT_OF_MEMORY;
  hipStream_t s = d.stream;
  const hipMemcpyKind h2d = hipMemcpyHostToDevice;
  hipError_t e = hipSuccess;
  if (b1 > b0) e = hipMemcpyAsync(w.leaf_bytes.p, b->leaf_bytes + b0, b1 - b0, h2d, s);
  e = e ? e : hipMemcpyAsync(w.leaf_off.p, loff.data(), (nleaves + 1) * 8, h2d, s);
  e = e ? e : hipMemcpyAsync(w.tx_leaf_off.p, toff.data(), (ntx + 1) * 8, h2d, s);
  if (ntok) {
    e = e ? e : hipMemcpyAsync(w.tok.p, b->tok + k0, ntok, h2d, s);
    e = e ? e : hipMemcpyAsync(w.tok_hash.p, b->tok_hash + k0 * 32, ntok * 32, h2d, s);
  }
  e = e ? e : hipMemcpyAsync(w.tx_tok_off.p, koff.data(), (ntx + 1) * 8, h2d, s);
  e = e ? e : hipMemcpyAsync(w.root.p, b->root + t0 * 32, ntx * 32, h2d, s);
  e = e ? e : launch_sha256_leaves(w.leaf_bytes.as<uint8_t>(), w.leaf_off.as<uint64_t>(), nleaves,
                                   w.hashes.as<uint32_t>(), s);
  e = e ? e : launch_pmt_verify(w.hashes.as<uint32_t>(), w.tx_leaf_off.as<uint64_t>(), w.tok.as<uint8_t>(),
                                w.tok_hash.as<uint8_t>(), w.tx_tok_off.as<uint64_t>(), w.root.as<uint8_t>(), ntx,
                                w.stack.as<uint32_t>(), w.tx_status.as<uint8_t>(), s);
  e = e ? e : hipMemcpyAsync(b->tx_status + t0, w.tx_status.p, ntx, hipMemcpyDeviceToHost, s);
  e = e ? e : hipEventRecord(S.tx_ev, s);
  e = e ? e : hipEventSynchronize(S.tx_ev);
  if (e != hipSuccess) (void)hipStreamSynchronize(s);
  return hip_err(e);
}

int filtered_tx_impl(cordahip_ctx* ctx, const cordahip_filtered_tx_batch* b) {
  const uint64_t n = b->ntx;
  if (n == 0) return CORDAHIP_SUCCESS;
  if (!b->leaf_off || !b->tx_leaf_off || !b->tx_tok_off || !b->root || !b->tx_status ||
      (!b->tok && b->tx_tok_off[n]) || (!b->tok_hash && b->tx_tok_off[n]))
    return CORDAHIP_ERR_INVALID_ARG;
  if (!check_filtered_batch(PoolPar{*ctx->host}, b)) return CORDAHIP_ERR_INVALID_ARG;  // before any enqueue
  return for_shards(ctx->devs, n, 1, [&](Device& d, uint64_t t0, uint64_t t1) { return filtered_tx_shard(d, b, t0, t1); });
}

Device* dev_at(cordahip_ctx* ctx, int device) {
  if (!ctx || device < 0 || device >= (int)ctx->devs.size()) return nullptr;
  return ctx->devs[device].get();
}

void free_device(Device& d) {
  (void)hipSetDevice(d.id);
  for (PackStage& st : d.ped) {
    for (auto& b : st.h) b.release();
    for (auto& b : st.d) b.release();
    for (hipEvent_t ev : {st.copied, st.done})
      if (ev) (void)hipEventDestroy(ev);
  }
  for (TxSet& S : d.set) {
    for (BatchStage& st : S.pb) {
      for (auto& b : st.h) b.release();
      for (auto& b : st.d) b.release();
      for (auto& b : st.hidx) b.release();
      for (auto& b : st.didx) b.release();
      st.dverdict.release();
      for (hipEvent_t ev : {st.copied, st.ed_done, st.ec_done})
        if (ev) (void)hipEventDestroy(ev);
    }
    TxWork& w = S.tx;
    for (DevBuf* b : {&w.leaf_bytes, &w.leaf_off, &w.tx_leaf_off, &w.hashes, &w.txid, &w.tx_status, &w.tx_sig_off,
                      &w.msgs, &w.comp_items, &w.payload, &w.comp_status, &w.tok, &w.tok_hash, &w.tx_tok_off, &w.root,
                      &w.stack})
      b->release();
    if (S.kryo_usage) (void)hipHostFree(S.kryo_usage);
    S.kryo_usage = S.kryo_usage_dev = nullptr;
    for (hipEvent_t* pe : {&S.tx_ev, &S.fork, &S.ids, &S.ed_fork, &S.ed_join}) {
      if (*pe) (void)hipEventDestroy(*pe);
      *pe = nullptr;
    }
  }
  for (auto& st : d.sstage) {
    for (DevBuf* b : {&st.ed_keys, &st.ed_sigs, &st.ed_msgs, &st.ed_status, &st.ec_scheme, &st.ec_keys,
                      &st.ec_key_len, &st.ec_sigs, &st.ec_sig_len, &st.ec_msgs, &st.ec_status})
      b->release();
    for (hipEvent_t ev : {st.ed_copied, st.ec_copied, st.ed_done, st.ec_done})
      if (ev) (void)hipEventDestroy(ev);
  }
  for (hipStream_t ss : {d.s_copy, d.s_ed, d.s_ec, d.s_idcopy, d.s_ed2})  // s_ec2 is s_idcopy
    if (ss) (void)hipStreamDestroy(ss);
  for (DevBuf* b : {&d.ec[0].counters, &d.ec[0].perm, &d.ec[0].ws, &d.ec[1].counters, &d.ec[1].perm, &d.ec[1].ws,
                    &d.kryo_sizes, &d.kryo_temp, &d.kryo_ws, &d.kryo_fixed, &d.kryo_items})
    b->release();
  for (auto& w : d.ed_ws) w.release();
  if (d.kryo_usage) (void)hipHostFree(d.kryo_usage);
  d.kryo_usage = d.kryo_usage_dev = nullptr;
  for (hipEvent_t ev : {d.ec[0].ev, d.ec[1].ev, d.ed_ev[0], d.ed_ev[1], d.kryo_ev})
    if (ev) (void)hipEventDestroy(ev);
  for (auto& tc : d.ring)
    for (hipEvent_t ev : {tc.a, tc.b})
      if (ev) (void)hipEventDestroy(ev);
  if (d.btab && d.gtab_k1 && d.gtab_r1) mem_acct(d.id).sub(ed25519_btable_bytes() + 2 * ecdsa_gtable_bytes());
  if (d.gtab_k1) (void)hipFree(d.gtab_k1);
  if (d.gtab_r1) (void)hipFree(d.gtab_r1);
  if (d.btab) (void)hipFree(d.btab);
  if (d.stream) (void)hipStreamDestroy(d.stream);
}

}  // namespace

// Synchronous entry points run host code that allocates (staging vectors,
// worker threads): no C++ exception may cross the C ABI into the JVM.
template <class F>
int guarded(F&& f) noexcept {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return CORDAHIP_ERR_OUT_OF_MEMORY;
  } catch (...) {
    return CORDAHIP_ERR_HIP;
  }
}

extern "C" {

uint32_t cordahip_abi_version(void) { return CORDAHIP_ABI_VERSION; }

const char* cordahip_strerror(int code) {
  switch (code) {
    case CORDAHIP_SUCCESS: return "success";
    case CORDAHIP_ERR_INVALID_ARG: return "invalid argument";
    case CORDAHIP_ERR_HIP: return "HIP runtime error";
    case CORDAHIP_ERR_NO_DEVICE: return "no usable HIP device";
    case CORDAHIP_ERR_OUT_OF_MEMORY: return "out of device memory";
    case CORDAHIP_ERR_TIMEOUT: return "timed out";
    case CORDAHIP_ERR_UNKNOWN_TICKET: return "unknown ticket";
    case CORDAHIP_ERR_NOT_IMPLEMENTED: return "not implemented on the GPU path";
    default: return "unknown error";
  }
}

void cordahip_shard_range(uint64_t n, uint32_t nshards, uint32_t shard, uint64_t align, uint64_t* lo, uint64_t* hi) {
  uint64_t a, b;
  shard_range(n, nshards, shard, align, a, b);
  if (lo) *lo = a;
  if (hi) *hi = b;
}

static int init_impl(uint32_t device_mask, cordahip_ctx** out);

int cordahip_init(uint32_t device_mask, cordahip_ctx** out) {
  if (!out) return CORDAHIP_ERR_INVALID_ARG;
  *out = nullptr;
  return guarded([&] { return init_impl(device_mask, out); });
}

static int init_impl(uint32_t device_mask, cordahip_ctx** out) {
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return CORDAHIP_ERR_NO_DEVICE;
  auto ctx = std::make_unique<cordahip_ctx>();
  int rc = CORDAHIP_SUCCESS;
  // Test-only: CORDAHIP_TEST_DEVICE_REPLICAS=k gives the context k Device
  // objects per selected HIP device (each with its own streams, buffers and
  // tables), so the N-device code -- shard split, per-device workers, tails,
  // verdict reassembly -- runs on a one-GPU box. Unset in production.
  int replicas = 1;
  if (const char* v = getenv("CORDAHIP_TEST_DEVICE_REPLICAS")) replicas = std::max(1, std::min(8, atoi(v)));
  std::vector<int> ids;
  for (int d = 0; d < count && d < 32; d++)
    if (!device_mask || ((device_mask >> d) & 1u))
      for (int r = 0; r < replicas; r++) ids.push_back(d);
  for (int d : ids) {
    if (rc != CORDAHIP_SUCCESS) break;
    ctx->devs.push_back(std::make_unique<Device>());
    Device& dev = *ctx->devs.back();
    dev.id = d;
    dev.uid = g_device_uid.fetch_add(1);
    if (hipSetDevice(d) != hipSuccess || hipStreamCreateWithFlags(&dev.stream, hipStreamNonBlocking) != hipSuccess) {
      rc = CORDAHIP_ERR_HIP;
      break;
    }
    for (TxSet& S : dev.set)
      for (hipEvent_t* pe : {&S.tx_ev, &S.fork, &S.ids, &S.ed_fork, &S.ed_join})
        if (hipEventCreateWithFlags(pe, hipEventDisableTiming) != hipSuccess) rc = CORDAHIP_ERR_HIP;
    if (rc != CORDAHIP_SUCCESS) break;
    for (auto& tc : dev.ring)
      if (hipEventCreate(&tc.a) != hipSuccess || hipEventCreate(&tc.b) != hipSuccess) rc = CORDAHIP_ERR_HIP;
    if (rc != CORDAHIP_SUCCESS) break;
    if (hipMalloc(reinterpret_cast<void**>(&dev.btab), ed25519_btable_bytes()) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&dev.gtab_k1), ecdsa_gtable_bytes()) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&dev.gtab_r1), ecdsa_gtable_bytes()) != hipSuccess) {
      rc = CORDAHIP_ERR_OUT_OF_MEMORY;
      break;
    }
    mem_acct(d).add(ed25519_btable_bytes() + 2 * ecdsa_gtable_bytes());
    device_budget(dev);
    static const bool id_prio = !(getenv("CORDAHIP_ID_PRIO") && getenv("CORDAHIP_ID_PRIO")[0] == '0');
    if (!id_prio && (tx_set_id_priority(0) != hipSuccess || kryo_set_priority(0) != hipSuccess)) {
      rc = CORDAHIP_ERR_HIP;
      break;
    }
    if (launch_ed25519_btable(dev.btab, dev.stream) != hipSuccess ||
        launch_ecdsa_gtables(dev.gtab_k1, dev.gtab_r1, dev.stream) != hipSuccess ||
        hipStreamSynchronize(dev.stream) != hipSuccess)
      rc = CORDAHIP_ERR_HIP;
  }
  if (rc == CORDAHIP_SUCCESS && ctx->devs.empty()) rc = CORDAHIP_ERR_NO_DEVICE;
  if (rc != CORDAHIP_SUCCESS) {
    for (auto& d : ctx->devs) free_device(*d);
    return rc;
  }
  ctx->pool = std::make_unique<WorkerPool>((int)std::max<size_t>(2, 2 * ctx->devs.size()));
  // host threads. Per device (numa_place.hpp): a pool bound to CPUs of the GPU's
  // NUMA node -- the devices of one node split its CPUs -- of CORDAHIP_HOST_THREADS
  // threads at most (default 16: the pipelines are PCIe / kernel bound beyond that,
  // tools/pack_bench.cpp); CORDAHIP_NUMA=0 leaves them unbound. Context-wide: a
  // pool for the batch-level passes (CSR checks, verdict words) of at most 16.
  int cap = 16;
  if (const char* v = getenv("CORDAHIP_HOST_THREADS")) cap = std::max(1, std::min(256, atoi(v)));
  std::vector<int> allowed;
  {
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0)
      for (int c = 0; c < CPU_SETSIZE; c++)
        if (CPU_ISSET(c, &cs)) allowed.push_back(c);
  }
  if (allowed.empty())
    for (int c = 0; c < (int)std::max(1u, std::thread::hardware_concurrency()); c++) allowed.push_back(c);
  std::vector<std::string> pci(ctx->devs.size());
  const bool numa = !(getenv("CORDAHIP_NUMA") && getenv("CORDAHIP_NUMA")[0] == '0');
  for (size_t i = 0; i < ctx->devs.size() && numa; i++) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, ctx->devs[i]->id) == hipSuccess) {
      pci[i] = bus;
      for (char& ch : pci[i]) ch = (char)tolower((unsigned char)ch);
    }
  }
  const char* root = getenv("CORDAHIP_SYSFS_ROOT");  // tests: a fake tree
  const std::vector<NumaPlace> plan = numa_plan(root ? root : "/sys", pci, allowed, cap);
  for (size_t i = 0; i < ctx->devs.size(); i++) {
    Device& d = *ctx->devs[i];
    d.place = plan[i];
    if (!numa) d.place.cpus.clear();
    d.pool = std::make_unique<HostPool>(d.place.threads, d.place.cpus);
    if (tracing())
      fprintf(stderr, "[cordahip] dev %d (%s): NUMA node %d, %zu CPUs, %d host threads%s%s\n", d.id, pci[i].c_str(),
              d.place.node, d.place.cpus.size(), d.place.threads, d.place.why.empty() ? "" : ": ",
              d.place.why.c_str());
  }
  ctx->host = std::make_unique<HostPool>(std::max(1, std::min<int>((int)allowed.size(), 16)));
  // the idle release: a device with no call for CORDAHIP_IDLE_RELEASE_MS (default 30 s;
  // 0: never) gives its grow-only buffers back (trim_device)
  const char* iv = getenv("CORDAHIP_IDLE_RELEASE_MS");
  const int64_t idle_ms = iv ? strtoll(iv, nullptr, 10) : 30000;
  if (idle_ms > 0) {
    cordahip_ctx* c = ctx.get();
    c->reaper = std::thread([c, idle_ms] {
      std::vector<int64_t> trimmed_at(c->devs.size(), 0);  // the last call's end when last trimmed
      std::unique_lock<std::mutex> g(c->reaper_mu);
      while (!c->reaper_stop) {
        c->reaper_cv.wait_for(g, std::chrono::milliseconds(std::min<int64_t>(250, idle_ms)));
        if (c->reaper_stop) break;
        for (size_t i = 0; i < c->devs.size(); i++) {
          Device& d = *c->devs[i];
          const int64_t last = d.last_use_ms.load();
          if (d.active.load() > 0 || last == 0 || last == trimmed_at[i] || (int64_t)now_ms() - last < idle_ms)
            continue;
          g.unlock();
          trim_device(d);
          g.lock();
          trimmed_at[i] = last;
        }
      }
    });
  }
  *out = ctx.release();
  return CORDAHIP_SUCCESS;
}

void cordahip_shutdown(cordahip_ctx* ctx) {
  if (!ctx) return;
  if (ctx->reaper.joinable()) {
    {
      std::lock_guard<std::mutex> g(ctx->reaper_mu);
      ctx->reaper_stop = true;
    }
    ctx->reaper_cv.notify_all();
    ctx->reaper.join();
  }
  ctx->pool.reset();  // runs every queued job to completion, joins the workers
  ctx->host.reset();
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    ctx->jobs.clear();
  }
  for (auto& d : ctx->devs) free_device(*d);
  delete ctx;
}

int cordahip_device_count(const cordahip_ctx* ctx) { return ctx ? (int)ctx->devs.size() : 0; }

int cordahip_device_mem(cordahip_ctx* ctx, int device, uint64_t* in_use, uint64_t* peak, uint64_t* budget) {
  Device* d = dev_at(ctx, device);
  if (!d) return CORDAHIP_ERR_INVALID_ARG;
  const MemAcct& m = mem_acct(d->id);
  if (in_use) *in_use = m.in_use.load();
  if (peak) *peak = m.peak.load();
  if (budget) *budget = d->mem_budget;
  return CORDAHIP_SUCCESS;
}

int cordahip_trim(cordahip_ctx* ctx) {
  if (!ctx) return CORDAHIP_ERR_INVALID_ARG;
  return guarded([&] {
    for (auto& d : ctx->devs) trim_device(*d);
    return (int)CORDAHIP_SUCCESS;
  });
}

int cordahip_alloc_pinned(cordahip_ctx* ctx, size_t bytes, void** host) {
  if (!ctx || !host) return CORDAHIP_ERR_INVALID_ARG;
  return hipHostMalloc(host, bytes, hipHostMallocPortable) == hipSuccess ? CORDAHIP_SUCCESS
                                                                          : CORDAHIP_ERR_OUT_OF_MEMORY;
}

int cordahip_free_pinned(cordahip_ctx* ctx, void* host) {
  if (!ctx) return CORDAHIP_ERR_INVALID_ARG;
  return hip_err(hipHostFree(host));
}

int cordahip_sig_verify(cordahip_ctx* ctx, const cordahip_sig_batch* batch) {
  if (!ctx || !batch) return CORDAHIP_ERR_INVALID_ARG;
  return guarded([&] { return sig_verify_impl(ctx, batch); });
}

int cordahip_sig_submit(cordahip_ctx* ctx, const cordahip_sig_batch* batch, uint64_t* ticket) {
  if (!ctx || !batch || !ticket) return CORDAHIP_ERR_INVALID_ARG;
  const cordahip_sig_batch copy = *batch;  // descriptor by value; buffers stay caller-owned
  return guarded([&] {
    *ticket = submit_job(ctx, [ctx, copy] { return sig_verify_impl(ctx, &copy); });
    return CORDAHIP_SUCCESS;
  });
}

int cordahip_tx_submit(cordahip_ctx* ctx, const cordahip_signed_tx_batch* batch, uint64_t* ticket) {
  if (!ctx || !batch || !ticket) return CORDAHIP_ERR_INVALID_ARG;
  const cordahip_signed_tx_batch copy = *batch;
  return guarded([&] {
    *ticket = submit_job(ctx, [ctx, copy] { return signed_tx_impl(ctx, &copy); });
    return CORDAHIP_SUCCESS;
  });
}

int cordahip_txcomp_submit(cordahip_ctx* ctx, const cordahip_signed_txcomp_batch* batch, uint64_t* ticket) {
  if (!ctx || !batch || !ticket) return CORDAHIP_ERR_INVALID_ARG;
  const cordahip_signed_txcomp_batch copy = *batch;
  return guarded([&] {
    *ticket = submit_job(ctx, [ctx, copy] { return signed_txcomp_impl(ctx, &copy); });
    return CORDAHIP_SUCCESS;
  });
}

int cordahip_signed_txcomp_verify(cordahip_ctx* ctx, const cordahip_signed_txcomp_batch* batch) {
  if (!ctx || !batch) return CORDAHIP_ERR_INVALID_ARG;
  return guarded([&] { return signed_txcomp_impl(ctx, batch); });
}

int cordahip_txid_submit(cordahip_ctx* ctx, const cordahip_txid_batch* batch, uint64_t* ticket) {
  if (!ctx || !batch || !ticket) return CORDAHIP_ERR_INVALID_ARG;
  const cordahip_txid_batch copy = *batch;
  return guarded([&] {
    *ticket = submit_job(ctx, [ctx, copy] { return tx_ids_impl(ctx, &copy); });
    return CORDAHIP_SUCCESS;
  });
}

int cordahip_filtered_tx_submit(cordahip_ctx* ctx, const cordahip_filtered_tx_batch* batch, uint64_t* ticket) {
  if (!ctx || !batch || !ticket) return CORDAHIP_ERR_INVALID_ARG;
  const cordahip_filtered_tx_batch copy = *batch;
  return guarded([&] {
    *ticket = submit_job(ctx, [ctx, copy] { return filtered_tx_impl(ctx, &copy); });
    return CORDAHIP_SUCCESS;
  });
}

int cordahip_wait(cordahip_ctx* ctx, uint64_t ticket, int64_t timeout_ns) {
  if (!ctx) return CORDAHIP_ERR_INVALID_ARG;
  std::shared_ptr<JobState> st;
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    auto it = ctx->jobs.find(ticket);
    if (it == ctx->jobs.end()) return CORDAHIP_ERR_UNKNOWN_TICKET;
    st = it->second;
  }
  int rc;
  {
    std::unique_lock<std::mutex> g(st->m);
    if (timeout_ns < 0) st->cv.wait(g, [&] { return st->done; });
    else if (!st->cv.wait_for(g, std::chrono::nanoseconds(timeout_ns), [&] { return st->done; }))
      return CORDAHIP_ERR_TIMEOUT;
    rc = st->rc;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  ctx->jobs.erase(ticket);  // released: the ticket is single-use
  return rc;
}

int cordahip_poll(cordahip_ctx* ctx, uint64_t ticket) {
  if (!ctx) return CORDAHIP_ERR_INVALID_ARG;
  std::shared_ptr<JobState> st;
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    auto it = ctx->jobs.find(ticket);
    if (it == ctx->jobs.end()) return CORDAHIP_ERR_UNKNOWN_TICKET;
    st = it->second;
  }
  std::lock_guard<std::mutex> g(st->m);
  return st->done ? 1 : 0;
}

int cordahip_ed25519_verify_device(cordahip_ctx* ctx, int device, const void* d_keys, const void* d_sigs,
                                   const void* d_msgs, uint32_t msg_len, uint64_t n, void* d_status,
                                   void* d_verdict, void* hip_stream) {
  Device* d = dev_at(ctx, device);
  if (!d || (!d_keys && n) || (!d_sigs && n) || (!d_status && n)) return CORDAHIP_ERR_INVALID_ARG;
  if ((reinterpret_cast<uintptr_t>(d_keys) | reinterpret_cast<uintptr_t>(d_sigs)) & 15)
    return CORDAHIP_ERR_INVALID_ARG;
  if (msg_len == 32 && (reinterpret_cast<uintptr_t>(d_msgs) & 15)) return CORDAHIP_ERR_INVALID_ARG;
  const Activity act(*d);
  if (hipSetDevice(d->id) != hipSuccess) return CORDAHIP_ERR_HIP;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);  // NULL = the device's null stream
  TimedCall* tc = timed_begin(*d, s);
  if (!tc) return CORDAHIP_ERR_HIP;
  hipError_t e = ed_verify_enqueue(*d, static_cast<const uint8_t*>(d_keys), static_cast<const uint8_t*>(d_sigs),
                                   static_cast<const uint8_t*>(d_msgs), msg_len, n, nullptr,
                                   static_cast<uint8_t*>(d_status), static_cast<unsigned long long*>(d_verdict), 0u, s);
  e = e ? e : hipEventRecord(tc->b, s);
  return hip_err(e);
}

int cordahip_ecdsa_verify_device(cordahip_ctx* ctx, int device, const void* d_scheme, const void* d_keys,
                                 const void* d_key_len, const void* d_sigs, const void* d_sig_len, const void* d_msgs,
                                 uint32_t msg_len, uint64_t n, void* d_status, void* d_verdict, void* hip_stream) {
  Device* d = dev_at(ctx, device);
  if (!d || (n && (!d_scheme || !d_keys || !d_key_len || !d_sigs || !d_sig_len || !d_status || (msg_len && !d_msgs))))
    return CORDAHIP_ERR_INVALID_ARG;
  const Activity act(*d);
  std::lock_guard<std::mutex> g(d->ec_mu[0]);
  if (hipSetDevice(d->id) != hipSuccess) return CORDAHIP_ERR_HIP;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  TimedCall* tc = timed_begin(*d, s);
  if (!tc) return CORDAHIP_ERR_HIP;
  hipError_t e = ec_verify_enqueue(*d, static_cast<const uint8_t*>(d_scheme), static_cast<const uint8_t*>(d_keys),
                                   static_cast<const uint8_t*>(d_key_len), static_cast<const uint8_t*>(d_sigs),
                                   static_cast<const uint8_t*>(d_sig_len), static_cast<const uint8_t*>(d_msgs), nullptr,
                                   msg_len, n, nullptr, static_cast<uint8_t*>(d_status),
                                   static_cast<unsigned long long*>(d_verdict), 0u, s);
  e = e ? e : hipEventRecord(tc->b, s);
  return hip_err(e);
}

double cordahip_last_kernel_ms(cordahip_ctx* ctx, int device) {
  Device* d = dev_at(ctx, device);
  if (!d) return -1.0;
  auto it = tl_last_call.find(d->uid);
  if (it == tl_last_call.end()) return -1.0;
  const TimedCall& tc = d->ring[it->second.first];
  {
    std::lock_guard<std::mutex> g(d->tmu);
    if (tc.gen != it->second.second) return -1.0;  // the slot was reused: > kTimingRing calls since
  }
  if (hipEventSynchronize(tc.b) != hipSuccess) return -1.0;
  float ms = -1.f;
  if (hipEventElapsedTime(&ms, tc.a, tc.b) != hipSuccess) return -1.0;
  {
    // a concurrent timed_begin may have re-recorded the slot's events between
    // the check above and the read: then ms mixes two calls, so report none
    std::lock_guard<std::mutex> g(d->tmu);
    if (tc.gen != it->second.second) return -1.0;
  }
  return ms;
}

int cordahip_ed25519_verify_host(cordahip_ctx* ctx, const uint8_t* keys, const uint8_t* sigs, const uint8_t* msgs,
                                 uint32_t msg_len, uint64_t n, uint8_t* status, uint64_t* verdict) {
  if (!ctx || (n && (!keys || !sigs || !status || (msg_len && !msgs)))) return CORDAHIP_ERR_INVALID_ARG;
  return guarded([&] { return ed25519_dense_host(ctx, keys, sigs, msgs, msg_len, n, status, verdict); });
}

int cordahip_filtered_tx_verify(cordahip_ctx* ctx, const cordahip_filtered_tx_batch* batch) {
  if (!ctx || !batch) return CORDAHIP_ERR_INVALID_ARG;
  return guarded([&] { return filtered_tx_impl(ctx, batch); });
}

int cordahip_stream_verify(cordahip_ctx* ctx, const cordahip_stream_batch* batch) {
  if (!ctx || !batch) return CORDAHIP_ERR_INVALID_ARG;
  return guarded([&] { return stream_verify_impl(ctx, batch); });
}

int cordahip_ed25519_sign_device(cordahip_ctx* ctx, int device, const void* d_seeds, const void* d_msgs,
                                 uint32_t msg_len, uint64_t n, void* d_pubs, void* d_sigs, void* hip_stream) {
  Device* d = dev_at(ctx, device);
  if (!d || (n && (!d_seeds || !d_pubs || !d_sigs))) return CORDAHIP_ERR_INVALID_ARG;
  if (hipSetDevice(d->id) != hipSuccess) return CORDAHIP_ERR_HIP;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);  // NULL = the device's null stream
  return hip_err(launch_ed25519_sign(static_cast<const uint8_t*>(d_seeds), static_cast<const uint8_t*>(d_msgs),
                                     msg_len, n, d->btab, static_cast<uint8_t*>(d_pubs),
                                     static_cast<uint8_t*>(d_sigs), s));
}

int cordahip_ecdsa_sign_device(cordahip_ctx* ctx, int device, const void* d_scheme, const void* d_seeds,
                               const void* d_msgs, uint32_t msg_len, uint64_t n, void* d_keys, void* d_key_len,
                               void* d_sigs, void* d_sig_len, void* hip_stream) {
  Device* d = dev_at(ctx, device);
  if (!d || (n && (!d_scheme || !d_seeds || !d_keys || !d_key_len || !d_sigs || !d_sig_len || (msg_len && !d_msgs))))
    return CORDAHIP_ERR_INVALID_ARG;
  if (hipSetDevice(d->id) != hipSuccess) return CORDAHIP_ERR_HIP;
  return hip_err(launch_ecdsa_sign(static_cast<const uint8_t*>(d_scheme), static_cast<const uint8_t*>(d_seeds),
                                   static_cast<const uint8_t*>(d_msgs), msg_len, n, d->gtab_k1, d->gtab_r1,
                                   static_cast<uint8_t*>(d_keys), static_cast<uint8_t*>(d_key_len),
                                   static_cast<uint8_t*>(d_sigs), static_cast<uint8_t*>(d_sig_len),
                                   static_cast<hipStream_t>(hip_stream)));
}

int cordahip_tx_ids(cordahip_ctx* ctx, const cordahip_txid_batch* batch) {
  if (!ctx || !batch) return CORDAHIP_ERR_INVALID_ARG;
  return guarded([&] { return tx_ids_impl(ctx, batch); });
}

int cordahip_signed_tx_verify(cordahip_ctx* ctx, const cordahip_signed_tx_batch* batch) {
  if (!ctx || !batch) return CORDAHIP_ERR_INVALID_ARG;
  return guarded([&] { return signed_tx_impl(ctx, batch); });
}

int cordahip_signed_tx_verify_ed25519_device(cordahip_ctx* ctx, int device, const void* d_leaf_bytes,
                                             const void* d_leaf_off, uint64_t nleaves, const void* d_tx_leaf_off,
                                             uint64_t ntx, const void* d_tx_sig_off, const void* d_keys,
                                             const void* d_sigs, uint64_t nsig, void* d_txid, void* d_tx_status,
                                             void* d_first_bad, void* d_sig_status, void* hip_stream) {
  Device* d = dev_at(ctx, device);
  if (!d || (ntx && (!d_leaf_off || !d_tx_leaf_off || !d_tx_sig_off || !d_txid || !d_tx_status || !d_first_bad)) ||
      (nsig && (!d_keys || !d_sigs || !d_sig_status)))
    return CORDAHIP_ERR_INVALID_ARG;
  // a buffer set for the enqueue; its event then fences the set's hashes / msgs
  // until these kernels finish (the next holder waits on it)
  const Activity act(*d);
  SetLease lease(*d);
  TxSet& S = lease.get();
  if (hipSetDevice(d->id) != hipSuccess) return CORDAHIP_ERR_HIP;
  TxWork& w = S.tx;
  if (w.hashes.cap < std::max<uint64_t>(nleaves, 1) * 32 || w.msgs.cap < std::max<uint64_t>(nsig, 1) * 32) {
    // growing frees the old buffers: the previous user's kernels must be done
    if (hipEventSynchronize(S.tx_ev) != hipSuccess) return CORDAHIP_ERR_HIP;
    if (w.hashes.ensure(std::max<uint64_t>(nleaves, 1) * 32) || w.msgs.ensure(std::max<uint64_t>(nsig, 1) * 32))
      return CORDAHIP_ERR_OUT_OF_MEMORY;
  }
  if (ensure_streams(*d) != hipSuccess) return CORDAHIP_ERR_HIP;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  // CORDAHIP_DEVICE_SPLIT=1: the id kernels fork onto the device's id stream beside the
  // key half of the Ed25519 prep on s (off by default: slower, see the component call)
  static const bool split = getenv("CORDAHIP_DEVICE_SPLIT") && getenv("CORDAHIP_DEVICE_SPLIT")[0] == '1';
  hipStream_t x = split ? d->s_idcopy : s;
  TimedCall* tc = timed_begin(*d, s);
  if (!tc) return CORDAHIP_ERR_HIP;
  hipError_t e = hipStreamWaitEvent(s, S.tx_ev, 0);  // the previous user of w.hashes / w.msgs is done
  if (split) {
    e = e ? e : hipEventRecord(S.fork, s);
    e = e ? e : hipStreamWaitEvent(x, S.fork, 0);
  }
  e = e ? e : launch_sha256_leaves(static_cast<const uint8_t*>(d_leaf_bytes), static_cast<const uint64_t*>(d_leaf_off),
                                   nleaves, w.hashes.as<uint32_t>(), x);
  e = e ? e : launch_merkle_root(w.hashes.as<uint32_t>(), static_cast<const uint64_t*>(d_tx_leaf_off), ntx,
                                 static_cast<uint8_t*>(d_txid), static_cast<uint8_t*>(d_tx_status), x);
  if (split) e = e ? e : hipEventRecord(S.ids, x);
  const std::function<hipError_t()> join = [&]() -> hipError_t {  // the ids, then the signatures' messages
    hipError_t r = split ? hipStreamWaitEvent(s, S.ids, 0) : hipSuccess;
    return r ? r : launch_gather_txid(static_cast<const uint8_t*>(d_txid), static_cast<const uint64_t*>(d_tx_sig_off),
                                      ntx, w.msgs.as<uint8_t>(), s);
  };
  // unforked, the ids come first and the prep runs fused (its key and message halves
  // as two launches cost ~0.6 ms more per 2.5 M signatures with nothing beside them)
  if (nsig == 0 || !split) e = e ? e : join();
  if (split)
    e = e ? e : ed_verify_enqueue(*d, static_cast<const uint8_t*>(d_keys), static_cast<const uint8_t*>(d_sigs),
                                  w.msgs.as<uint8_t>(), 32, nsig, nullptr, static_cast<uint8_t*>(d_sig_status), nullptr,
                                  0u, s, 0, nsig ? &join : nullptr);
  else
    e = e ? e : ed_verify_device_chunks(*d, S, static_cast<const uint8_t*>(d_keys), static_cast<const uint8_t*>(d_sigs),
                                        w.msgs.as<uint8_t>(), nsig, static_cast<uint8_t*>(d_sig_status), s);
  e = e ? e : hipEventRecord(S.tx_ev, s);  // fences w.hashes / w.msgs for the next user
  e = e ? e : launch_tx_reduce(static_cast<uint8_t*>(d_sig_status), static_cast<const uint64_t*>(d_tx_sig_off),
                               ntx, static_cast<int64_t*>(d_first_bad), static_cast<uint8_t*>(d_tx_status), s);
  e = e ? e : hipEventRecord(tc->b, s);
  return hip_err(e);
}

int cordahip_kryo_encode_device(cordahip_ctx* ctx, int device, const void* d_items, uint64_t n, uint32_t group,
                                void* d_out, uint64_t cap, void* d_off, void* d_status, void* hip_stream) {
  Device* d = dev_at(ctx, device);
  if (!d || !d_off || (n && (!d_items || !d_status))) return CORDAHIP_ERR_INVALID_ARG;
  if (n >= (1ull << 31) - 1) return CORDAHIP_ERR_INVALID_ARG;  // the scan counts items in an int
  return guarded([&]() -> int {
    const Activity act(*d);
    std::lock_guard<std::mutex> g(d->kryo_mu);
    if (hipSetDevice(d->id) != hipSuccess) return CORDAHIP_ERR_HIP;
    if (!d->kryo_ev && hipEventCreateWithFlags(&d->kryo_ev, hipEventDisableTiming) != hipSuccess)
      return CORDAHIP_ERR_HIP;
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    // the direct encoder's writers (items without a template): 2^13 threads,
    // 7 KB of level buffers each (56 MB)
    const uint64_t dwriters = 1u << 13;
    size_t temp_bytes = 0;
    if (kryo_scan_bytes(temp_bytes, n + 1, s) != hipSuccess) return CORDAHIP_ERR_HIP;
    if (d->kryo_sizes.cap < (n + 1) * 8 || d->kryo_temp.cap < temp_bytes || d->kryo_items.cap < n * 8 + 8 ||
        d->kryo_ws.cap < kryo_direct_ws_bytes(dwriters) || d->kryo_fixed.cap < kryo_fixed_scratch_bytes()) {
      // growing frees the old buffers: the previous user's kernels must be done
      if (hipEventSynchronize(d->kryo_ev) != hipSuccess) return CORDAHIP_ERR_HIP;
      if (d->kryo_sizes.ensure((n + 1) * 8) || d->kryo_temp.ensure(std::max<size_t>(temp_bytes, 16)) ||
          d->kryo_items.ensure(n * 8 + 8) || d->kryo_ws.ensure(kryo_direct_ws_bytes(dwriters)) ||
          kryo_fixed_ensure(*d))
        return CORDAHIP_ERR_OUT_OF_MEMORY;
    }
    TimedCall* tc = timed_begin(*d, s);
    if (!tc) return CORDAHIP_ERR_HIP;
    uint32_t* slots = d->kryo_items.as<uint32_t>();
    hipError_t e = hipStreamWaitEvent(s, d->kryo_ev, 0);  // the previous user of the scratch is done
    e = e ? e : kryo_state_ready(*d, s);
    e = e ? e
          : launch_kryo_encode(static_cast<const cordahip_kryo_item*>(d_items), nullptr, 0, n, group,
                               d->kryo_fixed.as<uint8_t>(),
                               slots, slots + n, d->kryo_sizes.as<uint64_t>(), static_cast<uint64_t*>(d_off),
                               static_cast<uint8_t*>(d_out), d_out ? cap : 0, static_cast<uint8_t*>(d_status),
                               d->kryo_ws.as<uint8_t>(), dwriters, d->kryo_temp.p, d->kryo_temp.cap, s);
    e = e ? e : kryo_usage_report(*d, nullptr, s);
    e = e ? e : hipEventRecord(d->kryo_ev, s);
    e = e ? e : hipEventRecord(tc->b, s);
    return hip_err(e);
  });
}

int cordahip_signed_txcomp_verify_ed25519_device(cordahip_ctx* ctx, int device, const void* d_items,
                                                 uint64_t n_items, uint32_t group, const void* d_payload,
                                                 uint64_t payload_len, const void* d_tx_item_off, uint64_t ntx,
                                                 const void* d_tx_sig_off, const void* d_keys, const void* d_sigs,
                                                 uint64_t nsig, void* d_txid, void* d_tx_status, void* d_first_bad,
                                                 void* d_sig_status, void* hip_stream) {
  Device* d = dev_at(ctx, device);
  if (!d || (ntx && (!d_tx_item_off || !d_tx_sig_off || !d_txid || !d_tx_status || !d_first_bad)) ||
      (n_items && !d_items) || (payload_len && !d_payload) || (nsig && (!d_keys || !d_sigs || !d_sig_status)))
    return CORDAHIP_ERR_INVALID_ARG;
  if (n_items >= (1ull << 31) - 1) return CORDAHIP_ERR_INVALID_ARG;  // the encoder's item slots and lists are 32-bit
  if ((reinterpret_cast<uintptr_t>(d_keys) | reinterpret_cast<uintptr_t>(d_sigs)) & 15) return CORDAHIP_ERR_INVALID_ARG;
  return guarded([&]() -> int {
    // a buffer set for the enqueue (its hashes, messages and component statuses, fenced
    // by its event until these kernels finish) and the encoder's scratch (kryo_mu, kryo_ev)
    const Activity act(*d);
    SetLease lease(*d);
    TxSet& S = lease.get();
    std::lock_guard<std::mutex> gk(d->kryo_mu);
    if (hipSetDevice(d->id) != hipSuccess) return CORDAHIP_ERR_HIP;
    if (!d->kryo_ev && hipEventCreateWithFlags(&d->kryo_ev, hipEventDisableTiming) != hipSuccess) return CORDAHIP_ERR_HIP;
    TxWork& w = S.tx;
    const uint64_t dwriters = CompPlan::kDirectWriters;
    if (w.hashes.cap < std::max<uint64_t>(n_items, 1) * 32 || w.msgs.cap < std::max<uint64_t>(nsig, 1) * 32 ||
        w.comp_status.cap < std::max<uint64_t>(n_items, 1)) {
      // growing frees the old buffers: the set's previous user must be done
      if (hipEventSynchronize(S.tx_ev) != hipSuccess) return CORDAHIP_ERR_HIP;
      if (w.hashes.ensure(std::max<uint64_t>(n_items, 1) * 32) || w.msgs.ensure(std::max<uint64_t>(nsig, 1) * 32) ||
          w.comp_status.ensure(std::max<uint64_t>(n_items, 1)))
        return CORDAHIP_ERR_OUT_OF_MEMORY;
    }
    if (d->kryo_sizes.cap < (n_items + 1) * 8 || d->kryo_items.cap < n_items * 8 + 8 ||
        d->kryo_ws.cap < kryo_direct_ws_bytes(dwriters) || d->kryo_fixed.cap < kryo_fixed_scratch_bytes()) {
      if (hipEventSynchronize(d->kryo_ev) != hipSuccess) return CORDAHIP_ERR_HIP;
      if (d->kryo_sizes.ensure((n_items + 1) * 8) || d->kryo_items.ensure(n_items * 8 + 8) ||
          d->kryo_ws.ensure(kryo_direct_ws_bytes(dwriters)) || kryo_fixed_ensure(*d))
        return CORDAHIP_ERR_OUT_OF_MEMORY;
    }
    if (ensure_streams(*d) != hipSuccess) return CORDAHIP_ERR_HIP;
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    // CORDAHIP_DEVICE_SPLIT=1: the id chain forks onto the device's id stream and runs
    // beside the key half of the Ed25519 prep (key and R decoding: no dependence on the
    // ids) on s, which joins it before the message half. Off: the split prep's two
    // launches cost more than the overlap gains (c4 --device-encode 87.3-87.4 against
    // 89.1-89.2 M sig/s, c4 95.6-95.9 against 96.1-96.5; profiles/r06_device_split_ab/)
    static const bool split = getenv("CORDAHIP_DEVICE_SPLIT") && getenv("CORDAHIP_DEVICE_SPLIT")[0] == '1';
    hipStream_t x = split ? d->s_idcopy : s;
    TimedCall* tc = timed_begin(*d, s);
    if (!tc) return CORDAHIP_ERR_HIP;
    uint32_t* slots = d->kryo_items.as<uint32_t>();
    hipError_t e = hipStreamWaitEvent(s, S.tx_ev, 0);  // the previous users of the set's buffers
    e = e ? e : hipStreamWaitEvent(s, d->kryo_ev, 0);  // and of the encoder's scratch are done
    if (split) {
      e = e ? e : hipEventRecord(S.fork, s);
      e = e ? e : hipStreamWaitEvent(x, S.fork, 0);
    }
    e = e ? e : kryo_state_ready(*d, x);
    // leaf hashes from the templates (misses impossible: new shapes are built, the rest
    // hashed by the direct encoder), then the ids, with a rejected component making its
    // transaction CORDAHIP_TX_BAD_COMPONENT
    e = e ? e
          : launch_kryo_hash_chain(static_cast<const cordahip_kryo_item*>(d_items),
                                   static_cast<const uint8_t*>(d_payload), payload_len, n_items, group,
                                   d->kryo_fixed.as<uint8_t>(), slots, slots + n_items, d->kryo_sizes.as<uint64_t>(),
                                   w.comp_status.as<uint8_t>(), w.hashes.as<uint32_t>(), d->kryo_ws.as<uint8_t>(),
                                   dwriters, x);
    e = e ? e : kryo_usage_report(*d, nullptr, x);
    e = e ? e : hipEventRecord(d->kryo_ev, x);
    e = e ? e : launch_merkle_root(w.hashes.as<uint32_t>(), static_cast<const uint64_t*>(d_tx_item_off), ntx,
                                   static_cast<uint8_t*>(d_txid), static_cast<uint8_t*>(d_tx_status), x,
                                   w.comp_status.as<uint8_t>());
    if (split) e = e ? e : hipEventRecord(S.ids, x);
    const std::function<hipError_t()> join = [&]() -> hipError_t {  // the ids, then the signatures' messages
      hipError_t r = split ? hipStreamWaitEvent(s, S.ids, 0) : hipSuccess;
      return r ? r : launch_gather_txid(static_cast<const uint8_t*>(d_txid), static_cast<const uint64_t*>(d_tx_sig_off),
                                        ntx, w.msgs.as<uint8_t>(), s);
    };
    if (nsig == 0 || !split) e = e ? e : join();  // unforked: ids first, then the fused prep
    if (split)
      e = e ? e : ed_verify_enqueue(*d, static_cast<const uint8_t*>(d_keys), static_cast<const uint8_t*>(d_sigs),
                                    w.msgs.as<uint8_t>(), 32, nsig, nullptr, static_cast<uint8_t*>(d_sig_status),
                                    nullptr, 0u, s, 0, nsig ? &join : nullptr);
    else
      e = e ? e : ed_verify_device_chunks(*d, S, static_cast<const uint8_t*>(d_keys),
                                          static_cast<const uint8_t*>(d_sigs), w.msgs.as<uint8_t>(), nsig,
                                          static_cast<uint8_t*>(d_sig_status), s);
    e = e ? e : hipEventRecord(S.tx_ev, s);  // fences the set's buffers for the next user
    e = e ? e : launch_tx_reduce(static_cast<uint8_t*>(d_sig_status), static_cast<const uint64_t*>(d_tx_sig_off), ntx,
                                 static_cast<int64_t*>(d_first_bad), static_cast<uint8_t*>(d_tx_status), s);
    e = e ? e : hipEventRecord(tc->b, s);
    return hip_err(e);
  });
}

}  // extern "C"
