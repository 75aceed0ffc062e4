// libcordahip's internal runtime types (not ABI): per-device state, buffers,
// the ticket pool, the host thread pool and the enqueue helpers shared by
// cordahip.cpp (C-ABI, tx / stream / device paths) and host_batch.cpp (the
// generic CSR signature batch).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/cordahip.h"
#include "numa_place.hpp"

namespace cordahip {
hipError_t launch_ed25519_btable(uint32_t* tab, hipStream_t s);
size_t ed25519_btable_bytes();
hipError_t launch_ed25519_verify(const uint8_t* keys, const uint8_t* sigs, const uint8_t* msgs, uint32_t msg_len,
                                 uint64_t n, const uint32_t* btab, const uint8_t* pre_status, uint8_t* status,
                                 unsigned long long* verdict, uint32_t* ws, uint64_t ws_lanes, uint32_t flags,
                                 hipStream_t s,
                                 const std::function<hipError_t()>* before_msgs = nullptr);
size_t ed25519_ws_lane_bytes();
hipError_t launch_ed25519_sign(const uint8_t* seeds, const uint8_t* msgs, uint32_t msg_len, uint64_t n,
                               const uint32_t* btab, uint8_t* pubs, uint8_t* sigs, hipStream_t s);
hipError_t launch_sha256_leaves(const uint8_t* bytes, const uint64_t* off, uint64_t nleaves, uint32_t* hashes,
                                hipStream_t s);
hipError_t launch_merkle_root(uint32_t* hashes, const uint64_t* tx_leaf_off, uint64_t ntx, uint8_t* txid,
                              uint8_t* tx_status, hipStream_t s, const uint8_t* item_status = nullptr,
                              uint8_t* map_txid = nullptr, uint8_t* map_status = nullptr);
hipError_t launch_gather_txid(const uint8_t* txid, const uint64_t* tx_sig_off, uint64_t ntx, uint8_t* msgs,
                              hipStream_t s);
hipError_t launch_store_to_host(const void* src, void* dst, uint64_t n, hipStream_t s);
hipError_t tx_set_id_priority(uint32_t on);  // the id kernels' raised wave priority (current device)
hipError_t kryo_set_priority(uint32_t on);   // the same for the Kryo encoder's kernels
// kryo_device.hip: the GPU Kryo leaf encoder (shapes, templates, sizes, scan, writes)
size_t kryo_fixed_scratch_bytes();                     // shape table, records, templates (persistent per device)
size_t kryo_direct_ws_bytes(uint64_t writers);         // the direct encoder's level buffers
hipError_t kryo_scan_bytes(size_t& bytes, uint64_t n1, hipStream_t s);
hipError_t kryo_clear(uint8_t* fixed, hipStream_t s);  // empty the shape table (and the template arena)
// device: [templates in the arena, table slots in use, misses of buffer set 0, of set 1]
// (each set's since its kryo_reset_misses)
const uint32_t* kryo_usage_src(uint8_t* fixed);
constexpr size_t kKryoUsageBytes = 16;
hipError_t kryo_reset_misses(uint8_t* fixed, uint32_t set, hipStream_t s);
uint32_t kryo_clear_threshold_slots();
uint32_t kryo_clear_threshold_templates();
// data_base != nullptr: items' `data` are offsets into data_len bytes at data_base.
// templates_only: the steady-state chain -- no new shapes built, no direct encoder;
// an item that would need either is a miss (counted, its leaf not written, status
// kKryoMiss) and the caller redoes the batch with templates_only false.
constexpr uint8_t kKryoMiss = 4;
hipError_t launch_kryo_encode(const cordahip_kryo_item* items, const uint8_t* data_base, uint64_t data_len,
                              uint64_t n, uint32_t group, uint8_t* fixed,
                              uint32_t* item_slot, uint32_t* direct, uint64_t* sizes, uint64_t* off, uint8_t* out,
                              uint64_t cap, uint8_t* status, uint8_t* dws, uint64_t dwriters, void* scan_temp,
                              size_t scan_bytes, hipStream_t s, bool templates_only = false, uint32_t set = 0);
// the shape pass alone (sizes, item_slot, statuses; kCMiss counts misses)
hipError_t launch_kryo_shape(const cordahip_kryo_item* items, const uint8_t* data_base, uint64_t data_len, uint64_t n,
                             uint32_t group, uint8_t* fixed, uint32_t* item_slot, uint32_t* direct, uint64_t* sizes,
                             uint8_t* status, hipStream_t s, bool templates_only, uint32_t set = 0);
// SHA-256 of every item's leaf straight from its template (after a templates-only shape
// pass): hashes[n][8] big-endian words, zero for items with a nonzero status
hipError_t launch_kryo_shape_hash(const cordahip_kryo_item* d_items, const uint8_t* data_base, uint64_t data_len,
                                  uint64_t n, uint32_t group, uint8_t* fixed, uint8_t* status, uint32_t* hashes,
                                  hipStream_t s, uint32_t set);
hipError_t launch_kryo_hash(const cordahip_kryo_item* items, const uint8_t* data_base, uint64_t data_len, uint64_t n,
                            uint32_t group, uint8_t* fixed, const uint32_t* item_slot, const uint64_t* sizes,
                            const uint8_t* status, uint32_t* hashes, hipStream_t s);
// the device hash chain (no misses, no leaf bytes): shapes -> build -> tsize ->
// kryo_hash -> kryo_dhash (the direct encoder into a SHA-256 sink); hashes[n][8]
// big-endian words, zero for an item the encoder rejects (status 1)
hipError_t launch_kryo_hash_chain(const cordahip_kryo_item* items, const uint8_t* data_base, uint64_t data_len,
                                  uint64_t n, uint32_t group, uint8_t* fixed, uint32_t* item_slot, uint32_t* direct,
                                  uint64_t* sizes, uint8_t* status, uint32_t* hashes, uint8_t* dws, uint64_t dwriters,
                                  hipStream_t s);
hipError_t launch_gather_rows32(const uint8_t* txid, const uint32_t* idx, uint64_t n, uint8_t* rows, hipStream_t s);
hipError_t launch_tx_reduce(uint8_t* sig_status, const uint64_t* tx_sig_off, uint64_t ntx, int64_t* first_bad,
                            uint8_t* tx_status, hipStream_t s);
hipError_t launch_pmt_verify(const uint32_t* leaf_hashes, const uint64_t* tx_leaf_off, const uint8_t* tok,
                             const uint8_t* tok_hash, const uint64_t* tx_tok_off, const uint8_t* root, uint64_t ntx,
                             uint32_t* stack, uint8_t* tx_status, hipStream_t s);
size_t ecdsa_gtable_bytes();
hipError_t launch_ecdsa_gtables(uint32_t* k1, uint32_t* r1, hipStream_t s);
hipError_t launch_ecdsa_verify(const uint8_t* scheme, const uint8_t* keys, const uint8_t* key_len,
                               const uint8_t* sigs, const uint8_t* sig_len, const uint8_t* msgs,
                               const uint64_t* msg_off, uint32_t msg_len, uint64_t n, const uint32_t* gk1,
                               const uint32_t* gr1, const uint8_t* pre_status, uint8_t* status,
                               unsigned long long* verdict, unsigned int* counters6, unsigned int* perm,
                               uint32_t* ws, uint64_t ws_slots, uint32_t flags, hipStream_t s);
size_t ecdsa_ws_slot_bytes();
hipError_t launch_ecdsa_sign(const uint8_t* scheme, const uint8_t* seeds, const uint8_t* msgs, uint32_t msg_len,
                             uint64_t n, const uint32_t* gk1, const uint32_t* gr1, uint8_t* keys, uint8_t* key_len,
                             uint8_t* sigs, uint8_t* sig_len, hipStream_t s);

namespace rt {

// The library's device memory per HIP device (every DevBuf, the fixed tables):
// bytes in use and their peak, for cordahip_device_mem and the budget
// (CORDAHIP_DEVICE_MEM_BUDGET) that sizes the workspaces.
constexpr int kMaxHipDevices = 64;
struct MemAcct {
  std::atomic<uint64_t> in_use{0}, peak{0};
  void add(uint64_t b) {
    const uint64_t now = in_use.fetch_add(b) + b;
    uint64_t p = peak.load();
    while (now > p && !peak.compare_exchange_weak(p, now)) {
    }
  }
  void sub(uint64_t b) { in_use.fetch_sub(b); }
};
MemAcct& mem_acct(int dev);

// grow-only device buffer (accounted on the device it was allocated on)
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int dev = -1;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    release();
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) d = 0;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) {
      cap = bytes;
      dev = d;
      mem_acct(dev).add(bytes);
    } else {
      p = nullptr;
    }
    return e;
  }
  void release() {
    if (p) {
      (void)hipFree(p);
      mem_acct(dev).sub(cap);
    }
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// grow-only page-locked host buffer (staging for the packed host pipelines)
struct PinBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// one stage (buffer set) of the C5 streaming pipeline (cordahip_stream_verify);
// its events order the reuse of the buffers, so the host never waits per chunk
struct StreamStage {
  hipEvent_t ed_copied = nullptr, ec_copied = nullptr;  // this chunk's H2D of each section done
  hipEvent_t ed_done = nullptr, ec_done = nullptr;      // its kernels and status D2H done: buffers free
  DevBuf ed_keys, ed_sigs, ed_msgs, ed_status;
  DevBuf ec_scheme, ec_keys, ec_key_len, ec_sigs, ec_sig_len, ec_msgs, ec_status;
};
constexpr int kStreamStages = 3;
// lanes per chunk, both sections together (C5 A/B on one box, profiles/r02_c5_stream_ab.json:
// 2^21 76.7, 2^22 82.4, 2^23 84.9, 2^24 84.6 M verifs/s with the single-stream stages)
constexpr uint64_t kStreamChunk = 1ull << 23;

// one stage of a packed host pipeline (host_batch.cpp): the host packs a chunk
// of lanes into the pinned buffers, they cross PCIe into the device buffers,
// the kernels run, the statuses come back into h_status; `done` marks the
// stage reusable (the host scatters its statuses first)
struct PackStage {
  hipEvent_t copied = nullptr, done = nullptr;
  PinBuf h[9];
  DevBuf d[9];
  bool pending = false;
  uint64_t tag0 = 0, tag1 = 0, tag2 = 0;  // which chunk is in flight (pipeline-defined)
};
constexpr int kPackStages = 3;
// Signed-tx batches keep more of their small (2^17-signature) chunks in flight:
// a chunk's prep waits for its id slice, and with three stages the pipeline could
// not run far enough ahead of the id chain -- c4h --components at two calls in
// flight 79.4-82.5 M sig/s with 3 stages, 84.7-85.7 with 4, 86.3-87.1 with 5,
// 86.4-87.6 with 6; c4h 90.3-91.5 / 90.6-91.5 / 89.3-92.6 / 92.4-92.5
// (profiles/r06_pack_stages_ab/). Generic batches (4 M-lane chunks, ~0.55 GB of
// pinned rows each) keep three.
#ifndef CORDAHIP_TX_STAGES
#define CORDAHIP_TX_STAGES 6  // A/B builds: -DCORDAHIP_TX_STAGES=N
#endif
constexpr int kTxStages = CORDAHIP_TX_STAGES;

// one stage of the generic-batch pipeline (host_batch.cpp): a chunk of the
// batch's lanes, classified and packed into BOTH sections' pinned buffers
// (h/d[0..4] Ed25519 keys, sigs, msgs, pre-status, status; [5..13] ECDSA
// scheme, keys, key_len, sigs, sig_len, msgs, msg_off, pre-status, status);
// the lane lists say where each row's status goes back
struct BatchStage {
  hipEvent_t copied = nullptr, ed_done = nullptr, ec_done = nullptr;
  PinBuf h[14];
  DevBuf d[14];
  PinBuf hidx[2];  // device-id messages (MsgView::dev): per Ed25519 / ECDSA row, its tx's id index
  DevBuf didx[2];
  std::vector<uint64_t> ed_lanes, ec_lanes;
  uint64_t a = 0, b = 0;  // the chunk's lanes [a, b) (per-chunk verdict words)
  bool direct = false;    // rows == lanes: statuses / verdict words went straight to the caller's pinned arrays
  DevBuf dverdict;        // the direct chunks' verdict words (wave ballots of the Ed25519 kernel)
  bool pending = false;
};

struct TxWork {  // device buffers of the transaction paths (grow-only)
  DevBuf leaf_bytes, leaf_off, tx_leaf_off, hashes, txid, tx_status, tx_sig_off, msgs;
  DevBuf comp_items, payload, comp_status;  // component-level batches: items, their payload, encoder statuses
  DevBuf tok, tok_hash, tx_tok_off, root, stack;  // filtered-tx (partial Merkle tree) path
};

// One set of a device's transaction and signature-pipeline buffers. A call
// holds its set from start to finish; tx_ev marks the completion of the last
// work enqueued on the set's device buffers (the next holder's first wait).
struct TxSet {
  TxWork tx;
  hipEvent_t tx_ev = nullptr;
  BatchStage pb[kTxStages];  // generic CSR batches (the first kPackStages) and the signed-tx signature chunks
  // component calls: the encoder's usage counters after this set's last call,
  // host-mapped: [templates in the arena, table slots in use, misses of set 0, of set 1]
  uint32_t* kryo_usage = nullptr;
  uint32_t* kryo_usage_dev = nullptr;
  // the device signed-tx calls' fork / join: the id chain runs on the id stream beside
  // the key half of the Ed25519 prep on the caller's stream
  hipEvent_t fork = nullptr, ids = nullptr;
  // their chunked Ed25519 section (ed_verify_device_chunks): s_ed2 forks off the
  // caller's stream and joins it again
  hipEvent_t ed_fork = nullptr, ed_join = nullptr;
};
constexpr int kTxSets = 2;

struct EcWork {  // device buffers of the ECDSA paths (grow-only)
  DevBuf counters, perm;
  DevBuf ws;                 // split-kernel workspace (kEcWsSlots records)
  hipEvent_t ev = nullptr;   // last enqueued user of counters/perm/ws (cross-stream reuse)
};

// Per-call timing of the *_device entry points: a ring of event pairs per
// device, one pair per call, so concurrent callers never share events; a
// slot's generation tells a reader whether its call's events are still there.
constexpr int kTimingRing = 64;
struct TimedCall {
  hipEvent_t a = nullptr, b = nullptr;
  uint64_t gen = 0;
};

class HostPool;

struct Device {
  int id = 0;
  uint64_t uid = 0;  // process-unique: keys the per-thread timing slot
  // host threads next to this GPU (numa_place.hpp): the packing / scattering /
  // reduce pool of its pipelines, bound to CPUs of its NUMA node; the thread that
  // runs a pipeline binds itself there for the call (NodeBind), so the pinned
  // stages it allocates are first-touched on that node too
  NumaPlace place;
  std::unique_ptr<HostPool> pool;
  // device memory (CORDAHIP_DEVICE_MEM_BUDGET, cordahip_init): the workspace sizes
  // the budget allows -- Ed25519 slots 0 / 1 (lanes), ECDSA (slots) -- and the
  // activity the idle release reads (calls in progress, the last one's end)
  uint64_t mem_budget = 0;
  uint64_t ed_ws_lanes[2] = {0, 0};
  uint64_t ec_ws_slots = 0;
  std::atomic<int> active{0};
  std::atomic<int64_t> last_use_ms{0};
  uint32_t* btab = nullptr;
  uint32_t* gtab_k1 = nullptr;  // [k]G tables, k = 0..128, secp256k1 / P-256
  uint32_t* gtab_r1 = nullptr;
  // ECDSA workspaces: slot 0 for the device path and the stream drain, slot 1 for the
  // host pipelines' alternate chunks (capped at half of slot 0), each with its lock;
  // ec_turn alternates the host chunks between them (s_ec / s_ec2)
  std::mutex ec_mu[2];
  EcWork ec[2];
  std::atomic<uint32_t> ec_turn{0};
  hipStream_t stream = nullptr;  // context stream (init-time work and host tx paths)
  std::mutex tmu;
  TimedCall ring[kTimingRing];
  uint64_t ring_next = 0;
  // Transaction / signature-pipeline buffer sets (TxSet): a call holds one set
  // from start to finish (acquire_set / SetLease); two sets let a signed-tx call
  // drain while the next one enqueues. tx_order_mu is the enqueue token of the
  // signed-tx path: held from a call's start until its last chunk is enqueued,
  // so consecutive calls' work reaches the shared streams in call order.
  TxSet set[kTxSets];
  std::mutex set_m;
  std::condition_variable set_cv;
  bool set_busy[kTxSets] = {};
  std::mutex tx_order_mu;
  // consecutive Ed25519 chunks of every pipeline call alternate workspace slots and
  // streams (s_ed / s_ed2) across calls too, so call k + 1's first prep overlaps
  // call k's last ladder
  std::atomic<uint32_t> ed_turn{0};
  // Ed25519 split-kernel workspace, shared by every stream that verifies on
  // this device: ed_mu orders the enqueues, ed_ev makes each user's stream
  // wait for the previous user's kernels before it reuses the buffer.
  // Two workspace slots: the host pipelines alternate consecutive chunks between
  // them and between s_ed / s_ed2, so chunk k + 1's kernels fill the CUs chunk
  // k's end-of-grid tail leaves idle (slot 0 alone serves the device paths).
  std::mutex ed_mu[2];
  DevBuf ed_ws[2];
  hipEvent_t ed_ev[2] = {nullptr, nullptr};
  // The pipelines' three streams, created together and shared by the C5 drain
  // and the packed host pipelines: every H2D on s_copy (PCIe in chunk order),
  // each section's kernels + status D2H on its own stream. Three active
  // streams, not one per stage and section: HIP maps streams onto
  // GPU_MAX_HW_QUEUES (4) hardware queues, and streams sharing a queue
  // serialise (with 6 stage streams C5 ran 90.6 M/s at 4 queues, 93.4 at 8).
  std::mutex streams_mu;
  hipStream_t s_copy = nullptr, s_ed = nullptr, s_ec = nullptr, s_ed2 = nullptr;
  hipStream_t s_ec2 = nullptr;  // = s_idcopy: generic batches' alternate ECDSA chunks
  // signed-tx batches: the id slices' leaf-byte H2D on a stream of its own, so
  // slice j + 1's bytes cross PCIe while slice j hashes (d.stream)
  hipStream_t s_idcopy = nullptr;
  std::mutex stream_mu;  // serialises use of sstage (C5)
  StreamStage sstage[kStreamStages];
  // packed dense Ed25519 rows (cordahip_ed25519_verify_host); the generic CSR
  // batches' stages live in the TxSets
  std::mutex ped_mu;
  PackStage ped[kPackStages];
  // GPU Kryo encoder scratch (cordahip_kryo_encode_device): leaf sizes, the
  // scan's temporary storage, the shape table and templates, per-item shape
  // slots and the direct-encoder list, the direct writers' OutputChunked level
  // buffers; kryo_mu orders the enqueues, kryo_ev fences reuse
  std::mutex kryo_mu;
  DevBuf kryo_sizes, kryo_temp, kryo_ws, kryo_fixed, kryo_items;
  // the fixed part is persistent (shape table, records, templates): zeroed when
  // allocated, cleared when a call reports it over half full (TxSet::kryo_usage:
  // a host-mapped copy of its usage counters, stored after each call)
  bool kryo_fresh = false;
  bool kryo_templates_ok = false;  // the last component batch had no encoder misses (cordahip.cpp)
  uint32_t* kryo_usage = nullptr;      // cordahip_kryo_encode_device's own report
  uint32_t* kryo_usage_dev = nullptr;
  uint64_t kryo_gen = 0;           // table clears so far (kryo_mu): a call's end updates kryo_templates_ok
                                   // only if no clear came after its start
  hipEvent_t kryo_ev = nullptr;
};

// Fork-join pool for host-side packing and scattering. parallel_for splits
// [0, n) into pieces of at least `grain` lanes; the caller runs pieces too,
// so concurrent callers (one pipeline per device and section) all progress.
class HostPool {
 public:
  // cpus non-empty: every worker thread is bound to them (a device's NUMA node)
  explicit HostPool(int nthreads, const std::vector<int>& cpus = {});
  ~HostPool();
  int threads() const { return (int)threads_.size() + 1; }
  void parallel_for(uint64_t n, uint64_t grain, const std::function<void(uint64_t, uint64_t)>& fn);

 private:
  struct Job {
    const std::function<void(uint64_t, uint64_t)>* fn = nullptr;
    uint64_t n = 0, piece = 0, npieces = 0;
    std::atomic<uint64_t> next{0}, done{0};
    std::mutex m;
    std::condition_variable cv;
  };
  static void run_pieces(Job& j);
  void worker();
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::shared_ptr<Job>> q_;
  std::vector<std::thread> threads_;
  bool stop_ = false;
};

// The calling thread bound to a device's CPUs for a scope (its previous affinity
// restored after): pipelines pack rows and first-touch pinned stages on the GPU's
// NUMA node. No-op when the device has no placement.
class NodeBind {
 public:
  explicit NodeBind(const Device& d);
  ~NodeBind();
  NodeBind(const NodeBind&) = delete;
  NodeBind& operator=(const NodeBind&) = delete;

 private:
  bool bound_ = false;
  std::vector<unsigned char> saved_;  // cpu_set_t bytes
};
// the pool a device's host work runs on
HostPool& pool_of(cordahip_ctx* ctx, Device& d);


// ---- ticket pool -------------------------------------------------------------
struct JobState {
  std::mutex m;
  std::condition_variable cv;
  bool done = false;
  int rc = CORDAHIP_SUCCESS;
};

class WorkerPool {
 public:
  explicit WorkerPool(int nthreads);
  ~WorkerPool();
  void push(std::shared_ptr<JobState> st, std::function<int()> fn);

 private:
  void run();
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::pair<std::shared_ptr<JobState>, std::function<int()>>> q_;
  std::vector<std::thread> threads_;
  bool stop_ = false;
};

// CORDAHIP_TRACE=1: host-side phase timings of the host pipelines on stderr
// (wait for a stage, classify, pack, enqueue; tx-id / signature phases), to
// see whether the host or the GPU bounds a host batch
inline double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
inline bool tracing() {
  static const bool on = getenv("CORDAHIP_TRACE") != nullptr;
  return on;
}

// a call in progress on a device (the idle release waits for none)
class Activity {
 public:
  explicit Activity(Device& d) : d_(d) { d_.active.fetch_add(1); }
  ~Activity() {
    d_.last_use_ms.store((int64_t)now_ms());
    d_.active.fetch_sub(1);
  }
  Activity(const Activity&) = delete;
  Activity& operator=(const Activity&) = delete;

 private:
  Device& d_;
};

// The device address of pinned host memory p (nullptr when p is pageable or
// unknown to HIP): kernels store results there directly, since a D2H
// hipMemcpyAsync queued behind busy compute streams can hold the enqueuing
// thread for milliseconds (7-9 ms per call in profiles/r04_q)
inline void* host_mapped(const void* p) {
  hipPointerAttribute_t at;
  void* dp = nullptr;
  if (!p || hipPointerGetAttributes(&at, p) != hipSuccess || at.type != hipMemoryTypeHost ||
      hipHostGetDevicePointer(&dp, const_cast<void*>(p), 0) != hipSuccess)
    dp = nullptr;
  (void)hipGetLastError();
  return dp;
}

// under CORDAHIP_TRACE: report a HIP call that held the host for over 1 ms
template <class F>
hipError_t blocked(const char* what, F&& f) {
  if (!tracing()) return f();
  const double t = now_ms();
  const hipError_t e = f();
  const double dt = now_ms() - t;
  if (dt > 1.0) fprintf(stderr, "[cordahip] %s held the host %.2f ms\n", what, dt);
  return e;
}

int hip_err(hipError_t e);
hipError_t ensure_streams(Device& d);
// before_msgs != nullptr: the messages are produced on stream s by that callback,
// which runs after the keys' half of the prep is enqueued (launch_ed25519_verify)
hipError_t ed_verify_enqueue(Device& d, const uint8_t* keys, const uint8_t* sigs, const uint8_t* msgs,
                             uint32_t msg_len, uint64_t n, const uint8_t* pre, uint8_t* status,
                             unsigned long long* verdict, uint32_t flags, hipStream_t s, int slot = 0,
                             const std::function<hipError_t()>* before_msgs = nullptr);
// d.ec_mu[slot] must be held
hipError_t ec_verify_enqueue(Device& d, const uint8_t* scheme, const uint8_t* keys, const uint8_t* key_len,
                             const uint8_t* sigs, const uint8_t* sig_len, const uint8_t* msgs, const uint64_t* msg_off,
                             uint32_t msg_len, uint64_t n, const uint8_t* pre, uint8_t* status,
                             unsigned long long* verdict, uint32_t flags, hipStream_t s, int slot = 0);
void shard_range(uint64_t n, uint64_t nshards, uint64_t shard, uint64_t align, uint64_t& lo, uint64_t& hi);
uint64_t env_lanes(const char* name, uint64_t dflt);

// Run fn(device, lo, hi) for every non-empty shard of n lanes, one host thread
// per device; returns the first failure.
template <class F>
int for_shards(std::vector<std::unique_ptr<Device>>& devs, uint64_t n, uint64_t align, F fn) {
  const uint64_t nd = devs.size();
  std::vector<std::future<int>> fs;
  for (uint64_t i = 0; i < nd; i++) {
    uint64_t lo, hi;
    shard_range(n, nd, i, align, lo, hi);
    if (lo >= hi) break;
    Device* d = devs[i].get();
    if (nd == 1) return fn(*d, lo, hi);
    fs.push_back(std::async(std::launch::async, [=, &fn] { return fn(*d, lo, hi); }));
  }
  int rc = CORDAHIP_SUCCESS;
  for (auto& f : fs) {
    const int r = f.get();
    if (r != CORDAHIP_SUCCESS && rc == CORDAHIP_SUCCESS) rc = r;
  }
  return rc;
}

// A device's buffer set for one call: the first free one (blocks while both are
// held); `prefer` is tried first. The holder then waits on set.tx_ev before
// touching device buffers an asynchronous device-path call may still use.
class SetLease {
 public:
  // exact: set `prefer` itself (the idle release takes both)
  explicit SetLease(Device& d, int prefer = 0, bool exact = false) : d_(d) {
    std::unique_lock<std::mutex> g(d.set_m);
    for (;;) {
      for (int k = 0; k < (exact ? 1 : kTxSets); k++) {
        const int i = (prefer + k) % kTxSets;
        if (!d.set_busy[i]) {
          d.set_busy[i] = true;
          idx_ = i;
          return;
        }
      }
      d.set_cv.wait(g);
    }
  }
  ~SetLease() {
    {
      std::lock_guard<std::mutex> g(d_.set_m);
      d_.set_busy[idx_] = false;
    }
    d_.set_cv.notify_one();
  }
  SetLease(const SetLease&) = delete;
  SetLease& operator=(const SetLease&) = delete;
  int index() const { return idx_; }
  TxSet& get() const { return d_.set[idx_]; }

 private:
  Device& d_;
  int idx_ = 0;
};

}  // namespace rt
}  // namespace cordahip

struct cordahip_ctx {
  std::vector<std::unique_ptr<cordahip::rt::Device>> devs;
  std::mutex mu;  // guards next_ticket and jobs
  uint64_t next_ticket = 1;
  std::unordered_map<uint64_t, std::shared_ptr<cordahip::rt::JobState>> jobs;
  std::unique_ptr<cordahip::rt::WorkerPool> pool;
  std::unique_ptr<cordahip::rt::HostPool> host;  // packing / scattering threads
  // signed-tx batches' signature -> transaction maps, kept for reuse across
  // calls (a fresh 20 MB map per C4 call page-faulted for 0.8-3.9 ms): taken
  // by a call, returned after it; at most kTxOfCache kept
  static constexpr size_t kTxOfCache = 4;
  std::mutex txof_mu;
  std::vector<std::pair<std::unique_ptr<uint64_t[]>, uint64_t>> txof_free;
  // the idle release (CORDAHIP_IDLE_RELEASE_MS): a thread that frees an idle
  // device's grow-only buffers (cordahip.cpp trim_device)
  std::thread reaper;
  std::mutex reaper_mu;
  std::condition_variable reaper_cv;
  bool reaper_stop = false;
};

namespace cordahip {
namespace rt {
// The ids of one device's transaction shard as its id slices leave them in HBM
// (signed-tx batches): txid[t - t0] is transaction t's id once the event of the
// slice holding t has completed; the signatures are verified in chunks whose
// message rows the device gathers from there (no host round trip for the ids).
struct DeviceIds {
  const uint8_t* txid = nullptr;           // device pointer, the shard's ids
  uint64_t t0 = 0;                         // the shard's first transaction
  std::vector<uint64_t> tx_bound;          // slice j = transactions [tx_bound[j], tx_bound[j + 1])
  std::vector<hipEvent_t> ready;           // ready[j]: slice j's ids are in txid (recorded on the id stream)
  std::vector<uint64_t> chunk_bound;       // the signature pipeline's chunk boundaries (signature indices)
  // Ed25519 chunks run the prep's key half before waiting for their ids (leaf
  // batches: +1.5% c4h interleaved; component batches, whose heavier id kernels
  // then meet more prep beside them: -1.8%, profiles/r05_prep_split_ab/)
  bool split_prep = false;
  // called before a chunk's copies are enqueued (after = false: the id slices
  // the chunk ending at sig_end needs) and after them (after = true: a few more)
  std::function<hipError_t(uint64_t sig_end, bool after)> advance;
  // called when the statuses of signatures [a, b) are final on the host (a
  // chunk has finished): the per-transaction reduce of the transactions whose
  // signatures all lie in [a, b) runs there, while later chunks verify
  std::function<hipError_t(uint64_t a, uint64_t b)> done;
  // called once every chunk is enqueued, before the pipeline drains: the signed-tx
  // call enqueues its remaining id slices and hands the enqueue token to the next call
  std::function<hipError_t()> enqueued;
  hipEvent_t wait_for(uint64_t tx) const {  // the event after which transaction tx's id is on the device
    const size_t j = (size_t)(std::upper_bound(tx_bound.begin(), tx_bound.end(), tx) - tx_bound.begin());
    return ready[j ? j - 1 : 0];
  }
};

// Where lane i's message is: the batch's CSR (msg + msg_off), or -- for the
// signatures of a transaction batch, each over its transaction's id
// (SignedTransaction.kt:98) -- the 32-byte id of transaction tx_of[i]: on the
// host at base (dev == nullptr) or on the device (dev).
struct MsgView {
  const uint8_t* base;
  const uint64_t* off;
  const uint64_t* tx_of;
  const DeviceIds* dev = nullptr;
  uint64_t chunk = 0;  // lanes per pipeline chunk (0: the default, CORDAHIP_HOST_CHUNK)
  const uint8_t* ptr(uint64_t i) const { return tx_of ? base + 32 * tx_of[i] : base + off[i]; }
  uint64_t len(uint64_t i) const { return tx_of ? 32 : off[i + 1] - off[i]; }
};
// generic CSR batches (host_batch.cpp); sig_verify_msgs takes the messages
// from mv instead of b->msg / b->msg_off
int sig_verify_impl(cordahip_ctx* ctx, const cordahip_sig_batch* b);
int sig_verify_msgs(cordahip_ctx* ctx, const cordahip_sig_batch* b, const MsgView& mv);
// lanes [lo, hi) of b on device d only, through the stages of the caller's set
// (the signed-tx path's per-device signatures)
int sig_verify_range(cordahip_ctx* ctx, Device& d, TxSet& set, const cordahip_sig_batch* b, const MsgView& mv,
                     uint64_t lo, uint64_t hi);
// dense Ed25519 rows in host memory through the packed pipeline (host_batch.cpp)
int ed25519_dense_host(cordahip_ctx* ctx, const uint8_t* keys, const uint8_t* sigs, const uint8_t* msgs,
                       uint32_t msg_len, uint64_t n, uint8_t* status, uint64_t* verdict);
void verdict_from_status(cordahip_ctx* ctx, const uint8_t* status, uint64_t n, uint64_t* verdict);
}  // namespace rt
}  // namespace cordahip
