// Native Kryo leaf encoder on the GPU: the same leaf
// preimages as cordahip_kryo_encode (kryo_core.hpp, one encoder for both
// sides), for batches whose component payloads are already in HBM -- a
// transaction batch's ids then need no host serialisation and no leaf bytes
// over PCIe (c4h with native leaves moves 1,717 B of leaves per cash-issue
// transaction; its components are ~600 B).
//
// Leaves are written from per-shape templates (kryo_template.hpp), not by
// running the byte-sequential encoder once per item:
//   1. kryo_shape: every item's shape hash (a streaming walk of the inputs the
//      encoder branches on) picks a slot of a 2^16-slot table; an empty slot is
//      claimed with one 64-bit CAS (hash | item) and the item becomes the
//      shape's representative. Items of shapes built by earlier calls are
//      compared with the slot's exact record (shape_matches; the hash only
//      picks the slot) and sized here.
//   2. kryo_build: one wave per NEW shape records the representative's shape
//      (structure words and span bytes, ShapeRec) in the slot and traces it
//      through the encoder (KoutT<true>, the OutputChunked level buffers in
//      LDS): a symbol per leaf byte -- a constant, payload byte k, or byte j of
//      the item's value; then 16 copies of the constant bytes shifted by 0..15,
//      a descriptor per 16-byte block and shift, and the SHA-256 midstate of the
//      leading all-constant blocks.
//   3. kryo_tsize: items of shapes claimed in this call, compared and sized
//      after kryo_build; items without a shape, with a hash collision, or whose
//      shape has no template go on a list for the direct encoder, which sizes
//      them (kryo_dsize, counting mode).
//   4. an exclusive scan of the sizes into the CSR offsets (hipcub).
//   5. kryo_twrite: a wave writes the output span of 16 consecutive leaves in
//      16-byte blocks, one per lane (1 KB per store instruction): the constant
//      copy for the block's alignment with the descriptor's payload window
//      merged in; the rare blocks (leaf boundaries, value bytes, RAW edges) go
//      to a per-wave LDS queue and are written byte by byte afterwards.
//   6. kryo_dwrite: the listed items through the direct encoder (per-thread
//      level buffers in a workspace); its byte stores share no byte with
//      kryo_twrite's.
//   7. kryo_hash (the component-level signed-tx slices, once every shape is
//      built): each leaf's SHA-256 straight from its template, no leaf bytes.
// The table, the records and the templates persist across calls on a device
// (a template is derived metadata of a shape, never a cached leaf: every call
// writes every leaf from its own items), so batches of recurring shapes build
// nothing; the host clears the table when it passes half full.
// r04 ran the direct encoder for every item: 80.5 KB of L2-fabric traffic per
// cash-issue transaction (the level buffers' round trips) against 1,717 B of
// leaves, 5.0 + 17.9 ms per 6.25 M leaves (profiles/r04_pmc_kryo_traffic.json).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "kryo_template.hpp"
#include "sha2_device.hpp"

namespace cordahip {

namespace {

using kryo::kChunk;

constexpr uint32_t kSlots = 1u << 16;      // shape table slots (a power of two)
constexpr uint32_t kMaxProbe = 64;         // linear probes before an item goes to the direct encoder
constexpr uint32_t kBuilders = 512;        // templates the arena holds (more shapes: direct encoder)
constexpr uint32_t kTmplSyms = 4096;       // leaf bytes a template covers (longer leaves: direct encoder)
// One template in the arena (byte offsets; kryo_build writes it, kryo_twrite reads it):
//   syms [kTmplSyms] u32   the traced symbols, one per leaf byte (the byte-by-byte path)
//   tb   [16][kTB] u8      copy c: leaf byte i at 16 + c + i if it is a constant, 0 where it
//                          is patched and in the pads -- for a leaf starting at output address
//                          a, copy (a & 15) lines its bytes up with the 16-byte output blocks
//   desc [16][kBlk] u64    per copy and 16-byte block: the patched bytes' mask (bits 0..15),
//                          the block's kind (bits 16..17: 0 constants only, 1 every patched
//                          byte t is payload byte delta + t, 2 anything else: byte by byte),
//                          delta (bits 32..63, signed)
//   mid  [16] u32          leaf hashing: [0] kc, the leading 64-byte blocks whose bytes are
//                          all constants, [1..8] the SHA-256 state after them (kryo_hash
//                          starts there: 6 of a cash-issue transaction's 30 blocks)
constexpr uint32_t kTB = kTmplSyms + 48;   // 16 pad + up to 15 shift + the leaf + 16 pad + 1 (a multiple of 16)
constexpr uint32_t kBlk = kTB / 16;        // blocks per copy
constexpr size_t kOffTb = (size_t)kTmplSyms * 4, kOffDesc = kOffTb + 16 * (size_t)kTB,
                 kOffMid = kOffDesc + 16 * (size_t)kBlk * 8,
                 kTmplBytes = (kOffMid + 64 + 255) / 256 * 256;
constexpr size_t kTmplWords = kTmplBytes / 4;
constexpr uint32_t kDescConst = 0, kDescLinear = 1, kDescBytes = 2;
constexpr uint32_t kNoSlot = 0xffffffffu;  // item_slot: no shape (direct encoder)
constexpr uint32_t kRawSlot = 0xfffffffeu; // item_slot: a RAW leaf (copied)
constexpr int32_t kNoTemplate = -2, kUnbuilt = -3;  // slot_size values besides a size (-1: an invalid shape)
constexpr uint32_t kDefer = 0x80000000u;  // item_slot: the slot was claimed this call (verified in kryo_tsize)
constexpr uint32_t kLeavesPerWave = 16;  // a wave writes the output span of this many leaves
constexpr uint32_t kBuildWaves = 16;     // kryo_build: waves (new shapes taken in turn)
constexpr uint32_t kDsizeBlocks = 64;    // kryo_dsize: blocks of 256 (direct items taken in turn)
constexpr uint32_t kLevelSyms = kryo::kLevelBytes;  // levels 1..7 (level 0 is the leaf itself)
// counters: [0] new shapes this call, [1] direct items this call, [2] templates
// in the arena, [3] table slots in use (the last two persist with the table),
// [4 + k] misses of the runtime's buffer set k: items that needed a new template
// or the direct encoder since the host last reset it (a templates-only chain did
// not write their leaves); one counter per set, as two calls' slices may both be
// on the device
enum { kCNew = 0, kCDirect = 1, kCArena = 2, kCUsed = 3, kCMiss = 4 };
constexpr uint8_t kKryoMiss = 4;  // item status of a miss (runtime.hpp)

// Items as the encoder sees them. base == nullptr: `data` are device pointers
// (cordahip_kryo_encode_device). Otherwise `data` are offsets into a payload of
// `limit` bytes at base (the component-level tx batches): rebased here, and an
// item whose payload would run past the end gets no data (the encoder then
// rejects it, as it rejects a missing payload).
struct ItemSrc {
  const cordahip_kryo_item* items;
  const uint8_t* base;
  uint64_t limit;
  __device__ cordahip_kryo_item operator[](uint64_t i) const {
    cordahip_kryo_item it = items[i];
    if (base) {
      const uint64_t off = (uint64_t)(uintptr_t)it.data;
      const uint64_t bytes = (it.kind == CORDAHIP_KRYO_STRING || it.kind == CORDAHIP_KRYO_KOTLIN_OBJECT) ? 2 * it.len
                                                                                                        : it.len;
      const bool fits = off <= limit && bytes <= limit - off && it.len < (1ull << 62);
      it.data = fits ? base + off : nullptr;
    }
    return it;
  }
};

// the encoder's kernels run at the id kernels' raised wave priority (tx.hip g_id_prio)
__device__ uint32_t g_kryo_prio = 1;
__device__ inline void kryo_priority() {
  if (g_kryo_prio) __builtin_amdgcn_s_setprio(3);
}

// Thread j's item when the batch is records of `group` items (a transaction's
// components): kind-major within tiles of 64 records, one tile per block of
// 64 x group threads, so each wave takes one kind (the shape walk does not
// diverge) while one CU reads the tile's items and payload. (r05's first
// mapping was kind-major over the whole batch: every record's lines were
// fetched once per kind, 5.1 KB of L2-fabric reads per cash-issue
// transaction; tiles of 256-thread blocks split a record's kinds over two
// XCDs' L2s; profiles/r05_pmc_kryo_*.) Threads past the last record: n.
__device__ inline uint64_t item_of(uint64_t j, uint64_t n, uint32_t group) {
  if (group <= 1 || n % group) return j;
  const uint64_t tile = j / (64ull * group), r = j % (64ull * group), rec = tile * 64 + r % 64;
  return rec < n / group ? rec * group + r / 64 : n;
}
inline bool grouped(uint64_t n, uint32_t group) { return group > 1 && group <= 16 && n % group == 0; }
// the shape pass's block size and threads for n items (whole tiles of 64 records)
inline uint32_t shape_block(uint64_t n, uint32_t group) { return grouped(n, group) ? 64 * group : 256; }
inline uint64_t item_threads(uint64_t n, uint32_t group) {
  if (!grouped(n, group)) return n;
  return (n / group + 63) / 64 * 64 * group;
}

// one atomic add per wave for the lanes (of those active) where pred holds
__device__ inline void wave_count(uint32_t* p, bool pred) {
  const uint64_t b = __ballot(pred);
  if (pred && (uint32_t)__lane_id() == (uint32_t)(__ffsll((unsigned long long)b) - 1)) atomicAdd(p, (uint32_t)__popcll(b));
}

// ---- 1. shapes ------------------------------------------------------------------
// An item whose slot holds a shape built by an earlier call is compared with
// the slot's record and sized here; one whose slot was claimed in this call
// (slot_size still kUnbuilt) is compared after kryo_build, in kryo_tsize.
__device__ inline void direct_item(uint32_t* direct, uint32_t* counters, uint64_t i) {
  direct[atomicAdd(&counters[kCDirect], 1u)] = (uint32_t)i;  // sized by kryo_dsize
}

// the size and status of an item of slot `slot` (built): false when it goes to the direct encoder
__device__ inline bool template_item(const cordahip_kryo_item& it, const kryo::ShapeRec& rec, int32_t z,
                                     uint64_t& size, uint8_t& st) {
  if (z == kNoTemplate || !kryo::shape_matches(it, rec)) return false;  // exact: a hash collision goes direct
  size = z >= 0 ? (uint64_t)z : 0;
  st = z >= 0 ? 0 : 1;  // an invalid shape: the encoder rejects every item of it
  return true;
}

// The slot of shape hash h: found (its tag), claimed (an empty slot, CAS), or
// kNoSlot (no room within kMaxProbe probes; templates_only: not in the table).
// The probes are agent-scope loads (another XCD may claim a slot during the
// kernel), which the L2 does not keep: one per wave per distinct hash, not one
// per item (r05: 5 x 128 B of fabric reads per cash-issue transaction).
__device__ inline uint32_t probe_slot(unsigned long long* table, uint64_t h, uint64_t i, bool templates_only,
                                      bool& claimed) {
  const uint32_t tag = (uint32_t)(h >> 32);
  const unsigned long long mine = ((unsigned long long)tag << 32) | (unsigned long long)(i + 1);
  uint32_t k = (uint32_t)h & (kSlots - 1);
  claimed = false;
  for (uint32_t probe = 0; probe < kMaxProbe; probe++, k = (k + 1) & (kSlots - 1)) {
    unsigned long long v = __hip_atomic_load(&table[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == 0 && templates_only) return kNoSlot;  // an unknown shape: a miss
    if (v == 0) {
      v = atomicCAS(&table[k], 0ull, mine);
      if (v == 0) {  // claimed: this item represents a new shape
        claimed = true;
        return k;
      }
    }
    if ((uint32_t)(v >> 32) == tag) return k;
  }
  return kNoSlot;
}

// templates_only: no slot is claimed and nothing goes to the direct encoder; an
// item without a built template of its shape is a miss (kKryoMiss, size 0,
// item_slot kNoSlot: kryo_twrite does not write it).
__global__ void __launch_bounds__(1024) kryo_shape_kernel(ItemSrc items, uint64_t n, uint32_t group, bool templates_only,
                                                          bool hash_chain,
                                                          unsigned long long* __restrict__ table,
                                                          const int32_t* __restrict__ slot_size,
                                                          const kryo::ShapeRec* __restrict__ rec,
                                                          uint32_t* __restrict__ item_slot, uint32_t* __restrict__ shape_list,
                                                          uint64_t* __restrict__ sizes, uint8_t* __restrict__ status,
                                                          uint32_t* __restrict__ direct, uint32_t* __restrict__ counters,
                                                          uint32_t* __restrict__ misses) {
  kryo_priority();
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j == 0) sizes[n] = 0;  // the scan's last element: off[n] = the total
  const uint64_t i = item_of(j, n, group);
  if (i >= n) return;
  const cordahip_kryo_item it = items[i];
  uint64_t size = 0;
  uint8_t st = 0;
  if (it.kind == CORDAHIP_KRYO_RAW) {
    item_slot[i] = kRawSlot;
    if (it.len && !it.data) {
      st = 1;
    } else if (hash_chain && it.len >> 29) {  // kryo_hash takes leaves under 2^29 bytes (32-bit bit counts
                                              // and block indices): larger RAW leaves take the full chain
      item_slot[i] = kNoSlot;
      if (templates_only) {
        st = kKryoMiss;
        atomicAdd(misses, 1u);
      } else {
        direct_item(direct, counters, i);  // the device hash chain: hashed by kryo_dhash
      }
    } else {
      size = it.len;
    }
    sizes[i] = size;
    status[i] = st;
    return;
  }
  // 1. The wave's first lane hashes its item and finds its slot. 2. When that slot
  // holds a built template, every lane compares its item with the slot's record
  // (copied to LDS): one walk per item in the common case, a wave of one kind of
  // the same shape (r05: a hash walk plus a compare walk per item). 3. Lanes that
  // do not match hash their own item and probe (new shapes, other kinds, collisions).
  __shared__ kryo::ShapeRec srec[16];
  const uint64_t act = __ballot(true);
  const int lead = __ffsll((unsigned long long)act) - 1;
  const bool is_lead = (int)__lane_id() == lead;
  uint32_t slot = kNoSlot;
  bool claimed = false;
  if (is_lead) {
    uint64_t h = 0;
    if (kryo::shape_hash_of(it, h)) slot = probe_slot(table, h, i, templates_only, claimed);
  }
  const uint32_t s0 = (uint32_t)__shfl((int)slot, lead);
  const bool c0 = __shfl((int)claimed, lead) != 0;
  const int32_t z0 = (s0 != kNoSlot && !c0) ? slot_size[s0] : kUnbuilt;
  const bool built0 = z0 != kUnbuilt && z0 != kNoTemplate;
  bool done = false;
  if (built0) {
    kryo::ShapeRec* mine = &srec[threadIdx.x >> 6];
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0));
    const uint32_t nact = (uint32_t)__popcll(act);
    constexpr uint32_t kQ = sizeof(kryo::ShapeRec) / 16;
    static_assert(sizeof(kryo::ShapeRec) % 16 == 0, "ShapeRec in uint4s");
    for (uint32_t q = rank; q < kQ; q += nact)
      reinterpret_cast<uint4*>(mine)[q] = reinterpret_cast<const uint4*>(rec + s0)[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (template_item(it, *mine, z0, size, st)) {
      slot = s0;
      done = true;
    } else if (is_lead) {
      slot = kNoSlot;  // the slot's record is another shape (a hash collision): direct
      done = true;
    }
  }
  if (!done && !is_lead) {
    uint64_t h = 0;
    if (kryo::shape_hash_of(it, h)) slot = probe_slot(table, h, i, templates_only, claimed);
  }
  if (claimed) {
    shape_list[atomicAdd(&counters[kCNew], 1u)] = slot;
    atomicAdd(&counters[kCUsed], 1u);
  }
  bool deferred = false;
  if (!done && slot != kNoSlot) {
    const int32_t z = claimed ? kUnbuilt : slot_size[slot];
    if (z == kUnbuilt && !templates_only) {  // built after this kernel: compared in kryo_tsize
      deferred = true;
    } else if (z == kUnbuilt || !template_item(it, rec[slot], z, size, st)) {
      slot = kNoSlot;
    }
  }
  // an item the encoder rejects before writing a byte (no payload, an unknown kind)
  // is decided here: neither a direct item nor a miss (one such item from untrusted
  // input would otherwise redo every templates-only call)
  const bool reject = slot == kNoSlot && kryo::rejected_outright(it);
  wave_count(misses, deferred || (slot == kNoSlot && !reject));
  if (deferred) {
    item_slot[i] = slot | kDefer;
    return;
  }
  item_slot[i] = slot;
  if (reject) {
    size = 0;
    st = 1;
  } else if (slot == kNoSlot) {
    if (templates_only) {
      size = 0;
      st = kKryoMiss;
    } else {
      direct_item(direct, counters, i);
    }
  }
  sizes[i] = size;
  status[i] = st;
}

// The templates-only shape pass for one lane, as kryo_shape_kernel decides it, in
// a form every lane of a wave calls (no early return: the fused shape + hash
// kernel synchronises its block afterwards). live: the lane holds item i. Out: the
// item's slot (kRawSlot / a built template's slot / kNoSlot), its leaf size and its
// status (0, 1 rejected, kKryoMiss); misses counted per wave.
__device__ inline void shape_templates_only(const ItemSrc& items, uint64_t i, bool live,
                                            unsigned long long* __restrict__ table,
                                            const int32_t* __restrict__ slot_size,
                                            const kryo::ShapeRec* __restrict__ rec, kryo::ShapeRec* srec_wave,
                                            uint32_t* misses, uint32_t& slot_o, uint32_t& len_o, uint8_t& st_o) {
  cordahip_kryo_item it{};
  if (live) it = items[i];
  uint64_t size = 0;
  uint8_t st = 0;
  uint32_t slot = kNoSlot;
  bool miss = false;
  const bool raw = live && it.kind == CORDAHIP_KRYO_RAW;
  if (raw) {
    slot = kRawSlot;
    if (it.len && !it.data) {
      st = 1;
    } else if (it.len >> 29) {  // kryo_hash's 32-bit bit counts: the full chain takes it
      slot = kNoSlot;
      st = kKryoMiss;
      miss = true;
    } else {
      size = it.len;
    }
  }
  const bool part = live && !raw;
  const uint64_t act = __ballot(part);
  if (act) {
    const int lead = __ffsll((unsigned long long)act) - 1;
    const bool is_lead = (int)__lane_id() == lead;
    bool claimed = false;
    if (is_lead) {
      uint64_t h = 0;
      if (kryo::shape_hash_of(it, h)) slot = probe_slot(table, h, i, true, claimed);
    }
    const uint32_t s0 = (uint32_t)__shfl((int)slot, lead);
    const int32_t z0 = s0 != kNoSlot ? slot_size[s0] : kUnbuilt;
    const bool built0 = z0 != kUnbuilt && z0 != kNoTemplate;
    bool done = false;
    if (built0) {
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0));
      const uint32_t nact = (uint32_t)__popcll(act);
      constexpr uint32_t kQ = sizeof(kryo::ShapeRec) / 16;
      if (part)
        for (uint32_t q = rank; q < kQ; q += nact)
          reinterpret_cast<uint4*>(srec_wave)[q] = reinterpret_cast<const uint4*>(rec + s0)[q];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (part && template_item(it, *srec_wave, z0, size, st)) {
        slot = s0;
        done = true;
      } else if (part && is_lead) {
        slot = kNoSlot;  // the slot's record is another shape (a hash collision)
        done = true;
      }
    }
    if (part && !done && !is_lead) {
      uint64_t h = 0;
      slot = kNoSlot;
      if (kryo::shape_hash_of(it, h)) slot = probe_slot(table, h, i, true, claimed);
    }
    if (part && !done && slot != kNoSlot) {
      const int32_t z = slot_size[slot];
      if (z == kUnbuilt || !template_item(it, rec[slot], z, size, st)) slot = kNoSlot;
    }
    if (part && slot == kNoSlot) {
      size = 0;
      if (kryo::rejected_outright(it)) {
        st = 1;
      } else {
        st = kKryoMiss;
        miss = true;
      }
    }
  }
  wave_count(misses, miss);
  slot_o = slot;
  len_o = (uint32_t)size;
  st_o = st;
}

// ---- 2. records and templates ----------------------------------------------------------
// One wave per new shape: lane 0 records the representative's shape and traces
// it (the level buffers in LDS) into the template's symbols; then the wave
// writes the 16 shifted copies of the constant bytes and every block's
// descriptor.
__global__ void __launch_bounds__(64) kryo_build_kernel(ItemSrc items, const unsigned long long* __restrict__ table,
                                                        const uint32_t* __restrict__ shape_list,
                                                        uint32_t* __restrict__ counters, kryo::ShapeRec* __restrict__ rec,
                                                        int32_t* __restrict__ slot_size, uint32_t* __restrict__ slot_map,
                                                        uint32_t* __restrict__ arena) {
  __shared__ uint32_t levels[kLevelSyms];
  __shared__ int32_t sh_size;
  __shared__ uint32_t sh_idx;
  const uint32_t nnew = counters[kCNew];
  for (uint32_t b = blockIdx.x; b < nnew; b += gridDim.x) {
    const uint32_t slot = shape_list[b];
    if (threadIdx.x == 0) {
      const cordahip_kryo_item it = items[(uint32_t)table[slot] - 1];
      kryo::ShapeRecord rv(rec[slot]);
      kryo::shape_walk(it, rv);
      int32_t size = kNoTemplate;
      uint32_t idx = kBuilders;
      if (rec[slot].ok) {
        idx = atomicAdd(&counters[kCArena], 1u);
        if (idx < kBuilders) size = (int32_t)kryo::trace_leaf(it, arena + idx * kTmplWords, kTmplSyms, levels);
      }
      slot_map[slot] = idx;
      slot_size[slot] = size;  // the size, or -1 (an invalid shape) / kNoTemplate
      sh_size = size;
      sh_idx = idx;
    }
    __syncthreads();
    if (sh_size > 0) {
      const uint32_t* syms = arena + sh_idx * kTmplWords;
      uint8_t* base = reinterpret_cast<uint8_t*>(arena + sh_idx * kTmplWords);
      const int32_t size = sh_size;
      // the 16 shifted copies of the constant bytes, a dword at a time
      for (uint32_t x = threadIdx.x; x < 16 * kTB / 4; x += blockDim.x) {
        const uint32_t c = x / (kTB / 4), o = (x % (kTB / 4)) * 4;
        uint32_t tw = 0;
        for (uint32_t q = 0; q < 4; q++) {
          const int32_t i = (int32_t)(o + q) - 16 - (int32_t)c;
          if (i >= 0 && i < size && (syms[i] & kryo::kSymTypeMask) == kryo::kSymConst)
            tw |= (syms[i] & 0xffu) << (8 * q);
        }
        reinterpret_cast<uint32_t*>(base + kOffTb)[x] = tw;
      }
      // the descriptors: block k of copy c covers leaf bytes 16 k + t - 16 - c
      for (uint32_t x = threadIdx.x; x < 16 * kBlk; x += blockDim.x) {
        const uint32_t c = x / kBlk, k = x % kBlk;
        uint32_t pm = 0, kind = kDescConst;
        int64_t delta = 0;
        for (uint32_t t = 0; t < 16; t++) {
          const int32_t i = (int32_t)(16 * k + t) - 16 - (int32_t)c;
          if (i < 0 || i >= size) continue;
          const uint32_t sym = syms[i];
          if ((sym & kryo::kSymTypeMask) == kryo::kSymConst) continue;
          const int64_t o = (int64_t)((sym >> 8) & (kryo::kMaxPayloadOff - 1)) - t;
          const bool lin = (sym & kryo::kSymTypeMask) == kryo::kSymPayload && !(sym & kryo::kSymOr80);
          if (!pm) {
            kind = lin ? kDescLinear : kDescBytes;
            delta = o;
          } else if (!lin || o != delta) {
            kind = kDescBytes;
          }
          pm |= 1u << t;
        }
        reinterpret_cast<uint64_t*>(base + kOffDesc)[x] =
            (uint64_t)pm | ((uint64_t)kind << 16) | ((uint64_t)(uint32_t)(int32_t)delta << 32);
      }
      if (threadIdx.x == 0) {  // the midstate of the leading all-constant message blocks
        uint32_t st[8], kc = 0;
        sha256_init(st);
        for (; 64 * (kc + 1) <= (uint32_t)size; kc++) {
          uint32_t w[16];
          bool cst = true;
          for (uint32_t q = 0; q < 16; q++) {
            uint32_t x = 0;
            for (uint32_t t = 0; t < 4; t++) {
              const uint32_t sym = syms[64 * kc + 4 * q + t];
              cst = cst && (sym & kryo::kSymTypeMask) == kryo::kSymConst;
              x = (x << 8) | (sym & 0xffu);
            }
            w[q] = x;
          }
          if (!cst) break;
          sha256_block(st, w);
        }
        uint32_t* mid = reinterpret_cast<uint32_t*>(base + kOffMid);
        mid[0] = kc;
        for (int q = 0; q < 8; q++) mid[1 + q] = st[q];
      }
    }
    __syncthreads();
  }
}

// ---- 3. sizes of the shapes built this call ------------------------------------------
__global__ void __launch_bounds__(256) kryo_tsize_kernel(ItemSrc items, uint64_t n,
                                                         uint32_t* __restrict__ item_slot,
                                                         const int32_t* __restrict__ slot_size,
                                                         const kryo::ShapeRec* __restrict__ rec,
                                                         uint64_t* __restrict__ sizes, uint8_t* __restrict__ status,
                                                         uint32_t* __restrict__ direct, uint32_t* __restrict__ counters) {
  kryo_priority();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t slot = item_slot[i];
  if (slot == kNoSlot || slot == kRawSlot || !(slot & kDefer)) return;  // resolved by kryo_shape
  slot &= ~kDefer;
  const cordahip_kryo_item it = items[i];
  uint64_t size = 0;
  uint8_t st = 0;
  if (!template_item(it, rec[slot], slot_size[slot], size, st)) {
    slot = kNoSlot;
    direct_item(direct, counters, i);
  }
  item_slot[i] = slot;
  sizes[i] = size;
  status[i] = st;
}

// the direct encoder's count pass over the listed items
__global__ void __launch_bounds__(256) kryo_dsize_kernel(ItemSrc items,
                                                         const uint32_t* __restrict__ direct,
                                                         const uint32_t* __restrict__ counters,
                                                         uint64_t* __restrict__ sizes, uint8_t* __restrict__ status) {
  const uint32_t nd = counters[kCDirect];
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nd; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t i = direct[j];
    kryo::Kout o(nullptr, 0, nullptr);  // counting mode
    const cordahip_kryo_item it = items[i];
    const bool ok = kryo::encode_leaf(o, it);
    sizes[i] = ok ? o.pos : 0;
    status[i] = ok ? 0 : 1;
  }
}

// ---- 5. template writes -------------------------------------------------------------
// A leaf's source: kind 0 template (its copy 0), 1 RAW, 2 direct (not written here).
struct LeafSrc {
  uint32_t kind;
  const uint32_t* syms;
  const uint8_t* data;
  int64_t value;
};

__device__ inline LeafSrc leaf_src(const ItemSrc& items, const uint32_t* item_slot, const uint32_t* slot_map,
                                   const uint32_t* arena, uint64_t L) {
  const cordahip_kryo_item it = items[L];
  const uint32_t slot = item_slot[L];
  LeafSrc s;
  s.data = it.data;
  s.value = it.value;
  s.syms = nullptr;
  if (slot == kRawSlot) {
    s.kind = 1;
  } else if (slot == kNoSlot) {
    s.kind = 2;
  } else {
    s.kind = 0;
    s.syms = arena + (size_t)slot_map[slot] * kTmplWords;
  }
  return s;
}

__device__ inline uint8_t src_byte(uint32_t kind, const uint32_t* syms, const uint8_t* data, int64_t value,
                                   uint64_t p) {
  return kind == 1 ? data[p] : kryo::sym_byte(syms[p], data, value);
}

// Byte q of the output when it lies in a leaf after `from` (the end of a dword
// whose first byte is in an earlier leaf): false when that leaf is not written
// here (direct encoder, or beyond cap).
__device__ inline bool spill_byte(const ItemSrc& items, uint64_t n, const uint64_t* off, const uint32_t* item_slot,
                                  const uint32_t* slot_map, const uint32_t* arena, uint64_t cap, uint64_t from,
                                  uint64_t q, uint8_t& byte) {
  uint64_t L = from;
  while (L < n && off[L + 1] <= q) L++;
  if (L >= n || off[L + 1] > cap) return false;
  const LeafSrc s = leaf_src(items, item_slot, slot_map, arena, L);
  if (s.kind == 2) return false;
  byte = src_byte(s.kind, s.syms, s.data, s.value, q - off[L]);
  return true;
}

// A wave writes the output span of kLeavesPerWave consecutive leaves as 16-byte
// output blocks, one per lane per pass (1 KB per store instruction). A block
// that lies inside one template leaf reads that leaf's constant bytes from the
// copy shifted to its alignment and the block's descriptor: constants only, or
// every patched byte t = payload byte delta + t (one 16-byte window of the
// item: at most two aligned 16-byte loads). Every other block -- a leaf
// boundary, value bytes, a RAW or direct leaf's edge, the buffer's ends -- goes
// on a per-wave queue in LDS and is written byte by byte afterwards, 16 lanes
// per block, so the rare paths do not diverge the common one. (r05's first
// writer walked symbols per byte: ~4,500 VALU instructions per wave of 16
// leaves, the TA busy for the whole kernel; profiles/r05_pmc_kryo_encoder.json.)
constexpr uint32_t kQueue = 256;

struct LeafMeta {
  uint32_t kind;  // 0 template, 1 RAW, 2 not written here (direct encoder, empty, beyond cap)
  uint32_t sh;    // (output address of the leaf) & 15: the template copy aligned to the blocks
  uint32_t a, b;  // the leaf's bytes, relative to the span's start
  const uint32_t* tmpl;  // the template (its syms; tb / desc at fixed offsets)
  const uint8_t* data;
  int64_t value;
};

// the leaf holding span byte x (0 <= x < bound[nl], nl <= 16): the last leaf starting at or
// before it (empty leaves start where the next one does; the search passes over them)
__device__ inline uint32_t leaf_at(const uint32_t* bound, uint32_t nl, uint32_t x) {
  uint32_t lo = 0;
#pragma unroll
  for (uint32_t step = 8; step; step >>= 1) {
    const uint32_t c = lo + step;
    if (c < nl && bound[c] <= x) lo = c;
  }
  return lo;
}

__device__ inline uint32_t byte_mask32(uint32_t m4) {  // 4 mask bits -> 4 byte masks
  return ((m4 * 0x00204081u) & 0x01010101u) * 0xffu;
}

// bytes q[t0 .. t1] (t0 <= t1 < 16) as a 16-byte window w[t] = q[t]: at most two aligned
// 16-byte loads, each holding one of the wanted bytes (so both are mapped)
__device__ inline void load_window(const uint8_t* q, uint32_t t0, uint32_t t1, uint32_t* w) {
  const uintptr_t qa = (uintptr_t)q, ca = qa & ~(uintptr_t)15;
  const uint32_t s = (uint32_t)(qa - ca);
  uint4 u0 = make_uint4(0, 0, 0, 0), u1 = make_uint4(0, 0, 0, 0);
  if (s + t0 < 16) u0 = *reinterpret_cast<const uint4*>(ca);
  if (s + t1 >= 16) u1 = *reinterpret_cast<const uint4*>(ca + 16);
  const uint32_t d[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
  const uint32_t dw = s >> 2, sb = s & 3;
  uint32_t e[5];
#pragma unroll
  for (int i = 0; i < 5; i++)
    e[i] = dw == 0 ? d[i] : dw == 1 ? d[i + 1] : dw == 2 ? d[i + 2] : (i + 3 < 8 ? d[i + 3] : 0);
#pragma unroll
  for (int i = 0; i < 4; i++) w[i] = __builtin_amdgcn_alignbyte(e[i + 1], e[i], sb);
}

__global__ void __launch_bounds__(256) kryo_twrite_kernel(ItemSrc items, uint64_t n,
                                                          const uint64_t* __restrict__ off,
                                                          const uint32_t* __restrict__ item_slot,
                                                          const uint32_t* __restrict__ slot_map,
                                                          const uint32_t* __restrict__ arena, uint8_t* __restrict__ out,
                                                          uint64_t cap, uint8_t* __restrict__ status) {
  kryo_priority();
  __shared__ LeafMeta meta_s[4][kLeavesPerWave];
  __shared__ uint32_t bound_s[4][kLeavesPerWave + 1];
  __shared__ uint32_t queue_s[4][kQueue];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  LeafMeta* meta = meta_s[wv];
  uint32_t* bound = bound_s[wv];
  uint32_t* queue = queue_s[wv];
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + wv;
  const uint64_t L0 = wave * kLeavesPerWave;
  if (L0 >= n) return;
  const uint32_t nl = (uint32_t)(L0 + kLeavesPerWave < n ? kLeavesPerWave : n - L0);
  const uint64_t base = (uint64_t)(uintptr_t)out;
  const uint64_t P0 = off[L0], P1 = off[L0 + nl];  // the span (< 2^32 bytes: kLeavesPerWave leaves)
  if (lane <= nl) bound[lane] = (uint32_t)(off[L0 + lane] - P0);
  if (lane < nl) {
    const uint64_t a = off[L0 + lane], b = off[L0 + lane + 1];
    const LeafSrc s = leaf_src(items, item_slot, slot_map, arena, L0 + lane);
    LeafMeta m;
    m.kind = (b == a || b > cap) ? 2 : s.kind;
    m.sh = (uint32_t)((base + a) & 15);
    m.a = (uint32_t)(a - P0);
    m.b = (uint32_t)(b - P0);
    m.tmpl = s.syms;
    m.data = s.data;
    m.value = s.value;
    meta[lane] = m;
    if (b > cap && b > a && s.kind != 2) status[L0 + lane] = 2;  // not written (nor the leaves after it)
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the wave's LDS stores before its loads
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (P1 == P0) return;
  // the 16-byte blocks whose first output byte is in the span (the span at
  // output position 0 also takes the block that starts before the buffer)
  const uint64_t lo = P0 == 0 ? (base & ~15ull) : ((base + P0 + 15) & ~15ull);
  const uint64_t hi = (base + P1 + 15) & ~15ull;
  const uint32_t nblk = (uint32_t)((hi - lo) / 16);
  const int64_t span = (int64_t)(P1 - P0);

  // the queued blocks, byte by byte: 16 lanes per block
  auto flush = [&](uint32_t nq) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (uint32_t j = lane; j < nq * 16; j += 64) {
      const uint64_t A = lo + 16ull * queue[j >> 4];
      const uint32_t t = j & 15;
      if (A + t < base) continue;  // before the buffer
      const int64_t xt = (int64_t)(A + t - base) - (int64_t)P0;
      uint8_t byte = 0;
      if (xt >= span) {  // past the span: the next wave's leaves
        if (!spill_byte(items, n, off, item_slot, slot_map, arena, cap, L0 + nl, A + t - base, byte)) continue;
      } else {
        const LeafMeta& m = meta[leaf_at(bound, nl, (uint32_t)xt)];
        if (m.kind == 2) continue;
        const uint32_t p = (uint32_t)xt - m.a;
        byte = m.kind == 1 ? m.data[p] : kryo::sym_byte(m.tmpl[p], m.data, m.value);
      }
      reinterpret_cast<uint8_t*>(A)[t] = byte;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the queue is refilled after this
    __builtin_amdgcn_wave_barrier();
  };

  uint32_t nq = 0;  // wave-uniform
  for (uint32_t b0 = 0; b0 < nblk; b0 += 64) {
    if (nq + 64 > kQueue) {
      flush(nq);
      nq = 0;
    }
    const uint32_t bi = b0 + lane;
    bool fast = false;
    if (bi < nblk) {
      const uint64_t A = lo + 16ull * bi;
      const int64_t x = (int64_t)(A - base) - (int64_t)P0;  // span position of the block's byte 0
      const LeafMeta& m = meta[leaf_at(bound, nl, x < 0 ? 0u : (uint32_t)x)];
      if (A >= base && x >= (int64_t)m.a && x + 16 <= (int64_t)m.b && m.kind != 2) {
        const int64_t pb = x - (int64_t)m.a;  // leaf position of the block's byte 0
        uint32_t v[4];
        if (m.kind == 1) {  // RAW: the item's bytes
          load_window(m.data + pb, 0, 15, v);
          fast = true;
        } else {
          const uint8_t* tp = reinterpret_cast<const uint8_t*>(m.tmpl);
          const uint32_t idx = (uint32_t)(16 + (int64_t)m.sh + pb);  // a multiple of 16
          // the descriptor and the constant copy load together (the copy's address needs
          // no descriptor); the payload window follows the descriptor
          const uint64_t desc = reinterpret_cast<const uint64_t*>(tp + kOffDesc)[m.sh * kBlk + idx / 16];
          const uint4 tv = *reinterpret_cast<const uint4*>(tp + kOffTb + (size_t)m.sh * kTB + idx);
          const uint32_t pm = (uint32_t)desc & 0xffff, kind = (uint32_t)(desc >> 16) & 3;
          if (kind != kDescBytes) {
            v[0] = tv.x, v[1] = tv.y, v[2] = tv.z, v[3] = tv.w;
            if (pm) {
              uint32_t w[4];
              load_window(m.data + (int32_t)(desc >> 32), __builtin_ctz(pm), 31 - __builtin_clz(pm), w);
#pragma unroll
              for (int i = 0; i < 4; i++) {
                const uint32_t mk = byte_mask32((pm >> (4 * i)) & 15);
                v[i] = (v[i] & ~mk) | (w[i] & mk);
              }
            }
            fast = true;
          }
        }
        if (fast) *reinterpret_cast<uint4*>(A) = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
    // the others to the queue (in block order; positions by ballot prefix)
    const bool need = bi < nblk && !fast;
    const uint64_t ball = __ballot(need);
    if (need) queue[nq + __builtin_amdgcn_mbcnt_hi((uint32_t)(ball >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ball, 0))] = bi;
    nq += (uint32_t)__popcll(ball);
  }
  flush(nq);
}

// ---- 6. direct writes ---------------------------------------------------------------
__global__ void __launch_bounds__(256) kryo_dwrite_kernel(ItemSrc items, const uint32_t* __restrict__ direct,
                                                          const uint32_t* __restrict__ counters,
                                                          const uint64_t* __restrict__ off, uint8_t* __restrict__ out,
                                                          uint64_t cap, uint8_t* __restrict__ status,
                                                          uint8_t* __restrict__ ws) {
  const uint32_t nd = counters[kCDirect];
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t* levels = ws + t * (uint64_t)kLevelSyms;  // levels 1..7 of this thread's OutputChunked buffers
  for (uint64_t j = t; j < nd; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t i = direct[j];
    if (status[i] != 0) continue;
    const uint64_t a = off[i], b = off[i + 1];
    if (b > cap) {  // beyond the caller's buffer: not written
      status[i] = 2;
      continue;
    }
    kryo::Kout o(out + a, b - a, levels);
    const cordahip_kryo_item it = items[i];
    if (!kryo::encode_leaf(o, it) || o.pos != b - a) status[i] = 3;  // cannot happen: same encoder
  }
}

// ---- 6b. direct hashes --------------------------------------------------------------
// The device hash chain (cordahip_signed_txcomp_verify_ed25519_device) needs the
// direct items' leaves only as SHA-256 input: the direct encoder runs with a
// level-0 sink that compresses the bytes as they come (no leaf buffer, no size
// pass, no scan). A byte at a time through a per-thread block: slow per byte,
// but the direct list is empty in steady state (new shapes get templates).
struct ShaSink {
  static constexpr bool kActive = true;
  uint32_t st[8];
  uint32_t w[16];
  uint32_t n = 0;  // bytes in the current block; a full block is compressed when the next byte arrives
  __device__ ShaSink() {
    sha256_init(st);
    for (int k = 0; k < 16; k++) w[k] = 0;
  }
  __device__ void compress() {
    uint32_t t[16];
    for (int k = 0; k < 16; k++) t[k] = w[k], w[k] = 0;
    sha256_block(st, t);
    n = 0;
  }
  __device__ void put(uint8_t b) {
    if (n == 64) compress();
    w[n >> 2] |= (uint32_t)b << (24 - 8 * (n & 3));
    n++;
  }
  // n bytes: whole blocks straight from p while more than a block remains behind
  // them (the last byte stays buffered for mark()), the rest through the block
  __device__ void write(const uint8_t* p, uint64_t len) {
    while (len) {
      if (n == 64) compress();
      if (n == 0 && len > 64) {
        uint32_t t[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
          t[k] = ((uint32_t)p[4 * k] << 24) | ((uint32_t)p[4 * k + 1] << 16) | ((uint32_t)p[4 * k + 2] << 8) | p[4 * k + 3];
        sha256_block(st, t);
        p += 64;
        len -= 64;
        continue;
      }
      const uint64_t take = len < 64 - n ? len : 64 - n;
      for (uint64_t i = 0; i < take; i++, n++) w[n >> 2] |= (uint32_t)p[i] << (24 - 8 * (n & 3));
      p += take;
      len -= take;
    }
  }
  __device__ void mark() { w[(n - 1) >> 2] |= 0x80u << (24 - 8 * ((n - 1) & 3)); }
  __device__ void finish(uint64_t total) {  // FIPS 180-4 padding after `total` bytes
    if (n == 64) compress();
    w[n >> 2] |= 0x80u << (24 - 8 * (n & 3));
    if (n >= 56) {
      n = 64;
      compress();
    }
    w[14] = (uint32_t)(total >> 29);
    w[15] = (uint32_t)(total << 3);
    compress();
  }
};

__global__ void __launch_bounds__(256) kryo_dhash_kernel(ItemSrc items, const uint32_t* __restrict__ direct,
                                                         const uint32_t* __restrict__ counters,
                                                         uint8_t* __restrict__ status, uint32_t* __restrict__ hashes,
                                                         uint8_t* __restrict__ ws) {
  const uint32_t nd = counters[kCDirect];
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t* levels = ws + t * (uint64_t)kLevelSyms;  // levels 1..7 of this thread's OutputChunked buffers
  for (uint64_t j = t; j < nd; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t i = direct[j];
    ShaSink sink;
    kryo::KoutT<false, ShaSink> o(nullptr, 0, levels);
    o.sink = &sink;
    const cordahip_kryo_item it = items[i];
    const bool ok = kryo::encode_leaf(o, it);
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (ok) {
      sink.finish(o.pos);
      for (int k = 0; k < 8; k++) h[k] = sink.st[k];
    }
    status[i] = ok ? 0 : 1;
    uint4* out = reinterpret_cast<uint4*>(hashes + (uint64_t)i * 8);
    out[0] = make_uint4(h[0], h[1], h[2], h[3]);
    out[1] = make_uint4(h[4], h[5], h[6], h[7]);
  }
}

// ---- 7. leaf hashes straight from the templates (the templates-only chain) ---------
// The component-level signed-tx slices need the leaves only as SHA-256 input:
// one lane per leaf assembles each 64-byte message block from its template in
// registers (the same 16-byte pieces kryo_twrite stores: the constant copy for
// the leaf's own alignment with the descriptor's payload window merged in;
// pieces of other kinds byte by byte from the symbols) and compresses it, so
// no leaf is written, scanned or read back (shape -> scan -> twrite ->
// sha256_leaves was 4 launches and 2 x 2.15 GB of leaf traffic per C4 call).
// Interleaved on one corpus: c4h --components 77.0 against 74.6 M sig/s with the
// writes (profiles/r05_fused_hash_ab.json); without the descriptors loaded a
// block ahead the fused kernel lost (73.3: a descriptor round trip before each
// block's payload loads).
// Threads take items as kryo_shape does (a wave = one kind of 64 transactions:
// equal lengths); a RAW leaf is its item's bytes; an item without a template
// (a miss, status != 0) gets a zero hash -- its call is redone or its
// transaction rejected.
struct HashSrc {
  uint32_t kind;  // 0 template, 1 RAW, 2 none
  const uint8_t* tmpl;
  const uint8_t* data;
  int64_t value;
  uint32_t len;
};

// bytes [16 p, 16 p + 16) of the leaf (len > 16 p), zero past its end, as 4 little-endian
// words; desc: the piece's descriptor (template leaves; loaded a block ahead by the caller)
__device__ inline uint64_t piece_desc(const HashSrc& h, uint32_t p) {
  return h.kind == 0 && 16 * p < h.len ? reinterpret_cast<const uint64_t*>(h.tmpl + kOffDesc)[p + 1] : 0;  // copy 0
}
__device__ inline void leaf_piece(const HashSrc& h, uint32_t p, uint64_t desc, uint32_t* v) {
  const uint32_t lo = 16 * p, last = min(15u, h.len - 1 - lo);
  if (h.kind == 1) {
    load_window(h.data + lo, 0, last, v);
  } else {
    const uint32_t pm = (uint32_t)desc & 0xffff, kind = (uint32_t)(desc >> 16) & 3;
    if (kind != kDescBytes) {
      const uint4 tv = *reinterpret_cast<const uint4*>(h.tmpl + kOffTb + 16 + lo);
      v[0] = tv.x, v[1] = tv.y, v[2] = tv.z, v[3] = tv.w;
      if (pm) {
        uint32_t w[4];
        load_window(h.data + (int32_t)(desc >> 32), __builtin_ctz(pm), 31 - __builtin_clz(pm), w);
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint32_t mk = byte_mask32((pm >> (4 * i)) & 15);
          v[i] = (v[i] & ~mk) | (w[i] & mk);
        }
      }
      return;  // the copy and the descriptor are zero past the leaf
    }
    // byte by byte from the symbols: the piece's 16 symbols in four 16-byte loads (the
    // same address in every lane of the wave), then every payload byte's load issued
    // before any is used (r05 walked them one dependent load pair at a time)
    const uint4* sp = reinterpret_cast<const uint4*>(h.tmpl + 4 * (size_t)lo);
    const uint4 q0 = sp[0], q1 = sp[1], q2 = sp[2], q3 = sp[3];
    const uint32_t sy[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                             q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
    uint32_t pb[16];
#pragma unroll
    for (uint32_t t = 0; t < 16; t++)
      pb[t] = (t <= last && (sy[t] & kryo::kSymTypeMask) == kryo::kSymPayload)
                  ? h.data[(sy[t] >> 8) & (kryo::kMaxPayloadOff - 1)] : 0u;
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = 0;
#pragma unroll
    for (uint32_t t = 0; t < 16; t++) {
      const uint32_t x = sy[t], ty = x & kryo::kSymTypeMask;
      uint32_t b = ty == kryo::kSymPayload ? (pb[t] | ((x & kryo::kSymOr80) ? 0x80u : 0u))
                   : ty == kryo::kSymConst ? (x & 0xffu) : (uint32_t)kryo::sym_byte(x, nullptr, h.value);
      v[t >> 2] |= (t <= last ? b : 0u) << (8 * (t & 3));
    }
    return;
  }
  if (last < 15) {  // RAW: the window holds only the leaf's bytes
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int keep = (int)last + 1 - 4 * i;  // bytes of word i inside the leaf
      v[i] = keep >= 4 ? v[i] : keep <= 0 ? 0u : v[i] & ((1u << (8 * keep)) - 1);
    }
  }
}

// The wave-uniform form of leaf_piece: every lane of the wave hashes a leaf of the
// same template, so the template's constant copies, descriptors and symbols are read
// through the scalar cache at one address per wave (constant address space: scalar
// loads into SGPRs), only the payload windows are per-lane vector loads, and the
// piece's control flow branches on scalars instead of exec masks.
typedef const __attribute__((address_space(4))) uint8_t* TmplPtr;
__device__ inline void leaf_piece_uniform(TmplPtr T, uint32_t len, const uint8_t* data, int64_t value, uint32_t p,
                                          uint32_t* v) {
  const uint32_t lo = 16 * p, last = min(15u, len - 1 - lo);
  const uint64_t desc = reinterpret_cast<const __attribute__((address_space(4))) uint64_t*>(T + kOffDesc)[p + 1];
  const uint32_t pm = (uint32_t)desc & 0xffff, kind = (uint32_t)(desc >> 16) & 3;
  if (kind != kDescBytes) {
    const __attribute__((address_space(4))) uint32_t* tv =
        reinterpret_cast<const __attribute__((address_space(4))) uint32_t*>(T + kOffTb + 16 + lo);
    v[0] = tv[0], v[1] = tv[1], v[2] = tv[2], v[3] = tv[3];
    if (pm) {
      uint32_t w[4];
      load_window(data + (int32_t)(desc >> 32), __builtin_ctz(pm), 31 - __builtin_clz(pm), w);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t mk = byte_mask32((pm >> (4 * i)) & 15);
        v[i] = (v[i] & ~mk) | (w[i] & mk);
      }
    }
    return;
  }
  const __attribute__((address_space(4))) uint32_t* sp =
      reinterpret_cast<const __attribute__((address_space(4))) uint32_t*>(T + 4 * (size_t)lo);
  uint32_t sy[16];
#pragma unroll
  for (int t = 0; t < 16; t++) sy[t] = sp[t];
  uint32_t pb[16];
#pragma unroll
  for (uint32_t t = 0; t < 16; t++)
    pb[t] = (t <= last && (sy[t] & kryo::kSymTypeMask) == kryo::kSymPayload)
                ? data[(sy[t] >> 8) & (kryo::kMaxPayloadOff - 1)] : 0u;
#pragma unroll
  for (int i = 0; i < 4; i++) v[i] = 0;
#pragma unroll
  for (uint32_t t = 0; t < 16; t++) {
    const uint32_t x = sy[t], ty = x & kryo::kSymTypeMask;
    uint32_t b = ty == kryo::kSymPayload ? (pb[t] | ((x & kryo::kSymOr80) ? 0x80u : 0u))
                 : ty == kryo::kSymConst ? (x & 0xffu) : (uint32_t)kryo::sym_byte(x, nullptr, value);
    v[t >> 2] |= (t <= last ? b : 0u) << (8 * (t & 3));
  }
}

// kryo_hash's blocks: 256 items of ONE kind (records of `group` items: 256
// consecutive records' component `kind`), the `group` blocks of a tile of 256
// records on one XCD (blocks go round-robin over the 8 XCDs, so block b's tile is
// chosen among those of XCD b % 8: the records' items and payload lines are read
// into one L2). Ungrouped batches: 256 consecutive items per block. Returns n past
// the last item.
__device__ inline uint64_t hash_item_of(uint32_t b, uint32_t t, uint64_t n, uint32_t group) {
  if (group <= 1 || group > 16 || n % group) return (uint64_t)b * 256 + t < n ? (uint64_t)b * 256 + t : n;
  const uint32_t q = b / 8, kind = q % group;
  const uint64_t tile = (uint64_t)(q / group) * 8 + b % 8, rec = tile * 256 + t;
  return rec < n / group ? rec * group + kind : n;
}
inline uint32_t hash_blocks(uint64_t n, uint32_t group) {
  if (!grouped(n, group)) return (uint32_t)((n + 255) / 256);
  const uint64_t tiles = (n / group + 255) / 256;
  return (uint32_t)((tiles + 7) / 8 * 8 * group);
}

// kFused (the host calls' templates-only chain): the block first runs the shape
// pass for its own items (shape_templates_only), keeps slot, size and status in
// LDS and stores only the status (merkle_root's BAD_COMPONENT input), so one launch
// per id slice replaces kryo_shape + kryo_hash.
struct FusedShape {
  unsigned long long* table;
  const int32_t* slot_size;
  const kryo::ShapeRec* rec;
  uint32_t* misses;
  uint8_t* status_out;
};

template <int kMinWaves, bool kFused = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kMinWaves, 8)))
kryo_hash_kernel(ItemSrc items, uint64_t n, uint32_t group,
                                                         const uint32_t* __restrict__ item_slot,
                                                         const uint32_t* __restrict__ slot_map,
                                                         const uint32_t* __restrict__ arena,
                                                         const uint64_t* __restrict__ sizes,
                                                         const uint8_t* __restrict__ status,
                                                         uint32_t* __restrict__ hashes /* [n][8] BE words */,
                                                         FusedShape fs = {}) {
  kryo_priority();
  // The block's items grouped by template before any lane hashes: a wave whose
  // lanes hold leaves of one template assembles its blocks on the scalar path, one
  // of several templates (a cash state's quantity and nonce varints give 2-3 shapes
  // per 64 transactions, each shifting every later byte) diverges at every piece.
  // Up to kGroups rounds each collect the lanes of the smallest remaining key
  // (the slot; status != 0 and past-the-end lanes last), in lane order; the rest
  // keep theirs.
  constexpr int kGroups = 8;
  __shared__ uint8_t order[256];
  __shared__ uint32_t s_min, s_cnt[4];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t i0 = hash_item_of(blockIdx.x, tid, n, group);
  __shared__ uint32_t f_slot[kFused ? 256 : 1], f_len[kFused ? 256 : 1];
  __shared__ uint8_t f_st[kFused ? 256 : 1];
  __shared__ kryo::ShapeRec f_rec[kFused ? 4 : 1];
  uint32_t key;
  if constexpr (kFused) {
    uint32_t sl, ln;
    uint8_t st0;
    shape_templates_only(items, i0, i0 < n, fs.table, fs.slot_size, fs.rec, &f_rec[wv], fs.misses, sl, ln, st0);
    f_slot[tid] = sl;
    f_len[tid] = ln;
    f_st[tid] = st0;
    if (i0 < n) fs.status_out[i0] = st0;
    key = i0 >= n ? 0xffffffffu : st0 != 0 ? 0xfffffffeu : sl;
  } else {
    key = i0 >= n ? 0xffffffffu : status[i0] != 0 ? 0xfffffffeu : item_slot[i0];
  }
  bool placed = i0 >= n;
  uint32_t base = 0;
  for (int r = 0; r <= kGroups; r++) {
    if (tid == 0) s_min = 0xffffffffu;
    __syncthreads();
    if (!placed && r < kGroups) atomicMin(&s_min, key);
    __syncthreads();
    const uint32_t cur = s_min;
    const bool pred = !placed && (r == kGroups || key == cur);
    const uint64_t bal = __ballot(pred);
    if (lane == 0) s_cnt[wv] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t off = base, tot = 0;
    for (uint32_t w = 0; w < 4; w++) {
      off += w < wv ? s_cnt[w] : 0u;
      tot += s_cnt[w];
    }
    if (pred) {
      order[off + (uint32_t)__popcll(bal & ((1ull << lane) - 1))] = (uint8_t)tid;
      placed = true;
    }
    base += tot;
    __syncthreads();
    if (r < kGroups && cur == 0xffffffffu) break;  // every lane with an item placed
  }
  if (tid >= base) return;
  const uint32_t src = order[tid];
  const uint64_t i = hash_item_of(blockIdx.x, src, n, group);
  HashSrc h;
  h.kind = 2;
  const uint8_t sti = kFused ? f_st[src] : status[i];
  if (sti == 0) {
    const cordahip_kryo_item it = items[i];
    const uint32_t slot = kFused ? f_slot[src] : item_slot[i];
    h.data = it.data;
    h.value = it.value;
    h.len = kFused ? f_len[src] : (uint32_t)sizes[i];
    if (slot == kRawSlot) {
      h.kind = 1;
    } else if (slot != kNoSlot && !(slot & kDefer)) {
      h.kind = 0;
      h.tmpl = reinterpret_cast<const uint8_t*>(arena + (size_t)slot_map[slot] * kTmplWords);
    }
  }
  uint32_t st[8];
  const uint64_t tp = h.kind == 0 ? (uint64_t)(uintptr_t)h.tmpl : 0;
  const uint64_t tp0 = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(tp >> 32)) << 32) |
                       __builtin_amdgcn_readfirstlane((uint32_t)tp);
  if (__all(tp != 0 && tp == tp0)) {  // one template in the whole wave: the scalar path
    TmplPtr T = (TmplPtr)(uintptr_t)tp0;
    const uint32_t len = __builtin_amdgcn_readfirstlane(h.len);  // one shape: one size
    const __attribute__((address_space(4))) uint32_t* mid =
        reinterpret_cast<const __attribute__((address_space(4))) uint32_t*>(T + kOffMid);
    const uint32_t b0 = mid[0];
    sha256_init(st);
    if (b0) {
#pragma unroll
      for (int k = 0; k < 8; k++) st[k] = mid[1 + k];
    }
    const uint32_t nb = (len + 9 + 63) / 64;
    for (uint32_t b = b0; b < nb; b++) {
      uint32_t w[16];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t p = 4 * b + q;
        uint32_t v[4] = {0, 0, 0, 0};
        if (16 * p < len) leaf_piece_uniform(T, len, h.data, h.value, p, v);
        if (len >= 16 * p && len < 16 * p + 16) {  // the padding's first byte
          const uint32_t t = len - 16 * p;
          v[t >> 2] |= 0x80u << (8 * (t & 3));
        }
#pragma unroll
        for (int k = 0; k < 4; k++) w[4 * q + k] = bswap32(v[k]);
      }
      if (b == nb - 1) {
        w[14] = len >> 29;
        w[15] = len << 3;
      }
      sha256_block(st, w);
    }
  } else if (h.kind == 2) {
#pragma unroll
    for (int k = 0; k < 8; k++) st[k] = 0;
  } else {
    sha256_init(st);
    uint32_t b0 = 0;
    if (h.kind == 0) {  // start after the template's all-constant blocks
      const uint32_t* mid = reinterpret_cast<const uint32_t*>(h.tmpl + kOffMid);
      b0 = mid[0];
      if (b0) {
#pragma unroll
        for (int k = 0; k < 8; k++) st[k] = mid[1 + k];
      }
    }
    const uint32_t nb = (h.len + 9 + 63) / 64;
    // the descriptors one block ahead: a block's payload loads then issue with its
    // constant-copy loads instead of after a descriptor round trip
    uint64_t dn[4];
#pragma unroll
    for (int q = 0; q < 4; q++) dn[q] = piece_desc(h, 4 * b0 + q);
    for (uint32_t b = b0; b < nb; b++) {
      uint32_t w[16];
      uint64_t dc[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        dc[q] = dn[q];
        dn[q] = piece_desc(h, 4 * (b + 1) + q);
      }
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t p = 4 * b + q;
        uint32_t v[4] = {0, 0, 0, 0};
        if (16 * p < h.len) leaf_piece(h, p, dc[q], v);
        if (h.len >= 16 * p && h.len < 16 * p + 16) {  // the padding's first byte
          const uint32_t t = h.len - 16 * p;
          v[t >> 2] |= 0x80u << (8 * (t & 3));
        }
#pragma unroll
        for (int k = 0; k < 4; k++) w[4 * q + k] = bswap32(v[k]);
      }
      if (b == nb - 1) {
        w[14] = h.len >> 29;  // the 64-bit bit length (0 below the 2^29-byte guard in kryo_shape)
        w[15] = h.len << 3;
      }
      sha256_block(st, w);
    }
  }
  uint4* o = reinterpret_cast<uint4*>(hashes + i * 8);
  o[0] = make_uint4(st[0], st[1], st[2], st[3]);
  o[1] = make_uint4(st[4], st[5], st[6], st[7]);
}

}  // namespace

// The encoder's persistent per-device state (cordahip.cpp allocates
// kryo_fixed_scratch_bytes() once, zeroed; kryo_clear() empties it).
struct KryoState {
  unsigned long long* table;  // [kSlots] tag | representative + 1
  kryo::ShapeRec* rec;        // [kSlots]
  int32_t* slot_size;         // [kSlots]
  uint32_t* slot_map;         // [kSlots] the slot's template in the arena
  uint32_t* shape_list;       // [kSlots] slots claimed this call
  uint32_t* counters;         // [16] kCNew, kCDirect, kCArena, kCUsed
  uint32_t* arena;            // [kBuilders * kTmplWords]
  explicit KryoState(uint8_t* p) {
    table = reinterpret_cast<unsigned long long*>(p);
    rec = reinterpret_cast<kryo::ShapeRec*>(table + kSlots);
    slot_size = reinterpret_cast<int32_t*>(rec + kSlots);
    slot_map = reinterpret_cast<uint32_t*>(slot_size + kSlots);
    shape_list = slot_map + kSlots;
    counters = shape_list + kSlots;
    arena = counters + 16;
  }
};

size_t kryo_fixed_scratch_bytes() {
  return (size_t)kSlots * (8 + sizeof(kryo::ShapeRec) + 4 + 4 + 4) + 64 + (size_t)kBuilders * kTmplBytes;
}
size_t kryo_direct_ws_bytes(uint64_t writers) { return (size_t)writers * kLevelSyms; }
// the table, records and templates emptied (the arena need not be)
hipError_t kryo_clear(uint8_t* fixed, hipStream_t s) {
  const KryoState k(fixed);
  hipError_t e = hipMemsetAsync(k.table, 0, (size_t)kSlots * 8, s);
  static_assert(kUnbuilt == -3, "kUnbuilt as a byte pattern");
  e = e ? e : hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(k.slot_size), (int)kUnbuilt, kSlots, s);
  return e ? e : hipMemsetAsync(k.counters, 0, 64, s);
}
// counters[kCArena .. kCMiss + 1] (device) -> usage[0..3] (host-mapped), after a call
const uint32_t* kryo_usage_src(uint8_t* fixed) { return KryoState(fixed).counters + kCArena; }
hipError_t kryo_reset_misses(uint8_t* fixed, uint32_t set, hipStream_t s) {
  return hipMemsetAsync(KryoState(fixed).counters + kCMiss + (set & 1), 0, 4, s);
}
uint32_t kryo_clear_threshold_slots() { return kSlots / 2; }
uint32_t kryo_clear_threshold_templates() { return kBuilders - 64; }

static hipError_t shape_launch(const cordahip_kryo_item* d_items, const uint8_t* data_base, uint64_t data_len,
                               uint64_t n, uint32_t group, uint8_t* fixed, uint32_t* item_slot, uint32_t* direct,
                               uint64_t* sizes, uint8_t* status, hipStream_t s, bool templates_only, bool hash_chain,
                               uint32_t set) {
  if (n == 0) return hipSuccess;
  const ItemSrc items{d_items, data_base, data_len};
  const KryoState k(fixed);
  const uint32_t sb = shape_block(n, group), g = grouped(n, group) ? group : 1;
  hipLaunchKernelGGL(kryo_shape_kernel, dim3((uint32_t)((item_threads(n, group) + sb - 1) / sb)), dim3(sb), 0, s, items,
                     n, g, templates_only, hash_chain, k.table, k.slot_size, k.rec, item_slot, k.shape_list, sizes,
                     status, direct, k.counters, k.counters + kCMiss + (set < 2 ? set : 2));  // [6]: the device hash chain's (unread)
  return hipGetLastError();
}

hipError_t launch_kryo_shape(const cordahip_kryo_item* d_items, const uint8_t* data_base, uint64_t data_len,
                             uint64_t n, uint32_t group, uint8_t* fixed, uint32_t* item_slot, uint32_t* direct,
                             uint64_t* sizes, uint8_t* status, hipStream_t s, bool templates_only, uint32_t set) {
  // the shape pass of the templates-only chain feeds kryo_hash: RAW leaves over its limit are misses
  return shape_launch(d_items, data_base, data_len, n, group, fixed, item_slot, direct, sizes, status, s,
                      templates_only, templates_only, set);
}

hipError_t launch_kryo_encode(const cordahip_kryo_item* d_items, const uint8_t* data_base, uint64_t data_len,
                              uint64_t n, uint32_t group, uint8_t* fixed, uint32_t* item_slot, uint32_t* direct,
                              uint64_t* sizes, uint64_t* off, uint8_t* out, uint64_t cap, uint8_t* status,
                              uint8_t* dws, uint64_t dwriters, void* scan_temp, size_t scan_bytes, hipStream_t s,
                              bool templates_only, uint32_t set) {
  const ItemSrc items{d_items, data_base, data_len};
  const KryoState k(fixed);
  // kCNew, kCDirect (the templates-only chain neither claims nor lists: no reset, one
  // launch less per id slice)
  hipError_t e = templates_only ? hipSuccess : hipMemsetAsync(k.counters, 0, 8, s);
  if (e || n == 0) {
    e = e ? e : hipMemsetAsync(off, 0, 8, s);
    return e;
  }
  e = shape_launch(d_items, data_base, data_len, n, group, fixed, item_slot, direct, sizes, status, s,
                   templates_only, templates_only, set);
  // build, tsize, dsize (and dwrite) serve new shapes and direct items; in steady
  // state they find nothing to do, yet beside the Ed25519 ladders of a component
  // batch each empty launch of build / dsize / dwrite took 0.07-0.47 ms on the
  // slice's critical path (profiles/r05_c4h_rare_ab: 57.8 -> 68.0 M sig/s without
  // them). The templates-only chain leaves them out and reports misses instead.
  if (!templates_only) {
    hipLaunchKernelGGL(kryo_build_kernel, dim3(kBuildWaves), dim3(64), 0, s, items, k.table, k.shape_list, k.counters,
                       k.rec, k.slot_size, k.slot_map, k.arena);
    hipLaunchKernelGGL(kryo_tsize_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, items, n, item_slot,
                       k.slot_size, k.rec, sizes, status, direct, k.counters);
    hipLaunchKernelGGL(kryo_dsize_kernel, dim3(kDsizeBlocks), dim3(256), 0, s, items, direct, k.counters, sizes, status);
  }
  e = hipGetLastError();
  size_t tb = scan_bytes;
  e = e ? e : hipcub::DeviceScan::ExclusiveSum(scan_temp, tb, sizes, off, (int)(n + 1), s);
  if (e || !out) return e;
  const uint64_t waves = (n + kLeavesPerWave - 1) / kLeavesPerWave;
  hipLaunchKernelGGL(kryo_twrite_kernel, dim3((uint32_t)((waves + 3) / 4)), dim3(256), 0, s, items, n, off, item_slot,
                     k.slot_map, k.arena, out, cap, status);
  if (templates_only) return hipGetLastError();
  hipLaunchKernelGGL(kryo_dwrite_kernel, dim3((uint32_t)std::max<uint64_t>(1, dwriters / 256)), dim3(256), 0, s, items,
                     direct, k.counters, off, out, cap, status, dws);
  return hipGetLastError();
}

hipError_t kryo_set_priority(uint32_t on) { return hipMemcpyToSymbol(HIP_SYMBOL(g_kryo_prio), &on, 4); }

hipError_t launch_kryo_hash(const cordahip_kryo_item* d_items, const uint8_t* data_base, uint64_t data_len,
                            uint64_t n, uint32_t group, uint8_t* fixed, const uint32_t* item_slot,
                            const uint64_t* sizes, const uint8_t* status, uint32_t* hashes, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const ItemSrc items{d_items, data_base, data_len};
  const KryoState k(fixed);
  const uint32_t sb = shape_block(n, group), g = grouped(n, group) ? group : 1;
  // waves per SIMD the register allocation must allow (CORDAHIP_KRYO_HASH_WAVES, A/B): 5
  // (96 VGPRs, 40 B of spills) against 4 (117 VGPRs): 2.43 against 2.67 ms per 6.25 M
  // leaves of C4 on the device chain, 6 (80 VGPRs, 112 B of spills) 2.56 (profiles/r06_kryo_hash_waves_ab/)
  static const int waves = [] {
    const char* v = getenv("CORDAHIP_KRYO_HASH_WAVES");
    return v ? atoi(v) : 5;
  }();
  const dim3 grid(hash_blocks(n, group)), blk(256);
  (void)sb;
  if (waves >= 6)
    hipLaunchKernelGGL(kryo_hash_kernel<6>, grid, blk, 0, s, items, n, g, item_slot, k.slot_map, k.arena, sizes, status,
                       hashes);
  else if (waves == 5)
    hipLaunchKernelGGL(kryo_hash_kernel<5>, grid, blk, 0, s, items, n, g, item_slot, k.slot_map, k.arena, sizes, status,
                       hashes);
  else
    hipLaunchKernelGGL(kryo_hash_kernel<1>, grid, blk, 0, s, items, n, g, item_slot, k.slot_map, k.arena, sizes, status,
                       hashes);
  return hipGetLastError();
}

// The host calls' templates-only chain in one launch per id slice: shapes and leaf
// hashes (kryo_hash_kernel<5, true>); statuses into `status`, misses into set's counter.
hipError_t launch_kryo_shape_hash(const cordahip_kryo_item* d_items, const uint8_t* data_base, uint64_t data_len,
                                  uint64_t n, uint32_t group, uint8_t* fixed, uint8_t* status, uint32_t* hashes,
                                  hipStream_t s, uint32_t set) {
  if (n == 0) return hipSuccess;
  const ItemSrc items{d_items, data_base, data_len};
  const KryoState k(fixed);
  const uint32_t g = grouped(n, group) ? group : 1;
  const FusedShape fs{k.table, k.slot_size, k.rec, k.counters + kCMiss + (set < 2 ? set : 2), status};
  hipLaunchKernelGGL((kryo_hash_kernel<5, true>), dim3(hash_blocks(n, group)), dim3(256), 0, s, items, n, g,
                     (const uint32_t*)nullptr, k.slot_map, k.arena, (const uint64_t*)nullptr, (const uint8_t*)nullptr,
                     hashes, fs);
  return hipGetLastError();
}

// The device hash chain: every item's leaf hash without a leaf in memory and
// without misses. The shape pass claims new shapes (as the full chain does),
// kryo_build traces their templates, kryo_tsize resolves the items of shapes
// built in this launch set; kryo_hash hashes every template and RAW item from
// its template or bytes, and kryo_dhash runs the direct encoder into a SHA-256
// sink for the rest (collisions, leaves beyond a template, a full arena, RAW
// leaves of 2^29 bytes or more). Steady state: build / tsize / dhash find
// nothing to do. dwriters: the dhash threads (ws holds kLevelSyms bytes each).
hipError_t launch_kryo_hash_chain(const cordahip_kryo_item* d_items, const uint8_t* data_base, uint64_t data_len,
                                  uint64_t n, uint32_t group, uint8_t* fixed, uint32_t* item_slot, uint32_t* direct,
                                  uint64_t* sizes, uint8_t* status, uint32_t* hashes, uint8_t* dws, uint64_t dwriters,
                                  hipStream_t s) {
  if (n == 0) return hipSuccess;
  const ItemSrc items{d_items, data_base, data_len};
  const KryoState k(fixed);
  hipError_t e = hipMemsetAsync(k.counters, 0, 8, s);  // kCNew, kCDirect
  e = e ? e : shape_launch(d_items, data_base, data_len, n, group, fixed, item_slot, direct, sizes, status, s, false,
                           true, 2);
  if (e) return e;
  hipLaunchKernelGGL(kryo_build_kernel, dim3(kBuildWaves), dim3(64), 0, s, items, k.table, k.shape_list, k.counters,
                     k.rec, k.slot_size, k.slot_map, k.arena);
  hipLaunchKernelGGL(kryo_tsize_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, items, n, item_slot,
                     k.slot_size, k.rec, sizes, status, direct, k.counters);
  e = hipGetLastError();
  e = e ? e : launch_kryo_hash(d_items, data_base, data_len, n, group, fixed, item_slot, sizes, status, hashes, s);
  if (e) return e;
  hipLaunchKernelGGL(kryo_dhash_kernel, dim3((uint32_t)std::max<uint64_t>(1, dwriters / 256)), dim3(256), 0, s, items,
                     direct, k.counters, status, hashes, dws);
  return hipGetLastError();
}

hipError_t kryo_scan_bytes(size_t& bytes, uint64_t n1, hipStream_t s) {
  bytes = 0;
  return hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)n1, s);
}

}  // namespace cordahip
