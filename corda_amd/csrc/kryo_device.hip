// Native Kryo leaf encoder on the GPU: the same leaf
// preimages as cordahip_kryo_encode (kryo_core.hpp, one encoder for both
// sides), for batches whose component payloads are already in HBM -- a
// transaction batch's ids then need no host serialisation and no leaf bytes
// over PCIe (c4h with native leaves moves 1,717 B of leaves per cash-issue
// transaction; its components are ~600 B).
//
// Leaves are written from per-shape templates (kryo_template.hpp), not by
// running the byte-sequential encoder once per item:
//   1. kryo_shape: every item's shape (the inputs the encoder branches on),
//      hashed into a 2^16-slot table; the first item of a shape claims a slot
//      (one 64-bit CAS: hash | item) and becomes its representative; equal
//      hashes are confirmed with same_shape, so a collision costs a probe,
//      never a wrong leaf.
//   2. kryo_build: one wave per shape traces its representative through the
//      encoder (KoutT<true>, the OutputChunked level buffers in LDS): a
//      symbol per leaf byte -- a constant, payload byte k, or byte j of the
//      item's value.
//   3. kryo_tsize: every item's size from its shape (RAW: its length); items
//      without a shape, or whose shape has no template, go on a list for the
//      direct encoder, which sizes them (kryo_dsize, counting mode).
//   4. an exclusive scan of the sizes into the CSR offsets (hipcub).
//   5. kryo_twrite: a wave per 8 consecutive leaves writes their bytes in
//      output order, one aligned dword per lane (64 lanes = 256 contiguous
//      bytes per store instruction), each byte from its template symbol; the
//      dword a leaf ends in carries the next leaves' first bytes.
//   6. kryo_dwrite: the listed items through the direct encoder (per-thread
//      level buffers in a workspace), after kryo_twrite: their byte stores
//      replace what kryo_twrite left in the dwords they share.
// r04 ran the direct encoder for every item: 80.5 KB of L2-fabric traffic per
// cash-issue transaction (the level buffers' round trips) against 1,717 B of
// leaves, 5.0 + 17.9 ms per 6.25 M leaves (profiles/r04_pmc_kryo_traffic.json).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "kryo_template.hpp"

namespace cordahip {

namespace {

using kryo::kChunk;

constexpr uint32_t kSlots = 1u << 16;      // shape table slots (a power of two)
constexpr uint32_t kMaxProbe = 64;         // linear probes before an item goes to the direct encoder
constexpr uint32_t kBuilders = 1024;       // templates per call (more shapes: direct encoder)
constexpr uint32_t kTmplSyms = 4096;       // symbols per template (longer leaves: direct encoder)
constexpr uint32_t kNoSlot = 0xffffffffu;  // item_slot: no shape (direct encoder)
constexpr uint32_t kRawSlot = 0xfffffffeu; // item_slot: a RAW leaf (copied)
constexpr int32_t kInvalid = -1, kNoTemplate = -2;
constexpr uint32_t kLeavesPerWave = 8;
constexpr uint32_t kLevelSyms = kryo::kLevelBytes;  // levels 1..7 (level 0 is the leaf itself)

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

__device__ inline uint64_t item_of(uint64_t j, uint64_t n, uint32_t group) {
  if (group <= 1 || n % group) return j;
  const uint64_t rec = n / group;  // records of `group` items: kind-major thread order
  return (j % rec) * group + j / rec;
}

// ---- 1. shapes ------------------------------------------------------------------
__global__ void __launch_bounds__(256) kryo_shape_kernel(ItemSrc items, uint64_t n,
                                                         uint32_t group, unsigned long long* __restrict__ table,
                                                         uint32_t* __restrict__ item_slot, uint32_t* __restrict__ shape_list,
                                                         uint32_t* __restrict__ counters) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t i = item_of(j, n, group);
  const cordahip_kryo_item it = items[i];
  if (it.kind == CORDAHIP_KRYO_RAW) {
    item_slot[i] = kRawSlot;
    return;
  }
  const kryo::Shape s = kryo::shape_of(it);
  uint32_t slot = kNoSlot;
  if (s.ok) {
    const uint64_t h = kryo::shape_hash(s);
    const unsigned long long mine = ((unsigned long long)(uint32_t)(h >> 32) << 32) | (unsigned long long)(i + 1);
    uint32_t k = (uint32_t)h & (kSlots - 1);
    for (uint32_t probe = 0; probe < kMaxProbe; probe++, k = (k + 1) & (kSlots - 1)) {
      unsigned long long v = __hip_atomic_load(&table[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v == 0) {
        v = atomicCAS(&table[k], 0ull, mine);
        if (v == 0) {  // claimed: this item represents the shape
          slot = k;
          const uint32_t idx = atomicAdd(&counters[0], 1u);
          if (idx < kSlots) shape_list[idx] = k;
          break;
        }
      }
      if ((uint32_t)(v >> 32) == (uint32_t)(h >> 32) &&
          kryo::same_shape(kryo::shape_of(items[(uint32_t)v - 1]), s)) {
        slot = k;
        break;
      }
    }
  }
  item_slot[i] = slot;
}

// ---- 2. templates -----------------------------------------------------------------
// One wave per shape (lane 0 traces; the level buffers live in LDS).
__global__ void __launch_bounds__(64) kryo_build_kernel(ItemSrc items,
                                                        const unsigned long long* __restrict__ table,
                                                        const uint32_t* __restrict__ shape_list,
                                                        const uint32_t* __restrict__ counters,
                                                        int32_t* __restrict__ slot_size, uint32_t* __restrict__ slot_map,
                                                        uint32_t* __restrict__ arena) {
  __shared__ uint32_t levels[kLevelSyms];
  const uint32_t nshapes = counters[0] < kSlots ? counters[0] : kSlots;
  for (uint32_t b = blockIdx.x; b < nshapes; b += gridDim.x) {
    if (threadIdx.x != 0) continue;
    const uint32_t slot = shape_list[b];
    if (b >= kBuilders) {  // beyond the arena: the shape's items use the direct encoder
      slot_size[slot] = kNoTemplate;
      continue;
    }
    slot_map[slot] = b;
    const uint64_t rep = (uint32_t)table[slot] - 1;
    const cordahip_kryo_item it = items[rep];
    const int64_t sz = kryo::trace_leaf(it, arena + (size_t)b * kTmplSyms, kTmplSyms, levels);
    slot_size[slot] = (int32_t)sz;  // the size, or kInvalid / kNoTemplate
  }
}

// ---- 3. sizes ---------------------------------------------------------------------
__global__ void __launch_bounds__(256) kryo_tsize_kernel(ItemSrc items, uint64_t n,
                                                         const uint32_t* __restrict__ item_slot,
                                                         const int32_t* __restrict__ slot_size,
                                                         uint64_t* __restrict__ sizes, uint8_t* __restrict__ status,
                                                         uint32_t* __restrict__ direct, uint32_t* __restrict__ counters) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) sizes[n] = 0;  // the scan's last element: off[n] = the total
  if (i >= n) return;
  const uint32_t slot = item_slot[i];
  uint64_t size = 0;
  uint8_t st = 0;
  bool dir = slot == kNoSlot;
  if (slot == kRawSlot) {
    const cordahip_kryo_item it = items[i];
    if (it.len && !it.data) st = 1;
    else size = it.len;
  } else if (!dir) {
    const int32_t z = slot_size[slot];
    if (z >= 0) size = (uint64_t)z;
    else if (z == kInvalid) st = 1;
    else dir = true;
  }
  if (dir) direct[atomicAdd(&counters[1], 1u)] = (uint32_t)i;  // sized by kryo_dsize
  sizes[i] = size;
  status[i] = st;
}

// the direct encoder's count pass over the listed items
__global__ void __launch_bounds__(256) kryo_dsize_kernel(ItemSrc items,
                                                         const uint32_t* __restrict__ direct,
                                                         const uint32_t* __restrict__ counters,
                                                         uint64_t* __restrict__ sizes, uint8_t* __restrict__ status) {
  const uint32_t nd = counters[1];
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
struct LeafSrc {
  uint32_t kind;  // 0 template, 1 raw, 2 direct (not written here)
  const uint32_t* syms;
  const uint8_t* data;
  int64_t value;
};

__device__ inline LeafSrc leaf_src(const ItemSrc& items, const uint32_t* item_slot,
                                   const int32_t* slot_size, const uint32_t* slot_map, const uint32_t* arena,
                                   uint64_t L) {
  const cordahip_kryo_item it = items[L];
  const uint32_t slot = item_slot[L];
  LeafSrc s;
  s.data = it.data;
  s.value = it.value;
  s.syms = nullptr;
  if (slot == kRawSlot) {
    s.kind = 1;
  } else if (slot == kNoSlot || slot_size[slot] < 0) {
    s.kind = 2;
  } else {
    s.kind = 0;
    s.syms = arena + (size_t)slot_map[slot] * kTmplSyms;
  }
  return s;
}

__device__ inline uint8_t src_byte(const LeafSrc& s, uint64_t p) {
  return s.kind == 1 ? s.data[p] : kryo::sym_byte(s.syms[p], s.data, s.value);
}

// Byte q of the output when it lies in a leaf after `from` (the end of a dword
// whose first byte is in an earlier leaf): false when that leaf is not written
// here (direct encoder, or beyond cap).
__device__ inline bool spill_byte(const ItemSrc& items, uint64_t n, const uint64_t* off,
                                  const uint32_t* item_slot, const int32_t* slot_size, const uint32_t* slot_map,
                                  const uint32_t* arena, uint64_t cap, uint64_t from, uint64_t q, uint8_t& byte) {
  uint64_t L = from;
  while (L < n && off[L + 1] <= q) L++;
  if (L >= n || off[L + 1] > cap) return false;
  const LeafSrc s = leaf_src(items, item_slot, slot_size, slot_map, arena, L);
  if (s.kind == 2) return false;
  byte = src_byte(s, q - off[L]);
  return true;
}

__global__ void __launch_bounds__(256) kryo_twrite_kernel(ItemSrc items, uint64_t n,
                                                          const uint64_t* __restrict__ off,
                                                          const uint32_t* __restrict__ item_slot,
                                                          const int32_t* __restrict__ slot_size,
                                                          const uint32_t* __restrict__ slot_map,
                                                          const uint32_t* __restrict__ arena, uint8_t* __restrict__ out,
                                                          uint64_t cap, uint8_t* __restrict__ status) {
  const uint32_t lane = threadIdx.x & 63;
  // wave-uniform (readfirstlane: the leaf loop and its loads stay scalar)
  const uint64_t wave = (uint64_t)__builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const uint64_t L0 = wave * kLeavesPerWave;
  if (L0 >= n) return;
  const uint64_t L1 = L0 + kLeavesPerWave < n ? L0 + kLeavesPerWave : n;
  const uint64_t base = (uint64_t)(uintptr_t)out;
  for (uint64_t L = L0; L < L1; L++) {
    const uint64_t a = off[L], b = off[L + 1];
    if (b == a) continue;  // invalid item (or an empty RAW leaf)
    const LeafSrc s = leaf_src(items, item_slot, slot_size, slot_map, arena, L);
    if (b > cap) {  // not written (nor are the leaves after it)
      if (lane == 0 && s.kind != 2) status[L] = 2;
      continue;
    }
    // the dwords whose first output byte is in this leaf (the leaf at output
    // position 0 also takes the dword that starts before the buffer)
    const uint64_t lo = a == 0 ? (base & ~3ull) : ((base + a + 3) & ~3ull);
    const uint64_t hi = (base + b + 3) & ~3ull;
    // a direct leaf's bytes come later (kryo_dwrite); only its last dword may
    // carry bytes of the next leaves
    const uint64_t start = s.kind == 2 ? (hi - 4 > lo ? hi - 4 : lo) : lo;
    for (uint64_t A = start + 4ull * lane; A < hi; A += 256) {
      uint32_t w = 0, valid = 0;
#pragma unroll
      for (uint32_t j = 0; j < 4; j++) {
        if (A + j < base) continue;
        const uint64_t q = A + j - base;
        uint8_t byte = 0;
        if (q < b) {
          if (s.kind == 2) continue;
          byte = src_byte(s, q - a);
        } else if (!spill_byte(items, n, off, item_slot, slot_size, slot_map, arena, cap, L + 1, q, byte)) {
          continue;
        }
        w |= (uint32_t)byte << (8 * j);
        valid |= 1u << j;
      }
      if (valid == 15) {
        *reinterpret_cast<uint32_t*>(A) = w;
      } else {
        for (uint32_t j = 0; j < 4; j++)
          if (valid >> j & 1) reinterpret_cast<uint8_t*>(A)[j] = (uint8_t)(w >> (8 * j));
      }
    }
  }
}

// ---- 6. direct writes ---------------------------------------------------------------
__global__ void __launch_bounds__(256) kryo_dwrite_kernel(ItemSrc items,
                                                          const uint32_t* __restrict__ direct,
                                                          const uint32_t* __restrict__ counters,
                                                          const uint64_t* __restrict__ off, uint8_t* __restrict__ out,
                                                          uint64_t cap, uint8_t* __restrict__ status,
                                                          uint8_t* __restrict__ ws) {
  const uint32_t nd = counters[1];
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // levels 1..7 of this thread's OutputChunked buffers (level 0 is the leaf)
  uint8_t* levels = ws + t * (uint64_t)kLevelSyms;
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

}  // namespace

// Scratch of one encode call (cordahip.cpp sizes it with kryo_scratch_bytes).
struct KryoScratch {
  unsigned long long* table;  // [kSlots]
  uint32_t* shape_list;       // [kSlots]
  int32_t* slot_size;         // [kSlots]
  uint32_t* slot_map;         // [kSlots] builder index of the slot's template
  uint32_t* counters;         // [0] shapes, [1] direct items
  uint32_t* item_slot;        // [n]
  uint32_t* direct;           // [n]
  uint32_t* arena;            // [kBuilders * kTmplSyms]
  uint8_t* dws;               // direct writers' level buffers
};

size_t kryo_fixed_scratch_bytes() {
  return (size_t)kSlots * (8 + 4 + 4 + 4) + 64 + (size_t)kBuilders * kTmplSyms * 4;
}
size_t kryo_direct_ws_bytes(uint64_t writers) { return (size_t)writers * kLevelSyms; }

hipError_t launch_kryo_encode(const cordahip_kryo_item* d_items, const uint8_t* data_base, uint64_t data_len,
                              uint64_t n, uint32_t group, uint8_t* fixed,
                              uint32_t* item_slot, uint32_t* direct, uint64_t* sizes, uint64_t* off, uint8_t* out,
                              uint64_t cap, uint8_t* status, uint8_t* dws, uint64_t dwriters, void* scan_temp,
                              size_t scan_bytes, hipStream_t s) {
  const ItemSrc items{d_items, data_base, data_len};
  KryoScratch k;
  k.table = reinterpret_cast<unsigned long long*>(fixed);
  k.shape_list = reinterpret_cast<uint32_t*>(k.table + kSlots);
  k.slot_size = reinterpret_cast<int32_t*>(k.shape_list + kSlots);
  k.slot_map = reinterpret_cast<uint32_t*>(k.slot_size + kSlots);
  k.counters = k.slot_map + kSlots;
  k.arena = k.counters + 16;
  hipError_t e = hipMemsetAsync(k.table, 0, (size_t)kSlots * 8, s);
  e = e ? e : hipMemsetAsync(k.counters, 0, 64, s);
  if (e || n == 0) {
    e = e ? e : hipMemsetAsync(off, 0, 8, s);
    return e;
  }
  const uint32_t blocks = (uint32_t)((n + 255) / 256);
  hipLaunchKernelGGL(kryo_shape_kernel, dim3(blocks), dim3(256), 0, s, items, n, group, k.table, item_slot,
                     k.shape_list, k.counters);
  hipLaunchKernelGGL(kryo_build_kernel, dim3(kBuilders), dim3(64), 0, s, items, k.table, k.shape_list, k.counters,
                     k.slot_size, k.slot_map, k.arena);
  hipLaunchKernelGGL(kryo_tsize_kernel, dim3((uint32_t)((n + 1 + 255) / 256)), dim3(256), 0, s, items, n, item_slot,
                     k.slot_size, sizes, status, direct, k.counters);
  hipLaunchKernelGGL(kryo_dsize_kernel, dim3(1024), dim3(256), 0, s, items, direct, k.counters, sizes, status);
  e = hipGetLastError();
  size_t tb = scan_bytes;
  e = e ? e : hipcub::DeviceScan::ExclusiveSum(scan_temp, tb, sizes, off, (int)(n + 1), s);
  if (e || !out) return e;
  const uint64_t waves = (n + kLeavesPerWave - 1) / kLeavesPerWave;
  hipLaunchKernelGGL(kryo_twrite_kernel, dim3((uint32_t)((waves + 3) / 4)), dim3(256), 0, s, items, n, off, item_slot,
                     k.slot_size, k.slot_map, k.arena, out, cap, status);
  hipLaunchKernelGGL(kryo_dwrite_kernel, dim3((uint32_t)std::max<uint64_t>(1, dwriters / 256)), dim3(256), 0, s, items,
                     direct, k.counters, off, out, cap, status, dws);
  return hipGetLastError();
}

hipError_t kryo_scan_bytes(size_t& bytes, uint64_t n1, hipStream_t s) {
  bytes = 0;
  return hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)n1, s);
}

}  // namespace cordahip
