// Transaction ids and per-transaction signature verdicts for gfx950 —
// kernels K3 (leaf hashes), K4 (Merkle roots) and K5 (per-tx reduction).
//
// Reference path:
//   WireTransaction.id = MerkleTree.getMerkleTree(availableComponentHashes).hash
//     WireTransaction.kt:48,120; MerkleTransaction.kt:69
//   leaf_i = SHA-256(serialised component i)                  MerkleTransaction.kt:16-18,
//            ("corda\0\0\1" + Kryo bytes, produced by the host)  Kryo.kt:95,101,165-176
//   padWithZeros to 2^k with SecureHash.zeroHash               MerkleTree.kt:33-41
//   node = SHA-256(left || right), no domain separation        MerkleTree.kt:57-63, SecureHash.kt:24
//   empty -> MerkleTreeException; one leaf -> root = leaf      MerkleTree.kt:49-52
//   SignedTransaction.checkSignaturesAreValid: sigs verified in list order,
//   the first failure throws                                   SignedTransaction.kt:95-100
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>

#include "sha2_device.hpp"
#include "status.hpp"

namespace cordahip {

// The transaction-id kernels run at raised wave priority (s_setprio 3): beside
// the Ed25519 ladders of a signed-tx batch they are the id slices' critical
// path -- a signature chunk's prep waits for its slice's ids -- and at equal
// priority the ladder waves took most of the issue slots (a 2^16-signature
// slice's SHA-256 0.46-0.51 ms beside a ladder against 0.13 ms alone,
// profiles/r05_c4h_components_timeline_skiprare_ab.txt). Total work is
// unchanged; the ladders take the slots the id waves leave. 0: off
// (CORDAHIP_ID_PRIO=0, tx_set_id_priority).
__device__ uint32_t g_id_prio = 1;

__device__ inline void id_priority() {
  if (g_id_prio) __builtin_amdgcn_s_setprio(3);
}

hipError_t tx_set_id_priority(uint32_t on) { return hipMemcpyToSymbol(HIP_SYMBOL(g_id_prio), &on, 4); }

// tx-level statuses beyond the lane statuses (include/cordahip.h)
static constexpr uint8_t kTxNoLeaves = 6;      // MerkleTreeException
static constexpr uint8_t kTxBadComponent = 9;  // a component the encoder rejected (cordahip.h)
static constexpr uint8_t kTxNoSignatures = 7;  // SignedTransaction init: require(sigs.isNotEmpty())

// SHA-256(a || b) for two 32-byte digests (state words, big-endian): the
// Merkle node hash. The second block is the constant padding of a 64-byte
// message.
CDEV void sha256_node(uint32_t out[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    w[i] = a[i];
    w[8 + i] = b[i];
  }
  sha256_init(out);
  sha256_block(out, w);
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = 0;
  w[0] = 0x80000000u;
  w[15] = 512;
  sha256_block(out, w);
}

// K3: one lane per leaf. A wave runs as many SHA-256 blocks as its longest
// leaf, and a transaction's components differ widely in length (C4: 8, 3, 3, 1
// and 1 blocks), so each 256-leaf tile is first counting-sorted in LDS by block
// count (buckets 1..7, 8+): waves then hold leaves of similar length
// (C4: ~15 instead of 32 wave-blocks per tile). Hashes are written by leaf index.
__global__ void __launch_bounds__(256) sha256_leaves_kernel(const uint8_t* __restrict__ bytes,
                                                           const uint64_t* __restrict__ off, uint64_t nleaves,
                                                           uint32_t* __restrict__ hashes /* [nleaves][8] BE words */) {
  id_priority();
  __shared__ unsigned int cnt[9], order[256];
  const uint64_t mine = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (threadIdx.x < 9) cnt[threadIdx.x] = 0;
  __syncthreads();
  int key = 8;  // past the end: last bucket, never hashed
  if (mine < nleaves) {
    const uint64_t nb = (off[mine + 1] - off[mine] + 9 + 63) / 64;
    key = nb >= 8 ? 7 : (int)nb - 1;
  }
  atomicAdd(&cnt[key], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {  // exclusive prefix over the 9 buckets -> cursors
    unsigned int run = 0;
    for (int k = 0; k < 9; k++) {
      const unsigned int c = cnt[k];
      cnt[k] = run;
      run += c;
    }
  }
  __syncthreads();
  order[atomicAdd(&cnt[key], 1u)] = threadIdx.x;
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + order[threadIdx.x];
  if (i >= nleaves) return;
  uint32_t h[8];
  const uint64_t lo = off[i], hi = off[i + 1];
  sha256_bytes(h, bytes + lo, hi - lo);
  uint4* o = reinterpret_cast<uint4*>(hashes + i * 8);
  o[0] = make_uint4(h[0], h[1], h[2], h[3]);
  o[1] = make_uint4(h[4], h[5], h[6], h[7]);
}

// K4: one lane per transaction; reduces the tx's leaf-hash range in place.
// Level j holds m_j real nodes; positions >= m_j are the padding constant
// Z_j (Z_0 = zeroHash, Z_{j+1} = H(Z_j, Z_j)), exactly the padded tree of
// MerkleTree.kt:33-66.
//
// Optional, for the pipelined signed-tx slices (one launch instead of three):
// item_status != nullptr -- component batches: a tx with a component the
// encoder rejected gets kTxBadComponent (item_status is indexed like hashes,
// by absolute leaf index); map_txid / map_status != nullptr -- the id and
// status also go to the caller's pinned arrays through their device mapping.
CDEV void merkle_emit(uint64_t t, const uint32_t root[8], uint8_t st, uint8_t* __restrict__ txid,
                      uint8_t* __restrict__ tx_status, uint8_t* __restrict__ map_txid, uint8_t* __restrict__ map_status) {
  const uint4 r0 = make_uint4(bswap32(root[0]), bswap32(root[1]), bswap32(root[2]), bswap32(root[3]));
  const uint4 r1 = make_uint4(bswap32(root[4]), bswap32(root[5]), bswap32(root[6]), bswap32(root[7]));
  uint4* o = reinterpret_cast<uint4*>(txid + t * 32);
  o[0] = r0;
  o[1] = r1;
  if (tx_status) tx_status[t] = st;
  if (map_txid) {
    uint8_t* d = map_txid + t * 32;
    if (((uintptr_t)d & 15) == 0) {
      reinterpret_cast<uint4*>(d)[0] = r0;
      reinterpret_cast<uint4*>(d)[1] = r1;
    } else {
      const uint8_t* b = reinterpret_cast<const uint8_t*>(o);
      for (int i = 0; i < 32; i++) d[i] = b[i];
    }
  }
  if (map_status) map_status[t] = st;
}

__global__ void __launch_bounds__(256) merkle_root_kernel(uint32_t* __restrict__ hashes,
                                                         const uint64_t* __restrict__ tx_leaf_off, uint64_t ntx,
                                                         uint8_t* __restrict__ txid, uint8_t* __restrict__ tx_status,
                                                         const uint8_t* __restrict__ item_status,
                                                         uint8_t* __restrict__ map_txid, uint8_t* __restrict__ map_status) {
  id_priority();
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntx) return;
  const uint64_t lo = tx_leaf_off[t], hi = tx_leaf_off[t + 1];
  uint64_t m = hi - lo;
  if (m == 0) {
    const uint32_t zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    merkle_emit(t, zero, kTxNoLeaves, txid, tx_status, map_txid, map_status);
    return;
  }
  uint8_t st = kStatusOk;
  if (item_status)
    for (uint64_t i = lo; i < hi; i++)
      if (item_status[i] != 0) st = kTxBadComponent;
  uint32_t* v = hashes + lo * 8;
  uint32_t z[8];  // Z_zlevel
#pragma unroll
  for (int i = 0; i < 8; i++) z[i] = 0;
  int zlevel = 0;
  for (int level = 0; m > 1; level++) {
    const uint64_t half = (m + 1) / 2;
    if (m & 1) {  // the last real node pairs with the padding constant Z_level
      for (; zlevel < level; zlevel++) {
        uint32_t zz[8];
        sha256_node(zz, z, z);
#pragma unroll
        for (int k = 0; k < 8; k++) z[k] = zz[k];
      }
    }
    for (uint64_t i = 0; i < half; i++) {
      uint32_t a[8], b[8], r[8];
      const uint4* pa = reinterpret_cast<const uint4*>(v + 16 * i);
      const uint4 a0 = pa[0], a1 = pa[1];
      a[0] = a0.x; a[1] = a0.y; a[2] = a0.z; a[3] = a0.w; a[4] = a1.x; a[5] = a1.y; a[6] = a1.z; a[7] = a1.w;
      if (2 * i + 1 < m) {
        const uint4 b0 = pa[2], b1 = pa[3];
        b[0] = b0.x; b[1] = b0.y; b[2] = b0.z; b[3] = b0.w; b[4] = b1.x; b[5] = b1.y; b[6] = b1.z; b[7] = b1.w;
      } else {
#pragma unroll
        for (int k = 0; k < 8; k++) b[k] = z[k];
      }
      sha256_node(r, a, b);
      uint4* po = reinterpret_cast<uint4*>(v + 8 * i);
      po[0] = make_uint4(r[0], r[1], r[2], r[3]);
      po[1] = make_uint4(r[4], r[5], r[6], r[7]);
    }
    m = half;
  }
  // root = v[0]; emit big-endian bytes (SecureHash byte order)
  const uint4* pv = reinterpret_cast<const uint4*>(v);
  const uint4 r0 = pv[0], r1 = pv[1];
  const uint32_t root[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
  merkle_emit(t, root, st, txid, tx_status, map_txid, map_status);
}

// gather: msgs[s] = txid[sig_tx[s]] (each signature signs its tx id, SignedTransaction.kt:98)
__global__ void __launch_bounds__(256) gather_txid_kernel(const uint8_t* __restrict__ txid,
                                                         const uint64_t* __restrict__ tx_sig_off, uint64_t ntx,
                                                         uint8_t* __restrict__ msgs) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntx) return;
  const uint4* src = reinterpret_cast<const uint4*>(txid + t * 32);
  const uint4 a = src[0], b = src[1];
  for (uint64_t s = tx_sig_off[t]; s < tx_sig_off[t + 1]; s++) {
    uint4* d = reinterpret_cast<uint4*>(msgs + s * 32);
    d[0] = a;
    d[1] = b;
  }
}

// Host signed-tx batches: the message rows of a pipeline chunk gathered on the
// device from the ids the id slices left in HBM (row r = txid[idx[r]]), so the
// signatures never wait for the ids to cross PCIe twice (D2H, then H2D as
// messages). Two lanes per row, one 16-byte load and store each.
__global__ void __launch_bounds__(256) gather_rows32_kernel(const uint8_t* __restrict__ txid,
                                                            const uint32_t* __restrict__ idx, uint64_t n,
                                                            uint8_t* __restrict__ rows) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * n) return;
  const uint64_t r = t >> 1, h = t & 1;
  reinterpret_cast<uint4*>(rows + r * 32)[h] = reinterpret_cast<const uint4*>(txid + (uint64_t)idx[r] * 32)[h];
}

// Device -> pinned host bytes by kernel stores (the host buffer is mapped, so
// the kernel writes it across PCIe directly): the pipelines' status returns.
// An SDMA hipMemcpyAsync D2H behind a compute stream's kernels held the
// enqueuing host thread ~7-18 ms whenever the DMA engine was busy with another
// stream's H2D (CORDAHIP_TRACE "launch" phase, profiles/r04_h), which stalled
// every later chunk's enqueue; a store kernel is ordered by the stream alone.
// 16 bytes per lane where both ends allow it, the ragged head/tail bytewise.
__global__ void __launch_bounds__(256) store_to_host_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                            uint64_t n) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    if (t < n / 16) reinterpret_cast<uint4*>(dst)[t] = reinterpret_cast<const uint4*>(src)[t];
    const uint64_t tail = n & ~15ull;
    if (t < n - tail) dst[tail + t] = src[tail + t];
  } else if (t < n) {
    dst[t] = src[t];
  }
}

// K5: checkSignaturesAreValid order — the first non-OK signature (list order)
// decides the tx outcome; -1 when every signature verified.
__global__ void __launch_bounds__(256) tx_reduce_kernel(uint8_t* __restrict__ sig_status,
                                                       const uint64_t* __restrict__ tx_sig_off, uint64_t ntx,
                                                       int64_t* __restrict__ first_bad, uint8_t* __restrict__ tx_status) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntx) return;
  const uint64_t lo = tx_sig_off[t], hi = tx_sig_off[t + 1];
  first_bad[t] = -1;
  // require(sigs.isNotEmpty()) runs in the constructor (SignedTransaction.kt:37-39),
  // before the lazy tx.id can throw MerkleTreeException
  if (lo == hi) {
    tx_status[t] = kTxNoSignatures;
    return;
  }
  if (tx_status[t] != kStatusOk) {  // the id itself could not be computed (no leaves, a bad component):
    for (uint64_t s = lo; s < hi; s++) sig_status[s] = tx_status[t];  // no signature was checked (host reduce_txs)
    return;
  }
  int64_t fb = -1;
  uint8_t st = kStatusOk;
  for (uint64_t s = lo; s < hi; s++) {
    const uint8_t v = sig_status[s];
    if (v != kStatusOk) {
      fb = (int64_t)(s - lo);
      st = v;
      break;
    }
  }
  first_bad[t] = fb;
  tx_status[t] = st;
}


// ---------------------------------------------------------------------------
// K6: FilteredTransaction.verify (MerkleTransaction.kt:134-140) ->
// PartialMerkleTree.verify (PartialMerkleTree.kt:132-158), one lane per
// filtered transaction. The partial tree arrives as its post-order token
// stream (0 IncludedLeaf, 1 Leaf, 2 Node) and is evaluated with a stack kept in
// HBM (the tx's own slice of `stack`, one 32-B slot per token): IncludedLeaf /
// Leaf push their hash, Node pops right then left and pushes
// hashConcat(left, right) = SHA-256(left || right) (SecureHash.kt:24). The
// included hashes, in token order, are the reference's usedHashes; verify()
// is true iff they equal the filtered leaves' hashes as multisets
// (groupBy equality) and the computed root equals the claimed root.
static constexpr uint8_t kTxBadTree = 8;
static constexpr uint8_t kTokIncluded = 0, kTokLeaf = 1, kTokNode = 2;

CDEV void load_hash_be(uint32_t w[8], const uint8_t* __restrict__ p) {  // 32 bytes -> SHA state words
  const uint4* p4 = reinterpret_cast<const uint4*>(p);
  const uint4 a = p4[0], b = p4[1];
  w[0] = bswap32(a.x); w[1] = bswap32(a.y); w[2] = bswap32(a.z); w[3] = bswap32(a.w);
  w[4] = bswap32(b.x); w[5] = bswap32(b.y); w[6] = bswap32(b.z); w[7] = bswap32(b.w);
}
CDEV void st_words(uint32_t* __restrict__ o, const uint32_t w[8]) {
  uint4* o4 = reinterpret_cast<uint4*>(o);
  o4[0] = make_uint4(w[0], w[1], w[2], w[3]);
  o4[1] = make_uint4(w[4], w[5], w[6], w[7]);
}
CDEV void ld_words(uint32_t w[8], const uint32_t* __restrict__ p) {
  const uint4* p4 = reinterpret_cast<const uint4*>(p);
  const uint4 a = p4[0], b = p4[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
CDEV bool words_eq(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b) {
  uint32_t d = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) d |= a[k] ^ b[k];
  return d == 0;
}

__global__ void __launch_bounds__(256) pmt_verify_kernel(const uint32_t* __restrict__ leaf_hashes,
                                                        const uint64_t* __restrict__ tx_leaf_off,
                                                        const uint8_t* __restrict__ tok,
                                                        const uint8_t* __restrict__ tok_hash,
                                                        const uint64_t* __restrict__ tx_tok_off,
                                                        const uint8_t* __restrict__ root, uint64_t ntx,
                                                        uint32_t* __restrict__ stack, uint8_t* __restrict__ tx_status) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntx) return;
  const uint64_t l0 = tx_leaf_off[t], l1 = tx_leaf_off[t + 1];
  if (l0 == l1) {  // filteredLeaves.availableComponentHashes empty: MerkleTreeException
    tx_status[t] = kTxNoLeaves;
    return;
  }
  const uint64_t k0 = tx_tok_off[t], k1 = tx_tok_off[t + 1];
  uint32_t* stk = stack + k0 * 8;
  uint64_t sp = 0, nincl = 0;
  bool ok = true;
  for (uint64_t k = k0; k < k1 && ok; k++) {
    const uint8_t tk = tok[k];
    if (tk == kTokIncluded || tk == kTokLeaf) {
      uint32_t h[8];
      load_hash_be(h, tok_hash + k * 32);
      st_words(stk + sp * 8, h);
      sp++;
      nincl += tk == kTokIncluded;
    } else if (tk == kTokNode && sp >= 2) {
      uint32_t a[8], b[8], r[8];
      ld_words(b, stk + (sp - 1) * 8);
      ld_words(a, stk + (sp - 2) * 8);
      sha256_node(r, a, b);
      st_words(stk + (sp - 2) * 8, r);
      sp--;
    } else {
      ok = false;
    }
  }
  if (!ok || sp != 1) {
    tx_status[t] = kTxBadTree;
    return;
  }
  uint32_t want[8];
  load_hash_be(want, root + t * 32);
  bool match = words_eq(stk, want) && nincl == l1 - l0;
  // multiset equality of the included token hashes and the leaf hashes
  for (uint64_t k = k0; k < k1 && match; k++) {
    if (tok[k] != kTokIncluded) continue;
    uint32_t h[8];
    load_hash_be(h, tok_hash + k * 32);
    uint64_t in_tree = 0, in_leaves = 0;
    for (uint64_t q = k0; q < k1; q++) {
      if (tok[q] != kTokIncluded) continue;
      uint32_t g[8];
      load_hash_be(g, tok_hash + q * 32);
      in_tree += words_eq(g, h);
    }
    for (uint64_t q = l0; q < l1; q++) in_leaves += words_eq(leaf_hashes + q * 8, h);
    match = in_tree == in_leaves;
  }
  tx_status[t] = match ? kStatusOk : kStatusBadSig;
}

hipError_t launch_pmt_verify(const uint32_t* leaf_hashes, const uint64_t* tx_leaf_off, const uint8_t* tok,
                             const uint8_t* tok_hash, const uint64_t* tx_tok_off, const uint8_t* root, uint64_t ntx,
                             uint32_t* stack, uint8_t* tx_status, hipStream_t s) {
  if (!ntx) return hipSuccess;
  hipLaunchKernelGGL(pmt_verify_kernel, dim3((uint32_t)((ntx + 255) / 256)), dim3(256), 0, s, leaf_hashes,
                     tx_leaf_off, tok, tok_hash, tx_tok_off, root, ntx, stack, tx_status);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
hipError_t launch_sha256_leaves(const uint8_t* bytes, const uint64_t* off, uint64_t nleaves, uint32_t* hashes,
                                hipStream_t s) {
  if (!nleaves) return hipSuccess;
  hipLaunchKernelGGL(sha256_leaves_kernel, dim3((uint32_t)((nleaves + 255) / 256)), dim3(256), 0, s, bytes, off,
                     nleaves, hashes);
  return hipGetLastError();
}
hipError_t launch_merkle_root(uint32_t* hashes, const uint64_t* tx_leaf_off, uint64_t ntx, uint8_t* txid,
                              uint8_t* tx_status, hipStream_t s, const uint8_t* item_status, uint8_t* map_txid,
                              uint8_t* map_status) {
  if (!ntx) return hipSuccess;
  hipLaunchKernelGGL(merkle_root_kernel, dim3((uint32_t)((ntx + 255) / 256)), dim3(256), 0, s, hashes, tx_leaf_off,
                     ntx, txid, tx_status, item_status, map_txid, map_status);
  return hipGetLastError();
}
hipError_t launch_gather_txid(const uint8_t* txid, const uint64_t* tx_sig_off, uint64_t ntx, uint8_t* msgs,
                              hipStream_t s) {
  if (!ntx) return hipSuccess;
  hipLaunchKernelGGL(gather_txid_kernel, dim3((uint32_t)((ntx + 255) / 256)), dim3(256), 0, s, txid, tx_sig_off,
                     ntx, msgs);
  return hipGetLastError();
}
hipError_t launch_store_to_host(const void* src, void* dst, uint64_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  const bool vec = (((uintptr_t)src | (uintptr_t)dst) & 15) == 0;
  const uint64_t threads = vec ? std::max<uint64_t>(n / 16, 16) : n;
  hipLaunchKernelGGL(store_to_host_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s,
                     static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), n);
  return hipGetLastError();
}
hipError_t launch_gather_rows32(const uint8_t* txid, const uint32_t* idx, uint64_t n, uint8_t* rows, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(gather_rows32_kernel, dim3((uint32_t)((2 * n + 255) / 256)), dim3(256), 0, s, txid, idx, n, rows);
  return hipGetLastError();
}
hipError_t launch_tx_reduce(uint8_t* sig_status, const uint64_t* tx_sig_off, uint64_t ntx, int64_t* first_bad,
                            uint8_t* tx_status, hipStream_t s) {
  if (!ntx) return hipSuccess;
  hipLaunchKernelGGL(tx_reduce_kernel, dim3((uint32_t)((ntx + 255) / 256)), dim3(256), 0, s, sig_status,
                     tx_sig_off, ntx, first_bad, tx_status);
  return hipGetLastError();
}

}  // namespace cordahip
