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

// The second block of every Merkle node hash is the constant padding of a
// 64-byte message (0x80, zeros, bit length 512): its message schedule is
// constant, so its rounds take K[i] + W[i] precomputed (tools/gen_merkle_consts.py):
// no schedule and one add less per round.
__device__ __constant__ static const uint32_t kPadKW[64] = {
    0xc28a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf374,
    0x649b69c1, 0xf0fe4786, 0x0fe1edc6, 0x240cf254, 0x4fe9346f, 0x6cc984be, 0x61b9411e, 0x16f988fa,
    0xf2c65152, 0xa88e5a6d, 0xb019fc65, 0xb9d99ec7, 0x9a1231c3, 0xe70eeaa0, 0xfdb1232b, 0xc7353eb0,
    0x3069bad5, 0xcb976d5f, 0x5a0f118f, 0xdc1eeefd, 0x0a35b689, 0xde0b7a04, 0x58f4ca9d, 0xe15d5b16,
    0x007f3e86, 0x37088980, 0xa507ea32, 0x6fab9537, 0x17406110, 0x0d8cd6f1, 0xcdaa3b6d, 0xc0bbbe37,
    0x83613bda, 0xdb48a363, 0x0b02e931, 0x6fd15ca7, 0x521afaca, 0x31338431, 0x6ed41a95, 0x6d437890,
    0xc39c91f2, 0x9eccabbd, 0xb5c9a0e6, 0x532fb63c, 0xd2c741c6, 0x07237ea3, 0xa4954b68, 0x4c191d76,
};
// Z_j: the root of a complete tree of 2^j zeroHash leaves (Z_0 = zeroHash,
// Z_{j+1} = SHA-256(Z_j || Z_j), MerkleTree.kt:33-41), the padding node of level j
// (tools/gen_merkle_consts.py; r05 hashed them in every transaction's tree)
__device__ __constant__ static const uint32_t kZeroHash[64][8] = {
    {0x00000000, 0x00000000, 0x00000000, 0x00000000, 0x00000000, 0x00000000, 0x00000000, 0x00000000},
    {0xf5a5fd42, 0xd16a2030, 0x2798ef6e, 0xd309979b, 0x43003d23, 0x20d9f0e8, 0xea9831a9, 0x2759fb4b},
    {0xdb56114e, 0x00fdd4c1, 0xf85c892b, 0xf35ac9a8, 0x9289aaec, 0xb1ebd0a9, 0x6cde606a, 0x748b5d71},
    {0xc78009fd, 0xf07fc56a, 0x11f12237, 0x0658a353, 0xaaa542ed, 0x63e44c4b, 0xc15ff4cd, 0x105ab33c},
    {0x536d9883, 0x7f2dd165, 0xa55d5eea, 0xe9148595, 0x4472d56f, 0x246df256, 0xbf3cae19, 0x352a123c},
    {0x9efde052, 0xaa15429f, 0xae05bad4, 0xd0b1d7c6, 0x4da64d03, 0xd7a1854a, 0x588c2cb8, 0x430c0d30},
    {0xd88ddfee, 0xd400a875, 0x5596b219, 0x42c1497e, 0x114c302e, 0x6118290f, 0x91e67729, 0x76041fa1},
    {0x87eb0ddb, 0xa57e35f6, 0xd2866738, 0x02a4af59, 0x75e22506, 0xc7cf4c64, 0xbb6be5ee, 0x11527f2c},
    {0x26846476, 0xfd5fc54a, 0x5d433851, 0x67c95144, 0xf2643f53, 0x3cc85bb9, 0xd16b782f, 0x8d7db193},
    {0x506d8658, 0x2d252405, 0xb8400187, 0x92cad2bf, 0x1259f1ef, 0x5aa5f887, 0xe13cb2f0, 0x094f51e1},
    {0xffff0ad7, 0xe659772f, 0x9534c195, 0xc815efc4, 0x014ef1e1, 0xdaed4404, 0xc06385d1, 0x1192e92b},
    {0x6cf04127, 0xdb05441c, 0xd833107a, 0x52be8528, 0x68890e43, 0x17e6a02a, 0xb47683aa, 0x75964220},
    {0xb7d05f87, 0x5f140027, 0xef5118a2, 0x247bbb84, 0xce8f2f0f, 0x11236230, 0x85daf796, 0x0c329f5f},
    {0xdf6af5f5, 0xbbdb6be9, 0xef8aa618, 0xe4bf8073, 0x96086717, 0x1e29676f, 0x8b284dea, 0x6a08a85e},
    {0xb58d900f, 0x5e182e3c, 0x50ef7496, 0x9ea16c77, 0x26c54975, 0x7cc23523, 0xc369587d, 0xa7293784},
    {0xd49a7502, 0xffcfb034, 0x0b1d7885, 0x688500ca, 0x308161a7, 0xf96b62df, 0x9d083b71, 0xfcc8f2bb},
    {0x8fe6b168, 0x9256c0d3, 0x85f42f5b, 0xbe2027a2, 0x2c1996e1, 0x10ba97c1, 0x71d3e594, 0x8de92beb},
    {0x8d0d63c3, 0x9ebade85, 0x09e0ae3c, 0x9c3876fb, 0x5fa112be, 0x18f905ec, 0xacfecb92, 0x057603ab},
    {0x95eec8b2, 0xe541cad4, 0xe91de383, 0x85f2e046, 0x619f5449, 0x6c2382cb, 0x6cacd5b9, 0x8c26f5a4},
    {0xf893e908, 0x917775b6, 0x2bff2329, 0x4dbbe3a1, 0xcd8e6cc1, 0xc35b4801, 0x887b646a, 0x6f81f17f},
    {0xcddba7b5, 0x92e31333, 0x93c16194, 0xfac7431a, 0xbf2f5485, 0xed711db2, 0x82183c81, 0x9e08ebaa},
    {0x8a8d7fe3, 0xaf8caa08, 0x5a7639a8, 0x32001457, 0xdfb9128a, 0x8061142a, 0xd0335629, 0xff23ff9c},
    {0xfeb3c337, 0xd7a51a6f, 0xbf00b9e3, 0x4c52e1c9, 0x195c969b, 0xd4e7a0bf, 0xd51d5c5b, 0xed9c1167},
    {0xe71f0aa8, 0x3cc32edf, 0xbefa9f4d, 0x3e0174ca, 0x85182eec, 0x9f3a09f6, 0xa6c0df63, 0x77a510d7},
    {0x31206fa8, 0x0a50bb6a, 0xbe290850, 0x58f16212, 0x212a60ee, 0xc8f049fe, 0xcb92d8c8, 0xe0a84bc0},
    {0x21352bfe, 0xcbeddde9, 0x93839f61, 0x4c3dac0a, 0x3ee37543, 0xf9b412b1, 0x6199dc15, 0x8e23b544},
    {0x619e3127, 0x24bb6d7c, 0x3153ed9d, 0xe791d764, 0xa366b389, 0xaf13c58b, 0xf8a8d904, 0x81a46765},
    {0x7cdd2986, 0x26825062, 0x8d0c10e3, 0x85c58c61, 0x91e6fbe0, 0x5191bcc0, 0x4f133f2c, 0xea72c1c4},
    {0x848930bd, 0x7ba8cac5, 0x46610721, 0x13fb2788, 0x69e07bb8, 0x587f9139, 0x2933374d, 0x017bcbe1},
    {0x8869ff2c, 0x22b28cc1, 0x0510d985, 0x32928033, 0x28be4fb0, 0xe80495e8, 0xbb8d271f, 0x5b889636},
    {0xb5fe28e7, 0x9f1b850f, 0x8658246c, 0xe9b6a1e7, 0xb49fc06d, 0xb7143e8f, 0xe0b4f2b0, 0xc5523a5c},
    {0x985e929f, 0x70af28d0, 0xbdd1a90a, 0x808f977f, 0x597c7c77, 0x8c489e98, 0xd3bd8910, 0xd31ac0f7},
    {0xc6f67e02, 0xe6e4e1bd, 0xefb994c6, 0x098953f3, 0x4636ba2b, 0x6ca20a47, 0x21d2b26a, 0x886722ff},
    {0x1c9a7e5f, 0xf1cf48b4, 0xad1582d3, 0xf4e4a100, 0x4f3b20d8, 0xc5a2b713, 0x87a4254a, 0xd933ebc5},
    {0x2f075ae2, 0x29646b6f, 0x6aed19a5, 0xe372cf29, 0x5081401e, 0xb893ff59, 0x9b3f9acc, 0x0c0d3e7d},
    {0x328921de, 0xb5961207, 0x6801e8cd, 0x61592107, 0xb5c67c79, 0xb846595c, 0xc6320c39, 0x5b46362c},
    {0xbfb909fd, 0xb236ad24, 0x11b4e488, 0x3810a074, 0xb8404646, 0x89986c3f, 0x8a809182, 0x7e17c327},
    {0x55d8fb36, 0x87ba3ba4, 0x9f342c77, 0xf5a1f89b, 0xec83d811, 0x446e1a46, 0x7139213d, 0x640b6a74},
    {0xf7210d4f, 0x8e7e1039, 0x790e7bf4, 0xefa20755, 0x5a10a6db, 0x1dd4b95d, 0xa313aaa8, 0x8b88fe76},
    {0xad21b516, 0xcbc645ff, 0xe34ab5de, 0x1c8aef8c, 0xd4e7f8d2, 0xb51e8e14, 0x56adc756, 0x3cda206f},
    {0x6bfe8d2b, 0xcc4237b7, 0x4a504705, 0x8ef45533, 0x9ecd7360, 0xcb63bfbb, 0x8ee5448e, 0x6430ba04},
    {0xa7f23ce9, 0x181740dc, 0x220c8147, 0x82654fee, 0x6aceb9f1, 0xec9222c4, 0xe2467d0a, 0xb1680837},
    {0xaef9476c, 0x89590a2c, 0x8cc9b3b7, 0x4f4967c7, 0x57c49d98, 0x66a44bac, 0xf21fa2ed, 0x675ddfa2},
    {0x9a42bcad, 0x82f6a9e4, 0x1284d808, 0xead319f2, 0x9f3b0820, 0x9d680f0e, 0x2ce71510, 0xd071e205},
    {0xd1a66d35, 0x4a67b9cf, 0x179571d8, 0xe5f97792, 0x716e8dd4, 0xec441968, 0x39a3f7c6, 0xb74f8bac},
    {0xfafa3025, 0xf2f89509, 0xc2c71c74, 0xfba0cd92, 0x858ef49b, 0x0780fb54, 0x79746c8a, 0x9bfcb346},
    {0x3334a7c1, 0xe7f6705a, 0xa6011a6a, 0x94964501, 0x6db4acde, 0x0ca9abd6, 0x6dc79d82, 0x66423056},
    {0x0796fd75, 0x664faef7, 0x44ee4e52, 0xd7271e2b, 0xbb769f91, 0xed6f9b74, 0xd8b694f5, 0x6606852c},
    {0x7ba3ae4a, 0x417fe854, 0x5b142bc8, 0x9f4adcd7, 0xae13941c, 0xbab7750b, 0x83e9f0a6, 0x6d16be64},
    {0x788fafcc, 0x4aa52039, 0x9adbaed1, 0x95f8b12c, 0x4eb31ec1, 0x0168e50a, 0xabc659a6, 0xaea516dc},
    {0xe833d7a6, 0x7160e68b, 0xf4c9044a, 0x53077df2, 0x727ad00c, 0xf36f4949, 0xc7b681a9, 0x12140cbb},
    {0x309eabf0, 0x95dc6714, 0xf9f4d864, 0xbba5affa, 0xe0b35ae2, 0xf5e3565b, 0xcc3a47b2, 0x12767701},
    {0x226a8ebe, 0xfa288665, 0xa644a502, 0x73335efb, 0xb610510f, 0x241b5b72, 0x0c8a368d, 0x59a69a5d},
    {0x41abfd99, 0x54258276, 0x25938131, 0xaf0c4f33, 0xfe0bd468, 0x8c222c21, 0xfa9da8e8, 0x9caa03f8},
    {0x442c642e, 0xf50fa1a6, 0x67a6e6d1, 0x05c77c5c, 0xc3fec8d7, 0xaa2570cf, 0x1a3077b5, 0x03c38069},
    {0xa0a08dfc, 0x9b42d96c, 0x2de19b6d, 0x127b8ae1, 0x36ddcf3e, 0x5ad0dce4, 0x22c45a56, 0xf61f6a74},
    {0x7d348382, 0xaf096dbe, 0x0bf086c7, 0xbb39b2a2, 0xc0bc36b6, 0x21ab0c73, 0x8e9885d7, 0x31d81740},
    {0x3ab13475, 0x1d191269, 0x026c8699, 0x4eaa8b43, 0xa83b4ad1, 0xf6d0e773, 0x81c4e297, 0x4afbc8f6},
    {0x9a745261, 0x1db2d23e, 0xae26f9bd, 0xbb88958e, 0xf44c64d0, 0xfe987be9, 0xf726adf9, 0x38f50f6c},
    {0x725c7f81, 0x6037bfe4, 0x52cd1e7b, 0xa35ac47e, 0xdcb49a9a, 0x2b27aeca, 0x70dce483, 0xcb7ded1f},
    {0x2cea1af5, 0x1fb28b62, 0x887c3999, 0x8ac9fef4, 0xdfdeda1f, 0x07e071ba, 0x558a173a, 0xfd06cbc3},
    {0xff1d59f9, 0x8b6c551d, 0x95089357, 0x057d5c8b, 0xe2640227, 0x9e9df0b1, 0xdf1a10b7, 0x2bf3927f},
    {0x2f8a181f, 0x7c99dd21, 0x5a7529bf, 0xe296a960, 0x3a144673, 0x7186d21a, 0xeb8bc7ae, 0x59e1fd21},
    {0xecc502c9, 0xb1145f39, 0x50cb7d3e, 0x3842446f, 0x81a4f0df, 0x1df537ce, 0xe139ef64, 0xea984bd9},
};

CDEV void sha256_rounds_kw(uint32_t h[8], const uint32_t* kw) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    const uint32_t t1 = hh + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + kw[i];
    const uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// SHA-256(a || b) for two 32-byte digests (state words, big-endian): the
// Merkle node hash.
CDEV void sha256_node(uint32_t out[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    w[i] = a[i];
    w[8 + i] = b[i];
  }
  sha256_init(out);
  sha256_block(out, w);
  sha256_rounds_kw(out, kPadKW);
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
  uint32_t z[8];  // Z_level
  for (int level = 0; m > 1; level++) {
    const uint64_t half = (m + 1) / 2;
    if (m & 1) {  // the last real node pairs with the padding constant Z_level
#pragma unroll
      for (int k = 0; k < 8; k++) z[k] = kZeroHash[level][k];
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
