// Shared layout of the Ed25519 split verification (kernel K1): the fixed-base
// table, the per-lane HBM workspace record prep writes and the ladder reads,
// and the point helpers both translation units use.
//
//   ed25519.hip         prep: i2p decode of A, strict decode of R, SHA-512,
//                       h mod L, S_eff, lattice reduction -> workspace record
//   ed25519_ladder.hip  ladder: [e]B + [c0](+-A) + [c1](-R) == O, verdict ballot
//
// The two live in separate translation units, each register-allocated for its
// own shape: prep is dominated by the two decompressions' square chains (run as
// one paired chain), the ladder by the group formulas' independent products;
// both issue those products as generated asm pairs (fe25519_asm.hpp).
#pragma once
#include "fe25519.hpp"
#include "ge25519.hpp"
#include "sc25519.hpp"

namespace cordahip {

// B tables for Booth windows of kBBits over e = e_lo + 2^128 e_hi: entry k
// (0..2^15) = [k]B as affine niels (y+x, y-x, 2d*x*y), 32 u32 per entry (30
// limbs + 2 pad); entries [kBTableEntries, 2 kBTableEntries) = [k]B',
// B' = [2^(kBDigits kBBits)]B = [2^128]B. 2 x 4.2 MB, L2/MALL-resident. 16-bit
// windows give 16 fixed-base additions per verification (12-bit: 22, 8-bit
// from LDS: 32; profiles/r02_c2_bwin12_ab.json); the window is a multiple of
// the ladder's 4-bit one so both share the doublings.
static constexpr int kBBits = 16;
static constexpr int kBDigits = 8;  // per half: 8 x 16 = 128 bits
static constexpr int kBTableEntries = (1 << (kBBits - 1)) + 1;
static constexpr int kBEntryWords = 32;
static constexpr uint8_t kStatusPending = 0xff;

// Per-lane workspace record (3,200 B = 50 x 64 B, so every record and every
// entry starts on a 64-B sector): entries [1..8](-A), [1..8](-R) in cached form
// (40 words) padded to 48 words, so a gather of one entry reads exactly three
// 64-B sectors (at 40-word stride an entry straddled 3-4 sectors and 2-3
// 128-B lines). Digit 0 gathers the shared identity entry kIdentityCached
// (L2-resident) instead of a per-lane copy.
static constexpr int kWhEntryWords = 48;
static constexpr int kWhTabA = 0;                       // [k](-A) at (k - 1) * kWhEntryWords, k = 1..8
static constexpr int kWhTabR = 8 * kWhEntryWords;       // [k](-R)
static constexpr int kWhKa = 16 * kWhEntryWords;        // |c0|, c1, e (8 words each)
static constexpr int kWhKr = kWhKa + 8;
static constexpr int kWhE = kWhKa + 16;
static constexpr int kWhFlags = kWhKa + 24;             // bit 0: c0 < 0
static constexpr int kWhLaneWords = kWhKa + 32;         // 800 words
static_assert(kWhLaneWords % 16 == 0, "records must start on 64-B sectors");

// the identity in cached form (Y+X, Y-X, Z, 2dT) = (1, 1, 1, 0), entry 0 of
// every per-lane table (defined in ed25519_ladder.hip)
extern __device__ const uint32_t kIdentityCached[kWhEntryWords];

// entry |d| of a per-lane table (tab = rec + kWhTabA or kWhTabR)
CDEV const uint32_t* table_entry(const uint32_t* tab, int absd) {
  return absd == 0 ? kIdentityCached : tab + (absd - 1) * kWhEntryWords;
}

CDEV void load_niels(ge_niels& n, const uint32_t* __restrict__ tab, int idx) {
  const uint4* e = reinterpret_cast<const uint4*>(tab + idx * kBEntryWords);
  uint32_t w[32];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint4 v = e[q];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 10; i++) {
    n.ypx.v[i] = w[i];
    n.ymx.v[i] = w[10 + i];
    n.xy2d.v[i] = w[20 + i];
  }
}

// conditional negation of a niels / cached point: swap (y+x, y-x), negate t
CDEV void niels_cneg(ge_niels& n, bool neg) {
  fe nt;
  fe_neg_loose(nt, n.xy2d);  // 2x: only ever the g-operand of fe_mul
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const uint32_t a = n.ypx.v[i], b = n.ymx.v[i];
    n.ypx.v[i] = neg ? b : a;
    n.ymx.v[i] = neg ? a : b;
    n.xy2d.v[i] = neg ? nt.v[i] : n.xy2d.v[i];
  }
}
CDEV void cached_cneg(ge_cached& c, bool neg) {
  fe nt;
  fe_neg_loose(nt, c.T2d);
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const uint32_t a = c.YpX.v[i], b = c.YmX.v[i];
    c.YpX.v[i] = neg ? b : a;
    c.YmX.v[i] = neg ? a : b;
    c.T2d.v[i] = neg ? nt.v[i] : c.T2d.v[i];
  }
}

CDEV void store_cached(uint32_t* __restrict__ o, const ge_cached& c) {
  uint4* o4 = reinterpret_cast<uint4*>(o);
  uint32_t w[40];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    w[i] = c.YpX.v[i];
    w[10 + i] = c.YmX.v[i];
    w[20 + i] = c.Z.v[i];
    w[30 + i] = c.T2d.v[i];
  }
#pragma unroll
  for (int q = 0; q < 10; q++) o4[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  // the pad too: whole 64-B sectors, no partial-sector writes
  o4[10] = o4[11] = make_uint4(0u, 0u, 0u, 0u);
}

CDEV void load_cached(ge_cached& c, const uint32_t* __restrict__ p) {
  const uint4* p4 = reinterpret_cast<const uint4*>(p);
  uint32_t w[40];
#pragma unroll
  for (int q = 0; q < 10; q++) {
    const uint4 v = p4[q];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 10; i++) {
    c.YpX.v[i] = w[i];
    c.YmX.v[i] = w[10 + i];
    c.Z.v[i] = w[20 + i];
    c.T2d.v[i] = w[30 + i];
  }
}

CDEV void store8(uint32_t* __restrict__ o, const uint32_t v[8]) {
  uint4* o4 = reinterpret_cast<uint4*>(o);
  o4[0] = make_uint4(v[0], v[1], v[2], v[3]);
  o4[1] = make_uint4(v[4], v[5], v[6], v[7]);
}
CDEV void load8(uint32_t v[8], const uint32_t* __restrict__ p) {
  const uint4* p4 = reinterpret_cast<const uint4*>(p);
  const uint4 a = p4[0], b = p4[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

CDEV int mp8_bitlen(const uint32_t a[8]) {
  int n = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) n = a[i] ? 32 * i + 32 - __builtin_clz(a[i]) : n;
  return n;
}

CDEV int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}

// stops the machine scheduler from interleaving the phases on either side
// (independent phases interleaved = both phases' registers live at once)
#define PHASE_BARRIER() __builtin_amdgcn_sched_barrier(0)

// host-side launcher of the ladder (ed25519_ladder.hip)
hipError_t launch_ed25519_ladder(uint64_t base, uint64_t m, const uint32_t* btab, const uint32_t* ws, uint8_t* status,
                                 unsigned long long* verdict, hipStream_t s);

}  // namespace cordahip
