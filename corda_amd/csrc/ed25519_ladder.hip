// Ed25519 verification ladder for gfx950 — second kernel of K1.
//
// Per lane (record written by ed25519_prep_half_kernel, ed25519.hip): decide
//   [e]B + [c0](+-A) + [c1](-R) == O
// with |c0|, c1 ~ 2^128 (c0 == c1 h mod 8L, c1 odd) and e = c1 S_eff mod L: the
// i2p 0.2.0 cofactorless check encode([S]B - [h]A) == R rewritten over
// half-size scalars (T. Pornin, ePrint 2020/454; the equivalence argument is in
// ed25519.hip above half_scalars). 4-bit Booth windows over the per-lane
// [0..8](-A), [0..8](-R) tables (gathered from the workspace one window ahead,
// so the four doublings hide the load), 16-bit Booth windows over B and
// B' = [2^128]B from L2/MALL-resident tables (ed25519_ws.hpp). Digit positions are the same in every lane, so the
// ladder never diverges; P == O is X == 0 and Y == Z (no inversion).
// Verdict word per wave by ballot.
// field products in hand-scheduled pairs (ge25519.hpp fe_mul_pair, fe25519_asm.hpp)
#ifndef FE_USE_ASM2
#define FE_USE_ASM2 1
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ed25519_ws.hpp"
#include "status.hpp"

namespace cordahip {

__device__ __attribute__((aligned(64))) const uint32_t kIdentityCached[kWhEntryWords] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0,   // Y + X
                                                            1, 0, 0, 0, 0, 0, 0, 0, 0, 0,   // Y - X
                                                            1, 0, 0, 0, 0, 0, 0, 0, 0, 0,   // Z
                                                            0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // 2dT

// booth_digit (sc25519.hpp) over a scalar stored word-major in LDS: word w of
// this thread's scalar at col[w * 256]
template <int W>
CDEV int booth_digit_col(const uint32_t* col, int j) {
  const int lo = W * j - 1;  // may be -1
  uint32_t v;
  if (lo < 0) {
    v = (col[0] << 1) & ((1u << (W + 1)) - 1);
  } else {
    const int w = lo >> 5, sh = lo & 31;
    const uint64_t hi = w + 1 <= 7 ? col[(w + 1) * 256] : 0u;
    v = (uint32_t)(((hi << 32) | col[w * 256]) >> sh) & ((1u << (W + 1)) - 1);
  }
  return (int)((v + 1) >> 1) - (int)((v >> W) << W);
}

// waves per SIMD the register allocation targets (2: up to 256 VGPRs)
#ifndef ED_LADDER_WAVES
#define ED_LADDER_WAVES 2
#endif
// the generated asm blocks (fe25519_asm.hpp) clobber the fixed accumulator
// VGPRs v160..v167, so the kernel needs a budget of >= 168 VGPRs: 512 / waves
static_assert(512 / ED_LADDER_WAVES >= 168, "fe25519_asm.hpp's v160..v167 accumulators need >= 168 VGPRs per lane");

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ED_LADDER_WAVES))) ed25519_ladder_half_kernel(
    uint64_t base, uint64_t m, const uint32_t* __restrict__ btab, const uint32_t* __restrict__ ws,
    uint8_t* __restrict__ status, unsigned long long* __restrict__ verdict) {
  const uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = li < m;
  const uint64_t lc = active ? li : m - 1;  // inactive lanes replay the last record, discard it
  const uint32_t* rec = ws + lc * kWhLaneWords;
  // |c0|, c1 and e live in LDS (word-major, one column per thread): each window
  // reads two words of each, and the 24 VGPRs they would pin across the loop
  // go to the group formulas' wider product blocks instead
  __shared__ uint32_t sk[24][256];
  const uint32_t* ska = &sk[0][threadIdx.x];
  const uint32_t* skr = &sk[8][threadIdx.x];
  const uint32_t* ske = &sk[16][threadIdx.x];
  int bits;
  {
    uint32_t ka[8], kr[8], e[8];
    load8(ka, rec + kWhKa);
    load8(kr, rec + kWhKr);
    load8(e, rec + kWhE);
#pragma unroll
    for (int q = 0; q < 8; q++) {
      sk[q][threadIdx.x] = ka[q];
      sk[8 + q][threadIdx.x] = kr[q];
      sk[16 + q][threadIdx.x] = e[q];
    }
    bits = max(mp8_bitlen(ka), mp8_bitlen(kr));
  }
  const bool c0neg = rec[kWhFlags] & 1u;  // [c0](-A) with c0 < 0 is [|c0|]A: flip the digit signs
  // at least the windows the fixed-base digits need (e's low half: kBDigits
  // digits of kBBits bits); |c0|, c1 ~ 2^128 give 33
  const int W = max(wave_max((bits + 1 + 3) / 4), (kBDigits - 1) * (kBBits / 4) + 1);
  const uint32_t* btab2 = btab + kBTableEntries * kBEntryWords;
  ge_p3 P;
  ge_identity(P);
  for (int j = W - 1; j >= 0; j--) {
    const int da = booth_digit_col<4>(ska, j), dr = booth_digit_col<4>(skr, j);
    ge_cached ca, cr;  // issued before the doublings, consumed after them
    load_cached(ca, table_entry(rec + kWhTabA, da < 0 ? -da : da));
    load_cached(cr, table_entry(rec + kWhTabR, dr < 0 ? -dr : dr));
    if (j != W - 1) {
      ge_dbl<false>(P, P);
      ge_dbl<false>(P, P);
      ge_dbl<false>(P, P);
      ge_dbl<true>(P, P);
    }
    cached_cneg(ca, (da < 0) != c0neg);
    ge_add<true>(P, P, ca);
    // fixed-base window: the L2 gather of each niels entry is issued one
    // addition ahead of its use (registers allow no more)
    // (W is the wave's maximum and may exceed 33: the low half's windows end at
    // digit kBDigits - 1, the high half's digits ride on B')
    const bool bwin = j % (kBBits / 4) == 0 && j < kBDigits * (kBBits / 4);
    cached_cneg(cr, dr < 0);
    if (bwin) {
      const int d0 = booth_digit_col<kBBits>(ske, j / (kBBits / 4));
      const int d1 = booth_digit_col<kBBits>(ske, j / (kBBits / 4) + kBDigits);
      ge_niels nb0, nb1;
      load_niels(nb0, btab, d0 < 0 ? -d0 : d0);
      ge_add<true>(P, P, cr);
      load_niels(nb1, btab2, d1 < 0 ? -d1 : d1);
      niels_cneg(nb0, d0 < 0);
      ge_madd<true>(P, P, nb0);
      niels_cneg(nb1, d1 < 0);
      ge_madd<false>(P, P, nb1);
    } else {
      ge_add<false>(P, P, cr);
    }
  }
  fe d;
  fe_sub(d, P.Y, P.Z);
  const bool zero = fe_iszero(P.X) && fe_iszero(d);
  const uint64_t i = base + li;
  uint8_t st = kStatusBadSig;
  if (active) {
    st = status[i];
    if (st == kStatusPending) {
      st = zero ? kStatusOk : kStatusBadSig;
      status[i] = st;
    }
  }
  const unsigned long long ok = __ballot(active && st == kStatusOk);
  // base is a multiple of 64 (workspace chunks are), so lane 0 of a wave owns a whole verdict word
  if ((threadIdx.x & 63) == 0 && active && verdict) verdict[i >> 6] = ok;
}

hipError_t launch_ed25519_ladder(uint64_t base, uint64_t m, const uint32_t* btab, const uint32_t* ws, uint8_t* status,
                                 unsigned long long* verdict, hipStream_t s) {
  const uint32_t blocks = (uint32_t)((m + 255) / 256);
  hipLaunchKernelGGL(ed25519_ladder_half_kernel, dim3(blocks), dim3(256), 0, s, base, m, btab, ws, status, verdict);
  return hipGetLastError();
}

}  // namespace cordahip
