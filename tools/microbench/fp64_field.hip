// FP64-FMA field products for the two base fields of the hot path (VERDICT r03
// item 5: a bounded A/B of the one lever the integer kernels have not tried).
//
// v_fma_f64 issues at the v_mad_u64_u32 rate on gfx950 (profiles/r01_int_rates.jsonl),
// and a 53-bit significand carries more bits per multiply than the 29-bit or
// 25.5-bit integer limbs. An EXACT limb product needs its rounding error too:
//   T' = fma(a, b, T)   the running column sum T, kept in the binade
//                       [2^95, 2^96) whose ulp is the limb radix 2^43, rounded
//   D  = T - T'         exact (same binade)
//   l  = fma(a, b, D)   = a*b - (T' - T): the rounding error, exact, |l| <= 2^42
//   L += l              the column's low part, exact (|L| < 2^53)
// -- four FP64 VALU instructions per 43x43-bit limb product (three for a
// column's first). Radix 2^43 x 6 limbs (258 bits) leaves the headroom the
// 53-bit significand needs (radix 2^51 x 5 does not: a 5-product column of
// 102-bit products overflows the binade whose ulp is 2^51).
//
//   f6_mul  GF(2^255-19): 36 products -> 11 columns (T, L) -> 12 signed limbs
//           -> carry the high half (magic-number rounding) -> fold x152
//           (2^258 = 8 * 19 mod p) -> carry the low half -> 6 signed limbs
//           |r| <= 2^42 + 2^15, valid inputs of the next product
//   f6_sq   the same with 21 products (cross terms through 2a_i)
//   p6_cols the P-256 product WITHOUT any reduction (36 products -> 12 limbs):
//           a lower bound for an FP64 P-256 product, to set against the
//           complete radix-2^29 asm product + REDC (152 instructions)
// The integer fe_mul / fe_sq of corda_amd/csrc/fe25519.hpp run in the same
// harness. Output: JSON lines (ps per field op at full occupancy), then, for
// the correctness check (tools/microbench/fp64_field_check.py), the inputs and
// outputs of the first 512 lanes of one f6_mul and one f6_sq as hex.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../corda_amd/csrc/fe25519.hpp"

using namespace cordahip;

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e = (x);                                                                       \
    if (e != hipSuccess) {                                                                    \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);         \
      return 1;                                                                               \
    }                                                                                         \
  } while (0)

struct f6 {
  double v[6];
};

#define FD __device__ __forceinline__
constexpr double kCT = 0x1.8p95;       // 1.5 * 2^95: column sums stay in [2^95, 2^96), ulp 2^43
constexpr double kRound = 0x1.8p95;    // magic for rounding a |x| < 2^52 limb to a multiple of 2^43
constexpr double kInv43 = 0x1p-43;
constexpr double kK = 0x1.8p52;        // CT * 2^-43: pre-subtracted from L so r = fma(T, 2^-43, L)

// 11 columns of a 6x6 product (the a_i b_j with i + j = k) as (T_k, L_k)
template <int NI>
FD void columns(const double* a, const double* b, double* T, double* L) {
#pragma unroll
  for (int k = 0; k < 11; k++) {
    T[k] = kCT;
    L[k] = -kK;
  }
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int j = 0; j < 6; j++) {
      if (NI == 1 && j < i) continue;  // squaring: cross terms once, a already doubled off the diagonal
      const double x = (NI == 1 && j != i) ? a[i] * 2.0 : a[i];
      const double t1 = __fma_rn(x, b[j], T[i + j]);
      const double d = T[i + j] - t1;
      L[i + j] += __fma_rn(x, b[j], d);
      T[i + j] = t1;
    }
}

// r (12 signed limbs, radix 2^43) from the columns: r_k = L_k + (T_{k-1} - CT) 2^-43
FD void normalize(const double* T, const double* L, double* r) {
  r[0] = L[0] + kK;
#pragma unroll
  for (int k = 1; k < 11; k++) r[k] = __fma_rn(T[k - 1], kInv43, L[k]);
  r[11] = __fma_rn(T[10], kInv43, -kK);
}

// one carry step: x -> x - q, next += q 2^-43 (q = x rounded to a multiple of 2^43)
FD void carry(double& x, double& next) {
  const double q = (x + kRound) - kRound;
  x -= q;
  next = __fma_rn(q, kInv43, next);
}

FD void reduce25519(double* r, f6& out) {
  double top = 0.0;
#pragma unroll
  for (int k = 6; k < 11; k++) carry(r[k], r[k + 1]);
  carry(r[11], top);  // weight 2^516 = 152^2 mod p
#pragma unroll
  for (int k = 0; k < 6; k++) r[k] = __fma_rn(152.0, r[k + 6], r[k]);
  r[0] = __fma_rn(23104.0, top, r[0]);
  double c = 0.0;
#pragma unroll
  for (int k = 0; k < 5; k++) carry(r[k], r[k + 1]);
  carry(r[5], c);
  r[0] = __fma_rn(152.0, c, r[0]);
#pragma unroll
  for (int k = 0; k < 6; k++) out.v[k] = r[k];
}

FD void f6_mul(f6& o, const f6& a, const f6& b) {
  double T[11], L[11], r[12];
  columns<0>(a.v, b.v, T, L);
  normalize(T, L, r);
  reduce25519(r, o);
}

FD void f6_sq(f6& o, const f6& a) {
  double T[11], L[11], r[12];
  columns<1>(a.v, a.v, T, L);
  normalize(T, L, r);
  reduce25519(r, o);
}

// P-256 product columns only (no reduction): 12 signed limbs folded into 6 by
// plain addition so the chain stays bounded -- NOT a field product, a cost probe
FD void p6_cols(f6& o, const f6& a, const f6& b) {
  double T[11], L[11], r[12];
  columns<0>(a.v, b.v, T, L);
  normalize(T, L, r);
#pragma unroll
  for (int k = 0; k < 6; k++) o.v[k] = (r[k] + r[k + 6]) * 0x1p-6;  // keep magnitudes in range
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
f6_chain(const double* __restrict__ in, double* __restrict__ out, int iters, int kind) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const double* p = in + i * 24;
  f6 a, b, c, d;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    a.v[k] = p[k];
    b.v[k] = p[6 + k];
    c.v[k] = p[12 + k];
    d.v[k] = p[18 + k];
  }
  for (int it = 0; it < iters; it++) {  // 4 independent chains, as the integer harness
    if (kind == 0) {
      f6_mul(a, a, b);
      f6_mul(b, b, c);
      f6_mul(c, c, d);
      f6_mul(d, d, a);
    } else if (kind == 1) {
      f6_sq(a, a);
      f6_sq(b, b);
      f6_sq(c, c);
      f6_sq(d, d);
    } else {
      p6_cols(a, a, b);
      p6_cols(b, b, c);
      p6_cols(c, c, d);
      p6_cols(d, d, a);
    }
  }
  double* o = out + i * 24;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    o[k] = a.v[k];
    o[6 + k] = b.v[k];
    o[12 + k] = c.v[k];
    o[18 + k] = d.v[k];
  }
}

// single products for the correctness check: out = a * b, out2 = a^2
__global__ void f6_once(const double* __restrict__ in, double* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  f6 a, b, m, s;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    a.v[k] = in[i * 24 + k];
    b.v[k] = in[i * 24 + 6 + k];
  }
  f6_mul(m, a, b);
  f6_sq(s, a);
#pragma unroll
  for (int k = 0; k < 6; k++) {
    out[i * 12 + k] = m.v[k];
    out[i * 12 + 6 + k] = s.v[k];
  }
}

CDEV void ld_fe(fe& a, const uint32_t* p) {
#pragma unroll
  for (int i = 0; i < 10; i++) a.v[i] = p[i];
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
int_chain(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int iters, int kind) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t* p = in + i * 40;
  fe a, b, c, d;
  ld_fe(a, p);
  ld_fe(b, p + 10);
  ld_fe(c, p + 20);
  ld_fe(d, p + 30);
  for (int it = 0; it < iters; it++) {
    if (kind == 0) {
      fe_mul(a, a, b);
      fe_mul(b, b, c);
      fe_mul(c, c, d);
      fe_mul(d, d, a);
    } else {
      fe_sq(a, a);
      fe_sq(b, b);
      fe_sq(c, c);
      fe_sq(d, d);
    }
  }
  uint32_t* o = out + i * 40;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    o[k] = a.v[k];
    o[10 + k] = b.v[k];
    o[20 + k] = c.v[k];
    o[30 + k] = d.v[k];
  }
}

template <class K, class T>
static int timed(const char* name, K kern, const T* din, T* dout, int lanes, int iters, int kind) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(lanes / 256), dim3(256), 0, 0, din, dout, 2, kind);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(lanes / 256), dim3(256), 0, 0, din, dout, iters, kind);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  const double ps = best * 1e9 / ((double)lanes * iters * 4);
  printf("{\"bench\": \"%s\", \"lanes\": %d, \"iters\": %d, \"ms\": %.3f, \"ps_per_field_op\": %.3f}\n", name, lanes,
         iters, best, ps);
  return 0;
}

int main(int argc, char** argv) {
  const int lanes = 1 << 20, iters = argc > 1 ? atoi(argv[1]) : 256;
  uint64_t s = 0x9E3779B97F4A7C15ull;
  auto rnd = [&]() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  };
  double* hf = (double*)malloc((size_t)lanes * 24 * 8);
  for (size_t i = 0; i < (size_t)lanes * 24; i++) hf[i] = (double)(rnd() & ((1ull << 43) - 1));  // 43-bit limbs
  uint32_t* hi = (uint32_t*)malloc((size_t)lanes * 40 * 4);
  for (size_t i = 0; i < (size_t)lanes * 40; i++) hi[i] = (uint32_t)rnd() & (((i % 10) & 1) ? M25 : M26);
  double *df, *dfo;
  uint32_t *di, *dio;
  CHECK(hipMalloc(&df, (size_t)lanes * 24 * 8));
  CHECK(hipMalloc(&dfo, (size_t)lanes * 24 * 8));
  CHECK(hipMalloc(&di, (size_t)lanes * 40 * 4));
  CHECK(hipMalloc(&dio, (size_t)lanes * 40 * 4));
  CHECK(hipMemcpy(df, hf, (size_t)lanes * 24 * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(di, hi, (size_t)lanes * 40 * 4, hipMemcpyHostToDevice));
  if (timed("int_fe_mul_radix25.5", int_chain, di, dio, lanes, iters, 0)) return 1;
  if (timed("int_fe_sq_radix25.5", int_chain, di, dio, lanes, iters, 1)) return 1;
  if (timed("fp64_f6_mul_radix43", f6_chain, df, dfo, lanes, iters, 0)) return 1;
  if (timed("fp64_f6_sq_radix43", f6_chain, df, dfo, lanes, iters, 1)) return 1;
  if (timed("fp64_p256_product_columns_only", f6_chain, df, dfo, lanes, iters, 2)) return 1;
  // correctness sample: the first 512 lanes' a, b (limbs 0..11 of the input) and a*b, a^2
  const int n = 512;
  hipLaunchKernelGGL(f6_once, dim3(n / 256), dim3(256), 0, 0, df, dfo, n);
  CHECK(hipDeviceSynchronize());
  double* ho = (double*)malloc((size_t)n * 12 * 8);
  CHECK(hipMemcpy(ho, dfo, (size_t)n * 12 * 8, hipMemcpyDeviceToHost));
  for (int i = 0; i < n; i++) {
    printf("CHK");
    for (int k = 0; k < 12; k++) printf(" %.17g", hf[i * 24 + k]);
    for (int k = 0; k < 12; k++) printf(" %.17g", ho[i * 12 + k]);
    printf("\n");
  }
  return 0;
}
