// Radix 2^32 vs radix 2^29 field products on gfx950: a
// bounded A/B of the P-256 base-field product the ECDSA ladder spends ~70% of
// its issue cycles in, and of GF(2^255-19) at radix 2^32.
//
//   r29_mul / r29_sqr   the production products: fp29_asm.hpp f29a_mul_r1 /
//                       f29a_sqr_r1 (radix 2^29 x 9 limbs, Montgomery, special
//                       REDC: 81 / 45 operand MACs + 36 REDC MACs, one asm chain)
//   p32_mul / p32_sqr   radix 2^32 x 8 limbs: product scanning with a 3-word
//                       column accumulator, each MAC a v_mad_u64_u32 whose carry
//                       out (VCC) a v_addc_co_u32 counts (64 MACs; squaring: 28
//                       cross MACs, one doubling pass, 8 diagonal MACs), then
//                       NIST's word-aligned reduction (FIPS 186-4 D.2.3: the
//                       s1 + 2 s2 + 2 s3 + s4 + s5 - s6 - s7 - s8 - s9 word sums
//                       in signed 64-bit, a carry pass, the top folded with
//                       2^256 == 2^224 - 2^192 - 2^96 + 1, a final pass): value
//                       < 2p (a lazy output, as r29's)
//   q32_mul             GF(2^255-19) radix 2^32 x 8: the same 64-MAC product,
//                       the high half folded with 38 (8 MACs) and 2^256 == 38
//                       again, output < 2^256 (lazy)
//   fe_mul              the production GF(2^255-19) product (fe25519.hpp, radix
//                       2^25.5 x 10, 100 MACs)
// Timing: 4 independent chains per lane (x = x*y round robin), 2^20 lanes, 2
// waves per SIMD, as tools/microbench/fp64_field.hip. Output: one JSON line
// per variant, then CHK lines (the first 512 lanes' operands and one product /
// square of each radix-32 variant) that tools/microbench/radix32_ab.py checks
// against Python integers.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../corda_amd/csrc/fe25519.hpp"
#include "../../corda_amd/csrc/fp29_asm.hpp"

using namespace cordahip;

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

struct w8 {
  uint32_t v[8];
};

// acc (64 bits) + a b, the carry out of bit 64 counted in c
CDEV void mac(uint64_t& acc, uint32_t& c, uint32_t a, uint32_t b) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(c)
      : "v"(a), "v"(b)
      : "vcc");
}

// 512-bit product, 16 words (product scanning)
CDEV void mul512(uint32_t* w, const w8& a, const w8& b) {
  uint64_t acc = 0;
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int j = (k > 7 ? k - 7 : 0); j <= (k < 7 ? k : 7); j++) mac(acc, c, a.v[j], b.v[k - j]);
    w[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c << 32);
    c = 0;
  }
  w[15] = (uint32_t)acc;
}

// 512-bit square: cross products once, doubled by one shift pass, + diagonals
CDEV void sqr512(uint32_t* w, const w8& a) {
  uint32_t x[16];
  uint64_t acc = 0;
  uint32_t c = 0;
  x[0] = 0;
#pragma unroll
  for (int k = 1; k < 14; k++) {
#pragma unroll
    for (int j = (k > 7 ? k - 7 : 0); 2 * j < k; j++) mac(acc, c, a.v[j], a.v[k - j]);
    x[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c << 32);
    c = 0;
  }
  x[14] = (uint32_t)acc;
  x[15] = (uint32_t)(acc >> 32);
  // 2x + diagonals, one carry chain
  uint32_t prev = 0;
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    const uint64_t d = (uint64_t)a.v[k / 2] * a.v[k / 2];
    const uint32_t x0 = __builtin_amdgcn_alignbit(x[k], prev, 31), x1 = __builtin_amdgcn_alignbit(x[k + 1], x[k], 31);
    prev = x[k + 1];
    const uint64_t s0 = carry + x0 + (uint32_t)d;
    const uint64_t s1 = (s0 >> 32) + x1 + (d >> 32);
    w[k] = (uint32_t)s0;
    w[k + 1] = (uint32_t)s1;
    carry = s1 >> 32;
  }
}

// P-256: p = 2^256 - 2^224 + 2^192 + 2^96 - 1 (words, little-endian)
__constant__ uint32_t kP[8] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0, 0, 0, 1, 0xffffffffu};

// NIST fast reduction of a 512-bit c (16 words) to < 2p
CDEV void nist_p256_reduce(w8& r, const uint32_t* c) {
  int64_t t[8];
  const int64_t C[16] = {c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7],
                         c[8], c[9], c[10], c[11], c[12], c[13], c[14], c[15]};
  t[0] = C[0] + C[8] + C[9] - C[11] - C[12] - C[13] - C[14];
  t[1] = C[1] + C[9] + C[10] - C[12] - C[13] - C[14] - C[15];
  t[2] = C[2] + C[10] + C[11] - C[13] - C[14] - C[15];
  t[3] = C[3] + 2 * C[11] + 2 * C[12] + C[13] - C[15] - C[8] - C[9];
  t[4] = C[4] + 2 * C[12] + 2 * C[13] + C[14] - C[9] - C[10];
  t[5] = C[5] + 2 * C[13] + 2 * C[14] + C[15] - C[10] - C[11];
  t[6] = C[6] + 3 * C[14] + 2 * C[15] + C[13] - C[8] - C[9];
  t[7] = C[7] + 3 * C[15] + C[8] - C[10] - C[11] - C[12] - C[13];
  // carry pass (signed); the top carry q in [-4, 7]
  int64_t q = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    t[i] += q;
    q = t[i] >> 32;  // arithmetic shift
    t[i] &= 0xffffffffll;
  }
  // fold q 2^256 == q (2^224 - 2^192 - 2^96 + 1), then one more pass
  t[0] += q;
  t[3] -= q;
  t[6] -= q;
  t[7] += q;
  q = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    t[i] += q;
    q = t[i] >> 32;
    t[i] &= 0xffffffffll;
  }
  // q in {-1, 0, 1}: add / subtract p once more (value then in [0, 2p))
  const int64_t sgn = q;
  q = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    t[i] += q - sgn * (int64_t)kP[i];
    q = t[i] >> 32;
    t[i] &= 0xffffffffll;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = (uint32_t)t[i];
}

CDEV void p32_mul(w8& r, const w8& a, const w8& b) {
  uint32_t w[16];
  mul512(w, a, b);
  nist_p256_reduce(r, w);
}
CDEV void p32_sqr(w8& r, const w8& a) {
  uint32_t w[16];
  sqr512(w, a);
  nist_p256_reduce(r, w);
}

// GF(2^255-19), radix 2^32: lo + 38 hi, then the top word again (output < 2^256)
CDEV void q32_mul(w8& r, const w8& a, const w8& b) {
  uint32_t w[16];
  mul512(w, a, b);
  uint64_t acc = 0;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc += w[i];
    mac(acc, c, w[8 + i], 38u);
    r.v[i] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c << 32);
    c = 0;
  }
  // acc < 39: fold once more (2^256 == 38); a final carry is absorbed (value < 2^256 after)
  uint64_t s = (uint64_t)r.v[0] + acc * 38;
  r.v[0] = (uint32_t)s;
#pragma unroll
  for (int i = 1; i < 8; i++) {
    s = (s >> 32) + r.v[i];
    r.v[i] = (uint32_t)s;
  }
  r.v[0] += (uint32_t)(s >> 32) * 38u;  // at most once, cannot carry again
}

template <class T>
CDEV void ld(T& a, const uint32_t* p, int n) {
#pragma unroll
  for (int i = 0; i < n; i++) a.v[i] = p[i];
}
template <class T>
CDEV void st(uint32_t* p, const T& a, int n) {
#pragma unroll
  for (int i = 0; i < n; i++) p[i] = a.v[i];
}

// kind: 0 r29_mul, 1 r29_sqr, 2 p32_mul, 3 p32_sqr, 4 q32_mul, 5 fe_mul (one
// kernel per kind, so each loop body's ISA can be counted by name)
template <int kind>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
chain(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int iters) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t* p = in + i * 40;
  uint32_t* o = out + i * 40;
  if constexpr (kind <= 1) {
    f29 a, b, c, d;
    ld(a, p, 9);
    ld(b, p + 10, 9);
    ld(c, p + 20, 9);
    ld(d, p + 30, 9);
    for (int it = 0; it < iters; it++) {
      if constexpr (kind == 0) {
        f29a_mul_r1(a, a, b);
        f29a_mul_r1(b, b, c);
        f29a_mul_r1(c, c, d);
        f29a_mul_r1(d, d, a);
      } else {
        f29a_sqr_r1(a, a);
        f29a_sqr_r1(b, b);
        f29a_sqr_r1(c, c);
        f29a_sqr_r1(d, d);
      }
    }
    st(o, a, 9);
    st(o + 10, b, 9);
    st(o + 20, c, 9);
    st(o + 30, d, 9);
  } else if constexpr (kind <= 4) {
    w8 a, b, c, d;
    ld(a, p, 8);
    ld(b, p + 10, 8);
    ld(c, p + 20, 8);
    ld(d, p + 30, 8);
    for (int it = 0; it < iters; it++) {
      if constexpr (kind == 2) {
        p32_mul(a, a, b);
        p32_mul(b, b, c);
        p32_mul(c, c, d);
        p32_mul(d, d, a);
      } else if constexpr (kind == 3) {
        p32_sqr(a, a);
        p32_sqr(b, b);
        p32_sqr(c, c);
        p32_sqr(d, d);
      } else {
        q32_mul(a, a, b);
        q32_mul(b, b, c);
        q32_mul(c, c, d);
        q32_mul(d, d, a);
      }
    }
    st(o, a, 8);
    st(o + 10, b, 8);
    st(o + 20, c, 8);
    st(o + 30, d, 8);
  } else {
    fe a, b, c, d;
    ld(a, p, 10);
    ld(b, p + 10, 10);
    ld(c, p + 20, 10);
    ld(d, p + 30, 10);
    for (int it = 0; it < iters; it++) {
      fe_mul(a, a, b);
      fe_mul(b, b, c);
      fe_mul(c, c, d);
      fe_mul(d, d, a);
    }
    st(o, a, 10);
    st(o + 10, b, 10);
    st(o + 20, c, 10);
    st(o + 30, d, 10);
  }
}

// one product / square per lane for the correctness check
__global__ void once(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  w8 a, b, m, s, q;
  ld(a, in + i * 40, 8);
  ld(b, in + i * 40 + 10, 8);
  p32_mul(m, a, b);
  p32_sqr(s, a);
  q32_mul(q, a, b);
  st(out + i * 24, m, 8);
  st(out + i * 24 + 8, s, 8);
  st(out + i * 24 + 16, q, 8);
}

template <int kind>
static int timed(const char* name, const uint32_t* din, uint32_t* dout, int lanes, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(chain<kind>, dim3(lanes / 256), dim3(256), 0, 0, din, dout, 2);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(chain<kind>, dim3(lanes / 256), dim3(256), 0, 0, din, dout, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  printf("{\"bench\": \"%s\", \"lanes\": %d, \"iters\": %d, \"ms\": %.3f, \"ps_per_field_op\": %.3f}\n", name, lanes,
         iters, best, best * 1e9 / ((double)lanes * iters * 4));
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
  // operands: radix-29 limbs (< 2^29) for r29, full words for the radix-32
  // variants (interpreted < 2^256; p32 inputs need not be reduced), 25/26-bit
  // limbs for fe_mul: one buffer per family
  const size_t words = (size_t)lanes * 40;
  uint32_t* h29 = (uint32_t*)malloc(words * 4);
  uint32_t* h32 = (uint32_t*)malloc(words * 4);
  uint32_t* hfe = (uint32_t*)malloc(words * 4);
  for (size_t i = 0; i < words; i++) {
    h29[i] = (uint32_t)rnd() & (((i % 10) == 8) ? 0xffffffu : 0x1fffffffu);
    h32[i] = (uint32_t)rnd();
    hfe[i] = (uint32_t)rnd() & (((i % 10) & 1) ? 0x1ffffffu : 0x3ffffffu);
  }
  uint32_t *d29, *d32, *dfe, *dout;
  CHECK(hipMalloc(&d29, words * 4));
  CHECK(hipMalloc(&d32, words * 4));
  CHECK(hipMalloc(&dfe, words * 4));
  CHECK(hipMalloc(&dout, words * 4));
  CHECK(hipMemcpy(d29, h29, words * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d32, h32, words * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dfe, hfe, words * 4, hipMemcpyHostToDevice));
  if (timed<0>("r29_mul_p256_asm", d29, dout, lanes, iters)) return 1;
  if (timed<1>("r29_sqr_p256_asm", d29, dout, lanes, iters)) return 1;
  if (timed<2>("p32_mul_p256_nist", d32, dout, lanes, iters)) return 1;
  if (timed<3>("p32_sqr_p256_nist", d32, dout, lanes, iters)) return 1;
  if (timed<4>("q32_mul_25519", d32, dout, lanes, iters)) return 1;
  if (timed<5>("fe_mul_25519_radix25.5", dfe, dout, lanes, iters)) return 1;
  const int n = 512;
  hipLaunchKernelGGL(once, dim3(n / 256), dim3(256), 0, 0, d32, dout, n);
  CHECK(hipDeviceSynchronize());
  uint32_t* ho = (uint32_t*)malloc((size_t)n * 24 * 4);
  CHECK(hipMemcpy(ho, dout, (size_t)n * 24 * 4, hipMemcpyDeviceToHost));
  for (int i = 0; i < n; i++) {
    printf("CHK");
    for (int k = 0; k < 8; k++) printf(" %u", h32[i * 40 + k]);
    for (int k = 0; k < 8; k++) printf(" %u", h32[i * 40 + 10 + k]);
    for (int k = 0; k < 24; k++) printf(" %u", ho[i * 24 + k]);
    printf("\n");
  }
  return 0;
}
