// GPU check + timing of the radix-2^29 Montgomery products on both ECDSA
// curves: the generated asm pairs (corda_amd/csrc/fp29_asm.hpp) and fp29.hpp's
// special-form C f29_mul / f29_sqr against a generic nine-limb REDC (below):
// identical limbs for random operands within f29_mul's input bounds (limbs
// < 2^29 with a top limb < 2^25, i.e. < 2^257), then the issue cost of long
// chains of each form.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../corda_amd/csrc/fp29_asm.hpp"
#include "../../corda_amd/csrc/fp29_consts.hpp"

using namespace cordahip;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

__device__ uint32_t xs(uint32_t& s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return s;
}
__device__ void rnd(f29& a, uint32_t& s) {
  for (int i = 0; i < 8; i++) a.v[i] = xs(s) & kMask29;
  a.v[8] = xs(s) & ((1u << 25) - 1);
}

// generic product-scanning REDC over p's nine limbs (fp29.hpp before the
// special-form reduction)
template <class F>
__device__ void gen_mul(f29& r, const f29& a, const f29& b, bool sq) {
  const f29& bb = sq ? a : b;
  uint32_t q[9];
  uint64_t acc = 0;
  for (int k = 0; k < 9; k++) {
    for (int j = 0; j < k; j++) acc += (uint64_t)a.v[j] * bb.v[k - j] + (uint64_t)q[j] * F::m(k - j);
    acc += (uint64_t)a.v[k] * bb.v[0];
    q[k] = ((uint32_t)acc * F::kMinv) & kMask29;
    acc += (uint64_t)q[k] * F::m(0);
    acc >>= 29;
  }
  f29 t;
  for (int k = 9; k < 17; k++) {
    for (int j = k - 8; j < 9; j++) acc += (uint64_t)a.v[j] * bb.v[k - j] + (uint64_t)q[j] * F::m(k - j);
    t.v[k - 9] = (uint32_t)acc & kMask29;
    acc >>= 29;
  }
  t.v[8] = (uint32_t)acc;
  r = t;
}

template <class F, int C>  // C: 0 k1, 1 r1 (which generated functions)
__device__ void pair_mm(f29& r0, const f29& a0, const f29& b0, f29& r1, const f29& a1, const f29& b1) {
  if (C == 0) f29a_mul_mul_k1(r0, a0, b0, r1, a1, b1); else f29a_mul_mul_r1(r0, a0, b0, r1, a1, b1);
}
template <class F, int C>
__device__ void pair_ss(f29& r0, const f29& a0, f29& r1, const f29& a1) {
  if (C == 0) f29a_sqr_sqr_k1(r0, a0, r1, a1); else f29a_sqr_sqr_r1(r0, a0, r1, a1);
}
template <class F, int C>
__device__ void pair_sm(f29& r0, const f29& a0, f29& r1, const f29& a1, const f29& b1) {
  if (C == 0) f29a_sqr_mul_k1(r0, a0, r1, a1, b1); else f29a_sqr_mul_r1(r0, a0, r1, a1, b1);
}

template <class F, int C>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) check(uint32_t* bad, uint32_t seed) {
  uint32_t s = seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
  for (int it = 0; it < 32; it++) {
    f29 f0, g0, f1, g1, a0, a1, b0, b1;
    rnd(f0, s); rnd(g0, s); rnd(f1, s); rnd(g1, s);
    uint32_t d = 0;
    f29 c0, c1;
    gen_mul<F>(a0, f0, g0, false);
    gen_mul<F>(a1, f1, g1, false);
    pair_mm<F, C>(b0, f0, g0, b1, f1, g1);
    f29_mul<F>(c0, f0, g0);
    f29_mul<F>(c1, f1, g1);
    for (int i = 0; i < 9; i++) d |= (a0.v[i] ^ b0.v[i]) | (a1.v[i] ^ b1.v[i]) | (a0.v[i] ^ c0.v[i]) | (a1.v[i] ^ c1.v[i]);
    gen_mul<F>(a0, f0, f0, true);
    gen_mul<F>(a1, f1, f1, true);
    pair_ss<F, C>(b0, f0, b1, f1);
    f29_sqr<F>(c0, f0);
    f29_sqr<F>(c1, f1);
    uint32_t e = 0;
    for (int i = 0; i < 9; i++) e |= (a0.v[i] ^ b0.v[i]) | (a1.v[i] ^ b1.v[i]) | (a0.v[i] ^ c0.v[i]) | (a1.v[i] ^ c1.v[i]);
    gen_mul<F>(a0, g0, g0, true);
    gen_mul<F>(a1, f1, g0, false);
    pair_sm<F, C>(b0, g0, b1, f1, g0);
    uint32_t g = 0;
    for (int i = 0; i < 9; i++) g |= (a0.v[i] ^ b0.v[i]) | (a1.v[i] ^ b1.v[i]);
    const uint32_t flags = (d ? 1u : 0u) | (e ? 2u : 0u) | (g ? 4u : 0u);
    if (flags) atomicOr(bad, flags);
  }
}

template <class F, int C, int MODE>  // 0: f29_mul x2, 1: pair, 2: f29_sqr x2, 3: pair
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) chain(uint32_t* out, uint32_t seed, int iters) {
  uint32_t s = seed ^ (blockIdx.x * 256 + threadIdx.x);
  f29 x, y, z, w;
  rnd(x, s); rnd(y, s); rnd(z, s); rnd(w, s);
  for (int it = 0; it < iters; it++) {
    if (MODE == 0) { f29_mul<F>(x, x, y); f29_mul<F>(z, z, w); }
    if (MODE == 1) pair_mm<F, C>(x, x, y, z, z, w);
    if (MODE == 2) { f29_sqr<F>(x, x); f29_sqr<F>(z, z); }
    if (MODE == 3) pair_ss<F, C>(x, x, z, z);
  }
  uint32_t a = 0;
  for (int i = 0; i < 9; i++) a ^= x.v[i] ^ z.v[i];
  out[blockIdx.x * 256 + threadIdx.x] = a;
}

template <class F, int C, int MODE>
static int time_chain(const char* name, uint32_t* dout, int ncu, int per_simd_waves) {
  const int blocks = ncu * per_simd_waves;
  const int iters = 2000;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((chain<F, C, MODE>), dim3(blocks), dim3(256), 0, 0, dout, 7u, 10);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL((chain<F, C, MODE>), dim3(blocks), dim3(256), 0, 0, dout, 7u, iters);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double ns_per_product = ms * 1e6 / ((double)per_simd_waves * iters * 2);
  printf("{\"curve\": \"%s\", \"form\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"ns_per_product_per_simd\": %.2f}\n",
         C == 0 ? "secp256k1" : "P-256", name, per_simd_waves, ms, ns_per_product);
  return 0;
}

template <class F, int C>
static int run(uint32_t* dbad, uint32_t* dout, int ncu) {
  CHECK(hipMemset(dbad, 0, 4));
  hipLaunchKernelGGL((check<F, C>), dim3(2048), dim3(256), 0, 0, dbad, 12345u + C);
  uint32_t bad = 0;
  CHECK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
  printf("{\"check\": \"fp29 asm pairs and special-form f29_mul/f29_sqr vs generic REDC\", \"curve\": \"%s\", \"lanes\": %d, "
         "\"mul_mul_mismatch\": %d, \"sqr_sqr_mismatch\": %d, \"sqr_mul_mismatch\": %d}\n",
         C == 0 ? "secp256k1" : "P-256", 2048 * 256 * 32, bad & 1, (bad >> 1) & 1, (bad >> 2) & 1);
  if (time_chain<F, C, 0>("f29_mul x2 (C)", dout, ncu, 2)) return 1;
  if (time_chain<F, C, 1>("mul_mul (asm)", dout, ncu, 2)) return 1;
  if (time_chain<F, C, 2>("f29_sqr x2 (C)", dout, ncu, 2)) return 1;
  if (time_chain<F, C, 3>("sqr_sqr (asm)", dout, ncu, 2)) return 1;
  return bad ? 2 : 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  uint32_t *dbad, *dout;
  CHECK(hipMalloc(&dbad, 4));
  CHECK(hipMalloc(&dout, (size_t)p.multiProcessorCount * 8 * 256 * 4));
  const int a = run<K1F, 0>(dbad, dout, p.multiProcessorCount);
  const int b = run<R1F, 1>(dbad, dout, p.multiProcessorCount);
  return a ? a : b;
}
