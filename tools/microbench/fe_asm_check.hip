// GPU check + timing of the generated multi-product field multiplies
// (corda_amd/csrc/fe25519_asm.hpp: fe_mul2/3/4, fe_sq2/4, fe_mul3x/4x) against fe25519.hpp's
// carry-chained C versions: identical limbs for random loose operands (limbs
// < 2^27, the group formulas' bound), then the issue cost of long chains.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../corda_amd/csrc/fe25519_asm.hpp"

using namespace cordahip;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

__device__ uint32_t xs(uint32_t& s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return s;
}
__device__ void rnd(fe& a, uint32_t& s, int lbits) {
  for (int i = 0; i < 10; i++) a.v[i] = xs(s) & ((1u << lbits) - 1);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) check(uint32_t* bad, uint32_t seed) {
  uint32_t s = seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
  for (int it = 0; it < 64; it++) {
    fe f0, g0, f1, g1, a0, a1, b0, b1;
    const int lb = 25 + (it & 3);  // 25..28-bit limbs (up to the loose bound)
    rnd(f0, s, lb); rnd(g0, s, it & 1 ? 27 : 26); rnd(f1, s, lb); rnd(g1, s, 26);
    fe_mul(a0, f0, g0);
    fe_mul(a1, f1, g1);
    fe_mul2(b0, f0, g0, b1, f1, g1);
    uint32_t d = 0;
    for (int i = 0; i < 10; i++) d |= (a0.v[i] ^ b0.v[i]) | (a1.v[i] ^ b1.v[i]);
    rnd(f0, s, 27); rnd(f1, s, 26);
    fe_sq(a0, f0);
    fe_sq(a1, f1);
    fe_sq2(b0, f0, b1, f1);
    for (int i = 0; i < 10; i++) d |= ((a0.v[i] ^ b0.v[i]) | (a1.v[i] ^ b1.v[i])) << 1;
    // 3- and 4-chain blocks
    fe f2, g2, f3, g3, a2, a3, b2, b3;
    rnd(f0, s, lb); rnd(g0, s, 26); rnd(f1, s, 26); rnd(g1, s, 27);
    rnd(f2, s, 27); rnd(g2, s, 25); rnd(f3, s, 26); rnd(g3, s, 26);
    fe_mul(a0, f0, g0); fe_mul(a1, f1, g1); fe_mul(a2, f2, g2); fe_mul(a3, f3, g3);
    fe_mul4(b0, f0, g0, b1, f1, g1, b2, f2, g2, b3, f3, g3);
    for (int i = 0; i < 10; i++)
      d |= ((a0.v[i] ^ b0.v[i]) | (a1.v[i] ^ b1.v[i]) | (a2.v[i] ^ b2.v[i]) | (a3.v[i] ^ b3.v[i])) ? 4u : 0u;
    fe_mul3(b0, f0, g0, b1, f1, g1, b2, f2, g2);
    for (int i = 0; i < 10; i++) d |= ((a0.v[i] ^ b0.v[i]) | (a1.v[i] ^ b1.v[i]) | (a2.v[i] ^ b2.v[i])) ? 8u : 0u;
    fe_sq(a0, f0); fe_sq(a1, f1); fe_sq(a2, f2); fe_sq(a3, f3);
    fe_sq4(b0, f0, b1, f1, b2, f2, b3, f3);
    for (int i = 0; i < 10; i++)
      d |= ((a0.v[i] ^ b0.v[i]) | (a1.v[i] ^ b1.v[i]) | (a2.v[i] ^ b2.v[i]) | (a3.v[i] ^ b3.v[i])) ? 16u : 0u;
    // outer-product blocks (the output stage: F, H up to 5x / 2x; E tight, G <= 3x)
    rnd(f0, s, 28); rnd(f1, s, 27); rnd(g0, s, 26); rnd(g1, s, 27);
    fe_mul(a0, f0, g0); fe_mul(a1, f1, g1); fe_mul(a2, f0, g1); fe_mul(a3, f1, g0);
    fe_mul4x(b0, b1, b2, b3, f0, f1, g0, g1);
    for (int i = 0; i < 10; i++)
      d |= ((a0.v[i] ^ b0.v[i]) | (a1.v[i] ^ b1.v[i]) | (a2.v[i] ^ b2.v[i]) | (a3.v[i] ^ b3.v[i])) ? 32u : 0u;
    fe_mul3x(b0, b1, b2, f0, f1, g0, g1);
    for (int i = 0; i < 10; i++) d |= ((a0.v[i] ^ b0.v[i]) | (a1.v[i] ^ b1.v[i]) | (a2.v[i] ^ b2.v[i])) ? 64u : 0u;
    // the swapped operand order of Y = H G, T = H E against fe_mul(G, H), fe_mul(E, H)
    fe_mul(a1, g1, f1); fe_mul(a3, g0, f1);
    fe_mul4x(b0, b1, b2, b3, f0, f1, g0, g1);
    for (int i = 0; i < 10; i++) d |= ((a1.v[i] ^ b1.v[i]) | (a3.v[i] ^ b3.v[i])) ? 128u : 0u;
    if (d) atomicOr(bad, d);
  }
}

// 0: fe_mul x4 (C), 1: 2 x fe_mul2, 2: fe_mul4, 3: 2 x fe_sq2, 4: fe_sq4 (four products per iteration)
template <int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) chain(uint32_t* out, uint32_t seed,
                                                                                   int iters) {
  uint32_t s = seed ^ (blockIdx.x * 256 + threadIdx.x);
  fe x, y, z, w, u, v;
  rnd(x, s, 26); rnd(y, s, 26); rnd(z, s, 26); rnd(w, s, 26); rnd(u, s, 26); rnd(v, s, 26);
  for (int it = 0; it < iters; it++) {
    if (MODE == 0) { fe_mul(x, x, y); fe_mul(z, z, w); fe_mul(u, u, y); fe_mul(v, v, w); }
    if (MODE == 1) { fe_mul2(x, x, y, z, z, w); fe_mul2(u, u, y, v, v, w); }
    if (MODE == 2) fe_mul4(x, x, y, z, z, w, u, u, y, v, v, w);
    if (MODE == 3) { fe_sq2(x, x, z, z); fe_sq2(u, u, v, v); }
    if (MODE == 4) fe_sq4(x, x, z, z, u, u, v, v);
  }
  uint32_t a = 0;
  for (int i = 0; i < 10; i++) a ^= x.v[i] ^ z.v[i] ^ u.v[i] ^ v.v[i];
  out[blockIdx.x * 256 + threadIdx.x] = a;
}

template <int MODE>
static int time_chain(const char* name, uint32_t* dout, int ncu, int per_simd_waves) {
  const int blocks = ncu * per_simd_waves;  // 256 threads = 4 waves, one per SIMD
  const int iters = 2000;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(chain<MODE>, dim3(blocks), dim3(256), 0, 0, dout, 7u, 10);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(chain<MODE>, dim3(blocks), dim3(256), 0, 0, dout, 7u, iters);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  // per SIMD: per_simd_waves waves x iters x 4 products
  const double ns_per_product = ms * 1e6 / ((double)per_simd_waves * iters * 4);
  printf("{\"form\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"ns_per_product_per_simd\": %.2f}\n", name,
         per_simd_waves, ms, ns_per_product);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  uint32_t *dbad, *dout;
  CHECK(hipMalloc(&dbad, 4));
  CHECK(hipMemset(dbad, 0, 4));
  CHECK(hipMalloc(&dout, (size_t)p.multiProcessorCount * 8 * 256 * 4));
  hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, dbad, 12345u);
  uint32_t bad = 0;
  CHECK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
  printf("{\"check\": \"fe_mul2/3/4, fe_sq2/4, fe_mul3x/4x vs fe_mul/fe_sq\", \"lanes\": %d, \"mul2_mismatch\": %d, "
         "\"sq2_mismatch\": %d, \"mul4_mismatch\": %d, \"mul3_mismatch\": %d, \"sq4_mismatch\": %d, "
         "\"mul4x_mismatch\": %d, \"mul3x_mismatch\": %d, \"mul4x_swapped_mismatch\": %d}\n",
         4096 * 256 * 64, bad & 1, (bad >> 1) & 1, (bad >> 2) & 1, (bad >> 3) & 1, (bad >> 4) & 1, (bad >> 5) & 1,
         (bad >> 6) & 1, (bad >> 7) & 1);
  for (int w : {2, 4}) {
    if (time_chain<0>("fe_mul x4 (C)", dout, p.multiProcessorCount, w)) return 1;
    if (time_chain<1>("2 x fe_mul2 (asm)", dout, p.multiProcessorCount, w)) return 1;
    if (time_chain<2>("fe_mul4 (asm)", dout, p.multiProcessorCount, w)) return 1;
    if (time_chain<3>("2 x fe_sq2 (asm)", dout, p.multiProcessorCount, w)) return 1;
    if (time_chain<4>("fe_sq4 (asm)", dout, p.multiProcessorCount, w)) return 1;
  }
  return bad ? 2 : 0;
}
