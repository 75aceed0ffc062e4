// Field / group-op microbenchmark for the Ed25519 kernels (gfx950).
//
// Times the ladder's inner window (4 doublings + 1 cached addition) and raw
// fe_mul / fe_sq chains per lane, for whichever fe25519.hpp variant this file
// is compiled with (-DFE_CARRY_CHAIN=0|1), and prints a checksum of the
// canonical outputs so variants can be checked against each other for
// bit-exact agreement. Build: make -C tools/microbench fe_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../corda_amd/csrc/fe25519.hpp"
#include "../../corda_amd/csrc/ge25519.hpp"

using namespace cordahip;

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e = (x);                                                                       \
    if (e != hipSuccess) {                                                                    \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);         \
      return 1;                                                                               \
    }                                                                                         \
  } while (0)

CDEV void ld_fe(fe& a, const uint32_t* p) {
#pragma unroll
  for (int i = 0; i < 10; i++) a.v[i] = p[i];
}
CDEV void st_fe(uint32_t* o, const fe& a) {
  uint32_t w[8];
  fe_tobytes(w, a);
#pragma unroll
  for (int i = 0; i < 8; i++) o[i] = w[i];
}

// in: per lane 80 words (P: X Y Z T, Q: YpX YmX Z T2d, 10 limbs each); out: 32 words
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
window_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int iters) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t* p = in + i * 80;
  ge_p3 P;
  ge_cached Q;
  ld_fe(P.X, p);
  ld_fe(P.Y, p + 10);
  ld_fe(P.Z, p + 20);
  ld_fe(P.T, p + 30);
  ld_fe(Q.YpX, p + 40);
  ld_fe(Q.YmX, p + 50);
  ld_fe(Q.Z, p + 60);
  ld_fe(Q.T2d, p + 70);
  for (int it = 0; it < iters; it++) {
    ge_dbl<false>(P, P);
    ge_dbl<false>(P, P);
    ge_dbl<false>(P, P);
    ge_dbl<true>(P, P);
    ge_add<true>(P, P, Q);
  }
  uint32_t* o = out + i * 32;
  st_fe(o, P.X);
  st_fe(o + 8, P.Y);
  st_fe(o + 16, P.Z);
  st_fe(o + 24, P.T);
}

template <bool SQ>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
chain_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int iters) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t* p = in + i * 80;
  fe a, b, c, d;
  ld_fe(a, p);
  ld_fe(b, p + 10);
  ld_fe(c, p + 20);
  ld_fe(d, p + 30);
  for (int it = 0; it < iters; it++) {  // 4 independent chains (the ILP a group op offers)
    if (SQ) {
      fe_sq(a, a);
      fe_sq(b, b);
      fe_sq(c, c);
      fe_sq(d, d);
    } else {
      fe_mul(a, a, b);
      fe_mul(b, b, c);
      fe_mul(c, c, d);
      fe_mul(d, d, a);
    }
  }
  uint32_t* o = out + i * 32;
  st_fe(o, a);
  st_fe(o + 8, b);
  st_fe(o + 16, c);
  st_fe(o + 24, d);
}

static uint64_t fold(const uint32_t* h, size_t n) {
  uint64_t x = 1469598103934665603ull;
  for (size_t i = 0; i < n; i++) x = (x ^ h[i]) * 1099511628211ull;
  return x;
}

template <class K>
static int run(const char* name, K kern, const uint32_t* din, uint32_t* dout, uint32_t* hout, int lanes, int iters,
               double ops_per_iter) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(lanes / 256), dim3(256), 0, 0, din, dout, 2);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(lanes / 256), dim3(256), 0, 0, din, dout, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipMemcpy(hout, dout, (size_t)lanes * 32 * 4, hipMemcpyDeviceToHost));
  // ns per lane-iteration at full-chip occupancy, and per field op
  const double ns = ms * 1e6 / ((double)lanes * iters);
  printf("{\"bench\": \"%s\", \"carry_chain\": %d, \"lanes\": %d, \"iters\": %d, \"ms\": %.3f, "
         "\"ps_per_lane_iter\": %.2f, \"ps_per_field_op\": %.3f, \"checksum\": \"%016llx\"}\n",
         name, FE_CARRY_CHAIN, lanes, iters, ms, ns * 1e3, ns * 1e3 / ops_per_iter,
         (unsigned long long)fold(hout, (size_t)lanes * 32));
  return 0;
}

int main(int argc, char** argv) {
  const int lanes = 1 << 20, iters = argc > 1 ? atoi(argv[1]) : 64;
  uint32_t* hin = (uint32_t*)malloc((size_t)lanes * 80 * 4);
  uint32_t* hout = (uint32_t*)malloc((size_t)lanes * 32 * 4);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < (size_t)lanes * 80; i++) {  // tight random limbs
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    hin[i] = (uint32_t)s & (((i % 10) & 1) ? M25 : M26);
  }
  uint32_t *din, *dout;
  CHECK(hipMalloc(&din, (size_t)lanes * 80 * 4));
  CHECK(hipMalloc(&dout, (size_t)lanes * 32 * 4));
  CHECK(hipMemcpy(din, hin, (size_t)lanes * 80 * 4, hipMemcpyHostToDevice));
  // field ops per iteration: window = 4 dbl (4S + 3M, one with T) + add (9M) = 16S + 13M + 9M
  if (run("window_4dbl_add", window_kernel, din, dout, hout, lanes, iters, 38.0)) return 1;
  if (run("mul_x4", chain_kernel<false>, din, dout, hout, lanes, iters * 8, 4.0)) return 1;
  if (run("sq_x4", chain_kernel<true>, din, dout, hout, lanes, iters * 8, 4.0)) return 1;
  return 0;
}
