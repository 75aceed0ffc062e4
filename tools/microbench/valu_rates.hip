// VALU issue cost per instruction type on gfx950, at full occupancy.
//
// Each kernel runs 16 independent instances of ONE instruction per asm block
// (one asm statement per block, so no compiler-inserted s_nop between them),
// 8 waves per SIMD (2048 x 256-thread blocks, < 64 VGPRs), and reports the
// SIMD cycles per wave64 instruction at the measured in-kernel clock:
//   cycles = clock x time / (wave-instructions / 1024 SIMDs).
// This is the cost table the Ed25519 / ECDSA field arithmetic is written
// against (which instruction forms to prefer for carries, shifts, selects).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

// 16 copies of an instruction template over registers %0..%15 (32-bit) or the
// 64-bit pairs held in y[]; "I(k)" expands the template for instance k.
#define R16(T) T(0) T(1) T(2) T(3) T(4) T(5) T(6) T(7) T(8) T(9) T(10) T(11) T(12) T(13) T(14) T(15)
#define XS "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), \
  "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15])
#define YS "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]), \
  "+v"(y[8]), "+v"(y[9]), "+v"(y[10]), "+v"(y[11]), "+v"(y[12]), "+v"(y[13]), "+v"(y[14]), "+v"(y[15])

#define S(k) #k
// 32-bit: x[k] = op(x[k], m)      operand %16 = m, %17 = m2
#define T_ADD(k) "v_add_u32 %" S(k) ", %" S(k) ", %16\n"
#define T_AND(k) "v_and_b32 %" S(k) ", %" S(k) ", %16\n"
#define T_LSHL(k) "v_lshlrev_b32 %" S(k) ", 1, %" S(k) "\n"
#define T_LSHR(k) "v_lshrrev_b32 %" S(k) ", 3, %" S(k) "\n"
#define T_MULLO(k) "v_mul_lo_u32 %" S(k) ", %" S(k) ", %16\n"
#define T_MUL19(k) "v_mul_lo_u32 %" S(k) ", %" S(k) ", 19\n"
#define T_MAD24(k) "v_mad_u32_u24 %" S(k) ", %" S(k) ", %16, %17\n"
#define T_ALIGN(k) "v_alignbit_b32 %" S(k) ", %" S(k) ", %16, 26\n"
#define T_BFE(k) "v_bfe_u32 %" S(k) ", %" S(k) ", 3, 26\n"
#define T_ADD3(k) "v_add3_u32 %" S(k) ", %" S(k) ", %16, %17\n"
#define T_LSHLADD(k) "v_lshl_add_u32 %" S(k) ", %" S(k) ", 1, %16\n"
#define T_ANDOR(k) "v_and_or_b32 %" S(k) ", %" S(k) ", %16, %17\n"
#define T_CNDMASK(k) "v_cndmask_b32 %" S(k) ", %" S(k) ", %16, vcc\n"
#define T_CNDMASKS(k) "v_cndmask_b32_e64 %" S(k) ", %" S(k) ", %16, %18\n"
#define T_BFI(k) "v_bfi_b32 %" S(k) ", %17, %" S(k) ", %16\n"
#define T_XOR(k) "v_xor_b32 %" S(k) ", %" S(k) ", %16\n"
// mp256.hpp mac(): a 64-bit MAC whose carry-out (VCC) is caught by v_addc (VCC in);
// y[k] at %0..%15, x[k] at %16..%31, m at %32, m2 at %33; reported per instruction
#define T_MACP(k, h) "v_mad_u64_u32 %" S(k) ", vcc, %32, %33, %" S(k) "\n v_addc_co_u32 %" S(h) ", vcc, 0, %" S(h) ", vcc\n"
#define R16P(T) T(0, 16) T(1, 17) T(2, 18) T(3, 19) T(4, 20) T(5, 21) T(6, 22) T(7, 23) T(8, 24) T(9, 25) \
  T(10, 26) T(11, 27) T(12, 28) T(13, 29) T(14, 30) T(15, 31)
#define T_ADDCO(k) "v_add_co_u32 %" S(k) ", vcc, %" S(k) ", %16\n"
#define T_SUB(k) "v_sub_u32 %" S(k) ", %16, %" S(k) "\n"
#define T_MOV(k) "v_mov_b32 %" S(k) ", %16\n"
#define T_FMA32(k) "v_fma_f32 %" S(k) ", %" S(k) ", %16, %17\n"
// 64-bit: y[k] = op(y[k], ...)
#define T_MAD64(k) "v_mad_u64_u32 %" S(k) ", %18, %16, %17, %" S(k) "\n"
#define T_MAD64C(k) "v_mad_u64_u32 %" S(k) ", %18, %16, 19, %" S(k) "\n"
#define T_LSHR64(k) "v_lshrrev_b64 %" S(k) ", 26, %" S(k) "\n"
#define T_LSHLADD64(k) "v_lshl_add_u64 %" S(k) ", %" S(k) ", 0, %19\n"
#define T_ADD64(k) "v_lshl_add_u64 %" S(k) ", %19, 0, %" S(k) "\n"

enum { K_ADD, K_AND, K_LSHL, K_LSHR, K_MULLO, K_MUL19, K_MAD24, K_ALIGN, K_BFE, K_ADD3, K_LSHLADD, K_ANDOR,
       K_CNDMASK, K_ADDCO, K_SUB, K_MOV, K_FMA32, K_MAD64, K_MAD64C, K_LSHR64, K_LSHLADD64, K_CNDMASKS, K_BFI, K_XOR,
       K_MACP, K_N };
static const char* kName[K_N] = {"v_add_u32", "v_and_b32", "v_lshlrev_b32", "v_lshrrev_b32", "v_mul_lo_u32",
                                 "v_mul_lo_u32 x19", "v_mad_u32_u24", "v_alignbit_b32", "v_bfe_u32", "v_add3_u32",
                                 "v_lshl_add_u32", "v_and_or_b32", "v_cndmask_b32", "v_add_co_u32", "v_sub_u32",
                                 "v_mov_b32", "v_fma_f32", "v_mad_u64_u32", "v_mad_u64_u32 x19",
                                 "v_lshrrev_b64", "v_lshl_add_u64", "v_cndmask_b32_e64 (SGPR pair)",
                                 "v_bfi_b32", "v_xor_b32", "v_mad_u64_u32 + v_addc_co_u32 (VCC carry)"};

template <int K>
__global__ void __launch_bounds__(256) bench(uint32_t* out, uint32_t seed, int iters, unsigned long long* clk) {
  uint32_t x[16];
  uint64_t y[16];
  uint32_t m = seed ^ threadIdx.x, m2 = seed * 3u + threadIdx.x;
  uint64_t m64 = ((uint64_t)m2 << 32) | m;
  unsigned long long cc = 0;
  const unsigned long long sm = __builtin_amdgcn_read_exec() ^ (unsigned long long)seed;  // a uniform 64-bit lane mask
#pragma unroll
  for (int c = 0; c < 16; c++) {
    x[c] = seed * (c + 1) + threadIdx.x;
    y[c] = ((uint64_t)x[c] << 32) | (x[c] ^ 0x5555u);
  }
  asm volatile("v_cmp_lt_u32 vcc, %0, %1" ::"v"(m), "v"(m2) : "vcc");
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
#define BODY32(T) asm volatile(R16(T) : XS : "v"(m), "v"(m2) : "vcc")
#define BODY32S(T) asm volatile(R16(T) : XS : "v"(m), "v"(m2), "s"(sm) : "vcc")
#define BODY64(T) asm volatile(R16(T) : YS : "v"(m), "v"(m2), "s"(cc), "v"(m64) : "vcc")
      if (K == K_ADD) BODY32(T_ADD);
      if (K == K_AND) BODY32(T_AND);
      if (K == K_LSHL) BODY32(T_LSHL);
      if (K == K_LSHR) BODY32(T_LSHR);
      if (K == K_MULLO) BODY32(T_MULLO);
      if (K == K_MUL19) BODY32(T_MUL19);
      if (K == K_MAD24) BODY32(T_MAD24);
      if (K == K_ALIGN) BODY32(T_ALIGN);
      if (K == K_BFE) BODY32(T_BFE);
      if (K == K_ADD3) BODY32(T_ADD3);
      if (K == K_LSHLADD) BODY32(T_LSHLADD);
      if (K == K_ANDOR) BODY32(T_ANDOR);
      if (K == K_CNDMASK) BODY32(T_CNDMASK);
      if (K == K_ADDCO) BODY32(T_ADDCO);
      if (K == K_SUB) BODY32(T_SUB);
      if (K == K_MOV) BODY32(T_MOV);
      if (K == K_FMA32) BODY32(T_FMA32);
      if (K == K_MAD64) BODY64(T_MAD64);
      if (K == K_MAD64C) BODY64(T_MAD64C);
      if (K == K_LSHR64) BODY64(T_LSHR64);
      if (K == K_LSHLADD64) BODY64(T_LSHLADD64);
      if (K == K_CNDMASKS) BODY32S(T_CNDMASKS);
      if (K == K_BFI) BODY32(T_BFI);
      if (K == K_XOR) BODY32(T_XOR);
      if (K == K_MACP) asm volatile(R16P(T_MACP) : YS, XS : "v"(m), "v"(m2) : "vcc");
    }
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < 16; c++) acc ^= x[c] ^ (uint32_t)y[c] ^ (uint32_t)(y[c] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int K>
static int run(int blocks, int iters, uint32_t* dout, unsigned long long* dclk, int ncu, int waves) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(bench<K>, dim3(blocks), dim3(256), 0, 0, dout, 12345u, 16, dclk);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(bench<K>, dim3(blocks), dim3(256), 0, 0, dout, 12345u, iters, dclk);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long clk[2];
  CHECK(hipMemcpy(clk, dclk, sizeof(clk), hipMemcpyDeviceToHost));
  const double ghz = (double)clk[0] / ((double)clk[1] / 100e6) / 1e9;  // memrealtime ticks at 100 MHz
  const double wave_insts = (double)blocks * 4.0 * iters * 4.0 * 16.0 * (K == K_MACP ? 2.0 : 1.0);  // 4 waves/block, 4 x 16 per iter
  const double cyc = ghz * 1e9 * ms * 1e-3 / (wave_insts / (ncu * 4.0));
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_wave_inst\": %.2f, \"clock_ghz\": %.3f, \"ms\": %.3f}\n",
         kName[K], waves, cyc, ghz, ms);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

template <int K>
static int run_all(uint32_t* dout, unsigned long long* dclk, int ncu, int waves) {
  if (run<K>(ncu * waves, 2048, dout, dclk, ncu, waves)) return 1;
  if constexpr (K + 1 < K_N) return run_all<K + 1>(dout, dclk, ncu, waves);
  return 0;
}

int main(int argc, char** argv) {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  uint32_t* dout;
  unsigned long long* dclk;
  CHECK(hipMalloc(&dout, (size_t)p.multiProcessorCount * 8 * 256 * sizeof(uint32_t)));
  CHECK(hipMalloc(&dclk, 2 * sizeof(unsigned long long)));
  // waves per SIMD from argv (default 8: the issue-cost table); 256-thread
  // blocks = one wave per SIMD each
  const int waves = argc > 1 ? atoi(argv[1]) : 8;
  printf("{\"arch\": \"%s\", \"cus\": %d, \"waves_per_simd\": %d}\n", p.gcnArchName, p.multiProcessorCount, waves);
  return run_all<0>(dout, dclk, p.multiProcessorCount, waves);
}
