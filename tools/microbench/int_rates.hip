// Integer / FP64 VALU throughput microbenchmark for gfx950.
//
// Measures the per-CU issue rate of the instructions a multi-precision
// field multiply can be built from, so the Ed25519/ECDSA kernels pick the
// limb radix from measurements instead of assumptions (SURVEY.md §7 "Hard
// parts"). Each kernel runs NCHAIN independent dependency chains of ONE
// instruction per lane (inline asm so hipcc cannot fold or re-schedule it).
//
// Output: one line per instruction: lane-ops/s, lane-ops per CU-cycle at the
// measured in-kernel clock, and the single-chain (latency-bound) variant.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

enum Op { MAD_U64_U32, MUL_LO_U32, MUL_HI_U32, MAD_U32_U24, MUL_HI_U32_U24, MUL_U32_U24,
          ADD_CO_U32, ADDC_CO_U32, ADD_U32, FMA_F64, FMA_F32, ALIGNBIT, LSHL_ADD, ADD3_U32,
          MAD_U64_CARRY, NOPS };
static const char* kNames[NOPS] = {
  "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u32_u24", "v_mul_hi_u32_u24",
  "v_mul_u32_u24", "v_add_co_u32", "v_addc_co_u32", "v_add_u32", "v_fma_f64", "v_fma_f32",
  "v_alignbit_b32", "v_lshl_add_u32", "v_add3_u32", "mad_u64+addc(pair)"};

template <int OP, int NCHAIN>
__global__ void __launch_bounds__(256) bench(uint32_t* out, uint32_t seed, int iters,
                                             unsigned long long* clk) {
  uint32_t x[NCHAIN];
  uint64_t y[NCHAIN];
  double d[NCHAIN];
  float f[NCHAIN];
  uint32_t m = seed ^ threadIdx.x;
  double dm = 1.0000001 + (double)(threadIdx.x & 7) * 1e-9;
  float fm = 1.0000001f;
#pragma unroll
  for (int c = 0; c < NCHAIN; c++) {
    x[c] = seed * (c + 1) + threadIdx.x;
    y[c] = ((uint64_t)x[c] << 32) | (x[c] ^ 0x5555u);
    d[c] = (double)x[c] * 1e-7;
    f[c] = (float)x[c] * 1e-7f;
  }
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < 16; u++) {
      // SGPR-writing ops: all 8 chains in ONE asm statement, so hipcc's
      // conservative inline-asm hazard padding (s_nop between statements)
      // does not pollute the issue-rate measurement.
      if (NCHAIN == 8 && (OP == MAD_U64_U32 || OP == ADD_CO_U32 || OP == ADDC_CO_U32 || OP == MAD_U64_CARRY)) {
        unsigned long long cc;
        if (OP == MAD_U64_U32)
          asm volatile(
              "v_mad_u64_u32 %0, %8, %9, %10, %0\n\tv_mad_u64_u32 %1, %8, %9, %11, %1\n\t"
              "v_mad_u64_u32 %2, %8, %9, %12, %2\n\tv_mad_u64_u32 %3, %8, %9, %13, %3\n\t"
              "v_mad_u64_u32 %4, %8, %9, %14, %4\n\tv_mad_u64_u32 %5, %8, %9, %15, %5\n\t"
              "v_mad_u64_u32 %6, %8, %9, %16, %6\n\tv_mad_u64_u32 %7, %8, %9, %17, %7"
              : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]), "=s"(cc)
              : "v"(m), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]));
        else if (OP == ADD_CO_U32)
          asm volatile(
              "v_add_co_u32 %0, vcc, %0, %8\n\tv_add_co_u32 %1, vcc, %1, %8\n\t"
              "v_add_co_u32 %2, vcc, %2, %8\n\tv_add_co_u32 %3, vcc, %3, %8\n\t"
              "v_add_co_u32 %4, vcc, %4, %8\n\tv_add_co_u32 %5, vcc, %5, %8\n\t"
              "v_add_co_u32 %6, vcc, %6, %8\n\tv_add_co_u32 %7, vcc, %7, %8"
              : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
              : "v"(m) : "vcc");
        else if (OP == ADDC_CO_U32)
          asm volatile(
              "v_addc_co_u32 %0, vcc, %0, %8, vcc\n\tv_addc_co_u32 %1, vcc, %1, %8, vcc\n\t"
              "v_addc_co_u32 %2, vcc, %2, %8, vcc\n\tv_addc_co_u32 %3, vcc, %3, %8, vcc\n\t"
              "v_addc_co_u32 %4, vcc, %4, %8, vcc\n\tv_addc_co_u32 %5, vcc, %5, %8, vcc\n\t"
              "v_addc_co_u32 %6, vcc, %6, %8, vcc\n\tv_addc_co_u32 %7, vcc, %7, %8, vcc"
              : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
              : "v"(m) : "vcc");
        else
          asm volatile(
              "v_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32 %8, vcc, 0, %8, vcc\n\t"
              "v_mad_u64_u32 %1, vcc, %16, %17, %1\n\tv_addc_co_u32 %9, vcc, 0, %9, vcc\n\t"
              "v_mad_u64_u32 %2, vcc, %16, %17, %2\n\tv_addc_co_u32 %10, vcc, 0, %10, vcc\n\t"
              "v_mad_u64_u32 %3, vcc, %16, %17, %3\n\tv_addc_co_u32 %11, vcc, 0, %11, vcc\n\t"
              "v_mad_u64_u32 %4, vcc, %16, %17, %4\n\tv_addc_co_u32 %12, vcc, 0, %12, vcc\n\t"
              "v_mad_u64_u32 %5, vcc, %16, %17, %5\n\tv_addc_co_u32 %13, vcc, 0, %13, vcc\n\t"
              "v_mad_u64_u32 %6, vcc, %16, %17, %6\n\tv_addc_co_u32 %14, vcc, 0, %14, vcc\n\t"
              "v_mad_u64_u32 %7, vcc, %16, %17, %7\n\tv_addc_co_u32 %15, vcc, 0, %15, vcc"
              : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]),
                "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
              : "v"(m), "v"(seed)
              : "vcc");
        (void)cc;
        continue;
      }
#pragma unroll
      for (int c = 0; c < NCHAIN; c++) {
        if (OP == MAD_U64_U32 && NCHAIN == 1) {
          unsigned long long cc;
          asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(y[c]), "=s"(cc) : "v"(m), "v"(x[c]));
        } else if (OP == MUL_LO_U32) {
          asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[c]) : "v"(m));
        } else if (OP == MUL_HI_U32) {
          asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[c]) : "v"(m));
        } else if (OP == MAD_U32_U24) {
          asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(x[c]) : "v"(m));
        } else if (OP == MUL_HI_U32_U24) {
          asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x[c]) : "v"(m));
        } else if (OP == MUL_U32_U24) {
          asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[c]) : "v"(m));
        } else if (OP == ADD_CO_U32) {
          asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x[c]) : "v"(m) : "vcc");
        } else if (OP == ADDC_CO_U32) {
          asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(x[c]) : "v"(m) : "vcc");
        } else if (OP == ADD_U32) {
          asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(m));
        } else if (OP == FMA_F64) {
          asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[c]) : "v"(dm));
        } else if (OP == FMA_F32) {
          asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[c]) : "v"(fm));
        } else if (OP == ALIGNBIT) {
          asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x[c]) : "v"(m));
        } else if (OP == LSHL_ADD) {
          asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x[c]) : "v"(m));
        } else if (OP == ADD3_U32) {
          asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x[c]) : "v"(m));
        } else if (OP == MAD_U64_CARRY) {
          // the pattern of a product-scanning column: 64-bit acc + carry word
          unsigned long long cc;
          asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, 0, %2, %1"
                       : "+v"(y[c]), "=s"(cc), "+v"(x[c]) : "v"(m), "v"(x[(c + 1) % NCHAIN]));
        }
      }
    }
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < NCHAIN; c++)
    acc ^= x[c] ^ (uint32_t)y[c] ^ (uint32_t)(y[c] >> 32) ^ (uint32_t)(uint64_t)d[c] ^ (uint32_t)f[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP, int NCHAIN>
static int run(const char* tag, int blocks, int iters, uint32_t* dout, unsigned long long* dclk) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((bench<OP, NCHAIN>), dim3(blocks), dim3(256), 0, 0, dout, 12345u, 8, dclk);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((bench<OP, NCHAIN>), dim3(blocks), dim3(256), 0, 0, dout, 12345u, iters, dclk);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long clk[2];
  CHECK(hipMemcpy(clk, dclk, sizeof(clk), hipMemcpyDeviceToHost));
  double ghz = (double)clk[0] / ((double)clk[1] / 100e6) / 1e9;  // memrealtime = 100 MHz
  double lane_ops = (double)blocks * 256.0 * iters * 16.0 * NCHAIN;
  double rate = lane_ops / (ms * 1e-3);
  double per_cu_cycle = rate / (256.0 * ghz * 1e9);
  printf("{\"op\": \"%s\", \"mode\": \"%s\", \"nchain\": %d, \"blocks\": %d, \"ms\": %.3f, "
         "\"lane_ops_per_s\": %.4e, \"clock_ghz\": %.3f, \"lane_ops_per_cu_cycle\": %.2f}\n",
         kNames[OP], tag, NCHAIN, blocks, ms, rate, ghz, per_cu_cycle);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

#define BOTH(OP)                                                         \
  if (run<OP, 8>("throughput", 256 * 8, 2048, dout, dclk)) return 1;    \
  if (run<OP, 1>("latency_1wave_per_simd", 256, 2048, dout, dclk)) return 1;

int main() {
  uint32_t* dout;
  unsigned long long* dclk;
  CHECK(hipMalloc(&dout, 256 * 8 * 256 * sizeof(uint32_t)));
  CHECK(hipMalloc(&dclk, 2 * sizeof(unsigned long long)));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  printf("{\"device\": \"%s\", \"arch\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.name,
         p.gcnArchName, p.multiProcessorCount, p.clockRate);
  BOTH(MAD_U64_U32)
  BOTH(MUL_LO_U32)
  BOTH(MUL_HI_U32)
  BOTH(MAD_U32_U24)
  BOTH(MUL_HI_U32_U24)
  BOTH(MUL_U32_U24)
  BOTH(ADD_CO_U32)
  BOTH(ADDC_CO_U32)
  BOTH(ADD_U32)
  BOTH(FMA_F64)
  BOTH(FMA_F32)
  BOTH(ALIGNBIT)
  BOTH(LSHL_ADD)
  BOTH(ADD3_U32)
  BOTH(MAD_U64_CARRY)
  return 0;
}
