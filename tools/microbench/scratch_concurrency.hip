// Does a short kernel with private (scratch) memory wait while another stream's
// long VALU kernel runs? (r05: the GPU Kryo encoder's fallback kernels -- 1.5-1.7 KB
// of scratch per lane, no work in steady state -- took 0.2-0.47 ms per launch beside
// the Ed25519 ladders and 5 us alone.) Times, with HIP events on stream B, an empty
// scratch kernel and an empty scratch-free kernel, alone and while stream A runs a
// ~2 ms VALU loop at one wave per SIMD (and a loop with the ladder's 128 VGPRs and
// 24 KB of LDS per block); empty kernels that need 176 VGPRs or 29 KB of LDS
// besides. One JSON line per case.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));      \
      return 1;                                                    \
    }                                                              \
  } while (0)

__global__ void __launch_bounds__(256) spin_kernel(uint32_t* out, uint32_t iters) {
  uint32_t a = threadIdx.x, b = blockIdx.x | 1;
  for (uint32_t i = 0; i < iters; i++) {
    a = a * 1664525u + b;
    b = b ^ (a >> 7);
  }
  if (a == 0x12345678u) out[0] = b;  // keeps the loop
}

// returns at once when n == 0 (as the encoder's fallback kernels usually do); the
// dynamically indexed local array forces private memory
__global__ void __launch_bounds__(256) scratch_kernel(const uint32_t* __restrict__ cnt, uint32_t* out) {
  const uint32_t n = cnt[0];
  volatile uint32_t buf[384];
  for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
    for (uint32_t k = 0; k < 384; k++) buf[k] = j + k;
    out[j] = buf[(j * 7) % 384];
  }
}

__global__ void __launch_bounds__(256) plain_kernel(const uint32_t* __restrict__ cnt, uint32_t* out) {
  const uint32_t n = cnt[0];
  for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) out[j] = j;
}

// empty kernels with one resource each: 176 VGPRs (a clobbered v175), or 29 KB of LDS
__global__ void __launch_bounds__(256) vgpr_kernel(const uint32_t* __restrict__ cnt, uint32_t* out) {
  const uint32_t n = cnt[0];
  asm volatile("s_nop 0" ::: "v175");
  for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) out[j] = j;
}
__global__ void __launch_bounds__(256) lds_kernel(const uint32_t* __restrict__ cnt, uint32_t* out) {
  __shared__ uint32_t lds[7296];
  const uint32_t n = cnt[0];
  for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
    lds[j % 7296] = j;
    out[j] = lds[(j * 7) % 7296];
  }
}

// the Ed25519 ladder's footprint: 128 VGPRs, 24 KB of LDS per 256-thread block
__global__ void __launch_bounds__(256) ladder_like_kernel(uint32_t* out, uint32_t iters) {
  __shared__ uint32_t lds[6144];
  asm volatile("s_nop 0" ::: "v127");
  uint32_t a = threadIdx.x, b = blockIdx.x | 1;
  lds[threadIdx.x] = a;
  __syncthreads();
  for (uint32_t i = 0; i < iters; i++) {
    a = a * 1664525u + b;
    b = b ^ (a >> 7);
  }
  if (a == 0x12345678u) out[0] = b + lds[(threadIdx.x * 5) & 255];
}

int main() {
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  uint32_t *cnt, *out;
  CK(hipMalloc(&cnt, 4));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(cnt, 0, 4));
  hipEvent_t e0, e1, a0, a1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&a0));
  CK(hipEventCreate(&a1));
  const uint32_t spin_blocks = 256, iters = 200000;  // 4 waves per CU: one per SIMD
  // warm both kernels (code objects loaded, scratch set up once)
  hipLaunchKernelGGL(scratch_kernel, dim3(128), dim3(256), 0, b, cnt, out);
  hipLaunchKernelGGL(plain_kernel, dim3(128), dim3(256), 0, b, cnt, out);
  hipLaunchKernelGGL(vgpr_kernel, dim3(128), dim3(256), 0, b, cnt, out);
  hipLaunchKernelGGL(lds_kernel, dim3(128), dim3(256), 0, b, cnt, out);
  hipLaunchKernelGGL(ladder_like_kernel, dim3(spin_blocks), dim3(256), 0, a, out, iters / 10);
  hipLaunchKernelGGL(spin_kernel, dim3(spin_blocks), dim3(256), 0, a, out, iters / 10);
  CK(hipDeviceSynchronize());
  const char* names[] = {"plain", "scratch", "vgpr176", "lds29k"};
  for (int busy = 0; busy < 3; busy++)  // alone, beside the spin loop, beside the ladder-like kernel
    for (int kind = 0; kind < 4; kind++)
      for (uint32_t blocks : {16u, 128u, 1024u}) {
        float best = 1e30f, worst = 0, spin_ms = 0;
        for (int rep = 0; rep < 5; rep++) {
          if (busy) {
            CK(hipEventRecord(a0, a));
            if (busy == 1) hipLaunchKernelGGL(spin_kernel, dim3(spin_blocks), dim3(256), 0, a, out, iters);
            else hipLaunchKernelGGL(ladder_like_kernel, dim3(spin_blocks), dim3(256), 0, a, out, iters);
            CK(hipEventRecord(a1, a));
            CK(hipStreamWaitEvent(b, a0, 0));
            // let the long kernel occupy the GPU first
            hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, b, out, iters / 20);
          }
          CK(hipEventRecord(e0, b));
          if (kind == 0) hipLaunchKernelGGL(plain_kernel, dim3(blocks), dim3(256), 0, b, cnt, out);
          else if (kind == 1) hipLaunchKernelGGL(scratch_kernel, dim3(blocks), dim3(256), 0, b, cnt, out);
          else if (kind == 2) hipLaunchKernelGGL(vgpr_kernel, dim3(blocks), dim3(256), 0, b, cnt, out);
          else hipLaunchKernelGGL(lds_kernel, dim3(blocks), dim3(256), 0, b, cnt, out);
          CK(hipEventRecord(e1, b));
          CK(hipDeviceSynchronize());
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (ms < best) best = ms;
          if (ms > worst) worst = ms;
          if (busy) CK(hipEventElapsedTime(&spin_ms, a0, a1));
        }
        printf("{\"beside\": \"%s\", \"kernel\": \"%s\", \"blocks\": %u, \"best_ms\": %.4f, \"worst_ms\": %.4f, "
               "\"long_kernel_ms\": %.3f}\n", busy == 0 ? "nothing" : busy == 1 ? "spin" : "ladder_like", names[kind],
               blocks, best, worst, spin_ms);
      }
  return 0;
}
