// Native Kryo leaf encoder on the GPU: the same leaf
// preimages as cordahip_kryo_encode (kryo_core.hpp, one encoder for both
// sides), for batches whose component payloads are already in HBM -- a
// transaction batch's ids then need no host serialisation and no leaf bytes
// over PCIe (c4h with native leaves moves 1,717 B of leaves per cash-issue
// transaction; its components are ~600 B).
//
// Three launches: (1) every item's leaf size in the encoder's counting mode (no
// buffers), (2) an exclusive scan of the sizes into the CSR offsets
// (hipcub), (3) every leaf written at its offset. One thread per leaf; the
// threads of a wave take the same component kind of consecutive records when
// the items come as records of `group` components (a cash-issue transaction:
// 5), so a wave runs one encoder path. The byte stream is sequential per leaf
// (Kryo's nested chunk framing needs each level's pending bytes before its
// length prefix), so each writing thread owns kLevelBytes of workspace for its
// OutputChunked levels; the writing grid is capped at the workspace's threads
// and strides over the items.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "kryo_core.hpp"

// waves per SIMD the encoder kernels target: 2 (up to 256 VGPRs) beat 4 and 8,
// whose extra scratch traffic cost more than the waves hide (profiles/r04_kryo_device)
#ifndef KRYO_WAVES
#define KRYO_WAVES 2
#endif

namespace cordahip {

namespace {

__device__ inline uint64_t item_of(uint64_t j, uint64_t n, uint32_t group) {
  if (group <= 1 || n % group) return j;
  const uint64_t rec = n / group;  // records of `group` items: kind-major thread order
  return (j % rec) * group + j / rec;
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KRYO_WAVES))) kryo_size_kernel(const cordahip_kryo_item* __restrict__ items, uint64_t n,
                                                        uint32_t group, uint64_t* __restrict__ sizes,
                                                        uint8_t* __restrict__ status) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j == 0) sizes[n] = 0;  // the scan's last element: off[n] = the total
  if (j >= n) return;
  const uint64_t i = item_of(j, n, group);
  kryo::Kout o(nullptr, 0, nullptr);  // counting mode
  const bool ok = kryo::encode_leaf(o, items[i]);
  sizes[i] = ok ? o.pos : 0;
  status[i] = ok ? 0 : 1;
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KRYO_WAVES))) kryo_write_kernel(const cordahip_kryo_item* __restrict__ items, uint64_t n,
                                                         uint32_t group, const uint64_t* __restrict__ off,
                                                         uint8_t* __restrict__ out, uint64_t cap,
                                                         uint8_t* __restrict__ status, uint8_t* __restrict__ ws) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  // each thread's level buffers contiguous (lane-interleaved buffers, one
  // 64-byte line per byte position of a wave, ran 2.3x slower: the lanes' leaves
  // drift apart and the copies lose their wide accesses, profiles/r04_kryo_device)
  uint8_t* levels = ws + t * (uint64_t)kryo::kLevelBytes;
  for (uint64_t j = t; j < n; j += stride) {
    const uint64_t i = item_of(j, n, group);
    if (status[i] != 0) continue;
    const uint64_t a = off[i], b = off[i + 1];
    if (b > cap) {  // beyond the caller's buffer: not written
      status[i] = 2;
      continue;
    }
    kryo::Kout o(out + a, b - a, levels);
    if (!kryo::encode_leaf(o, items[i]) || o.pos != b - a) status[i] = 3;  // cannot happen: same encoder
  }
}

}  // namespace

hipError_t launch_kryo_size(const cordahip_kryo_item* items, uint64_t n, uint32_t group, uint64_t* sizes,
                            uint8_t* status, hipStream_t s) {
  hipLaunchKernelGGL(kryo_size_kernel, dim3((uint32_t)((n + 1 + 255) / 256)), dim3(256), 0, s, items, n, group, sizes,
                     status);
  return hipGetLastError();
}

hipError_t kryo_scan(void* temp, size_t& temp_bytes, const uint64_t* sizes, uint64_t* off, uint64_t n1,
                     hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, sizes, off, (int)n1, s);
}

hipError_t launch_kryo_write(const cordahip_kryo_item* items, uint64_t n, uint32_t group, const uint64_t* off,
                             uint8_t* out, uint64_t cap, uint8_t* status, uint8_t* ws, uint64_t ws_threads,
                             hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t threads = std::min<uint64_t>(n, ws_threads) / 256 * 256;
  const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, threads / 256);
  hipLaunchKernelGGL(kryo_write_kernel, dim3(blocks), dim3(256), 0, s, items, n, group, off, out, cap, status, ws);
  return hipGetLastError();
}

}  // namespace cordahip
