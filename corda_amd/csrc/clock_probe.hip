// libcordaprobe.so -- bench diagnostic, NOT part of the product ABI
// (include/cordahip.h): the shader clock the chip holds while a workload runs.
//
// The kernels are issue-bound, so a box's verifications/s scale with the clock
// it sustains under load, and MI355X boxes differ by up to ~12% there
// (MI355X_MICROARCH DVFS item 5). To make bench lines comparable across boxes,
// bench.py runs one extra, untimed step of the workload with this sampler
// resident beside it: a few one-wave workgroups (one per XCD: workgroups are
// dealt round-robin over the 8 XCDs) that stamp (s_memtime, s_memrealtime)
// pairs at fixed real-time intervals. Clock = d(s_memtime) / d(s_memrealtime)
// x 100 MHz per interval (DVFS item 6), median over intervals and XCDs. The
// sampler is scalar-only between stamps, so it takes one wave slot per XCD and
// no VALU issue slots from the workload; it exits after a fixed real time, so
// every wave reaches its end. The product kernels carry no stamps.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <thread>
#include <vector>

namespace {

constexpr uint32_t kMaxSamples = 4096;

__global__ void __launch_bounds__(64) clock_sampler_kernel(uint64_t* out, volatile uint32_t* started,
                                                            uint32_t nsamples, uint64_t interval_ticks) {
  // out[block][k] = {s_memtime, s_memrealtime}; written by lane 0 with vector stores
  uint64_t* o = out + (uint64_t)blockIdx.x * nsamples * 2;
  uint64_t r = __builtin_amdgcn_s_memrealtime();
  uint64_t t = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    o[0] = t;
    o[1] = r;
    started[blockIdx.x] = 1u;
    __threadfence_system();
  }
  for (uint32_t k = 1; k < nsamples; k++) {
    const uint64_t r_last = r;
    do {
      __builtin_amdgcn_s_sleep(2);
      r = __builtin_amdgcn_s_memrealtime();
    } while (r - r_last < interval_ticks);
    t = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
      o[2 * k] = t;
      o[2 * k + 1] = r;
    }
  }
}

struct Probe {
  int device = 0;
  hipStream_t stream = nullptr;
  uint64_t* d_out = nullptr;
  uint32_t* h_started = nullptr;
  hipEvent_t a = nullptr, b = nullptr;
  uint32_t nblocks = 0, nsamples = 0;
};

void destroy(Probe* p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  if (p->stream) (void)hipStreamSynchronize(p->stream);
  if (p->d_out) (void)hipFree(p->d_out);
  if (p->h_started) (void)hipHostFree(p->h_started);
  if (p->a) (void)hipEventDestroy(p->a);
  if (p->b) (void)hipEventDestroy(p->b);
  if (p->stream) (void)hipStreamDestroy(p->stream);
  delete p;
}

}  // namespace

extern "C" {

// Start the sampler on `device` for about duration_ms of real time (nsamples
// stamps per workgroup, nblocks one-wave workgroups), on a stream with a
// hardware queue of its own (CU-masked, all CUs), so it cannot queue behind the
// workload. Returns once every workgroup is resident (or -2 after 2 s).
int cordaprobe_clock_start(int device, double duration_ms, uint32_t nblocks, uint32_t nsamples, void** handle) {
  if (!handle || nblocks == 0 || nblocks > 256 || nsamples < 2 || nsamples > kMaxSamples || duration_ms <= 0)
    return -1;
  *handle = nullptr;
  Probe* p = new Probe;
  p->device = device;
  p->nblocks = nblocks;
  p->nsamples = nsamples;
  int ncu = 0;
  hipError_t e = hipSetDevice(device);
  e = e ? e : hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
  std::vector<uint32_t> mask((std::max(ncu, 1) + 31) / 32, 0xffffffffu);
  e = e ? e : hipExtStreamCreateWithCUMask(&p->stream, (uint32_t)mask.size(), mask.data());
  e = e ? e : hipMalloc(reinterpret_cast<void**>(&p->d_out), (size_t)nblocks * nsamples * 16);
  e = e ? e : hipHostMalloc(reinterpret_cast<void**>(&p->h_started), nblocks * 4, hipHostMallocCoherent);
  e = e ? e : hipEventCreate(&p->a);
  e = e ? e : hipEventCreate(&p->b);
  if (e != hipSuccess) {
    destroy(p);
    return -3;
  }
  for (uint32_t i = 0; i < nblocks; i++) p->h_started[i] = 0;
  // s_memrealtime runs at 100 MHz
  const uint64_t interval = std::max<uint64_t>(1, (uint64_t)(duration_ms * 1e5 / (nsamples - 1)));
  e = hipEventRecord(p->a, p->stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(clock_sampler_kernel, dim3(nblocks), dim3(64), 0, p->stream, p->d_out, p->h_started,
                       nsamples, interval);
    e = hipGetLastError();
  }
  e = e ? e : hipEventRecord(p->b, p->stream);
  if (e != hipSuccess) {
    destroy(p);
    return -3;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    uint32_t up = 0;
    for (uint32_t i = 0; i < nblocks; i++) up += __atomic_load_n(&p->h_started[i], __ATOMIC_ACQUIRE) ? 1 : 0;
    if (up == nblocks) break;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
      *handle = p;  // still running: the caller must finish (which waits for it)
      return -2;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  *handle = p;
  return 0;
}

// Wait for the sampler; per-interval clocks in GHz go to ghz[] (at most cap
// values, block-major), *n gets their count; *realtime_mhz the s_memrealtime
// rate implied by the kernel's event-timed duration (a sanity check of the
// 100 MHz assumption). Frees the probe.
int cordaprobe_clock_finish(void* handle, double* ghz, uint32_t cap, uint32_t* n, double* realtime_mhz) {
  Probe* p = static_cast<Probe*>(handle);
  if (!p) return -1;
  (void)hipSetDevice(p->device);
  hipError_t e = hipStreamSynchronize(p->stream);
  std::vector<uint64_t> h((size_t)p->nblocks * p->nsamples * 2);
  e = e ? e : hipMemcpy(h.data(), p->d_out, h.size() * 8, hipMemcpyDeviceToHost);
  float ms = 0.f;
  e = e ? e : hipEventElapsedTime(&ms, p->a, p->b);
  if (e != hipSuccess) {
    destroy(p);
    return -3;
  }
  uint32_t m = 0;
  uint64_t r_span = 0;
  for (uint32_t blk = 0; blk < p->nblocks; blk++) {
    const uint64_t* o = h.data() + (size_t)blk * p->nsamples * 2;
    r_span = std::max<uint64_t>(r_span, o[2 * (p->nsamples - 1) + 1] - o[1]);
    for (uint32_t k = 1; k < p->nsamples; k++) {
      const uint64_t dt = o[2 * k] - o[2 * (k - 1)], dr = o[2 * k + 1] - o[2 * (k - 1) + 1];
      if (dr && m < cap && ghz) ghz[m++] = (double)dt / (double)dr * 0.1;  // x 100 MHz, in GHz
    }
  }
  if (n) *n = m;
  if (realtime_mhz) *realtime_mhz = ms > 0 ? (double)r_span / (ms * 1e3) : 0.0;
  destroy(p);
  return 0;
}

}  // extern "C"
