// VALU instruction counts of the P-256 formulas: compile device-only,
// disassemble, count per kernel with tools/isa_count.py:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -c ec_isa_count.hip -o c.o
//   llvm-objdump -d --no-show-raw-insn c.o > c.s && python3 tools/isa_count.py c.s k_dbl k_maddne k_mul k_sqr
#include "../../corda_amd/csrc/ecdsa.hip"
namespace cordahip {
template <class C>
__device__ __forceinline__ void ldp(jpt& p, const uint32_t* io) {
  for (int i = 0; i < 9; i++) { p.X.v[i] = io[i * 64]; p.Y.v[i] = io[(9 + i) * 64]; p.Z.v[i] = io[(18 + i) * 64]; }
  p.inf = io[27 * 64] != 0;
}
__device__ __forceinline__ void stp(uint32_t* io, const jpt& p) {
  for (int i = 0; i < 9; i++) { io[i * 64] = p.X.v[i]; io[(9 + i) * 64] = p.Y.v[i]; io[(18 + i) * 64] = p.Z.v[i]; }
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) k_base(uint32_t* io) {
  io += threadIdx.x; jpt p; ldp<Curve<3>>(p, io); stp(io, p);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) k_dbl_r1(uint32_t* io) {
  io += threadIdx.x; jpt p; ldp<Curve<3>>(p, io); jdbl<Curve<3>>(p, p); stp(io, p);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) k_madd_r1(uint32_t* io) {
  io += threadIdx.x; jpt p; ldp<Curve<3>>(p, io); f29 x, y; for (int i = 0; i < 9; i++) { x.v[i] = io[(30 + i) * 64]; y.v[i] = io[(40 + i) * 64]; }
  jmadd<Curve<3>>(p, p, x, y); stp(io, p);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) k_mul_r1(uint32_t* io) {
  io += threadIdx.x; f29 x, y; for (int i = 0; i < 9; i++) { x.v[i] = io[(30 + i) * 64]; y.v[i] = io[(40 + i) * 64]; }
  f29_mul1<R1F>(x, x, y); for (int i = 0; i < 9; i++) io[i * 64] = x.v[i];
}
}
namespace cordahip {
template <class C>
CDEV void jmadd_noexc(jpt& r, const jpt& p, const f29& x2, const f29& y2) {
  using F = typename C::F;
  f29 z1z1, u2, s2, h, hh, i, j, rr, v, t, x3, y3, z3;
  f29_sqr_mul_pair<F>(z1z1, p.Z, t, y2, p.Z);
  f29_mul_pair<F>(u2, x2, z1z1, s2, t, z1z1);
  f29_sub_red<F>(h, u2, p.X);
  f29_sub_red<F>(rr, s2, p.Y);
  if (f29_iszero_norm<F>(h)) { r.inf = true; return; }
  f29_add(rr, rr, rr);
  f29_sqr_pair<F>(hh, h, x3, rr);
  f29_add(i, hh, hh);
  f29_add(i, i, i);
  f29_mul_pair<F>(j, h, i, v, p.X, i);
  f29_sub3_red<F>(x3, x3, j, v, v);
  f29_sub<F>(t, v, x3);
  f29_mul_pair<F>(y3, rr, t, t, p.Y, j);
  f29_sub2_red<F>(y3, y3, t, t);
  f29_add(t, p.Z, h);
  f29_sqr1<F>(t, t);
  f29_sub2_red<F>(z3, t, z1z1, hh);
  r.X = x3; r.Y = y3; r.Z = z3; r.inf = false;
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) k_maddne_r1(uint32_t* io) {
  io += threadIdx.x; jpt p; ldp<Curve<3>>(p, io); f29 x, y; for (int i = 0; i < 9; i++) { x.v[i] = io[(30 + i) * 64]; y.v[i] = io[(40 + i) * 64]; }
  jmadd_noexc<Curve<3>>(p, p, x, y); stp(io, p);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) k_sqr_r1(uint32_t* io) {
  io += threadIdx.x; f29 x; for (int i = 0; i < 9; i++) { x.v[i] = io[(30 + i) * 64]; }
  f29_sqr1<R1F>(x, x); for (int i = 0; i < 9; i++) io[i * 64] = x.v[i];
}
}
