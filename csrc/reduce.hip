// xdot — sum of split partials + cast, one pass (split-K weight gradients, csrc/gemm.hip
// partials): out[i] = (OUT) Σ_s part[s, i], fp32 accumulation in split order (deterministic).
#include "common.h"

namespace xdot {

template <int DTO>
__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ part, void* __restrict__ out,
                                                            int S, int64_t n4) {
  using TO = typename dt_traits<DTO>::T;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  f32x4 acc = *reinterpret_cast<const f32x4*>(part + 4 * i);
  for (int s = 1; s < S; ++s) acc += *reinterpret_cast<const f32x4*>(part + (int64_t)s * n4 * 4 + 4 * i);
  if constexpr (DTO == DT_F32) {
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(out) + 4 * i) = acc;
  } else {
    TO* o = reinterpret_cast<TO*>(out) + 4 * i;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (TO)acc[e];
  }
}

template <int DT>
__global__ __launch_bounds__(256) void prescale_rows_kernel(const u32x4* __restrict__ x, u32x4* __restrict__ out,
                                                             int64_t n8, float scale) {
  using T16 = typename dt_traits<DT>::T;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const float c2 = scale * 1.4426950408889634f;  // as flash_common.h: a.scale * LOG2E
  union { u32x4 u; T16 e[8]; } v;
  v.u = x[i];
#pragma unroll
  for (int e = 0; e < 8; ++e) v.e[e] = (T16)((float)v.e[e] * c2);
  out[i] = v.u;
}

}  // namespace xdot

extern "C" int xdot_prescale_rows_launch(const void* x, void* out, int64_t n, float scale, int dt, hipStream_t st) {
  using namespace xdot;
  if (n == 0) return 0;
  if (n % 8) return -1;
  const int64_t n8 = n / 8;
  const dim3 grid((unsigned)((n8 + 255) / 256));
  const u32x4* xi = reinterpret_cast<const u32x4*>(x);
  u32x4* o = reinterpret_cast<u32x4*>(out);
  if (dt == DT_BF16) hipLaunchKernelGGL(prescale_rows_kernel<DT_BF16>, grid, dim3(256), 0, st, xi, o, n8, scale);
  else if (dt == DT_F16) hipLaunchKernelGGL(prescale_rows_kernel<DT_F16>, grid, dim3(256), 0, st, xi, o, n8, scale);
  else return -1;
  return 0;
}

extern "C" int xdot_sum_partials_launch(const float* part, void* out, int S, int64_t n, int dto, hipStream_t st) {
  using namespace xdot;
  if (n == 0) return 0;
  if (n % 4) return -1;
  const int64_t n4 = n / 4;
  const dim3 grid((unsigned)((n4 + 255) / 256));
  if (dto == DT_F32) hipLaunchKernelGGL(sum_partials_kernel<DT_F32>, grid, dim3(256), 0, st, part, out, S, n4);
  else if (dto == DT_BF16) hipLaunchKernelGGL(sum_partials_kernel<DT_BF16>, grid, dim3(256), 0, st, part, out, S, n4);
  else if (dto == DT_F16) hipLaunchKernelGGL(sum_partials_kernel<DT_F16>, grid, dim3(256), 0, st, part, out, S, n4);
  else return -1;
  return 0;
}
