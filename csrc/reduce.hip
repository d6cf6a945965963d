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

}  // namespace xdot

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
