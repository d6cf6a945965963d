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

// the two products of one paired weight-gradient launch (csrc/gemm_wgrad.hip) summed by ONE
// launch: threads [0, n4a) sum problem a, the rest problem b (same per-element order as above)
template <int DTO>
__global__ __launch_bounds__(256) void sum_partials2_kernel(const float* __restrict__ pa, void* __restrict__ oa, int Sa,
                                                             int64_t n4a, const float* __restrict__ pb,
                                                             void* __restrict__ ob, int Sb, int64_t n4b) {
  using TO = typename dt_traits<DTO>::T;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool first = i < n4a;
  if (!first) i -= n4a;
  const int64_t n4 = first ? n4a : n4b;
  if (i >= n4) return;
  const float* part = first ? pa : pb;
  const int S = first ? Sa : Sb;
  f32x4 acc = *reinterpret_cast<const f32x4*>(part + 4 * i);
  for (int s = 1; s < S; ++s) acc += *reinterpret_cast<const f32x4*>(part + (int64_t)s * n4 * 4 + 4 * i);
  if constexpr (DTO == DT_F32) {
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(first ? oa : ob) + 4 * i) = acc;
  } else {
    TO* o = reinterpret_cast<TO*>(first ? oa : ob) + 4 * i;
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

// Fused MSE loss, forward half: one pass over (y, t) writes dy = (2 / n) (y - t) in the input
// dtype (the backward then only scales it by the incoming gradient) and one fp32 partial of
// sum (y - t)^2 per workgroup; mse_final sums the partials in order (deterministic) into the
// mean.  Replaces torch's MSELoss chain (sub, pow, mean-reduce, and a second pass over y and t
// plus fills in the backward).
template <int DT>
__global__ __launch_bounds__(256) void mse_fwd_kernel(const u32x4* __restrict__ y, const u32x4* __restrict__ t,
                                                       u32x4* __restrict__ dy, float* __restrict__ part, int64_t nv,
                                                       float g2) {
  using TT = typename dt_traits<DT>::T;
  constexpr int V = 16 / sizeof(TT);
  __shared__ float red[4];
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (int64_t)gridDim.x * 256) {
    union { u32x4 u; TT e[V]; } a, b, o;
    a.u = y[i];
    b.u = t[i];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const float d = (float)a.e[e] - (float)b.e[e];
      acc = __builtin_fmaf(d, d, acc);
      o.e[e] = (TT)(d * g2);
    }
    dy[i] = o.u;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

template <int DT>
__global__ __launch_bounds__(256) void mse_final_kernel(const float* __restrict__ part, int np, void* __restrict__ loss,
                                                         float inv_n) {
  using TT = typename dt_traits<DT>::T;
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < np; i += 256) acc += part[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) *reinterpret_cast<TT*>(loss) = (TT)(((red[0] + red[1]) + (red[2] + red[3])) * inv_n);
}

}  // namespace xdot

extern "C" int xdot_mse_fwd_launch(const void* y, const void* t, void* dy, float* part, int nparts, void* loss,
                                   int64_t n, int dt, hipStream_t st) {
  using namespace xdot;
  if (n == 0) return -1;
  const int V = dt == DT_F32 ? 4 : 8;
  if (n % V) return -1;
  const int64_t nv = n / V;
  const u32x4* yi = reinterpret_cast<const u32x4*>(y);
  const u32x4* ti = reinterpret_cast<const u32x4*>(t);
  u32x4* o = reinterpret_cast<u32x4*>(dy);
  const float g2 = 2.f / (float)n, inv_n = 1.f / (float)n;
#define MSE_CASE(D)                                                                                          \
  hipLaunchKernelGGL(mse_fwd_kernel<D>, dim3(nparts), dim3(256), 0, st, yi, ti, o, part, nv, g2);            \
  hipLaunchKernelGGL(mse_final_kernel<D>, dim3(1), dim3(256), 0, st, part, nparts, loss, inv_n);
  if (dt == DT_BF16) { MSE_CASE(DT_BF16) }
  else if (dt == DT_F16) { MSE_CASE(DT_F16) }
  else if (dt == DT_F32) { MSE_CASE(DT_F32) }
  else return -1;
#undef MSE_CASE
  return 0;
}

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

extern "C" int xdot_sum_partials2_launch(const float* pa, void* oa, int Sa, int64_t na, const float* pb, void* ob,
                                         int Sb, int64_t nb, int dto, hipStream_t st) {
  using namespace xdot;
  if ((na % 4) || (nb % 4)) return -1;
  const int64_t n4a = na / 4, n4b = nb / 4;
  if (n4a + n4b == 0) return 0;
  const dim3 grid((unsigned)((n4a + n4b + 255) / 256));
#define SP2(D) hipLaunchKernelGGL(sum_partials2_kernel<D>, grid, dim3(256), 0, st, pa, oa, Sa, n4a, pb, ob, Sb, n4b)
  if (dto == DT_F32) SP2(DT_F32);
  else if (dto == DT_BF16) SP2(DT_BF16);
  else if (dto == DT_F16) SP2(DT_F16);
  else return -1;
#undef SP2
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
