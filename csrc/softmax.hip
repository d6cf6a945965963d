// xdot — fused scale + boolean-mask + row-softmax, forward and backward (gfx950).
//
// Replaces three full passes of the reference over the (B, H, T/N, T) score block
// (reference: distributed_dot_product/module.py:65 `/ sqrt(dim)`, :66 `masked_fill(-inf)`,
// :67 `softmax(-1)`, and their autograd) with one read + one write per direction:
//   fwd: y = softmax(scale * x, masked -> -inf)          (fp32 math, bf16/fp16/fp32 io)
//   bwd: dx = scale * y * (dy - sum(dy * y))              (masked entries have y == 0)
// Rows are up to ~200k long (T = 200000), far past LDS, so:
//   * T <= 65536: the row is cached in registers (1024 threads x 8 x NPT elements), read once;
//   * longer rows: an online (max, sum) first pass, then a second streaming pass.
// The mask is the module's (B, R, T) bool mask broadcast over heads: score row `row` uses
// mask row (row / mdiv) * mmul + (row % mmod).  A fully masked row yields NaN exactly like
// torch.softmax over an all -inf row (reference parity).
#include "common.h"

namespace xdot {
namespace smx {


template <int BLOCK>
__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  v = is_max ? wave_max(v) : wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int NW = BLOCK / 64;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
  return r;
}

// Load 8 consecutive elements [e0, e0+8) of a row (bounded), as fp32.
template <typename T, bool VEC>
__device__ __forceinline__ void load8(float (&d)[8], const T* row, int64_t e0, int64_t T_, float fill) {
  if (VEC && e0 + 8 <= T_) {
    union { u32x4 u; T e[16 / sizeof(T)]; } b;
    if constexpr (sizeof(T) == 2) {
      b.u = *reinterpret_cast<const u32x4*>(row + e0);
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = (float)b.e[i];
    } else {
      b.u = *reinterpret_cast<const u32x4*>(row + e0);
#pragma unroll
      for (int i = 0; i < 4; ++i) d[i] = (float)b.e[i];
      b.u = *reinterpret_cast<const u32x4*>(row + e0 + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) d[4 + i] = (float)b.e[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = (e0 + i < T_) ? (float)row[e0 + i] : fill;
  }
}

template <typename T, bool VEC>
__device__ __forceinline__ void store8(T* row, int64_t e0, int64_t T_, const float (&d)[8]) {
  if (VEC && e0 + 8 <= T_) {
    if constexpr (sizeof(T) == 2) {
      union { u32x4 u; T e[8]; } b;
#pragma unroll
      for (int i = 0; i < 8; ++i) b.e[i] = (T)d[i];
      *reinterpret_cast<u32x4*>(row + e0) = b.u;
    } else {
      union { u32x4 u; T e[4]; } b;
#pragma unroll
      for (int i = 0; i < 4; ++i) b.e[i] = (T)d[i];
      *reinterpret_cast<u32x4*>(row + e0) = b.u;
#pragma unroll
      for (int i = 0; i < 4; ++i) b.e[i] = (T)d[4 + i];
      *reinterpret_cast<u32x4*>(row + e0 + 4) = b.u;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (e0 + i < T_) row[e0 + i] = (T)d[i];
  }
}

template <bool VEC>
__device__ __forceinline__ void load_mask8(bool (&m)[8], const uint8_t* mrow, int64_t e0, int64_t T_) {
  if (VEC && e0 + 8 <= T_) {
    uint64_t w = *reinterpret_cast<const uint64_t*>(mrow + e0);
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = (w >> (8 * i)) & 0xff;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = (e0 + i < T_) ? mrow[e0 + i] != 0 : false;
  }
}

// ---------------- forward, row cached in registers ----------------
template <typename T, int BLOCK, int NPT, bool VEC, bool MASK>
__global__ __launch_bounds__(BLOCK) void fwd_cached(Args a) {
  __shared__ float red[BLOCK / 64];
  const int64_t row = blockIdx.x;
  const T* x = reinterpret_cast<const T*>(a.x) + row * a.T;
  T* y = reinterpret_cast<T*>(a.out) + row * a.T;
  const uint8_t* mrow = MASK ? a.mask + ((row / a.mdiv) * a.mmul + (row % a.mmod)) * a.T : nullptr;
  const float NEG_INF = -__builtin_inff();
  float v[NPT][8];
  float mx = NEG_INF;
#pragma unroll
  for (int n = 0; n < NPT; ++n) {
    const int64_t e0 = ((int64_t)n * BLOCK + threadIdx.x) * 8;
    load8<T, VEC>(v[n], x, e0, a.T, NEG_INF);
    bool mk[8];
    if (MASK) load_mask8<VEC>(mk, mrow, e0, a.T);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float s = (e0 + i < a.T) ? v[n][i] * a.scale : NEG_INF;
      if (MASK && mk[i]) s = NEG_INF;
      v[n][i] = s;
      mx = fmaxf(mx, s);
    }
  }
  mx = block_reduce<BLOCK>(mx, red, true);
  float sum = 0.f;
#pragma unroll
  for (int n = 0; n < NPT; ++n)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float e = __expf(v[n][i] - mx);
      v[n][i] = e;
      sum += e;
    }
  sum = block_reduce<BLOCK>(sum, red, false);
  const float inv = 1.f / sum;
#pragma unroll
  for (int n = 0; n < NPT; ++n) {
    const int64_t e0 = ((int64_t)n * BLOCK + threadIdx.x) * 8;
    if (e0 < a.T) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[n][i] *= inv;
      store8<T, VEC>(y, e0, a.T, v[n]);
    }
  }
}

// ---------------- forward, streaming (very long rows) ----------------
template <typename T, int BLOCK, bool VEC, bool MASK>
__global__ __launch_bounds__(BLOCK) void fwd_stream(Args a) {
  __shared__ float red[BLOCK / 64];
  const int64_t row = blockIdx.x;
  const T* x = reinterpret_cast<const T*>(a.x) + row * a.T;
  T* y = reinterpret_cast<T*>(a.out) + row * a.T;
  const uint8_t* mrow = MASK ? a.mask + ((row / a.mdiv) * a.mmul + (row % a.mmod)) * a.T : nullptr;
  const float NEG_INF = -__builtin_inff();
  float mx = NEG_INF, sum = 0.f;
  for (int64_t e0 = (int64_t)threadIdx.x * 8; e0 < a.T; e0 += (int64_t)BLOCK * 8) {
    float v[8];
    bool mk[8];
    load8<T, VEC>(v, x, e0, a.T, NEG_INF);
    if (MASK) load_mask8<VEC>(mk, mrow, e0, a.T);
    float lm = NEG_INF;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float s = (e0 + i < a.T) ? v[i] * a.scale : NEG_INF;
      if (MASK && mk[i]) s = NEG_INF;
      v[i] = s;
      lm = fmaxf(lm, s);
    }
    const float nm = fmaxf(mx, lm);
    if (nm != NEG_INF) {
      sum *= __expf(mx - nm);
#pragma unroll
      for (int i = 0; i < 8; ++i) sum += __expf(v[i] - nm);
      mx = nm;
    }
  }
  // combine (max, sum) pairs across the block
  const float gmx = block_reduce<BLOCK>(mx, red, true);
  float part = (mx == NEG_INF) ? 0.f : sum * __expf(mx - gmx);
  const float gsum = block_reduce<BLOCK>(part, red, false);
  const float inv = 1.f / gsum;
  for (int64_t e0 = (int64_t)threadIdx.x * 8; e0 < a.T; e0 += (int64_t)BLOCK * 8) {
    float v[8];
    bool mk[8];
    load8<T, VEC>(v, x, e0, a.T, NEG_INF);
    if (MASK) load_mask8<VEC>(mk, mrow, e0, a.T);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float s = v[i] * a.scale;
      if (MASK && mk[i]) s = NEG_INF;
      v[i] = __expf(s - gmx) * inv;
    }
    store8<T, VEC>(y, e0, a.T, v);
  }
}

// ---------------- backward ----------------
template <typename T, int BLOCK, int NPT, bool VEC>
__global__ __launch_bounds__(BLOCK) void bwd_cached(Args a) {
  __shared__ float red[BLOCK / 64];
  const int64_t row = blockIdx.x;
  const T* y = reinterpret_cast<const T*>(a.x) + row * a.T;
  const T* dy = reinterpret_cast<const T*>(a.dy) + row * a.T;
  T* dx = reinterpret_cast<T*>(a.out) + row * a.T;
  float vy[NPT][8], vd[NPT][8];
  float dot = 0.f;
#pragma unroll
  for (int n = 0; n < NPT; ++n) {
    const int64_t e0 = ((int64_t)n * BLOCK + threadIdx.x) * 8;
    load8<T, VEC>(vy[n], y, e0, a.T, 0.f);
    load8<T, VEC>(vd[n], dy, e0, a.T, 0.f);
#pragma unroll
    for (int i = 0; i < 8; ++i) dot += vy[n][i] * vd[n][i];
  }
  dot = block_reduce<BLOCK>(dot, red, false);
#pragma unroll
  for (int n = 0; n < NPT; ++n) {
    const int64_t e0 = ((int64_t)n * BLOCK + threadIdx.x) * 8;
    if (e0 < a.T) {
#pragma unroll
      for (int i = 0; i < 8; ++i) vd[n][i] = a.scale * vy[n][i] * (vd[n][i] - dot);
      store8<T, VEC>(dx, e0, a.T, vd[n]);
    }
  }
}

template <typename T, int BLOCK, bool VEC>
__global__ __launch_bounds__(BLOCK) void bwd_stream(Args a) {
  __shared__ float red[BLOCK / 64];
  const int64_t row = blockIdx.x;
  const T* y = reinterpret_cast<const T*>(a.x) + row * a.T;
  const T* dy = reinterpret_cast<const T*>(a.dy) + row * a.T;
  T* dx = reinterpret_cast<T*>(a.out) + row * a.T;
  float dot = 0.f;
  for (int64_t e0 = (int64_t)threadIdx.x * 8; e0 < a.T; e0 += (int64_t)BLOCK * 8) {
    float vy[8], vd[8];
    load8<T, VEC>(vy, y, e0, a.T, 0.f);
    load8<T, VEC>(vd, dy, e0, a.T, 0.f);
#pragma unroll
    for (int i = 0; i < 8; ++i) dot += vy[i] * vd[i];
  }
  dot = block_reduce<BLOCK>(dot, red, false);
  for (int64_t e0 = (int64_t)threadIdx.x * 8; e0 < a.T; e0 += (int64_t)BLOCK * 8) {
    float vy[8], vd[8];
    load8<T, VEC>(vy, y, e0, a.T, 0.f);
    load8<T, VEC>(vd, dy, e0, a.T, 0.f);
#pragma unroll
    for (int i = 0; i < 8; ++i) vd[i] = a.scale * vy[i] * (vd[i] - dot);
    store8<T, VEC>(dx, e0, a.T, vd);
  }
}

template <typename T, bool VEC>
static void fwd_dispatch(const Args& a, hipStream_t st) {
  const dim3 g((unsigned)a.rows);
  const bool m = a.mask != nullptr;
#define XF(B, N) \
  { if (m) hipLaunchKernelGGL((fwd_cached<T, B, N, VEC, true>), g, dim3(B), 0, st, a); \
    else   hipLaunchKernelGGL((fwd_cached<T, B, N, VEC, false>), g, dim3(B), 0, st, a); return; }
  if (a.T <= 256 * 8) XF(256, 1)
  if (a.T <= 256 * 16) XF(256, 2)
  if (a.T <= 1024 * 8) XF(1024, 1)
  if (a.T <= 1024 * 16) XF(1024, 2)
  if (a.T <= 1024 * 32) XF(1024, 4)
  if (a.T <= 1024 * 64) XF(1024, 8)
#undef XF
  if (m) hipLaunchKernelGGL((fwd_stream<T, 1024, VEC, true>), g, dim3(1024), 0, st, a);
  else   hipLaunchKernelGGL((fwd_stream<T, 1024, VEC, false>), g, dim3(1024), 0, st, a);
}

template <typename T, bool VEC>
static void bwd_dispatch(const Args& a, hipStream_t st) {
  const dim3 g((unsigned)a.rows);
#define XB(B, N) { hipLaunchKernelGGL((bwd_cached<T, B, N, VEC>), g, dim3(B), 0, st, a); return; }
  if (a.T <= 256 * 8) XB(256, 1)
  if (a.T <= 256 * 16) XB(256, 2)
  if (a.T <= 1024 * 8) XB(1024, 1)
  if (a.T <= 1024 * 16) XB(1024, 2)
  if (a.T <= 1024 * 32) XB(1024, 4)
  if (a.T <= 1024 * 64) XB(1024, 8)
#undef XB
  hipLaunchKernelGGL((bwd_stream<T, 1024, VEC>), g, dim3(1024), 0, st, a);
}

}  // namespace smx
}  // namespace xdot

extern "C" int xdot_softmax_fwd_launch(const xdot::smx::Args* a, int dt, int vec, hipStream_t st) {
  using namespace xdot;
  if (a->rows == 0) return 0;
  if (dt == DT_F32) { vec ? smx::fwd_dispatch<float, true>(*a, st) : smx::fwd_dispatch<float, false>(*a, st); return 0; }
  if (dt == DT_BF16) { vec ? smx::fwd_dispatch<__bf16, true>(*a, st) : smx::fwd_dispatch<__bf16, false>(*a, st); return 0; }
  if (dt == DT_F16) { vec ? smx::fwd_dispatch<_Float16, true>(*a, st) : smx::fwd_dispatch<_Float16, false>(*a, st); return 0; }
  return -1;
}

extern "C" int xdot_softmax_bwd_launch(const xdot::smx::Args* a, int dt, int vec, hipStream_t st) {
  using namespace xdot;
  if (a->rows == 0) return 0;
  if (dt == DT_F32) { vec ? smx::bwd_dispatch<float, true>(*a, st) : smx::bwd_dispatch<float, false>(*a, st); return 0; }
  if (dt == DT_BF16) { vec ? smx::bwd_dispatch<__bf16, true>(*a, st) : smx::bwd_dispatch<__bf16, false>(*a, st); return 0; }
  if (dt == DT_F16) { vec ? smx::bwd_dispatch<_Float16, true>(*a, st) : smx::bwd_dispatch<_Float16, false>(*a, st); return 0; }
  return -1;
}
