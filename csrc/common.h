// xdot — shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
//
// Every kernel in csrc/ is written for wave64 / MFMA / 160 KiB LDS only; there is no
// portability layer.  Element types are carried as raw storage types:
//   DT_F32  -> float, DT_BF16 -> __bf16, DT_F16 -> _Float16
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kernels.h"

namespace xdot {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
// 16-byte vector at a 2-byte-aligned address: gfx950 under ROCm runs in unaligned-access mode,
// so this is still ONE global_load/store_dwordx4 (GEMM epilogues writing column blocks that start
// off 16-byte boundaries, e.g. nt's per-rank blocks at an odd T/N)
typedef u32x4 u32x4_ua __attribute__((aligned(2)));
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

constexpr int kWave = 64;

template <typename T> __device__ __forceinline__ float to_f32(T x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x) { return (T)x; }

// Element-type traits used by templated kernels.
template <int DT> struct dt_traits;
template <> struct dt_traits<DT_F32>  { using T = float;    static constexpr int kBytes = 4; };
template <> struct dt_traits<DT_BF16> { using T = __bf16;   static constexpr int kBytes = 2; };
template <> struct dt_traits<DT_F16>  { using T = _Float16; static constexpr int kBytes = 2; };

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// XCD-aware, bijective remap of a linear workgroup id (MI355X: 8 XCDs, blocks are dealt
// round-robin; remapping gives each XCD a contiguous run of logical tiles so neighbouring
// tiles that share operand panels share one L2).  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int wg, int nwg) {
  constexpr int NX = 8;
  if (nwg <= NX) return wg;
  int xcd = wg % NX, q = nwg / NX, r = nwg % NX;
  int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + wg / NX;
}

}  // namespace xdot
