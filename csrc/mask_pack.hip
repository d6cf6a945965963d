// xdot — compress the module's boolean attention mask (B, R, T) for the flash kernels.
//
// The reference materialises the expanded mask for every head and applies it with a full
// masked_fill pass over the (B, H, R, T) scores (reference: distributed_dot_product/
// module.py:47-50, :66).  Here the mask is read ONCE per forward (R*T bytes, shared by all
// heads and by the backward) and turned into
//   bits  (B, R, NKT) uint64 : bit k of word kt = mask[b, r, 64*kt + k]
//   bitsT (B, NRT, Tpad) uint64: the same bits column-major per 64-row tile (backward
//         column kernel: one word per lane covers its column's 64 rows)
//   flags (B, ceil(R/32), NKT4) uint8, NKT4 = NKT rounded up to 4: per 32-row x 64-col tile,
//         0 = nothing masked, 1 = everything masked (tile skipped), 2 = partial (bits applied
//         per element).  Rows are padded to 4 bytes so the kernels fetch a tile's flag with a
//         wave-uniform scalar load (s_load_dword), which does not wait on the vector-memory
//         counter that tracks their prefetched K/V tiles.
// An all-False mask (the reference example/benchmark) therefore costs the kernels nothing.
#include "common.h"

namespace xdot {

// One wave per 64-row x 64-column block of one batch: lane i reads row i's 64 mask bytes
// (eight 8-byte loads; rows only need 8-byte alignment, e.g. T = 25000), packs them into its
// row word, stores it (bits), turns the 64 row words into 64 column words with a 6-step
// butterfly transpose across lanes (bits_t) and derives both 32-row flags with two ballots.
// The mask is read exactly once; column tiles kt in [NKT, KT_ALL) only write padding.
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)v, m, 64), hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}

__global__ __launch_bounds__(256) void mask_pack_kernel(const uint8_t* __restrict__ m, uint64_t* __restrict__ bits,
                                                         uint64_t* __restrict__ bt, uint8_t* __restrict__ flags,
                                                         int B, int R, int T, int NKT, int NKT4, int NRT, int Tpad,
                                                         int KT_ALL, bool vec8) {
  const int lane = threadIdx.x & 63;
  const int64_t blk = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk >= (int64_t)B * NRT * KT_ALL) return;  // whole waves exit together
  const int kt = (int)(blk % KT_ALL);
  const int64_t brt = blk / KT_ALL;
  const int rt = (int)(brt % NRT), b = (int)(brt / NRT);
  const int r = rt * 64 + lane;
  const bool row_ok = r < R;
  uint64_t w = 0;
  if (row_ok && kt < NKT) {
    const int c0 = kt * 64;
    const uint8_t* p = m + ((int64_t)b * R + r) * T + c0;
    if (vec8 && c0 + 64 <= T) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint64_t x = *reinterpret_cast<const uint64_t*>(p + 8 * q);
#pragma unroll
        for (int k = 0; k < 8; ++k) w |= (uint64_t)(((x >> (8 * k)) & 0xff) != 0) << (8 * q + k);
      }
    } else {
      const int n = min(64, T - c0);
      for (int k = 0; k < n; ++k) w |= (uint64_t)(p[k] != 0) << k;
    }
    bits[((int64_t)b * R + r) * NKT + kt] = w;
  }
  // flags of the two 32-row halves (rows past R count as neither)
  if (kt < NKT4) {
    const int n = kt < NKT ? min(64, T - kt * 64) : 0;
    const uint64_t full = n == 64 ? ~0ull : ((1ull << n) - 1);
    const uint64_t any = __ballot(w != 0);
    const uint64_t all = __ballot(!row_ok || w == full);
    if ((lane & 31) == 0) {
      const int half = lane >> 5, rb = rt * 2 + half;
      if (rb < (R + 31) / 32) {
        const uint32_t a = (uint32_t)(any >> (32 * half)), l = (uint32_t)(all >> (32 * half));
        flags[((int64_t)b * ((R + 31) / 32) + rb) * NKT4 + kt] = kt >= NKT ? 1 : (a == 0 ? 0 : (l == 0xffffffffu ? 1 : 2));
      }
    }
  }
  // 64 x 64 bit transpose: lane c ends up with column c (bit i = row i)
  if (kt * 64 < Tpad) {
    const uint64_t M[6] = {0x00000000ffffffffull, 0x0000ffff0000ffffull, 0x00ff00ff00ff00ffull,
                           0x0f0f0f0f0f0f0f0full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const int j = 32 >> s;
      const uint64_t o = shfl_xor64(w, j);
      w = (lane & j) ? (((o >> j) & M[s]) | (w & ~M[s])) : ((w & M[s]) | ((o & M[s]) << j));
    }
    bt[((int64_t)b * NRT + rt) * Tpad + (int64_t)kt * 64 + lane] = w;
  }
}

}  // namespace xdot

extern "C" int xdot_mask_pack_launch(const uint8_t* mask, uint64_t* bits, uint64_t* bt, uint8_t* flags, int B, int R,
                                     int T, hipStream_t st) {
  using namespace xdot;
  const int NKT = (T + 63) / 64, NKT4 = (NKT + 3) & ~3, NRT = (R + 63) / 64, Tpad = (T + 127) / 128 * 128;
  const int KT_ALL = max(NKT4, Tpad / 64);
  const bool vec8 = (T % 8 == 0) && ((reinterpret_cast<uintptr_t>(mask) & 7) == 0);
  const int64_t nblk = (int64_t)B * NRT * KT_ALL;
  if (nblk == 0) return 0;
  hipLaunchKernelGGL(mask_pack_kernel, dim3((unsigned)((nblk + 3) / 4)), dim3(256), 0, st, mask, bits, bt, flags, B, R, T,
                     NKT, NKT4, NRT, Tpad, KT_ALL, vec8);
  return 0;
}
