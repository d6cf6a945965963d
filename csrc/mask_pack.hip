// xdot — compress the module's boolean attention mask (B, R, T) for the flash kernels.
//
// The reference materialises the expanded mask for every head and applies it with a full
// masked_fill pass over the (B, H, R, T) scores (reference: distributed_dot_product/
// module.py:47-50, :66).  Here the mask is read ONCE per forward (R*T bytes, shared by all
// heads and by the backward) and turned into
//   bits  (B, NKT, R) uint64 : bit k of word (kt, r) = mask[b, r, 64*kt + k] (kt-major: the
//         producer's stores and the row kernels' per-tile DMAs of 128/256 rows are contiguous)
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

// One wave per 64-row x 128-column block of one batch.  The wave reads the block with
// coalesced 8-byte lane pieces (8 lanes cover 64 contiguous bytes of a row; 8-byte loads when
// rows are 8-byte aligned, e.g. T = 25000, 4-byte or byte loads otherwise), packs every 8 bool bytes to one byte (4 bytes -> 4 bits with one
// 32-bit multiply), regroups the bytes per row through 1 KiB of LDS so lane i holds row i's
// two 64-bit words (a row-per-lane read of the mask was TA-bound: 64 cache lines per load
// instruction), stores them (bits), turns each set
// of 64 row words into 64 column words with a 6-step butterfly transpose across lanes (bits_t)
// and derives the 32-row flags with ballots.  Column tiles kt in [NKT, KT_ALL) only write padding.
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)v, m, 64), hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}

// 4 bool bytes (each 0 or 1: torch's bool storage) -> 4 bits, byte k -> bit k
__device__ __forceinline__ uint32_t pack4(uint32_t x) { return (x * 0x10204080u) >> 28; }

__global__ __launch_bounds__(256) void mask_pack_kernel(const uint8_t* __restrict__ m, uint64_t* __restrict__ bits,
                                                         uint64_t* __restrict__ bt, uint8_t* __restrict__ flags,
                                                         int B, int R, int T, int NKT, int NKT4, int NRT, int Tpad,
                                                         int KT_ALL, int va) {
  const int lane = threadIdx.x & 63;
  const int KT2 = (KT_ALL + 1) / 2;
  const int64_t blk = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk >= (int64_t)B * NRT * KT2) return;  // whole waves exit together
  const int kt0 = (int)(blk % KT2) * 2;
  const int64_t brt = blk / KT2;
  const int rt = (int)(brt % NRT), b = (int)(brt / NRT);
  const int r = rt * 64 + lane;
  const bool row_ok = r < R;
  uint64_t wv[2] = {0, 0};
  __shared__ __attribute__((aligned(16))) uint8_t stage[4][64 * 16];  // per wave: 64 rows x 128 bits
  uint8_t* sw = stage[threadIdx.x >> 6];
  const int c0 = kt0 * 64;
  if (kt0 < NKT && c0 + 128 <= T) {
    // coalesced: instruction (i, j) reads rows 8i..8i+7, bytes 64j..64j+63 of the block
    // (8 lanes x 8 B contiguous per row); each lane packs its 8 bytes to one byte in LDS
    uint64_t x[16];
    const int lr = lane >> 3, lc = (lane & 7) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rr = rt * 64 + 8 * i + lr;
      const uint8_t* p = m + ((int64_t)b * R + min(rr, R - 1)) * T + c0 + lc;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint8_t* q = p + 64 * j;
        uint64_t v;
        if (va == 8) {
          v = *reinterpret_cast<const uint64_t*>(q);
        } else if (va == 4) {  // rows 4-byte aligned (T % 8 == 4, e.g. T = 12500)
          v = (uint64_t)*reinterpret_cast<const uint32_t*>(q) | ((uint64_t)*reinterpret_cast<const uint32_t*>(q + 4) << 32);
        } else {               // odd row strides: byte loads, still 64 contiguous bytes per 8 lanes
          v = 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) v |= (uint64_t)q[e] << (8 * e);
        }
        x[2 * i + j] = rr < R ? v : 0ull;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint64_t v = x[2 * i + j];
        sw[(8 * i + lr) * 16 + 8 * j + (lane & 7)] = (uint8_t)(pack4((uint32_t)v) | (pack4((uint32_t)(v >> 32)) << 4));
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-private staging
    __builtin_amdgcn_wave_barrier();
    const u32x4 q = *reinterpret_cast<const u32x4*>(sw + lane * 16);
    wv[0] = ((uint64_t)q[1] << 32) | q[0];
    wv[1] = ((uint64_t)q[3] << 32) | q[2];
  } else if (row_ok && kt0 < NKT) {
    const uint8_t* p = m + ((int64_t)b * R + r) * T + c0;
    const int n = min(128, T - c0);
    for (int k = 0; k < n; ++k) wv[k >> 6] |= (uint64_t)(p[k] != 0) << (k & 63);
  }
  if (row_ok && kt0 < NKT) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (kt0 + h < NKT) bits[((int64_t)b * NKT + kt0 + h) * R + r] = wv[h];  // kt-major: coalesced
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int kt = kt0 + h;
    uint64_t w = wv[h];
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
}

}  // namespace xdot

extern "C" int xdot_mask_pack_launch(const uint8_t* mask, uint64_t* bits, uint64_t* bt, uint8_t* flags, int B, int R,
                                     int T, hipStream_t st) {
  using namespace xdot;
  const int NKT = (T + 63) / 64, NKT4 = (NKT + 3) & ~3, NRT = (R + 63) / 64, Tpad = (T + 127) / 128 * 128;
  const int KT_ALL = max(NKT4, Tpad / 64);
  // widest load every row start satisfies (the kernel reads each row's 128-column block as
  // 8-byte lane pieces; narrower alignment splits them, the access pattern stays coalesced)
  const uintptr_t base = reinterpret_cast<uintptr_t>(mask);
  const int va = (T % 8 == 0 && (base & 7) == 0) ? 8 : (T % 4 == 0 && (base & 3) == 0) ? 4 : 1;
  const int64_t nblk = (int64_t)B * NRT * ((KT_ALL + 1) / 2);
  if (nblk == 0) return 0;
  hipLaunchKernelGGL(mask_pack_kernel, dim3((unsigned)((nblk + 3) / 4)), dim3(256), 0, st, mask, bits, bt, flags, B, R, T,
                     NKT, NKT4, NRT, Tpad, KT_ALL, va);
  return 0;
}
