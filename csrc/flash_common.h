// xdot — shared pieces of the gfx950 flash-attention kernels (fwd + bwd).
//
// Conventions (see csrc/flash_fwd.hip for the full design):
//   "rows"  = local query-side rows of this rank (the module's projected `keys`, R rows)
//   "cols"  = gathered key-side rows (the module's projected `queries`/`values`, T rows)
//   All tensors are head-interleaved (..., H*D) so no transpose copies exist anywhere.
//   Gathered tensors are (B, T, ld): col t of batch b lives at (b*T + t)*ld + h*D (the RCCL
//   all-gather output (N, 1, R, ld) is exactly this layout for B = 1).  With the packed
//   [q | v] projection ld = 2*H*D and v starts H*D elements after q.
// MFMA: v_mfma_f32_32x32x16_{bf16,f16}.  For a 32x32 accumulator X, lane l holds column
// l&31 and rows (r&3) + 8*(r>>2) + 4*(l>>5), r = 0..15 (CDNA4 C/D map).
#pragma once
#include "common.h"

#include <cstdlib>
#include <utility>

namespace xdot {
namespace fa {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// ----------------------------------------------------------------------------------------
template <int DT> struct mfma32;
template <> struct mfma32<DT_BF16> {
  static __device__ __forceinline__ f32x16 run(u32x4 a, u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};
template <> struct mfma32<DT_F16> {
  static __device__ __forceinline__ f32x16 run(u32x4 a, u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
};

// pack two fp32 into one dword of two 16-bit values (round to nearest even)
template <int DT> __device__ __forceinline__ uint32_t pack2(float a, float b);
template <> __device__ __forceinline__ uint32_t pack2<DT_BF16>(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) __bf16 bf2;
  bf2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}
template <> __device__ __forceinline__ uint32_t pack2<DT_F16>(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) _Float16 h2;
  h2 v = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// accumulator registers 8s..8s+7 of a 32x32 tile -> MFMA operand fragment (k-step s)
template <int DT>
__device__ __forceinline__ u32x4 acc_to_frag(const f32x16& x, int s) {
  u32x4 r;
  r[0] = pack2<DT>(x[8 * s + 0], x[8 * s + 1]);
  r[1] = pack2<DT>(x[8 * s + 2], x[8 * s + 3]);
  r[2] = pack2<DT>(x[8 * s + 4], x[8 * s + 5]);
  r[3] = pack2<DT>(x[8 * s + 6], x[8 * s + 7]);
  return r;
}

// ---- LDS tile images -------------------------------------------------------------------
// One layout serves both ways a tile is read: rows of IMG_ROW bytes (D = 32/64/96/128 ->
// 64/192/192/320) whose 16-byte chunks are XOR-swizzled by (row >> 2) & 3.  Checked against
// the gfx950 LDS bank model (ds_read_b128: four 16-lane groups, ds_read_b64_tr_b16: two
// 32-lane halves, banks (addr/4) % 64): both the row-operand reads and the transposed reads
// below are conflict-free.
// Wide heads (flash_wide.hip, D > 128): 2D bytes, + 64 unless ROW/4 is already 16 or 48 mod 64
// dwords (the residues the bank analysis above holds for).
constexpr int wide_row(int D) { return ((D / 2) % 64 == 16 || (D / 2) % 64 == 48) ? 2 * D : 2 * D + 64; }
template <int D> struct Img {
  static constexpr int ROW = (D == 32) ? 64 : (D == 64 || D == 96) ? 192 : (D == 128) ? 320 : wide_row(D);
  static constexpr int BYTES = 64 * ROW;  // one 64-row tile
  static_assert((ROW / 4) % 64 == 16 || (ROW / 4) % 64 == 48, "image row residue");
};
template <int D>
__device__ __forceinline__ int img_off(int row, int chunk) {
  return row * Img<D>::ROW + ((chunk ^ ((row >> 2) & 3)) << 4);
}

// Per-lane byte bases into an image.  Every tile row offset used by the kernels (0, 16, 32,
// 48) is a multiple of 16 rows, so the swizzle term of a read depends only on the lane:
// two bases per read kind, everything else folds into the ds_read immediate offset.
struct Lanes {
  int rb0, rb1;  // row reads: even / odd k-step
  int tb0, tb1;  // transposed reads: rows k0 + 4h + q, and the same + 8
};
template <int D>
__device__ __forceinline__ Lanes make_lanes(int lane) {
  constexpr int ROW = Img<D>::ROW;
  Lanes L;
  const int hf = lane >> 5, r = lane & 31, f = (r >> 2) & 3;
  L.rb0 = r * ROW + ((hf ^ f) << 4);
  L.rb1 = r * ROW + (((2 + hf) ^ f) << 4);
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int cl = 2 * (g & 1) + (p >> 1);  // chunk bits below the d0 block (d0/8 is a multiple of 4)
  L.tb0 = (4 * hf + q) * ROW + ((cl ^ hf) << 4) + 8 * (p & 1);
  L.tb1 = (4 * hf + q + 8) * ROW + ((cl ^ (2 + hf)) << 4) + 8 * (p & 1);
  return L;
}

// Transposed operand from a [key][d] image, matching acc_to_frag's k order:
// lane l (d = d0 + (l&31), h = l>>5) gets elements j <-> key k0 + 8*(j>>2) + 4h + (j&3).
// k0 must be a multiple of 16, d0 a multiple of 32.
template <int D>
__device__ __forceinline__ u32x4 tr_frag(const char* img, int k0, int d0, const Lanes& L) {
  constexpr int ROW = Img<D>::ROW;
  // offsets added in the LDS address space: the constant part folds into the instruction's
  // 16-bit offset instead of a precomputed address register per (k0, d0)
  typedef const __attribute__((address_space(3))) char lds_char;
  lds_char* base = (lds_char*)img;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + L.tb0 + (k0 * ROW + d0 * 2)));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + L.tb1 + (k0 * ROW + d0 * 2)));
  union { struct { s16x4 a, b; } s; u32x4 u; } c;
  c.s.a = lo;
  c.s.b = hi;
  return c.u;
}

// Row-operand fragment (A or B of a 32x32x16 MFMA) from a [row][d] image:
// lane l: row r0 + (l&31), d = 16*s + 8*(l>>5) .. +7.  r0 must be a multiple of 16.
template <int D>
__device__ __forceinline__ u32x4 row_frag(const char* img, int r0, int s, const Lanes& L) {
  return *reinterpret_cast<const u32x4*>(img + ((s & 1) ? L.rb1 : L.rb0) + r0 * Img<D>::ROW + (s >> 1) * 64);
}

// global element offset of gathered col t (head offset excluded); ld = row stride
__device__ __forceinline__ int64_t col_off(int t, int b, int T, int64_t ld) {
  return ((int64_t)b * T + t) * ld;
}

// combine a value with the partner lane (lane ^ 32) through v_permlane32_swap (no LDS)
__device__ __forceinline__ float pair_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false, false);
  return __builtin_fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}
__device__ __forceinline__ float pair_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}


// ---- LDS-DMA staging ---------------------------------------------------------------------
// Tiles travel HBM -> LDS through global_load_lds (no VGPRs hold a tile in flight).  The DMA
// destination is lane-linear (wave-uniform M0 base + lane * size), so a swizzled image is
// produced by permuting the per-lane SOURCE addresses.  Kernels count their DMAs and wait
// with a counted `s_waitcnt vmcnt(N)` + raw s_barrier so the next tiles stay in flight.
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// tile index of accumulator register r for lane half hf
__device__ __forceinline__ int tidx(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }

// Score-buffer block I/O (exact-fp32 / split-bf16 / wide flash families, kernels.h BwdArgs::sbuf).  A 32x32 accumulator x holds element (a, b) with a = lane & 31 (lane
// index) and b = tidx(r, lane >> 5) (register r).  blk_store writes it TRANSPOSED into the
// reader's accumulator order: element (a, b) to [lane' = b + 32((a>>2)&1)][r' = (a&3) + 4(a>>3)],
// i.e. the reader whose lane index is b finds it in its register r' -> blk_load(blk, lane)[r'].
// (forward: a = row, b = column -> the column kernel's order; column kernel: a = column,
// b = row -> the row kernel's order.)  Per lane 16 scattered dword stores / 4 b128 loads.
__device__ __forceinline__ void blk_store(float* blk, const f32x16& x, int lane) {
  const int a = lane & 31, hf = lane >> 5;
  float* p = blk + 512 * ((a >> 2) & 1) + (a & 3) + 4 * (a >> 3);
#pragma unroll
  for (int r = 0; r < 16; ++r) p[16 * tidx(r, hf)] = x[r];
}
// The same through a wave-private 4-KiB LDS tile: the scatter goes to LDS (16 ds_write_b32, the
// 2-way bank conflicts of which cost nothing), then the block leaves as 4 coalesced 16-byte global
// stores per lane (64 lanes x 64 B contiguous) instead of 16 dword stores in 64-byte pieces
// (the direct scatter measured 2.5 % slower, the unswizzled tile the same: profiles/r5_fp32.md).
// Two halves, so the caller can put the tile's LDS writes before its next MFMA block and flush
// after it (the writes' latency then hides under the MFMAs instead of a wait in front of them).
// The tile position q of logical float q is q ^ 16 ((q >> 6) & 1) ^ 32 ((q >> 9) & 1): the 16
// scatter writes then cover all 64 banks (unswizzled: 16 banks, 4-way conflicts), and each
// reader lane's 16 floats stay one contiguous 64-byte slot (slot l ^ ((l >> 2) & 1) ^
// 2 ((l >> 5) & 1)), read chunk-rotated so every 16-lane b128 phase hits 16 bank quads.
__device__ __forceinline__ void blk_put_lds(float* wl, const f32x16& x, int lane) {
  const int a = lane & 31, hf = lane >> 5, sa = (a >> 2) & 1, k = hf + 2 * sa;
  float* p = wl + 512 * sa + (a & 3) + 4 * (a >> 3) + 64 * hf;
#pragma unroll
  for (int r = 0; r < 16; ++r) p[128 * (r >> 2) + 16 * ((r & 3) ^ k)] = x[r];
}
__device__ __forceinline__ void blk_flush_lds(float* blk, const float* wl, int lane) {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-private tile, no barrier
  const int slot = lane ^ ((lane >> 2) & 1) ^ (2 * ((lane >> 5) & 1));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = (i + (lane >> 2)) & 3;
    *reinterpret_cast<f32x4*>(blk + 16 * lane + 4 * c) = *reinterpret_cast<const f32x4*>(wl + 16 * slot + 4 * c);
  }
}
__device__ __forceinline__ void blk_store_lds(float* blk, float* wl, const f32x16& x, int lane) {
  blk_put_lds(wl, x, lane);
  blk_flush_lds(blk, wl, lane);
}
// float offset of the dump block after the last score block: writes of waves that own no block
// (rows past R, columns past T) go there, so every wave issues the same stores every tile
__device__ __forceinline__ int64_t sb_dump(int B, int H, int R, int T) {
  return (int64_t)B * H * ((R + 31) / 32) * ((T + 31) / 32) * 1024;
}
__device__ __forceinline__ f32x16 blk_load(const float* blk, int lane) {
  const f32x4* p = reinterpret_cast<const f32x4*>(blk + 16 * lane);
  f32x16 x;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x4 v = p[q];
#pragma unroll
    for (int t = 0; t < 4; ++t) x[4 * q + t] = v[t];
  }
  return x;
}

// flag of (32-row block rb32, 64-col tile kt64): 0 none / 1 all / 2 some masked
// The per-lane mask word of a partially masked tile, waited for INSIDE the `flag == 2` branch (an
// empty asm use): otherwise the wait lands at the branch join and even unmasked tiles drain this
// wave's whole vector-memory queue (the score-block and staging prefetches) every tile.
__device__ __forceinline__ uint32_t settle(uint32_t w) {
  asm volatile("" : "+v"(w));
  return w;
}
// A SCALAR load (constant address space, wave-uniform index; NKT4 % 4 == 0 keeps each flag row
// dword-aligned): it waits on lgkmcnt.  As a vector byte load it joined the in-order vector-memory
// queue behind the tile's prefetches, and its wait (at the join of the `mflags ? ... : 0` branch,
// so even without a mask) drained every prefetch each tile.
__device__ __forceinline__ int flag_at(const uint8_t* flags, int b, int NRB32, int NKT4, int rb32, int kt64) {
  const int64_t idx = ((int64_t)b * NRB32 + rb32) * NKT4 + kt64;
  typedef const __attribute__((address_space(4))) uint32_t cu32;
  const uint32_t w = reinterpret_cast<cu32*>(reinterpret_cast<uintptr_t>(flags))[idx >> 2];
  return (int)((w >> (8 * (idx & 3))) & 0xffu);
}

// Deep prefetch of a strided stream of score blocks (score-buffer kernels): SB_PF blocks in
// flight per wave in a register ring.  The loop is unrolled by the ring depth so that each step's
// slot is a compile-time index: no in-flight register is ever copied (a copy would wait for its
// load).  body(i, J) handles stream element i from slot J::value, then refills that slot with
// element i + PF.  One 4-KiB block per tile is too little to cover HBM latency when the tile's
// products are short (the dV and dK passes: one product per tile).
constexpr int SB_PF = 1;  // depths 1 / 2 / 3 measured equal (profiles/r5_fp32.md): no ring copies at 1
template <int N> struct Ic { static constexpr int value = N; };
template <int PF, class F> __device__ __forceinline__ void ring_loop(int beg, int end, F&& body) {
  static_assert(PF >= 1 && PF <= 4, "ring depth");
  for (int i0 = beg; i0 < end; i0 += PF) {
    body(i0, Ic<0>{});
    if constexpr (PF > 1)
      if (i0 + 1 < end) body(i0 + 1, Ic<1>{});
    if constexpr (PF > 2)
      if (i0 + 2 < end) body(i0 + 2, Ic<2>{});
    if constexpr (PF > 3)
      if (i0 + 3 < end) body(i0 + 3, Ic<3>{});
  }
}

// Row splits of a column-side launch: W workgroups of `nrt` 32-row tiles each, `slots` of them
// resident at once.  Fewest splits minimising ceil(W s / slots) / s (the idle share of the last
// round), each split >= 16 row tiles, 2 % charged per extra split (partials + their sum).
// (The fp32 forward / row kernels use it with up to 8 splits at 0.4 % each: their partials are
// ~1 % of an exact-fp32 kernel's time.)
inline int pick_csplit(int64_t W, int nrt, int slots, int maxs = 4, double per = 0.02) {
  int best = 1;
  double bc = 1e300;
  for (int s = 1; s <= maxs && (s == 1 || nrt / s >= 16); ++s) {
    const double c = (double)((W * s + slots - 1) / slots) / s * (1.0 + per * (s - 1));
    if (c < bc * 0.98) {
      bc = c;
      best = s;
    }
  }
  return best;
}
// resident workgroups per CU of one kernel instantiation (256 threads, `lds` bytes), cached
template <class K> int wg_per_cu(K kern, int lds) {
  static int v = 0;
  if (!v) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(kern), 256, lds) != hipSuccess || n < 1)
      n = 1;
    v = n;
  }
  return v;
}

// Pin MFMA accumulators to AGPRs (an empty asm with an "a" constraint).  Where accumulators and
// operand fragments together exceed the 256 VGPRs, the allocator otherwise keeps loop-carried
// accumulators in VGPRs and copies them into AGPRs around every product (2 VALU moves per
// register per product) or spills.
template <int N>
__device__ __forceinline__ void pin_agpr(f32x16 (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+a"(x[i]));
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// LDS-DMA of 16 / 4 bytes per lane: LDS[lds_wave_base + lane * size] <- global[base + off].
// Inline asm on purpose: for the builtin, hipcc inserts `s_waitcnt vmcnt(0)` in front of every
// ds_read_b64_tr_b16 while any DMA is pending (it cannot prove they do not alias), which
// would drain the prefetch ring every tile.  The kernel counts these DMAs itself (wait_vm).
// The dynamic LDS of the flash kernels: ONE symbol for all of them, so LDS-DMA destinations are
// its LDS address + a byte offset the compiler folds to a constant (converting an arbitrary
// generic pointer back to an LDS address costs ~8 SALU of null checks per DMA call).
extern __shared__ __attribute__((aligned(16))) char smem[];
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem + (uint32_t)((const char*)p - smem);
}
__device__ __forceinline__ void glds16(const void* base, uint32_t off, const char* lds_wave_base) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(off), "s"(base), "s"(lds_addr(lds_wave_base)) : "memory");
}
__device__ __forceinline__ void glds4(const void* base, uint32_t off, const char* lds_wave_base) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(off), "s"(base), "s"(lds_addr(lds_wave_base)) : "memory");
}


// IPW consecutive 1-KiB pieces of one wave (LDS destinations lds, lds + 1 KiB, ...) in ONE asm
// block: M0 is saved / restored once and stepped with s_add between pieces (per piece 1 SALU + 1
// wait state instead of 3 SALU + 2 wait states: 12 pieces per forward tile per wave)
template <int N> struct GldsRun;
template <> struct GldsRun<1> {
  static __device__ __forceinline__ void run(const void* base, const uint32_t* o, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(o[0]), "s"(lds), "s"(base) : "memory");
  }
};
template <> struct GldsRun<2> {
  static __device__ __forceinline__ void run(const void* base, const uint32_t* o, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %4\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %4\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(o[0]), "v"(o[1]), "s"(lds), "s"(base) : "memory", "scc");
  }
};
template <> struct GldsRun<4> {
  static __device__ __forceinline__ void run(const void* base, const uint32_t* o, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %5\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %6\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %6\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %6\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %6\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]), "s"(lds), "s"(base) : "memory", "scc");
  }
};
template <> struct GldsRun<3> {
  static __device__ __forceinline__ void run(const void* base, const uint32_t* o, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %5\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %5\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %5\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(o[0]), "v"(o[1]), "v"(o[2]), "s"(lds), "s"(base) : "memory", "scc");
  }
};
template <> struct GldsRun<5> {
  static __device__ __forceinline__ void run(const void* base, const uint32_t* o, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %7\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %7\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %7\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %7\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %5, %7\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]), "v"(o[4]), "s"(lds), "s"(base)
                 : "memory", "scc");
  }
};

// Per-lane DMA sources of one 64-row swizzled image, filled by the 4 waves of a workgroup in
// IPW 1-KiB pieces each: image position p holds chunk ((p % ROW) / 16) ^ ((row >> 2) & 3) of
// tile row p / ROW (padding positions of D = 64/128 images load chunk 0: any valid address).
template <int D> struct ImgDma {
  static constexpr int IPW = Img<D>::BYTES / 4096;
  int off[IPW], row[IPW];  // per lane: byte offset of its chunk in a full tile, tile row
  __device__ __forceinline__ void init(int wave, int lane, int stride_bytes) {
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int p = (wave * IPW + i) * 1024 + lane * 16, r = p / Img<D>::ROW;
      int c = ((p % Img<D>::ROW) >> 4) ^ ((r >> 2) & 3);
      if (c >= D / 8) c = 0;
      row[i] = r;
      off[i] = r * stride_bytes + c * 16;
    }
  }
  // base is the tile's first row; a full tile uses the precomputed offsets as the DMA's
  // 32-bit VGPR offset (no per-DMA address arithmetic), rows past rmax (tail tile) re-read
  // row rmax (callers mask them)
  __device__ __forceinline__ void issue(const char* base, int stride_bytes, int rmax, char* img, int wave) const {
    uint32_t o[IPW];
    if (rmax >= 63) {
#pragma unroll
      for (int i = 0; i < IPW; ++i) o[i] = (uint32_t)off[i];
    } else {
#pragma unroll
      for (int i = 0; i < IPW; ++i) o[i] = (uint32_t)(off[i] - (row[i] - min(row[i], rmax)) * stride_bytes);
    }
    GldsRun<IPW>::run(base, o, lds_addr(img + wave * IPW * 1024));
  }
};

// Ring stage of the row-block kernels (flash_fwd, flash_bwd_rows): the 64-column tile of the
// key/value side as two images + the 64-bit mask words of the workgroup's 128 rows for that
// column tile ([dword][128 rows]) + a 256-byte sink for the dummy DMA that keeps the count
// per wave constant when there is no mask.
template <int D> struct RowsCfg {
  static constexpr int IMG = Img<D>::BYTES;
  static constexpr int IPW = ImgDma<D>::IPW;
  static constexpr int OFF_W = 2 * IMG, OFF_X = OFF_W + 1024, OFF_F = OFF_X + 256;
  static constexpr int STAGE = OFF_F + 256;
  static constexpr int NBUF = (2 * 3 * STAGE <= 160 * 1024) ? 3 : 2;
  static constexpr int PF = NBUF - 1;
  static constexpr int NG = 2 * IPW + 2;
};

// Tile flags travel with their tile through the LDS ring (a scalar load per tile would put
// its ~µs latency and an lgkmcnt(0) on every iteration's critical path).  One 4-byte DMA per
// wave: lane i < nrows fetches dword `dw` of flag row i (rows `stride` bytes apart) into
// dst + 4 i (lanes >= nrows repeat row 0; the 256-byte area absorbs all 64 lanes).
__device__ __forceinline__ void glds_flags(const uint8_t* row0, int stride, int nrows, int dw, char* dst) {
  const int lane = threadIdx.x & 63;
  glds4(row0 + dw * 4, (uint32_t)((lane < nrows ? lane : 0) * stride), dst);
}
// byte `byte` of staged flag dword `idx` (wave-uniform)
__device__ __forceinline__ int staged_flag(const char* area, int idx, int byte) {
  const uint32_t v = __builtin_amdgcn_readfirstlane(reinterpret_cast<const uint32_t*>(area)[idx]);
  return (v >> (8 * byte)) & 0xff;
}

// mask word of workgroup row rr (0..ROWS-1) for the staged column tile ([dword][ROWS rows])
template <int ROWS = 128>
__device__ __forceinline__ uint64_t staged_word(const char* stage_w, int rr) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(stage_w);
  return (uint64_t)w[rr] | ((uint64_t)w[ROWS + rr] << 32);
}

// Masked-column bits of a 64-column tile for the lane's half (lane >> 5): bit j of the result
// covers tile column (j & 3) + 8 (j >> 2)... in the MFMA C/D order, i.e. register r of sub-tile
// tt tests bit tt*32 + (r&3) + 8*(r>>2) (constant positions: no per-lane column indices).
// Columns past T (tail tile) count as masked.
__device__ __forceinline__ uint64_t tile_bits(uint64_t w, int valid, int hf) {
  if (valid < 64) w |= ~0ull << valid;
  return w >> (4 * hf);
}
__device__ __forceinline__ bool bit_at(uint64_t w, int j) {
  return j < 32 ? ((uint32_t)w >> j) & 1u : ((uint32_t)(w >> 32) >> (j - 32)) & 1u;
}

// Masked-entry select: d[r] = (bit (r & 3) + 8 (r >> 2) of w) ? y : d[r] for the 16 registers of
// a 32x32 accumulator (the MFMA C/D row order of one lane half), y given as raw bits.  Per score
// v_bfe_i32 (bit -> 0 / -1) + v_bfi_b32 ((m & y) | (~m & x)), one asm statement each (hipcc
// turns plain C into a compare + v_cndmask form that measured +0.14 ms on the forward with a
// 10 % random mask; a single asm block over all 16 registers gave intermittently wrong
// results).  A random mask makes EVERY tile partial, so this runs on every score of every head.
template <int B>
__device__ __forceinline__ float sel_bit(uint32_t w, float x, uint32_t ybits) {
  uint32_t m, r;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(w), "n"(B));
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "s"(ybits), "v"(__builtin_bit_cast(uint32_t, x)));
  return __builtin_bit_cast(float, r);
}
template <int... R>
__device__ __forceinline__ void sel_bits16_(f32x16& d, uint32_t w, uint32_t ybits, std::integer_sequence<int, R...>) {
  ((d[R] = sel_bit<(R & 3) + 8 * (R >> 2)>(w, d[R], ybits)), ...);
}
__device__ __forceinline__ void sel_bits16(f32x16& d, uint32_t w, uint32_t ybits) {
  sel_bits16_(d, w, ybits, std::make_integer_sequence<int, 16>{});
}
constexpr uint32_t PINF_BITS = 0x7F800000u, NINF_BITS = 0xFF800000u;

// v_exp_f32 directly (exp2f would add a denormal-range fix-up of ~3 VALU ops per call;
// arguments here are <= 0 and results below 2^-126 are irrelevant to a softmax)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Scalar (SMEM) load of one dword at a wave-uniform address.  hipcc only emits s_load for
// memory it can prove unclobbered; otherwise it falls back to a vector load + readfirstlane
// whose `s_waitcnt vmcnt(0)` would also drain every tile prefetch in flight.
__device__ __forceinline__ uint32_t sload_u32(const uint32_t* p) {
  uint32_t v;
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p));
  return v;
}

// Flag of mask tile `kt` from a 4-byte padded flag row (wave-uniform row and kt).
__device__ __forceinline__ int tile_flag(const uint8_t* __restrict__ row, int kt) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(row) + __builtin_amdgcn_readfirstlane(kt >> 2);
  const uint32_t v = sload_u32(w);
  return (v >> (8 * (kt & 3))) & 0xff;
}


}  // namespace fa
}  // namespace xdot
