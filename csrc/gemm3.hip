// xdot — 8-phase 16-bit MFMA GEMM for gfx950 (the "v3" path of xdot.gemm).
//
//   C[z](m, n) = alpha * sum_{s < nseg} sum_{k < K} opA_s[z](m, k) * opB_s[z](k, n) + beta * C[z](m, n)
//
// Same addressing model as csrc/gemm.hip / csrc/gemm2.hip (2-level batch, K segments, each
// operand k- or mn-contiguous), so it carries the reference's three distributed products
// (distributed_dot_product/multiplication/functions.py:89-97 nt, :140-147 tn, :202-211 all).
// What changes against gemm2 (0.75x hipBLASLt on the plain large products,
// profiles/r2_gemm2_schedules_rejected.md):
//   * v_mfma_f32_16x16x32: at a power-limited clock the chip holds a higher clock on this
//     shape (1.13x the 32x32x16 rate on random data, profiles/r3_mfma_shape.md);
//   * the k-tile is split into four 16 KiB half-tile images (A rows 0-127 / 128-255, B
//     columns 0-127 / 128-255) and the loop into 4 phases per k-tile, each phase one
//     64x32 quadrant of the wave's 128x64 output x K=64 (16 MFMAs) and ONE half-tile of
//     LDS-DMA.  A half-tile is re-filled as soon as its last reader is two phases behind, so
//     four half-tiles (two k-tiles' worth of lookahead, ~4 phases of latency cover) stay in
//     flight across the raw barriers with counted `s_waitcnt vmcnt(8)` -- never 0 in the loop;
//   * the two waves of each SIMD run one barrier apart (waves 4-7 start one barrier late):
//     one wave's fragment reads and DMA issue overlap its partner's MFMAs;
//   * persistent grid walking (split, batch, tile) items; the k-tile stream runs straight
//     across items (the next item's tiles are in flight during this item's last phases); the
//     epilogue converts in registers and stores 16 bytes per lane (v_permlane16_swap pairs
//     two 16x16 accumulators into 8 consecutive columns), one output quadrant per phase of the
//     item's last k-tile -- no LDS round trip, no store burst for the DMA stream to queue behind;
//   * edge tiles are shifted inside the matrix (m0 = min(256 tm, M - 256)), so every DMA
//     source is in bounds with item-independent per-lane offsets; the overlap rows/columns
//     are recomputed bitwise identically and simply stored twice (hence beta = 0 only);
//   * K tails: operands stream through buffer_load ... lds; the tail k-tile's dead 16-byte
//     chunks / k rows get an out-of-range offset, so the DMA writes zeros (K % 8 == 0).
// Eligibility (checked by xdot_gemm3_launch): 16-bit A/B, beta = 0, M >= 256, N >= 256, 16-byte aligned
// operand bases, lda/ldb/batch/segment strides multiples of 8 elements, K % 8 == 0 unless both
// operands are mn-contiguous.
#include "flash_common.h"

namespace xdot {
namespace g3 {

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
#ifndef G3_FL
#define G3_FL 1  // whole-line epilogue stores for 16-bit C with k-contiguous B (A/B knob)
#endif
#ifndef G3_STORE_AUX
#define G3_STORE_AUX 0  // cache policy of the output stores (A/B knob of scripts/gemm3_ab.sh)
#endif
constexpr int HALF = 16384;       // one half-tile image (128 x 64 x 2 B)
constexpr int SLOT = 4 * HALF;    // [A 0-127 | A 128-255 | B 0-127 | B 128-255]
constexpr int TAB = 2 * SLOT;     // 128 KiB ring: two k-tiles; then the item table
constexpr int MAX_ITEMS = 2048;   // items per workgroup (16-byte entries, 32 KiB)
constexpr int LDS = TAB + 16 * MAX_ITEMS;

template <int DT> __device__ __forceinline__ f32x4 mfma16(u32x4 a, u32x4 b, f32x4 c) {
  if constexpr (DT == DT_BF16)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef f32x4 f32x4_ua __attribute__((aligned(4)));
// raw buffer descriptor over [base, base + 2 GiB): an offset >= 0x7FFFFFF0 is out of range and
// its LDS-DMA writes zeros (the K-tail lanes' offsets are set to 0x80000000)
constexpr uint32_t OOB = 0x80000000u;
__device__ __forceinline__ i32x4 rsrc_of(const void* base) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  i32x4 r;
  r[0] = (int)__builtin_amdgcn_readfirstlane((uint32_t)b);
  r[1] = (int)(__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) & 0xFFFFu);
  r[2] = 0x7FFFFFF0;
  r[3] = 0x00020000;
  return r;
}
// two consecutive 1 KiB LDS-DMA pieces of one wave through buffer_load ... lds (M0 stepped by
// s_add, saved once)
__device__ __forceinline__ void bdma2(i32x4 rsrc, uint32_t o0, uint32_t o1, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %4, 0 offen lds\n\t"
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %4, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(o0), "v"(o1), "s"(lds), "s"(rsrc) : "memory", "scc");
}

// swap lanes 16-31 <-> ... (odd 16-lane rows of x with even rows of y); returns {x', y'}
__device__ __forceinline__ void swap16(uint32_t& x, uint32_t& y) {
  const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}

}  // namespace g3

// Work item = (split zs, batch z, output tile).  Walked by a persistent grid: workgroup slot s
// takes items s, s + G, ...; the LDS ring runs straight across items.
template <int DTI, int DTO, bool A_MC, bool B_MC, int EPI>
__global__ __launch_bounds__(512) void gemm3_kernel(GemmArgs p, float* __restrict__ ws, int W, int batches, int nsplit) {
  using namespace g3;
  using fa::smem;
  using fa::lds_addr;
  using fa::s16x4;
  using TI = typename dt_traits<DTI>::T;
  using TO = typename dt_traits<DTO>::T;
  constexpr bool OUT16 = sizeof(TO) == 2;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int g = lane >> 4, l15 = lane & 15;
  const int G = gridDim.x;
  const int slot0 = xcd_remap(blockIdx.x, G);
  if (slot0 >= W) return;

  const int ktiles = (p.K + BK - 1) / BK;
  const int ntot = ktiles * p.nseg;
  const int ntile = p.tiles_m * p.tiles_n;
  constexpr int GM = 8, SB = 32;
  const int64_t lda2 = p.lda * 2, ldb2 = p.ldb * 2;
  // byte steps of one k-tile / one half-tile inside an operand
  const int64_t a_kstep = A_MC ? 64 * lda2 : 128, b_kstep = B_MC ? 64 * ldb2 : 128;
  // FL (16-bit C, k-contiguous B): wave wn owns the 64 contiguous output columns 64 wn .. +63
  // (its two 32-column n-halves side by side), B half i = columns {64 w + 32 i + c} (image row
  // 32 w + c), and the epilogue writes whole 128-byte row segments (see store_half).
  // Otherwise wave wn owns columns 128 i + 32 wn (an mn-contiguous B half is then one
  // contiguous 256-byte piece of a k row).
  constexpr bool FL = EPI == 0 && !B_MC && G3_FL;
  constexpr int WCOL = FL ? 64 : 32;  // column stride of the waves
  const int64_t a_half = A_MC ? 256 : 128 * lda2, b_half = B_MC ? 256 : (FL ? 32 : 128) * ldb2;
  // byte jump from the last k-tile of a K segment to the first of the next
  const int64_t a_segjump = 2 * p.sAseg - (int64_t)(ktiles - 1) * a_kstep;
  const int64_t b_segjump = 2 * p.sBseg - (int64_t)(ktiles - 1) * b_kstep;
  const int kl_t = p.K - (ktiles - 1) * BK;  // valid k of every segment's last k-tile

  struct Item {
    int m0, n0, mo, no, z, z1, z2, zs, tb, te;
    const char* a;  // operand bytes at (batch, tile mn origin)
    const char* b;
  };
  // Item table: at launch the workgroup decodes its items (slot0 + k G, k < nitems <= 2048) into
  // 16-byte LDS entries past the 128 KiB ring -- {tm | tn << 16, z1 | z2 << 16, tb | zs << 24, te}
  // -- so the loop looks an item up with one broadcast ds_read instead of ~10 integer divisions.
  // Tile order: super-blocks of SB x SB tiles (row-major over the super-block grid), inside one
  // super-block groups of GM m-tiles sweeping its n-tiles.  A super-block's panels are re-read
  // while at most SB^2 x 128 KiB of output streams out (<= 128 MiB: they stay in the 256 MiB
  // Infinity Cache; a whole-row sweep at N = 75000 wrote 300 MB between two uses).
  const int nitems = (W - slot0 + G - 1) / G;
  for (int k = tid; k < nitems; k += NT) {
    const int L = slot0 + k * G;
    const int zz = L / ntile, tl = L % ntile;
    const int zs = zz / batches, z = zz % batches;
    const int sbr = tl / (SB * p.tiles_n);
    const int sbm = min(SB, p.tiles_m - sbr * SB);
    const int r1 = tl - sbr * SB * p.tiles_n;
    const int sbc = r1 / (sbm * SB);
    const int sbn = min(SB, p.tiles_n - sbc * SB);
    const int r2 = r1 - sbc * sbm * SB;
    const int gi = r2 / (GM * sbn);
    const int gm_n = min(GM, sbm - gi * GM);
    const int r3 = r2 - gi * GM * sbn;
    const int tm = sbr * SB + gi * GM + r3 % gm_n, tn = sbc * SB + r3 / gm_n;
    const int tb = (int)((unsigned)(zs * ntot) / (unsigned)nsplit);
    const int te = (int)((unsigned)((zs + 1) * ntot) / (unsigned)nsplit);
    *reinterpret_cast<u32x4*>(smem + TAB + 16 * k) =
        u32x4{(uint32_t)tm | ((uint32_t)tn << 16), (uint32_t)(z / p.nb2) | ((uint32_t)(z % p.nb2) << 16),
              (uint32_t)tb | ((uint32_t)zs << 24), (uint32_t)te};
  }
  __syncthreads();
  auto item_of = [&](int k) __attribute__((always_inline)) {
    const u32x4 e = *reinterpret_cast<const u32x4*>(smem + TAB + 16 * k);
    const uint32_t e0 = __builtin_amdgcn_readfirstlane(e[0]), e1 = __builtin_amdgcn_readfirstlane(e[1]);
    const uint32_t e2 = __builtin_amdgcn_readfirstlane(e[2]), e3 = __builtin_amdgcn_readfirstlane(e[3]);
    Item it;
    it.mo = (int)(e0 & 0xFFFFu) * BM;
    it.no = (int)(e0 >> 16) * BN;
    it.m0 = min(it.mo, p.M - BM);  // (an mn-contiguous operand has M / N % 8 == 0: 16-byte DMA sources)
    it.n0 = min(it.no, p.N - BN);
    const int z1 = (int)(e1 & 0xFFFFu), z2 = (int)(e1 >> 16);
    it.z1 = z1;
    it.z2 = z2;
    it.z = z1 * p.nb2 + z2;
    it.zs = (int)(e2 >> 24);
    it.tb = (int)(e2 & 0xFFFFFFu);
    it.te = (int)e3;
    it.a = reinterpret_cast<const char*>(p.A) + 2 * (z1 * p.sA1 + z2 * p.sA2 + (A_MC ? (int64_t)it.m0 : (int64_t)it.m0 * p.lda));
    it.b = reinterpret_cast<const char*>(p.B) + 2 * (z1 * p.sB1 + z2 * p.sB2 + (B_MC ? (int64_t)it.n0 : (int64_t)it.n0 * p.ldb));
    return it;
  };

  // ---- issue side: cursor of one k-tile (item L, flattened k index k < te, k-tile kt of its
  // segment, valid k kl, operand bytes a / b of the k-tile).  Kept small: it lives in SGPRs
  // twice (the k-tiles one and two ahead of the compute side).
  // An item's k-tile count is padded to an even number (te2 = tb + round_up_even(te - tb)):
  // every item then starts on LDS-slot parity 0 and ends on parity 1 (see the item loop).  The
  // pad k-tile (k >= te) is DMA'd entirely out of range, i.e. zeros, and adds nothing.
  struct Cur {
    int L, k, te, te2, kt, kl;  // kl: valid k of this k-tile (0: pad)
    const char* a;
    const char* b;
  };
  // k-tile k of the workgroup's item L (table index; k < te2)
  auto cur_at = [&](int L, int k, int te) __attribute__((always_inline)) {
    Cur c;
    const Item it = item_of(L);
    c.L = L;
    c.k = k;
    c.te = te;
    c.te2 = te + ((te - it.tb) & 1);
    const int seg = k / ktiles;
    c.kt = k - seg * ktiles;
    c.kl = c.kt == ktiles - 1 ? kl_t : BK;
    c.a = it.a + 2 * (int64_t)seg * p.sAseg + (int64_t)c.kt * a_kstep;
    c.b = it.b + 2 * (int64_t)seg * p.sBseg + (int64_t)c.kt * b_kstep;
    return c;
  };
  // the k-tile after c in the workgroup's stream (after the end: c itself again -- its DMAs
  // are harmless repeats)
  auto next_of = [&](const Cur& c) __attribute__((always_inline)) {
    if (c.k + 1 < c.te) {
      Cur n = c;
      n.k = c.k + 1;
      if (c.kt + 1 == ktiles) {  // next K segment
        n.kt = 0;
        n.a = c.a + a_segjump;
        n.b = c.b + b_segjump;
      } else {
        n.kt = c.kt + 1;
        n.a = c.a + a_kstep;
        n.b = c.b + b_kstep;
      }
      n.kl = n.kt == ktiles - 1 ? kl_t : BK;
      return n;
    }
    if (c.k + 1 < c.te2) {  // the pad k-tile
      Cur n = c;
      n.k = c.k + 1;
      n.kl = 0;
      return n;
    }
    if (c.L + 1 < nitems) {
      const Item it = item_of(c.L + 1);
      return cur_at(c.L + 1, it.tb, it.te);
    }
    return c;
  };

  // per-lane DMA source offsets of the wave's two 1 KiB pieces of a half-tile image
  //   k-contiguous image [128 rows][128 B], chunk c of row r at 16 * (c ^ ((r >> 1) & 7))
  //   mn-contiguous image [64 k][256 B], chunk c of row k at 16 * (c ^ (2 (k & 3) + 8 ((k >> 3) & 1)))
  uint32_t oa[2], ob[2];
  int ta[2], tb_[2];  // tail test: chunk (k-contiguous) or k row (mn-contiguous)
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int pc = 2 * wave + pp;
    {
      if (!A_MC) {
        const int r = 8 * pc + (lane >> 3), c = (lane & 7) ^ ((r >> 1) & 7);
        oa[pp] = (uint32_t)(r * lda2 + 16 * c);
        ta[pp] = 8 * c;
      } else {
        const int k = 4 * pc + (lane >> 4), c = (lane & 15) ^ (2 * (k & 3) + 8 * ((k >> 3) & 1));
        oa[pp] = (uint32_t)(k * lda2 + 16 * c);
        ta[pp] = k;
      }
      if (!B_MC) {
        const int r = 8 * pc + (lane >> 3), c = (lane & 7) ^ ((r >> 1) & 7);
        const int rt = FL ? 64 * (r >> 5) + (r & 31) : r;  // tile row (output column) of image row r
        ob[pp] = (uint32_t)(rt * ldb2 + 16 * c);
        tb_[pp] = 8 * c;
      } else {
        const int k = 4 * pc + (lane >> 4), c = (lane & 15) ^ (2 * (k & 3) + 8 * ((k >> 3) & 1));
        ob[pp] = (uint32_t)(k * ldb2 + 16 * c);
        tb_[pp] = k;
      }
    }
  }
  // the same for the K-tail k-tile (every segment's tail has kl_t valid k)
  uint32_t oat[2], obt[2];
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    oat[pp] = ta[pp] < kl_t ? oa[pp] : g3::OOB;
    obt[pp] = tb_[pp] < kl_t ? ob[pp] : g3::OOB;
  }
  // which: 0 / 1 = A rows 0-127 / 128-255, 2 / 3 = B columns 0-127 / 128-255
  auto issue = [&](const Cur& c, const int which, const int s) __attribute__((always_inline)) {
    const bool isA = which < 2;
    const int h = which & 1;
    const uint32_t* o = isA ? oa : ob;
    const uint32_t dst = lds_addr(smem + s * SLOT + which * HALF + wave * 2048);
    const char* b0 = isA ? c.a + h * a_half : c.b + h * b_half;
    // full k-tile: the precomputed offsets; K tail: dead chunks / k rows out of range (zeros)
    const uint32_t* ot = isA ? oat : obt;
    const bool full = c.kl == BK, pad = c.kl == 0;
    bdma2(rsrc_of(b0), full ? o[0] : pad ? OOB : ot[0], full ? o[1] : pad ? OOB : ot[1], dst);
  };

  // ---- LDS fragment reads (16x16x32 operand: lane l holds mn = base + (l & 15), k = 8 (l >> 4) .. +7) ----
  typedef const __attribute__((address_space(3))) char lds_char;
  // k-contiguous: two lane bases (k-step 0 / 1), row offsets fold into the immediate
  const int kcb0 = l15 * 128 + 16 * ((0 + g) ^ (l15 >> 1));
  const int kcb1 = l15 * 128 + 16 * ((4 + g) ^ (l15 >> 1));
  // mn-contiguous transposed reads: lane 4q + p of group g reads row 8 g + q (+4, + 32 ks),
  // logical chunk (mn base / 8) + (p >> 1) of that row
  const int tq = (lane & 15) >> 2, tp = lane & 3;
  auto mc_base = [&](int chunk_bits123) __attribute__((always_inline)) {  // mn base / 8 (even) -> lane base
    const int c = (tp >> 1) | ((chunk_bits123 ^ (2 * tq + 8 * (g & 1))) & 14);
    return (8 * g + tq) * 256 + 16 * c + 8 * (tp & 1);
  };
  int mca[4], mcb[2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) mca[mt] = mc_base(8 * wm + 2 * mt);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) mcb[nt] = mc_base(4 * wn + 2 * nt);

  auto frag = [&](const char* img, const bool mc, const int mnb, const int mci, const int ks) __attribute__((always_inline)) -> u32x4 {
    if (!mc) {
      return *reinterpret_cast<const u32x4*>(img + (ks ? kcb1 : kcb0) + mnb * 128);
    } else {
      lds_char* b = (lds_char*)img + mci + ks * 32 * 256;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((fa::lds_s16x4*)(b));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((fa::lds_s16x4*)(b + 4 * 256));
      union { struct { s16x4 a, b; } s; u32x4 u; } r;
      r.s.a = lo;
      r.s.b = hi;
      return r.u;
    }
  };
  // A quarter j of the wave: rows 128 j + 64 wm + 16 mt (+ l15); image = A half j
  auto read_a = [&](u32x4 (&fa_)[4][2], const char* st, const int j) __attribute__((always_inline)) {
    const char* img = st + j * HALF;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) fa_[mt][ks] = frag(img, A_MC, 64 * wm + 16 * mt, mca[mt], ks);
  };
  // B half i of the wave: columns 128 i + 32 wn + 16 nt (+ l15); image = B half i
  auto read_b = [&](u32x4 (&fb_)[2][2], const char* st, const int i) __attribute__((always_inline)) {
    const char* img = st + (2 + i) * HALF;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) fb_[nt][ks] = frag(img, B_MC, 32 * wn + 16 * nt, mcb[nt], ks);
  };

  // acc[4 j + mt][2 i + nt]: C rows m0 + 128 j + 64 wm + 16 mt + l15, columns n0 + 128 i + 32 wn + 16 nt + 4 g + r
  // (the MFMA computes the C^T tile: B fragment as its A operand, so each lane holds 4 consecutive columns)
  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto quad = [&](const u32x4 (&fa_)[4][2], const u32x4 (&fb_)[2][2], const int j, const int i) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          f32x4& c = acc[4 * j + mt][2 * i + nt];
          c = mfma16<DTI>(fb_[nt][ks], fa_[mt][ks], c);
        }
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- epilogue: the wave's 128 x 64 block of item `it` (no control flow: a branch here splits
  // the accumulators' live ranges and the register allocator starts copying them around) ----
  //   EPI 0: 16-bit C, beta = 0: 16-byte stores, the two 16x16 tiles of a 32-column strip paired
  //          by v_permlane16_swap into 8 consecutive columns per lane;
  //   EPI 1: split-K fp32 slices (unscaled; the reduce applies alpha / beta);
  //   EPI 3: fp32 C, beta = 0.
  // Stores go through buffer descriptors: the 64-bit row base is scalar (one descriptor per
  // 16-row strip), the lane's 32-bit offset is the same for every strip of every item -- no
  // per-store 64-bit address registers next to the 128 accumulator registers.
  const int64_t ldo = EPI == 1 ? (int64_t)p.N : p.ldc;
  const int voff = EPI == 0 ? (int)((l15 * ldo + 16 * (g & 1) + 8 * (g >> 1)) * 2) : (int)((l15 * ldo + 4 * g) * 4);
  // Output quadrant (j, i) of the wave (acc[4 j + mt][2 i + nt], mt < 4, nt < 2): stored as soon
  // as its last MFMA of the item has issued -- in the next phase's load segment, so an item's
  // 16 (32 fp32) store instructions per wave spread over 4 phases instead of one burst that the
  // DMA stream queues behind -- then zeroed for the next item.
  auto store_quad = [&](const Item& it, const int j, const int i) __attribute__((always_inline)) {
    const int z1 = it.z1, z2 = it.z2;
    const float alpha = p.alpha;
    const char* cb;
    if constexpr (EPI == 1)
      cb = reinterpret_cast<const char*>(ws + ((int64_t)it.zs * batches + it.z) * (int64_t)p.M * p.N + it.n0 + WCOL * wn);
    else
      cb = reinterpret_cast<const char*>(p.C) + sizeof(TO) * (z1 * p.sC1 + z2 * p.sC2 + it.n0 + WCOL * wn);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int r0 = it.m0 + 128 * j + 64 * wm + 16 * mt;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(cb + (int64_t)r0 * ldo * (EPI == 0 ? 2 : 4)), 0, 0x7FFFFFF0, 0x00020000);
      f32x4& xr = acc[4 * j + mt][2 * i];
      f32x4& yr = acc[4 * j + mt][2 * i + 1];
      f32x4 x = xr, y = yr;
      if constexpr (EPI == 0) {
        x *= alpha;
        y *= alpha;
        uint32_t X0 = fa::pack2<DTO>(x[0], x[1]), X1 = fa::pack2<DTO>(x[2], x[3]);
        uint32_t Y0 = fa::pack2<DTO>(y[0], y[1]), Y1 = fa::pack2<DTO>(y[2], y[3]);
        swap16(X0, Y0);
        swap16(X1, Y1);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{X0, X1, Y0, Y1}, rs, voff + 256 * i, 0, G3_STORE_AUX);
      } else {
        if constexpr (EPI == 3) {
          x *= alpha;
          y *= alpha;
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), rs, voff + 512 * i, 0, G3_STORE_AUX);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), rs, voff + 512 * i + 64, 0, G3_STORE_AUX);
      }
      xr = f32x4{0.f, 0.f, 0.f, 0.f};
      yr = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  // FL epilogue of output row block j (both n-halves final): per 16-row strip two stores of
  // 8 rows x 128 bytes each (whole cache lines; the plain form writes 16 rows x 64 bytes per
  // instruction).  After the permlane16 pairing a lane holds 8 columns of its row in each half
  // (chunk c0 = 2 (g & 1) + (g >> 1) of the 4 16-byte chunks of a 64-byte half); lanes l and
  // l ^ 8 of a 16-lane row exchange one half (DPP row_ror:8), so the first store carries rows
  // 0-7 (chunks 0-7) and the second rows 8-15.
  const bool lo8 = l15 < 8;
  const int voff_fl = (int)(((l15 & 7) * ldo + 8 * (2 * (g & 1) + (g >> 1) + 4 * (l15 >> 3))) * 2);
  auto store_half = [&](const Item& it, const int j) __attribute__((always_inline)) {
    if constexpr (FL) {
      const float alpha = p.alpha;
      const char* cb = reinterpret_cast<const char*>(p.C) + sizeof(TO) * (it.z1 * p.sC1 + it.z2 * p.sC2 + it.n0 + WCOL * wn);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int r0 = it.m0 + 128 * j + 64 * wm + 16 * mt;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(cb + (int64_t)r0 * ldo * 2), 0, 0x7FFFFFF0, 0x00020000);
        uint32_t d[2][4];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const f32x4 x = acc[4 * j + mt][2 * i] * alpha, y = acc[4 * j + mt][2 * i + 1] * alpha;
          d[i][0] = fa::pack2<DTO>(x[0], x[1]);
          d[i][1] = fa::pack2<DTO>(x[2], x[3]);
          d[i][2] = fa::pack2<DTO>(y[0], y[1]);
          d[i][3] = fa::pack2<DTO>(y[2], y[3]);
          swap16(d[i][0], d[i][2]);
          swap16(d[i][1], d[i][3]);
          acc[4 * j + mt][2 * i] = f32x4{0.f, 0.f, 0.f, 0.f};
          acc[4 * j + mt][2 * i + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        u32x4 va, vb;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t send = lo8 ? d[1][e] : d[0][e];
          const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)send, 0x128, 0xF, 0xF, false);  // row_ror:8
          va[e] = lo8 ? d[0][e] : recv;
          vb[e] = lo8 ? recv : d[1][e];
        }
        __builtin_amdgcn_raw_buffer_store_b128(va, rs, voff_fl, 0, G3_STORE_AUX);
        __builtin_amdgcn_raw_buffer_store_b128(vb, rs, voff_fl + (int)(8 * ldo * 2), 0, G3_STORE_AUX);
      }
    }
  };
  // store instructions of one quadrant per lane (exact: the vmcnt waits around an item boundary
  // count them)
  constexpr int SPQ = EPI == 0 ? 4 : 8;
  // FL: 8 stores per row block j: j = 0 in the last k-tile's q2, j = 1 after it
  constexpr int SPH = 2 * SPQ;

  // ---- prologue: k-tiles 0 (slot 0) and 1 (slot 1) in the steady-state issue order ----
  // steady state, k-tile v (slot v & 1, quadrant order by parity P = v & 1):
  //   q0: reads A quarter 0 + B half P ("first B")   issues B half P    of k-tile v + 1
  //   q1: reads B half 1 - P ("second B")            issues A half 1    of k-tile v + 1
  //   q2: reads A quarter 1                          issues A half 0    of k-tile v + 2
  //   q3: no reads                                   issues B half P    of k-tile v + 2
  // waits vmcnt(8) in q0, q1, q3 (after their issue): data waited in phase q is read in q+1.
  Cur c1;
  {
    const Item it = item_of(0);
    c1 = cur_at(0, it.tb, it.te);
  }
  issue(c1, 0, 0);
  issue(c1, 2, 0);
  issue(c1, 3, 0);
  issue(c1, 1, 0);
  c1 = next_of(c1);
  issue(c1, 0, 1);
  issue(c1, 3, 1);
  fa::wait_vm<8>();
  fa::raw_barrier();
  if (wm == 1) fa::raw_barrier();  // waves 4-7 run one barrier behind

  int cL = 0;  // compute side: table index of the item
  // compute side: flattened k index and its end
  int ck, cte;  // cte: the padded end
  {
    const Item it = item_of(cL);
    ck = it.tb;
    cte = it.te + ((it.te - it.tb) & 1);
  }
  bool first = false;  // this k-tile is an item's first after an item boundary
  Cur c2 = c1;

  u32x4 fa_[4][2], fb0[2][2], fb1[2][2];

  // One k-tile of parity P from slot P.  LAST: the item's last k-tile -- quadrants 0-2 are
  // stored in the load segments of phases 1-3, quadrant 3 after the k-tile.  The waits count the
  // quadrant stores issued after the DMAs they wait for (SPQ per quadrant): on the last k-tile
  // q1 +1, q3 +3 quadrants; on the next item's first k-tile q0 +4, q1 +3, q3 +1.
  auto ktile = [&](auto Pc, auto Lc, const Item& it) __attribute__((always_inline)) {
    constexpr int P = decltype(Pc)::value;
    constexpr bool LAST = decltype(Lc)::value;
    // stores issued after the DMA each wait is for: see the item loop
    constexpr int W0F = FL ? 8 + 2 * SPH : 8 + 4 * SPQ, W1F = FL ? 8 + 2 * SPH : 8 + 3 * SPQ, W3F = FL ? 8 + SPH : 8 + SPQ;
    constexpr int W1L = FL ? 8 : 8 + SPQ, W3L = FL ? 8 + SPH : 8 + 3 * SPQ;
    const char* st = smem + P * SLOT;
    // q0
    read_a(fa_, st, 0);
    read_b(P ? fb1 : fb0, st, P);
    issue(c1, 2 + P, 1 - P);
    if (!LAST && first) fa::wait_vm<W0F>(); else fa::wait_vm<8>();
    fa::raw_barrier();
    quad(fa_, P ? fb1 : fb0, 0, P);
    fa::raw_barrier();
    // q1
    if constexpr (LAST && !FL) store_quad(it, 0, P);
    read_b(P ? fb0 : fb1, st, 1 - P);
    issue(c1, 1, 1 - P);
    if constexpr (LAST) fa::wait_vm<W1L>();
    else if (first) fa::wait_vm<W1F>();
    else fa::wait_vm<8>();
    fa::raw_barrier();
    quad(fa_, P ? fb0 : fb1, 0, 1 - P);
    fa::raw_barrier();
    // q2
    if constexpr (LAST && !FL) store_quad(it, 0, 1 - P);
    if constexpr (LAST && FL) store_half(it, 0);
    read_a(fa_, st, 1);
    issue(c2, 0, P);
    fa::raw_barrier();
    quad(fa_, P ? fb0 : fb1, 1, 1 - P);
    fa::raw_barrier();
    // q3
    if constexpr (LAST && !FL) store_quad(it, 1, 1 - P);
    issue(c2, 2 + P, P);
    if constexpr (LAST) fa::wait_vm<W3L>();
    else if (first) fa::wait_vm<W3F>();
    else fa::wait_vm<8>();
    fa::raw_barrier();
    quad(fa_, P ? fb1 : fb0, 1, P);
    fa::raw_barrier();
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using BT = std::integral_constant<bool, true>;
  using BF = std::integral_constant<bool, false>;
  // Items have an even number n >= 2 of k-tiles (odd counts padded), so every item starts on
  // parity 0 and ends on parity 1: per item, (n / 2 - 1) pairs of plain k-tiles, then a plain
  // parity-0 k-tile and the LAST parity-1 one -- straight-line code, no branch between
  // alternative k-tile bodies (which makes the register allocator shuffle the accumulators).
  auto plain = [&](auto Pc) __attribute__((always_inline)) {
    c2 = next_of(c1);
    ktile(Pc, BF{}, Item{});
    c1 = c2;
    first = false;
  };
  while (true) {
    for (int k = ck; k + 2 < cte; k += 2) {
      plain(I0{});
      plain(I1{});
    }
    plain(I0{});
    c2 = next_of(c1);
    const Item it = item_of(cL);
    ktile(I1{}, BT{}, it);
    if constexpr (FL) store_half(it, 1);
    else store_quad(it, 1, 1);
    c1 = c2;
    first = true;
    if (++cL >= nitems) break;
    const Item nx = item_of(cL);
    ck = nx.tb;
    cte = nx.te + ((nx.te - nx.tb) & 1);
  }
  fa::wait_vm<0>();  // repeat DMAs of the final k-tiles must land before the LDS goes away
  if (wm == 0) fa::raw_barrier();  // balance the stagger
}

template <int DTI, int DTO, bool AMC, bool BMC>
static void launch3_t(const GemmArgs& a, int batches, int splits, float* ws, int ncu, hipStream_t st) {
  const int W = a.tiles_m * a.tiles_n * batches * splits;
  const int G = W < ncu ? W : ncu;
  float* w = splits > 1 ? ws : nullptr;
  // epilogue modes (see the kernel): split-K slices 1, 16-bit C 0, fp32 C 3
#define G3L(E) hipLaunchKernelGGL((gemm3_kernel<DTI, DTO, AMC, BMC, E>), dim3(G), dim3(g3::NT), g3::LDS, st, a, w, W, batches, splits)
  if (w) G3L(1);
  else if constexpr (DTO == DT_F32) G3L(3);
  else G3L(0);
#undef G3L
}

template <int DTI, int DTO>
static void launch3_d(const GemmArgs& a, int batches, bool amc, bool bmc, int splits, float* ws, int ncu, hipStream_t st) {
  if (!amc && !bmc) return launch3_t<DTI, DTO, false, false>(a, batches, splits, ws, ncu, st);
  if (!amc && bmc) return launch3_t<DTI, DTO, false, true>(a, batches, splits, ws, ncu, st);
  if (amc && !bmc) return launch3_t<DTI, DTO, true, false>(a, batches, splits, ws, ncu, st);
  return launch3_t<DTI, DTO, true, true>(a, batches, splits, ws, ncu, st);
}

}  // namespace xdot

extern "C" int xdot_num_cus();
extern "C" int xdot_gemm_reduce_launch(const xdot::GemmArgs* a, const float* ws, int splits, int batches, int dt_out,
                                       hipStream_t st);

// Eligibility: see the file header.  -3 = shape/layout not eligible (caller falls back).
extern "C" int xdot_gemm3_launch(const xdot::GemmArgs* a, int batches, int dt_in, int dt_out, int a_mc, int b_mc,
                                 int splits, float* ws, hipStream_t st) {
  using namespace xdot;
  GemmArgs g = *a;
  // K % 8: a k-contiguous operand's K tail is zero-filled per 16-byte chunk; two mn-contiguous
  // operands (the weight gradients dYᵀ·X, K = the sequence rows) are tail-filled per k row, any K
  if (g.M < g3::BM || g.N < g3::BN || ((g.K % 8) != 0 && !(a_mc && b_mc)) || g.beta != 0.f) return -3;
  g.tiles_m = (g.M + g3::BM - 1) / g3::BM;
  g.tiles_n = (g.N + g3::BN - 1) / g3::BN;
  if (batches == 0 || g.K == 0) return -3;
  if (splits < 1 || (splits > 1 && !ws)) return -2;
  const int ncu_ = xdot_num_cus();
  if ((int64_t)((g.K + g3::BK - 1) / g3::BK) * g.nseg < splits) return -3;  // every item >= 1 k-tile
  {
    const int64_t W = (int64_t)g.tiles_m * g.tiles_n * batches * splits;
    if ((W + ncu_ - 1) / ncu_ > g3::MAX_ITEMS || g.tiles_m > 65535 || g.tiles_n > 65535) return -3;
  }
  const int ncu = xdot_num_cus();
#define G3_DT(I, O) \
  if (dt_in == I && dt_out == O) { launch3_d<I, O>(g, batches, a_mc, b_mc, splits, ws, ncu, st); goto done; }
  G3_DT(DT_BF16, DT_BF16) G3_DT(DT_BF16, DT_F32) G3_DT(DT_F16, DT_F16) G3_DT(DT_F16, DT_F32)
#undef G3_DT
  return -1;
done:
  if (splits > 1) return xdot_gemm_reduce_launch(&g, ws, splits, batches, dt_out, st);
  return 0;
}

// ---------------------------------------------------------------------------------------------
// fp32 on the bf16 matrix pipe: x = hi + lo with hi = bf16(x), lo = bf16(x - hi) (the residual
// after lo is ~2^-17 |x|).  A x B ~= hi_A hi_B + lo_A hi_B + hi_A lo_B: three bf16 products, one
// GEMM with 3x the K segments over compact operand copies A' = [hi, lo, hi], B' = [hi, hi, lo]
// per (batch, segment): layout [z1][z2][part][seg][R][C] (uniform segment stride R*C).
namespace xdot {
struct Split3Args {
  const float* src;
  __bf16* dst;
  int64_t s1, s2, sseg, ld;  // source strides (elements)
  int nb2, nseg, R, C;       // C: contiguous extent of the source rows
  int lo_mask;               // bit p: part p holds the lo halves
  int64_t n;                 // nb1 * nb2 * nseg * R * C
};
__global__ __launch_bounds__(256) void split3_kernel(Split3Args a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const int c = (int)(i % a.C);
  int64_t t = i / a.C;
  const int r = (int)(t % a.R);
  t /= a.R;
  const int seg = (int)(t % a.nseg);
  t /= a.nseg;
  const int z2 = (int)(t % a.nb2);
  const int z1 = (int)(t / a.nb2);
  const float x = a.src[z1 * a.s1 + z2 * a.s2 + seg * a.sseg + (int64_t)r * a.ld + c];
  __bf16 hi = (__bf16)x;
  __bf16 lo = (__bf16)(x - (float)hi);
  if (!__builtin_isfinite(x)) {
    lo = (__bf16)0.f;  // inf / NaN: hi carries it (inf - inf would make lo a NaN)
  } else if (!__builtin_isfinite((float)hi)) {
    // |x| near FLT_MAX rounds up to inf in bf16: truncate toward zero instead, the residual stays finite
    const float ht = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, x) & 0xFFFF0000u);
    hi = (__bf16)ht;
    lo = (__bf16)(x - ht);
  }
  const int64_t RC = (int64_t)a.R * a.C;
  __bf16* d = a.dst + ((int64_t)(z1 * a.nb2 + z2) * 3 * a.nseg + seg) * RC + (int64_t)r * a.C + c;
#pragma unroll
  for (int p = 0; p < 3; ++p) d[(int64_t)p * a.nseg * RC] = ((a.lo_mask >> p) & 1) ? lo : hi;
}
}  // namespace xdot

extern "C" int xdot_split3_launch(const float* src, void* dst, int64_t s1, int64_t s2, int64_t sseg, int64_t ld,
                                  int nb1, int nb2, int nseg, int R, int C, int lo_mask, hipStream_t st) {
  xdot::Split3Args a{src, reinterpret_cast<__bf16*>(dst), s1, s2, sseg, ld, nb2, nseg, R, C, lo_mask,
                     (int64_t)nb1 * nb2 * nseg * R * C};
  if (a.n == 0) return 0;
  hipLaunchKernelGGL(xdot::split3_kernel, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, st, a);
  return 0;
}
