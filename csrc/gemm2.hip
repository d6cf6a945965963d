// xdot — large-tile 16-bit MFMA GEMM for gfx950 (the "v2" path of xdot.gemm).
//
//   C[z](m, n) = alpha * sum_{s < nseg} sum_{k < K} opA_s[z](m, k) * opB_s[z](k, n) + beta * C[z](m, n)
//
// Same addressing model as csrc/gemm.hip (2-level batch, K segments, each operand k- or
// mn-contiguous), so it carries the same three distributed products of the reference
// (distributed_dot_product/multiplication/functions.py:89-97 nt, :140-147 tn, :202-211 all)
// when the shapes are big enough to fill 256x256 tiles.  Why a second kernel: the 128x128 /
// 4-wave v1 tile needs 128 B/clk/CU of LDS fragment reads plus 64 B/clk/CU of ds_write_b128
// staging at MFMA peak — the register-staged writes alone run the LDS store path at ~80 % —
// and it measured 0.59x hipBLASLt on 75000x75000x768 bf16.  Here:
//   * 256x256 workgroup tile, 8 waves (2 per SIMD) in a 2 (M) x 4 (N) grid, each wave a
//     128x64 tile = 4x2 v_mfma_f32_32x32x16 accumulators (128 VGPRs);
//     LDS fragment reads drop to 96 B/clk/CU at peak (37 % of the 256 B/clk array);
//   * operands travel HBM -> LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR staging, no
//     ds_write), through a ring of BK = 64 tiles (64 KiB per stage, 2 stages: every
//     k-contiguous row segment is one whole 128-byte line; BK = 32 x 4 stages measured
//     7-8 % slower), one `s_waitcnt vmcnt` + barrier per tile, the next tile's DMAs
//     interleaved with the first two k-steps' MFMAs;
//   * persistent grid (one workgroup per CU) walking (split, batch, tile) items: the ring
//     continues across items, so each item's epilogue overlaps the next item's first DMAs;
//   * k-contiguous images [256 rows][2 BK bytes], 16-byte chunks XOR-swizzled by row bits:
//     ds_read_b128 fragment reads conflict-free; mn-contiguous images [BK k][512 B], chunks
//     XOR-swizzled by 4 (k & 3): ds_read_b64_tr_b16 (hardware transpose) conflict-free.  The
//     swizzle is applied to the DMA *source* addresses (the DMA destination is lane-linear);
//   * K tails (K % 32) are zero-patched in LDS after the DMA lands; M/N tails re-read the
//     last valid row/chunk (finite values, their outputs are never stored);
//   * optional split-K (grid.z): each slice writes an fp32 partial, gemm2_reduce sums the
//     slices in order (deterministic) and applies alpha / beta / the output cast;
//   * grouped (8 M-tiles) + XCD-aware workgroup order so concurrently running tiles share
//     operand panels in one XCD's L2.
#include "flash_common.h"

#include <cstdlib>

namespace xdot {
namespace g2 {

constexpr int BM = 256, BN = 256, NT = 512;
constexpr int EPI_ROWF = 68;           // fp32 epilogue staging row (64 + 4 pad)

// BK = k per ring stage (32: 64-byte k-contiguous rows, 4 stages; 64: whole 128-byte cache
// lines per row, 2 stages).  Images: KC [256 rows][2 BK bytes], MC [BK k-rows][512 bytes].
template <int BK_, int NBUF_> struct Cfg {
  static constexpr int BK = BK_, NBUF = NBUF_, PF = NBUF_ - 1;
  static constexpr int IMG = 512 * BK_;               // bytes per operand image
  static constexpr int STAGE = 2 * IMG;
  static constexpr int LDS = NBUF_ * STAGE;
  static constexpr int PPW = IMG / 1024 / 8;          // 1 KiB DMA pieces per wave per image
  static constexpr int NG = 2 * PPW;                  // DMAs per wave per tile
  static constexpr int KCH = BK_ / 8;                 // 16-byte chunks per KC row
  static_assert(LDS <= 160 * 1024 && 8 * 32 * EPI_ROWF * 4 <= LDS, "lds");
};
// KC swizzle: chunk ^ f(row) keeps every 16-lane ds_read_b128 group on 16 distinct 4-bank windows
template <int KCH> __device__ __forceinline__ int kc_swz(int row) {
  return KCH == 4 ? ((row >> 2) & 3) : ((row >> 1) & 7);
}

// Per-lane DMA source offsets (bytes, relative to the tile's first row / k) of the wave's
// 1 KiB pieces of one operand image, plus what the K-tail path needs.
template <class CF, bool MC>
struct OpDma {
  static constexpr int P = CF::PPW;
  uint32_t off[P];
  int r[P], c[P];  // KC: image row (mn), logical chunk; MC: k row, clamped mn element offset
  __device__ __forceinline__ void init(int wave, int lane, int64_t ld, int mn_left) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int p = (wave * P + i) * 1024 + lane * 16;
      if (!MC) {  // [256 rows][KCH chunks]
        const int row = p / (CF::KCH * 16), cp = (p >> 4) % CF::KCH;
        const int c8 = cp ^ kc_swz<CF::KCH>(row);
        const int rr = min(row, mn_left - 1);
        r[i] = rr;
        c[i] = c8;
        off[i] = (uint32_t)(((int64_t)rr * ld + 8 * c8) * 2);
      } else {    // [BK k rows][32 chunks]
        const int kr = p >> 9, cp = (p >> 4) & 31;
        const int c8 = cp ^ (4 * (kr & 3));
        const int mn = min(8 * c8, mn_left - 8);
        r[i] = kr;
        c[i] = mn;
        off[i] = (uint32_t)(((int64_t)kr * ld + mn) * 2);
      }
    }
  }
  // K-tail tile: clamp k into [0, kleft) so no byte beyond the operand is touched
  __device__ __forceinline__ uint32_t tail_off(int i, int64_t ld, int kleft) const {
    if (!MC) {
      const int c8 = min(c[i], kleft / 8 - 1);
      return (uint32_t)(((int64_t)r[i] * ld + 8 * c8) * 2);
    } else {
      const int kr = min(r[i], kleft - 1);
      return (uint32_t)(((int64_t)kr * ld + c[i]) * 2);
    }
  }
};

typedef const __attribute__((address_space(3))) char lds_char;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// Fragment of a 32x32x16 MFMA operand (lane l: mn = base + (l & 31), k = 16 ks + 8 (l >> 5) + j).
//   KC image: one ds_read_b128 at lane base (per ks) + base_mn * row bytes (immediate).
//   MC image: two ds_read_b64_tr_b16 at lane base (per (base_mn / 32) & 3) + immediate.
template <int KCH>
__device__ __forceinline__ u32x4 frag_kc(const char* img, int lane_off, int base_mn) {
  return *reinterpret_cast<const u32x4*>(img + lane_off + base_mn * (KCH * 16));
}
__device__ __forceinline__ u32x4 frag_mc(const char* img, int lane_off, int base_mn, int ks) {
  lds_char* b = (lds_char*)img + lane_off + (ks * 16 * 512 + 64 * ((base_mn >> 5) & 4));
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b + 4 * 512));
  union { struct { s16x4 a, b; } s; u32x4 u; } c;
  c.s.a = lo;
  c.s.b = hi;
  return c.u;
}

// wave-uniform pointer forced into SGPRs (the DMA's base operand must be scalar)
template <typename T> __device__ __forceinline__ const T* sgpr_ptr(const T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<const T*>(((uint64_t)hi << 32) | lo);
}

template <int DT> __device__ __forceinline__ f32x16 mfma(u32x4 a, u32x4 b, f32x16 c) {
  if constexpr (DT == DT_BF16)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

}  // namespace g2

// Persistent: gridDim.x workgroups (<= one per CU) walk the work items L = slot, slot + G, ...
// (item = (split, batch, output tile)); the LDS-DMA ring runs straight across item
// boundaries, so the next item's first k-tile streams in during this item's last k-tile and
// epilogue.  ws != nullptr: split-K partials ws[((split * batches) + batch) * M * N + m * N + n].
// ISS: where the next k-tile's 8 DMAs are issued -- 0: all before k-step 0's fragment reads,
// 1: 4 after k-step 0's and 4 after k-step 1's fragment reads (before their MFMAs)
// PST: persistent grid (epilogue strips beside the ring, overlapping the next item's DMAs);
// !PST: one item per workgroup, the epilogue reuses the drained ring (128 KiB LDS)
template <int DTI, int DTO, bool A_MC, bool B_MC, int ISS, bool PST>
__global__ __launch_bounds__(512) void gemm2_kernel(GemmArgs p, float* __restrict__ ws, int W, int batches, int nsplit) {
  using namespace g2;
  using CF = Cfg<64, 2>;
  using fa::glds16;
  using fa::wait_vm;
  using fa::raw_barrier;
  using TI = typename dt_traits<DTI>::T;
  using TO = typename dt_traits<DTO>::T;
  constexpr int BK = CF::BK, NG = CF::NG, IMG = CF::IMG, STAGE = CF::STAGE;
  constexpr int PPW = CF::PPW, KCH = CF::KCH, KS = BK / 16;
  constexpr int EPI_OFF = PST ? 2 * STAGE : 0;  // 32 KiB of wave-private epilogue strips

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int G = gridDim.x;
  const int slot = xcd_remap(blockIdx.x, G);  // XCD x runs a contiguous slot range
  if (slot >= W) return;

  const int ktiles = (p.K + BK - 1) / BK;
  const int ntot = ktiles * p.nseg;
  const int ntile = p.tiles_m * p.tiles_n;
  constexpr int GM = 8;
  const int gsz = GM * p.tiles_n;

  struct Item {
    int m0, n0, z, zs, tb, te;
    const TI* A;  // batch + mn base
    const TI* B;
  };
  auto item_of = [&](int L) {
    Item it;
    const int zz = L / ntile, tl = L % ntile;
    it.zs = zz / batches;
    it.z = zz % batches;
    const int g = tl / gsz, first_m = g * GM;
    const int gm_n = min(GM, p.tiles_m - first_m);
    it.m0 = (first_m + (tl % gsz) % gm_n) * BM;
    it.n0 = ((tl % gsz) / gm_n) * BN;
    it.tb = (int)((int64_t)it.zs * ntot / nsplit);
    it.te = (int)((int64_t)(it.zs + 1) * ntot / nsplit);
    const int z1 = it.z / p.nb2, z2 = it.z % p.nb2;
    it.te = __builtin_amdgcn_readfirstlane(it.te);
    it.tb = __builtin_amdgcn_readfirstlane(it.tb);
    it.A = reinterpret_cast<const TI*>(p.A) + z1 * p.sA1 + z2 * p.sA2 + (A_MC ? (int64_t)it.m0 : (int64_t)it.m0 * p.lda);
    it.B = reinterpret_cast<const TI*>(p.B) + z1 * p.sB1 + z2 * p.sB2 + (B_MC ? (int64_t)it.n0 : (int64_t)it.n0 * p.ldb);
    return it;
  };

  // ---- issue side: the k-tile whose DMAs go out next (item ii, flattened k index ik) ----
  int iL = slot;
  Item ii = item_of(iL);
  OpDma<CF, A_MC> da;
  OpDma<CF, B_MC> db;
  da.init(wave, lane, p.lda, p.M - ii.m0);
  db.init(wave, lane, p.ldb, p.N - ii.n0);
  int ik = ii.tb, iseg = ik / ktiles, ikt = ik % ktiles, istage = 0;
  bool ivalid = true;
  const TI* ia = ii.A + iseg * p.sAseg + (A_MC ? (int64_t)ikt * BK * p.lda : (int64_t)ikt * BK);
  const TI* ib = ii.B + iseg * p.sBseg + (B_MC ? (int64_t)ikt * BK * p.ldb : (int64_t)ikt * BK);
  auto reset_ptrs = [&]() {
    ia = ii.A + iseg * p.sAseg + (A_MC ? (int64_t)ikt * BK * p.lda : (int64_t)ikt * BK);
    ib = ii.B + iseg * p.sBseg + (B_MC ? (int64_t)ikt * BK * p.ldb : (int64_t)ikt * BK);
  };
  auto issue_part = [&](int d0, int d1) {
    char* st = smem + istage * STAGE;
    const TI* sa = sgpr_ptr(ia);
    const TI* sb = sgpr_ptr(ib);
    if ((ikt + 1) * BK <= p.K) {
#pragma unroll
      for (int d = 0; d < NG; ++d) {
        if (d < d0 || d >= d1) continue;
        if (d < PPW) glds16(sa, da.off[d], st + (wave * PPW + d) * 1024);
        else glds16(sb, db.off[d - PPW], st + IMG + (wave * PPW + d - PPW) * 1024);
      }
    } else {  // K-tail tile (once per segment at most)
      const int kl = p.K - ikt * BK;
#pragma unroll
      for (int d = 0; d < NG; ++d) {
        if (d < d0 || d >= d1) continue;
        if (d < PPW) glds16(sa, da.tail_off(d, p.lda, kl), st + (wave * PPW + d) * 1024);
        else glds16(sb, db.tail_off(d - PPW, p.ldb, kl), st + IMG + (wave * PPW + d - PPW) * 1024);
      }
    }
  };
  auto advance_issue = [&]() {
    istage ^= 1;
    ik = __builtin_amdgcn_readfirstlane(ik + 1);
    if (ik < ii.te) {
      ikt = __builtin_amdgcn_readfirstlane(ikt + 1);
      if (ikt == ktiles) {
        ikt = 0;
        ++iseg;
        reset_ptrs();
      } else {
        ia += A_MC ? (int64_t)BK * p.lda : (int64_t)BK;
        ib += B_MC ? (int64_t)BK * p.ldb : (int64_t)BK;
      }
      return;
    }
    iL += G;
    if (iL >= W) {
      ivalid = false;
      return;
    }
    ii = item_of(iL);
    da.init(wave, lane, p.lda, p.M - ii.m0);
    db.init(wave, lane, p.ldb, p.N - ii.n0);
    ik = __builtin_amdgcn_readfirstlane(ii.tb);
    iseg = __builtin_amdgcn_readfirstlane(ik / ktiles);
    ikt = __builtin_amdgcn_readfirstlane(ik % ktiles);
    reset_ptrs();
  };

  // zero the k >= K part of a tail tile's images (after its DMAs landed, before any read)
  auto patch_tail = [&](char* st, int kl) {
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      char* img = st + o * IMG;
      const bool mc = o == 0 ? A_MC : B_MC;
#pragma unroll
      for (int i = 0; i < IMG / 16 / NT; ++i) {
        const int e = tid + NT * i;  // 16-byte entries of the image
        bool dead;
        if (!mc) {
          const int row = e / KCH, cp = e % KCH;
          dead = 8 * (cp ^ kc_swz<KCH>(row)) >= kl;
        } else {
          dead = (e >> 5) >= kl;
        }
        if (dead) *reinterpret_cast<u32x4*>(img + 16 * e) = u32x4{0, 0, 0, 0};
      }
    }
  };

  // per-lane LDS fragment bases
  const int l31 = lane & 31;
  int kc_off[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) kc_off[ks] = l31 * (KCH * 16) + (((2 * ks + hf) ^ kc_swz<KCH>(l31)) << 4);
  int mc_off[4];
  {
    const int Gq = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
#pragma unroll
    for (int v = 0; v < 4; ++v) mc_off[v] = (8 * (Gq >> 1) + q) * 512 + 64 * (v ^ q) + 32 * (Gq & 1) + 8 * pp;
  }

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // ---- epilogue of one item: 8 passes of a 16 x 64 fp32 strip through the wave's LDS strip
  // (64-float rows, 16-byte chunks XOR-swizzled by row & 3: conflict-free both ways) ----
  float* ep = reinterpret_cast<float*>(smem + EPI_OFF) + wave * 16 * 64;
  auto epilogue = [&](const Item& it) {
    const int rrow = lane >> 2, rq = lane & 3;
    const int gn = it.n0 + wn * 64 + rq * 16;
    const int z1 = it.z / p.nb2, z2 = it.z % p.nb2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 8 * h; r < 8 * h + 8; ++r) {
            const int row = (r & 3) + 8 * ((r >> 2) - 2 * h) + 4 * hf;
            const int col = 32 * j + l31;
            ep[row * 64 + ((((col >> 2) ^ (row & 3))) << 2) + (col & 3)] = acc[i][j][r];
          }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-private strip
        __builtin_amdgcn_wave_barrier();
        f32x4 v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = *reinterpret_cast<const f32x4*>(ep + rrow * 64 + (((4 * rq + c) ^ (rrow & 3)) << 2));
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        const int gm = it.m0 + wm * 128 + 32 * i + 16 * h + rrow;
        if (gm >= p.M) continue;
        if (ws) {
          float* dst = ws + ((int64_t)it.zs * batches + it.z) * (int64_t)p.M * p.N + (int64_t)gm * p.N + gn;
          if (gn + 16 <= p.N && (p.N & 3) == 0) {
#pragma unroll
            for (int c = 0; c < 4; ++c) *reinterpret_cast<f32x4*>(dst + 4 * c) = v[c];
          } else {
#pragma unroll
            for (int e = 0; e < 16; ++e)
              if (gn + e < p.N) dst[e] = v[e >> 2][e & 3];
          }
        } else {
          TO* dst = reinterpret_cast<TO*>(p.C) + z1 * p.sC1 + z2 * p.sC2 + (int64_t)gm * p.ldc + gn;
          constexpr int EO = 16 / sizeof(TO);
          if (gn + 16 <= p.N) {  // 16-byte stores at any element-aligned address (u32x4_ua)
#pragma unroll
            for (int c = 0; c < 16 / EO; ++c) {
              union { u32x4 u; TO e[EO]; } o;
              if (p.beta != 0.f) o.u = *reinterpret_cast<const u32x4_ua*>(dst + c * EO);
#pragma unroll
              for (int e = 0; e < EO; ++e) {
                const float x = v[(c * EO + e) >> 2][(c * EO + e) & 3] * p.alpha;
                o.e[e] = (TO)(p.beta != 0.f ? x + p.beta * (float)o.e[e] : x);
              }
              *reinterpret_cast<u32x4_ua*>(dst + c * EO) = o.u;
            }
          } else {
#pragma unroll
            for (int e = 0; e < 16; ++e)
              if (gn + e < p.N) {
                const float x = v[e >> 2][e & 3] * p.alpha;
                dst[e] = (TO)(p.beta != 0.f ? x + p.beta * (float)dst[e] : x);
              }
          }
        }
      }
    }
  };

  // ---- main loop over this workgroup's k-tiles, item after item ----
  int cL = slot;
  Item ci = ii;
  int ck = ci.tb, ckt = ck % ktiles, cstage = 0;
  issue_part(0, NG);
  advance_issue();
  wait_vm<0>();
  raw_barrier();
  while (true) {
    char* st = smem + cstage * STAGE;
    const bool pre = ivalid;
    {
      const int kl = p.K - ckt * BK;
      if (kl < BK) {  // uniform across the workgroup
        patch_tail(st, kl);
        __syncthreads();
      }
    }
    const char* sa = st;
    const char* sb = st + IMG;
    if (ISS == 0 && pre) issue_part(0, NG);
    // ISS 1: the next k-tile's DMAs go out after k-steps 0 and 1's fragment reads, before
    // their MFMAs (a DMA issue costs ~60 cycles; interleaved, the SIMD's other wave issues MFMAs)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      u32x4 fa[4], fb[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mb = wm * 128 + 32 * i;
        fa[i] = A_MC ? g2::frag_mc(sa, mc_off[(mb >> 5) & 3], mb, ks) : g2::frag_kc<KCH>(sa, kc_off[ks], mb);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int nb = wn * 64 + 32 * j;
        fb[j] = B_MC ? g2::frag_mc(sb, mc_off[(nb >> 5) & 3], nb, ks) : g2::frag_kc<KCH>(sb, kc_off[ks], nb);
      }
      if (ISS == 1 && ks < 2 && pre) issue_part(ks * (NG / 2), (ks + 1) * (NG / 2));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = g2::mfma<DTI>(fa[i], fb[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    if (pre) advance_issue();
    ck = __builtin_amdgcn_readfirstlane(ck + 1);
    const bool last = ck == ci.te;
    if (PST && last) {  // epilogue while the next item's first k-tile is in flight
      epilogue(ci);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    }
    wait_vm<0>();
    raw_barrier();
    if (!PST && last) {
      epilogue(ci);
      break;
    }
    if (last) {
      cL += G;
      if (cL >= W) break;
      ci = item_of(cL);
      ck = ci.tb;
      ckt = ck % ktiles;
    } else if (++ckt == ktiles) {
      ckt = 0;
    }
    cstage ^= 1;
  }
}

// C[z](m, n) = alpha * sum_s ws[s, z, m, n] + beta * C[z](m, n)   (slices summed in order)
template <int DTO>
__global__ __launch_bounds__(256) void gemm2_reduce(GemmArgs p, const float* __restrict__ ws, int S, int batches) {
  using TO = typename dt_traits<DTO>::T;
  const int64_t MN = (int64_t)p.M * p.N;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= MN * batches) return;
  const int z = (int)(idx / MN);
  const int64_t mn = idx % MN;
  const int m = (int)(mn / p.N), n = (int)(mn % p.N);
  float acc = 0.f;
  for (int s = 0; s < S; ++s) acc += ws[((int64_t)s * batches + z) * MN + mn];
  TO* c = reinterpret_cast<TO*>(p.C) + (z / p.nb2) * p.sC1 + (z % p.nb2) * p.sC2 + (int64_t)m * p.ldc + n;
  const float x = acc * p.alpha;
  *c = (TO)(p.beta != 0.f ? x + p.beta * (float)*c : x);
}

inline int num_cus() {
  static const int v = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  return v;
}

// largest k-tile count per item that still runs persistent
constexpr int GEMM2_PERSIST_KT = 32;

// 4 consecutive columns per thread (N % 4 == 0, ldc % 4 == 0, C 16-byte aligned)
template <int DTO>
__global__ __launch_bounds__(256) void gemm2_reduce4(GemmArgs p, const float* __restrict__ ws, int S, int batches) {
  using TO = typename dt_traits<DTO>::T;
  const int64_t MN = (int64_t)p.M * p.N, MN4 = MN / 4;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= MN4 * batches) return;
  const int z = (int)(idx / MN4);
  const int64_t mn = (idx % MN4) * 4;
  const int m = (int)(mn / p.N), n = (int)(mn % p.N);
  f32x4 acc = *reinterpret_cast<const f32x4*>(ws + (int64_t)z * MN + mn);
  for (int s = 1; s < S; ++s) acc += *reinterpret_cast<const f32x4*>(ws + ((int64_t)s * batches + z) * MN + mn);
  TO* c = reinterpret_cast<TO*>(p.C) + (z / p.nb2) * p.sC1 + (z % p.nb2) * p.sC2 + (int64_t)m * p.ldc + n;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float x = acc[e] * p.alpha;
    c[e] = (TO)(p.beta != 0.f ? x + p.beta * (float)c[e] : x);
  }
}

template <int DTI, int DTO, bool AMC, bool BMC>
static void launch2_t(const GemmArgs& a, int batches, int splits, float* ws, hipStream_t st) {
  const int W = a.tiles_m * a.tiles_n * batches * splits;
  // persistent (one workgroup per CU) when items are short (the per-item prologue/epilogue is
  // then a large share that the ring overlaps); one workgroup per item for long K
  const int kt_item = ((a.K + 63) / 64) * a.nseg / splits;
  const int G = (W > num_cus() && kt_item <= GEMM2_PERSIST_KT) ? num_cus() : W;
  constexpr int LDS = g2::Cfg<64, 2>::LDS + 32768;  // ring + epilogue strips = 160 KiB
  const bool pst = G < W;
#define G2LAUNCH(PST, LDSB)                                                                                        \
  hipLaunchKernelGGL((gemm2_kernel<DTI, DTO, AMC, BMC, 1, PST>), dim3(G), dim3(g2::NT), LDSB, st, a,            \
                     splits > 1 ? ws : nullptr, W, batches, splits)
  if (pst) G2LAUNCH(true, LDS);
  else G2LAUNCH(false, LDS - 32768);
#undef G2LAUNCH
  if (splits > 1) {
    const int64_t n = (int64_t)a.M * a.N * batches;
    const bool v4 = a.N % 4 == 0 && a.ldc % 4 == 0 && a.sC1 % 4 == 0 && a.sC2 % 4 == 0 &&
                    (reinterpret_cast<uintptr_t>(a.C) & 15) == 0;
    if (v4)
      hipLaunchKernelGGL((gemm2_reduce4<DTO>), dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, st, a, ws, splits, batches);
    else
      hipLaunchKernelGGL((gemm2_reduce<DTO>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, ws, splits, batches);
  }
}

template <int DTI, int DTO>
static void launch2_d(const GemmArgs& a, int batches, bool amc, bool bmc, int splits, float* ws, hipStream_t st) {
  if (!amc && !bmc) return launch2_t<DTI, DTO, false, false>(a, batches, splits, ws, st);
  if (!amc && bmc) return launch2_t<DTI, DTO, false, true>(a, batches, splits, ws, st);
  if (amc && !bmc) return launch2_t<DTI, DTO, true, false>(a, batches, splits, ws, st);
  return launch2_t<DTI, DTO, true, true>(a, batches, splits, ws, st);
}

}  // namespace xdot

// Eligibility (checked by the caller, csrc/bindings.cpp): 16-bit A/B, every operand address
// 16-byte aligned with lda/ldb/batch/segment strides multiples of 8 elements, K % 8 == 0 when
// an operand is k-contiguous, the mn extent of an mn-contiguous operand a multiple of 8.
extern "C" int xdot_gemm2_launch(const xdot::GemmArgs* a, int batches, int dt_in, int dt_out, int a_mc, int b_mc,
                                 int splits, float* ws, hipStream_t st) {
  using namespace xdot;
  GemmArgs g = *a;
  g.tiles_m = (g.M + g2::BM - 1) / g2::BM;
  g.tiles_n = (g.N + g2::BN - 1) / g2::BN;
  if (g.tiles_m == 0 || g.tiles_n == 0 || batches == 0) return 0;
  if (splits < 1 || (splits > 1 && !ws)) return -2;
#define G2_DT(I, O) \
  if (dt_in == I && dt_out == O) { launch2_d<I, O>(g, batches, a_mc, b_mc, splits, ws, st); return 0; }
  G2_DT(DT_BF16, DT_BF16) G2_DT(DT_BF16, DT_F32) G2_DT(DT_F16, DT_F16) G2_DT(DT_F16, DT_F32)
#undef G2_DT
  return -1;
}

extern "C" int xdot_num_cus() { return xdot::num_cus(); }

// C = alpha * sum_s ws[s] + beta * C for a split-K GEMM's fp32 slices (slices summed in order)
extern "C" int xdot_gemm_reduce_launch(const xdot::GemmArgs* ap, const float* ws, int splits, int batches, int dt_out,
                                       hipStream_t st) {
  using namespace xdot;
  const GemmArgs& a = *ap;
  const int64_t n = (int64_t)a.M * a.N * batches;
  const bool v4 = a.N % 4 == 0 && a.ldc % 4 == 0 && a.sC1 % 4 == 0 && a.sC2 % 4 == 0 &&
                  (reinterpret_cast<uintptr_t>(a.C) & 15) == 0;
#define RED(DT)                                                                                                      \
  if (dt_out == DT) {                                                                                                \
    if (v4) hipLaunchKernelGGL((gemm2_reduce4<DT>), dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, st, a, ws, splits, batches); \
    else hipLaunchKernelGGL((gemm2_reduce<DT>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, ws, splits, batches);        \
    return 0;                                                                                                        \
  }
  RED(DT_BF16) RED(DT_F16) RED(DT_F32)
#undef RED
  return -1;
}

