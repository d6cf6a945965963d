// xdot — persistent 256x256 exact-fp32 GEMM for gfx950 (the fp32 member of the "v2" family).
//
//   C[z](m, n) = alpha * sum_{s < nseg} sum_{k < K} opA_s[z](m, k) * opB_s[z](k, n) + beta * C[z](m, n)
//
// Same GemmArgs addressing as csrc/gemm.hip / gemm2.hip, fp32 in and out, every product exact
// (v_mfma_f32_32x32x2_f32: a k-ordered fmaf chain).  These are the reference's own products
// (distributed_dot_product/multiplication/functions.py:96 nt, :142 tn, :209 all, fp32 buffers of
// :86,198) at large shapes.  Why a second fp32 kernel: the 128x128 register-staged kernel of
// csrc/gemm_f32.hip measured 0.86x hipBLASLt (78 % MFMA busy on 25000 x 75000 x 768): its
// per-tile prologue / epilogue (24 k-tiles per output tile at K = 768) and the register staging
// (8 global loads + 8 ds_write_b128 + predicates per k-tile) are exposed.  Here, as in gemm2.hip:
//   * 256x256 workgroup tile, 8 waves (2 per SIMD) in a 2 (M) x 4 (N) grid, each wave 128x64 =
//     4x2 blocks of 32x32 (128 accumulator registers), 128 MFMAs (8192 cycles) per k-tile;
//   * operands travel HBM -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR staging, no
//     ds_write), BK = 32 (a k-contiguous row segment is one whole 128-byte line), 2 stages of
//     64 KiB, one counted `s_waitcnt vmcnt` + barrier per k-tile, the next k-tile's 8 DMAs per
//     wave interleaved with the first two MFMA groups;
//   * persistent grid (one workgroup per CU) walking (split, batch, tile) items: the ring runs
//     across items, so an item's epilogue (through wave-private LDS strips: 64-byte row pieces
//     per lane) overlaps the next item's first DMAs;
//   * images: k-contiguous [256 rows][8 x 16-byte chunks], chunk ^= (row >> 1) & 7 (each 16-lane
//     ds_read_b128 group on 16 distinct bank quads); mn-contiguous [32 k][64 chunks], chunk ^=
//     8 ((k >> 4) & 1) (the two lane halves of a ds_read_b32 on opposite 32-bank halves).  The
//     swizzle is applied to the DMA SOURCE addresses (the DMA destination is lane-linear);
//   * K tails are zero-patched in LDS after their DMAs land; M/N tails re-read the last valid
//     row / chunk (finite values whose outputs are never stored);
//   * split-K (ws != nullptr): fp32 partial slices summed in order by gemm2_reduce (deterministic).
// MFMA k pairing as in gemm_f32.hip: MFMA 4g + t of a k-tile, lane half h, uses k = 16h + 4g + t
// for both operands, so one ds_read_b128 of a k-contiguous image feeds four MFMAs.
#include "flash_common.h"

namespace xdot {
namespace g2f {

constexpr int BM = 256, BN = 256, BK = 32, NT = 512;
constexpr int IMG = 256 * BK * 4;     // bytes per operand image (32 KiB)
constexpr int STAGE = 2 * IMG;        // A + B
constexpr int RING = 2 * STAGE;       // 2 stages: 128 KiB
constexpr int PPW = IMG / 1024 / 8;   // 1-KiB DMA pieces per wave per image
constexpr int NG = 2 * PPW;           // DMAs per wave per k-tile
constexpr int EPI = 8 * 16 * 64 * 4;  // wave-private 16 x 64 fp32 epilogue strips
constexpr int LDS = RING + EPI;       // 160 KiB
static_assert(LDS <= 160 * 1024, "lds");

__device__ __forceinline__ int kc_swz(int row) { return (row >> 1) & 7; }

// Per-lane DMA source offsets (bytes from the k-tile's first row / k) of the wave's pieces of
// one operand image, plus what the K-tail path needs.
template <bool MC> struct OpDma {
  uint32_t off[PPW];
  int r[PPW], c[PPW];  // k-contiguous: image row (clamped), logical chunk; mn-contiguous: k row, mn offset
  __device__ __forceinline__ void init(int wave, int lane, int64_t ld, int mn_left) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = (wave * PPW + i) * 1024 + lane * 16;
      if (!MC) {  // [256 rows][8 chunks]
        const int row = p >> 7, c4 = ((p >> 4) & 7) ^ kc_swz(row);
        const int rr = min(row, mn_left - 1);
        r[i] = rr;
        c[i] = c4;
        off[i] = (uint32_t)(((int64_t)rr * ld + 4 * c4) * 4);
      } else {    // [32 k rows][64 chunks]
        const int kr = p >> 10, c4 = ((p >> 4) & 63) ^ (8 * ((kr >> 4) & 1));
        const int mn = min(4 * c4, mn_left - 4);
        r[i] = kr;
        c[i] = mn;
        off[i] = (uint32_t)(((int64_t)kr * ld + mn) * 4);
      }
    }
  }
  // K-tail k-tile: no byte past the last valid chunk / row of the operand is touched
  __device__ __forceinline__ uint32_t tail_off(int i, int64_t ld, int kleft) const {
    if (!MC) return (uint32_t)(((int64_t)r[i] * ld + 4 * min(c[i], (kleft + 3) / 4 - 1)) * 4);
    return (uint32_t)(((int64_t)min(r[i], kleft - 1) * ld + c[i]) * 4);
  }
};

// wave-uniform pointer forced into SGPRs (the DMA's base operand is scalar)
__device__ __forceinline__ const float* sgpr_ptr(const float* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<const float*>(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ f32x16 mm(float a, float b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// four k-steps (k = 16 hf + 4 g + t) of one 32-row block
__device__ __forceinline__ f32x4 frag_kc(const char* img, int row_bytes, int lane_off) {
  return *reinterpret_cast<const f32x4*>(img + row_bytes + lane_off);
}
__device__ __forceinline__ f32x4 frag_mc(const char* img, int lane_off, int g) {
  const float* q = reinterpret_cast<const float*>(img + lane_off + g * 4096);
  return f32x4{q[0], q[256], q[512], q[768]};
}

}  // namespace g2f

template <bool A_MC, bool B_MC>
__global__ __launch_bounds__(512) void gemm2_f32_kernel(GemmArgs p, float* __restrict__ ws, int W, int batches,
                                                        int nsplit) {
  using namespace g2f;
  using fa::glds16;
  using fa::raw_barrier;
  using fa::wait_vm;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5, l31 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int G = gridDim.x;
  const int slot = xcd_remap(blockIdx.x, G);
  if (slot >= W) return;

  const int ktiles = (p.K + BK - 1) / BK;
  const int ntot = ktiles * p.nseg;
  const int ntile = p.tiles_m * p.tiles_n;
  constexpr int GM = 8;
  const int gsz = GM * p.tiles_n;

  struct Item {
    int m0, n0, z, zs, tb, te;
    const float* A;  // batch + mn base
    const float* B;
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
    it.tb = __builtin_amdgcn_readfirstlane((int)((int64_t)it.zs * ntot / nsplit));
    it.te = __builtin_amdgcn_readfirstlane((int)((int64_t)(it.zs + 1) * ntot / nsplit));
    const int z1 = it.z / p.nb2, z2 = it.z % p.nb2;
    it.A = reinterpret_cast<const float*>(p.A) + z1 * p.sA1 + z2 * p.sA2 + (A_MC ? (int64_t)it.m0 : (int64_t)it.m0 * p.lda);
    it.B = reinterpret_cast<const float*>(p.B) + z1 * p.sB1 + z2 * p.sB2 + (B_MC ? (int64_t)it.n0 : (int64_t)it.n0 * p.ldb);
    return it;
  };

  // ---- issue side: the k-tile whose DMAs go out next (item ii, flattened k index ik) ----
  int iL = slot;
  Item ii = item_of(iL);
  g2f::OpDma<A_MC> da;
  g2f::OpDma<B_MC> db;
  da.init(wave, lane, p.lda, p.M - ii.m0);
  db.init(wave, lane, p.ldb, p.N - ii.n0);
  int ik = ii.tb, iseg = ik / ktiles, ikt = ik % ktiles, istage = 0;
  bool ivalid = true;
  const float* ia = nullptr;
  const float* ib = nullptr;
  auto reset_ptrs = [&]() {
    ia = ii.A + iseg * p.sAseg + (A_MC ? (int64_t)ikt * BK * p.lda : (int64_t)ikt * BK);
    ib = ii.B + iseg * p.sBseg + (B_MC ? (int64_t)ikt * BK * p.ldb : (int64_t)ikt * BK);
  };
  reset_ptrs();
  auto issue_part = [&](int d0, int d1) {
    char* st = smem + istage * STAGE;
    const float* sa = g2f::sgpr_ptr(ia);
    const float* sb = g2f::sgpr_ptr(ib);
    if ((ikt + 1) * BK <= p.K) {
#pragma unroll
      for (int d = 0; d < NG; ++d) {
        if (d < d0 || d >= d1) continue;
        if (d < PPW) glds16(sa, da.off[d], st + (wave * PPW + d) * 1024);
        else glds16(sb, db.off[d - PPW], st + IMG + (wave * PPW + d - PPW) * 1024);
      }
    } else {  // K-tail k-tile (once per segment at most)
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

  // zero the k >= kl part of a tail k-tile's images (after its DMAs landed, before any read)
  auto patch_tail = [&](char* st, int kl) {
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      char* img = st + o * IMG;
      const bool mc = o == 0 ? A_MC : B_MC;
#pragma unroll
      for (int i = 0; i < IMG / 16 / NT; ++i) {
        const int e = tid + NT * i;  // 16-byte entries of the image
        f32x4* q = reinterpret_cast<f32x4*>(img + 16 * e);
        if (!mc) {
          const int k0 = 4 * ((e & 7) ^ g2f::kc_swz(e >> 3));
          if (k0 + 3 >= kl) {
            f32x4 v = *q;
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (k0 + j >= kl) v[j] = 0.f;
            *q = v;
          }
        } else if ((e >> 6) >= kl) {
          *q = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
  };

  // per-lane LDS fragment offsets
  int kc_off[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) kc_off[g] = l31 * 128 + 16 * ((4 * hf + g) ^ g2f::kc_swz(l31));
  int mca[4], mcb[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) mca[i] = 16 * hf * 1024 + 512 * wm + 128 * (i ^ hf) + 4 * l31;
#pragma unroll
  for (int j = 0; j < 2; ++j) mcb[j] = 16 * hf * 1024 + 256 * wn + 128 * (j ^ hf) + 4 * l31;
  auto fragA = [&](const char* sa, int i, int g) -> f32x4 {
    if constexpr (A_MC) return g2f::frag_mc(sa, mca[i], g);
    else return g2f::frag_kc(sa, (wm * 128 + 32 * i) * 128, kc_off[g]);
  };
  auto fragB = [&](const char* sb, int j, int g) -> f32x4 {
    if constexpr (B_MC) return g2f::frag_mc(sb, mcb[j], g);
    else return g2f::frag_kc(sb, (wn * 64 + 32 * j) * 128, kc_off[g]);
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  // ---- epilogue of one item: 8 passes of a 16 x 64 fp32 strip through the wave's LDS strip
  // (64-float rows, 16-byte chunks XOR-swizzled by row & 3: conflict-free both ways) ----
  float* ep = reinterpret_cast<float*>(smem + RING) + wave * 16 * 64;
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
        float* dst = ws ? ws + ((int64_t)it.zs * batches + it.z) * (int64_t)p.M * p.N + (int64_t)gm * p.N + gn
                        : reinterpret_cast<float*>(p.C) + z1 * p.sC1 + z2 * p.sC2 + (int64_t)gm * p.ldc + gn;
        const bool full = gn + 16 <= p.N;
        if (ws) {
          if (full && (p.N & 3) == 0) {
#pragma unroll
            for (int c = 0; c < 4; ++c) *reinterpret_cast<f32x4*>(dst + 4 * c) = v[c];
          } else {
#pragma unroll
            for (int e = 0; e < 16; ++e)
              if (gn + e < p.N) dst[e] = v[e >> 2][e & 3];
          }
        } else if (full) {  // 16-byte stores at any 4-byte-aligned address (u32x4_ua)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            f32x4 o = v[c] * p.alpha;
            if (p.beta != 0.f) o += p.beta * __builtin_bit_cast(f32x4, *reinterpret_cast<const u32x4_ua*>(dst + 4 * c));
            *reinterpret_cast<u32x4_ua*>(dst + 4 * c) = __builtin_bit_cast(u32x4, o);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 16; ++e)
            if (gn + e < p.N) {
              const float x = v[e >> 2][e & 3] * p.alpha;
              dst[e] = p.beta != 0.f ? x + p.beta * dst[e] : x;
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
    // 4 groups of 4 k-steps; fragment reads one group ahead; the next k-tile's DMAs go out
    // after groups 0 and 1's reads (a DMA issue costs ~60 cycles; the SIMD's other wave
    // issues MFMAs meanwhile)
    f32x4 fa0[4], fb0[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa0[i] = fragA(sa, i, 0);
#pragma unroll
    for (int j = 0; j < 2; ++j) fb0[j] = fragB(sb, j, 0);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 fa1[4], fb1[2];
      if (g + 1 < 4) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa1[i] = fragA(sa, i, g + 1);
#pragma unroll
        for (int j = 0; j < 2; ++j) fb1[j] = fragB(sb, j, g + 1);
      }
      // (staggered by wave half or spread over all 4 groups measured the same, profiles/r5_fp32.md §4)
      if (g < 2 && pre) issue_part(g * (NG / 2), (g + 1) * (NG / 2));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = g2f::mm(fa0[i][s], fb0[j][s], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (g + 1 < 4) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa0[i] = fa1[i];
#pragma unroll
        for (int j = 0; j < 2; ++j) fb0[j] = fb1[j];
      }
    }
    if (pre) advance_issue();
    ck = __builtin_amdgcn_readfirstlane(ck + 1);
    const bool last = ck == ci.te;
    if (last) {  // epilogue while the next item's first k-tile is in flight
      epilogue(ci);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
    }
    wait_vm<0>();
    raw_barrier();
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

}  // namespace xdot

// Eligibility (checked by the caller, csrc/bindings.cpp): fp32 A/B/C, operand bases 16-byte
// aligned with lda/ldb/batch/segment strides multiples of 4 elements, K % 4 == 0 when an operand
// is k-contiguous, the mn extent of an mn-contiguous operand a multiple of 4.  splits > 1 needs
// ws (splits * batches * M * N floats); the ordered sum runs after (xdot_gemm_reduce_launch).
extern "C" int xdot_gemm2_f32_launch(const xdot::GemmArgs* a, int batches, int a_mc, int b_mc, int splits, float* ws,
                                     hipStream_t st) {
  using namespace xdot;
  GemmArgs g = *a;
  g.tiles_m = (g.M + g2f::BM - 1) / g2f::BM;
  g.tiles_n = (g.N + g2f::BN - 1) / g2f::BN;
  if (g.tiles_m == 0 || g.tiles_n == 0 || batches == 0) return 0;
  if (g.K <= 0 || splits < 1 || (splits > 1 && !ws)) return -2;
  const int W = g.tiles_m * g.tiles_n * batches * splits;
  const int G = W < xdot_num_cus() ? W : xdot_num_cus();
#define G2F(AM, BM_)                                                                                          \
  if (a_mc == AM && b_mc == BM_) {                                                                            \
    hipLaunchKernelGGL((gemm2_f32_kernel<AM, BM_>), dim3(G), dim3(g2f::NT), g2f::LDS, st, g, splits > 1 ? ws : nullptr, \
                       W, batches, splits);                                                                   \
  }
  G2F(false, false) else G2F(false, true) else G2F(true, false) else G2F(true, true)
#undef G2F
  if (splits > 1) return xdot_gemm_reduce_launch(&g, ws, splits, batches, DT_F32, st);
  return 0;
}
