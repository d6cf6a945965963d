// xdot — projection GEMM for gfx950: the module's Linear layers (reference:
// distributed_dot_product/module.py:43-45 keys / queries / values, :75 composition), forward and
// input gradient.
//
//   NT:  C[M, N] = α (A[M, K] · B[N, K]ᵀ (+ bias[N]))   forward   y  = x · Wᵀ + b (α: the
//        attention's row-side pre-scale folded into the k projection, one rounding)
//   NN:  C[M, N] = A[M, K] · B[K, N]                 backward  dx = dy · W
//
// A is k-contiguous (activations / output gradients, row stride lda), C row-major (ldc).  The
// shapes are the per-rank projections: M = T/N rows (3125 at the N=8 headline rank, 25000 at
// N=1), N, K = 768 / 1536.  At M = 3125 the 256x256-tile kernels have 78 tiles for 256 CUs
// (fill-bound: profiles/r3_rank_host.md), so this kernel picks the tile size per shape
// (128x128, 64x128, 64x64) to put >= 2 workgroups on every CU, and runs the whole K = 768 /
// 1536 reduction in one workgroup (no split-K partials).
//
//   * 256 threads = 2x2 waves, each a (BM/2) x (BN/2) block of v_mfma_f32_16x16x32 tiles;
//   * k-tiles of 64 through a 2- or 3-stage LDS ring filled by global_load_lds_dwordx4 (no VGPRs
//     hold a tile in flight; the next k-tile's DMA runs under this one's MFMAs, and the
//     co-resident workgroups cover the rest of its latency);
//   * k-contiguous images [rows][128 B], 16-byte chunk c of row r at c ^ ((r >> 1) & 7):
//     conflict-free ds_read_b128 fragments (the gemm3 layout); NN's B is an mn-contiguous
//     image [64 k][256 B] read with ds_read_b64_tr_b16 (hardware transpose, gemm3's swizzle);
//   * the MFMA computes Cᵀ tiles (B fragment as its A operand), so each lane ends with 4
//     consecutive output columns of one row: + bias in fp32, one rounding, 8-byte stores;
//   * rows past M re-read row M-1 (no bounds branches in the loop) and are not stored.
#include "flash_common.h"

namespace xdot {
namespace gp {

constexpr int BK = 64;
#ifndef GP_PRIO
#define GP_PRIO 1  // s_setprio 1 around each k-step's MFMAs (A/B knob; 0-2 % faster, profiles/r4_s2.md)
#endif
#ifndef GP_PRE
#define GP_PRE 0  // read both k-steps' fragments before the first k-step's MFMAs (A/B knob)
#endif
#ifndef GP_BIG
#define GP_BIG 1  // 0: never the 128x128 tile (64x128 at every M)
#endif
#ifndef GP_HUGE
#define GP_HUGE 0  // 1: 256x128 tiles of 8 waves where they fill >= 4 rounds of the 256 CUs (A/B knob)
#endif

template <int DT> __device__ __forceinline__ f32x4 mfma16(u32x4 a, u32x4 b, f32x4 c) {
  if constexpr (DT == DT_BF16)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// N consecutive 1 KiB LDS-DMA pieces of one wave: LDS[lds + 1024 i + 16 lane] <- base + o[i]
template <int N> __device__ __forceinline__ void dma_run(const void* base, const uint32_t* o, uint32_t lds);
template <> __device__ __forceinline__ void dma_run<2>(const void* base, const uint32_t* o, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %4\n\t"
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %4\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(o[0]), "v"(o[1]), "s"(lds), "s"(base) : "memory", "scc");
}
template <> __device__ __forceinline__ void dma_run<4>(const void* base, const uint32_t* o, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %5\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %6\n\t"
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %6\n\t"
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %6\n\t"
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %6\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]), "s"(lds), "s"(base)
               : "memory", "scc");
}

// NS_: stages of both rings (2 or 3), or 32 = a 3-stage A ring beside a 2-stage B ring (the
// activations, streamed from HBM, are issued two k-tiles ahead; the L2-resident weights one):
// 80 KiB at 128x128, so two workgroups still share a CU
template <int BM, int BN, bool NN, int NS_> struct Cfg {
  static constexpr int NA = NS_ == 32 ? 3 : NS_, NB = NS_ == 32 ? 2 : NS_;
  static constexpr int WGM = BM == 256 ? 4 : 2, NW = 2 * WGM, NTH = 64 * NW;  // waves: WGM x 2
  static constexpr int A_BYTES = BM * 128;                 // [BM rows][64 k x 2 B]
  static constexpr int B_BYTES = NN ? 64 * BN * 2 : BN * 128;
  static constexpr int B_OFF = NA * A_BYTES;               // A ring, then B ring
  static constexpr int LDS = NA * A_BYTES + NB * B_BYTES;
  static constexpr int APW = A_BYTES / (1024 * NW), BPW = B_BYTES / (1024 * NW);  // 1 KiB pieces per wave
  static constexpr int WM = BM / WGM, WN = BN / 2, MT = WM / 16, NT = WN / 16;
};

// lanes 16-31 of x <-> lanes 0-15 of y, and 48-63 of x <-> 32-47 of y
__device__ __forceinline__ void swap16(uint32_t& x, uint32_t& y) {
  const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}

}  // namespace gp

template <int DT, int BM, int BN, bool NN, bool BIAS, int NS_, bool V16>
__global__ __launch_bounds__(BM == 256 ? 512 : 256) void gemm_proj_kernel(ProjArgs p) {
  using namespace gp;
  using fa::smem;
  using fa::lds_addr;
  using CF = Cfg<BM, BN, NN, NS_>;
  using T16 = typename dt_traits<DT>::T;
  static_assert(!NN || BN == 128, "NN: 256-byte mn-contiguous B rows");
  constexpr int MT = CF::MT, NT = CF::NT, APW = CF::APW, BPW = CF::BPW, NA = CF::NA, NB = CF::NB;
  static_assert((NA == 2 || NA == 3) && NB <= NA, "ring stages");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;  // WGM x 2 waves
  const int g = lane >> 4, l15 = lane & 15;
  const int tiles_n = p.N / BN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lin / tiles_n, tn = lin % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int KT = p.K / BK;
  const int64_t lda2 = (int64_t)p.lda * 2, ldb2 = (int64_t)p.ldb * 2;

  // ---- per-lane DMA source offsets (constant over k-tiles: the bases advance) ----
  uint32_t oa[APW], ob[BPW];
#pragma unroll
  for (int i = 0; i < APW; ++i) {
    const int pc = wave * APW + i;
    const int r = 8 * pc + (lane >> 3), c = (lane & 7) ^ ((r >> 1) & 7);
    const int rr = min(r, p.M - 1 - m0);  // rows past M re-read row M-1 (never stored)
    oa[i] = (uint32_t)(rr * lda2 + 16 * c);
  }
#pragma unroll
  for (int i = 0; i < BPW; ++i) {
    const int pc = wave * BPW + i;
    if constexpr (!NN) {
      const int r = 8 * pc + (lane >> 3), c = (lane & 7) ^ ((r >> 1) & 7);
      ob[i] = (uint32_t)(r * ldb2 + 16 * c);
    } else {
      const int k = 4 * pc + (lane >> 4), c = (lane & 15) ^ (2 * (k & 3) + 8 * ((k >> 3) & 1));
      ob[i] = (uint32_t)(k * ldb2 + 16 * c);
    }
  }
  const char* a_base = reinterpret_cast<const char*>(p.A) + (int64_t)m0 * lda2;
  const char* b_base = reinterpret_cast<const char*>(p.B) + (NN ? (int64_t)n0 * 2 : (int64_t)n0 * ldb2);
  const int64_t b_kstep = NN ? 64 * ldb2 : 128;
  auto issue_a = [&](int kt) __attribute__((always_inline)) {
    dma_run<APW>(a_base + (int64_t)kt * 128, oa, lds_addr(smem + (kt % NA) * CF::A_BYTES + wave * APW * 1024));
  };
  auto issue_b = [&](int kt) __attribute__((always_inline)) {
    dma_run<BPW>(b_base + (int64_t)kt * b_kstep, ob,
                 lds_addr(smem + CF::B_OFF + (kt % NB) * CF::B_BYTES + wave * BPW * 1024));
  };

  // ---- fragment reads (16x16x32 operand: lane l holds mn = base + (l & 15), k = 8 (l >> 4) .. +7) ----
  typedef const __attribute__((address_space(3))) char lds_char;
  const int kcb0 = l15 * 128 + 16 * ((0 + g) ^ (l15 >> 1));
  const int kcb1 = l15 * 128 + 16 * ((4 + g) ^ (l15 >> 1));
  auto kfrag = [&](const char* img, int mnb, int ks) __attribute__((always_inline)) -> u32x4 {
    return *reinterpret_cast<const u32x4*>(img + (ks ? kcb1 : kcb0) + mnb * 128);
  };
  // mn-contiguous transposed reads (NN's B): lane 4q + p of group g reads k row 8 g + q (+4,
  // + 32 ks), logical chunk (n base / 8) + (p >> 1) of that row
  const int tq = (lane & 15) >> 2, tp = lane & 3;
  auto mc_base = [&](int cb) __attribute__((always_inline)) {
    const int c = (tp >> 1) | ((cb ^ (2 * tq + 8 * (g & 1))) & 14);
    return (8 * g + tq) * 256 + 16 * c + 8 * (tp & 1);
  };
  int mcb[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) mcb[nt] = NN ? mc_base((CF::WN * wn + 16 * nt) / 8) : 0;
  auto bfrag = [&](const char* img, int nt, int ks) __attribute__((always_inline)) -> u32x4 {
    if constexpr (!NN) {
      return kfrag(img, CF::WN * wn + 16 * nt, ks);
    } else {
      lds_char* b = (lds_char*)img + mcb[nt] + ks * 32 * 256;
      fa::s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((fa::lds_s16x4*)(b));
      fa::s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((fa::lds_s16x4*)(b + 4 * 256));
      union { struct { fa::s16x4 a, b; } s; u32x4 u; } r;
      r.s.a = lo;
      r.s.b = hi;
      return r.u;
    }
  };

  // acc[mt][nt]: rows m0 + WM wm + 16 mt + l15, columns n0 + WN wn + 16 nt + 4 g .. +3
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Rings: k-tile kt's A in A-stage kt % NA, its B in B-stage kt % NB.  After the barrier of
  // iteration kt every wave is done with k-tile kt - 1, so A(kt + NA - 1) and B(kt + NB - 1) go into
  // the stages it used -- issued B first, then A, so the wait at the top of the next iteration can
  // leave exactly the A k-tiles beyond it in flight (APW instructions each; vmcnt counts in order).
  constexpr int NPW = APW + BPW;
#pragma unroll
  for (int i = 0; i < NA - 1; ++i) {
    if (i < KT) issue_a(i);
    if (i < NB - 1 && i < KT) issue_b(i);
  }
  for (int kt = 0; kt < KT; ++kt) {
    if constexpr (NA == 3 && NB == 3) {
      if (kt + 1 < KT) fa::wait_vm<NPW>(); else fa::wait_vm<0>();
    } else if constexpr (NA == 3) {
      if (kt + 1 < KT) fa::wait_vm<APW>(); else fa::wait_vm<0>();
    } else {
      fa::wait_vm<0>();
    }
    fa::raw_barrier();  // k-tile kt visible to every wave; every wave is done with k-tile kt - 1
    if (kt + NB - 1 < KT) issue_b(kt + NB - 1);
    if (kt + NA - 1 < KT) issue_a(kt + NA - 1);
    const char* ai = smem + (kt % NA) * CF::A_BYTES;
    const char* bi = smem + CF::B_OFF + (kt % NB) * CF::B_BYTES;
    // GP_PRE: both k-steps' fragments are read up front (the second k-step's reads fly under the
    // first k-step's MFMAs); else each k-step reads, then multiplies
    u32x4 fa_[2][MT], fb_[2][NT];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks == 0 || !GP_PRE) {
#pragma unroll
        for (int kk = ks; kk < (GP_PRE ? 2 : ks + 1); ++kk) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) fa_[kk][mt] = kfrag(ai, CF::WM * wm + 16 * mt, kk);
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) fb_[kk][nt] = bfrag(bi, nt, kk);
        }
      }
      if constexpr (GP_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16<DT>(fb_[ks][nt], fa_[ks][mt], acc[mt][nt]);
      if constexpr (GP_PRIO) __builtin_amdgcn_s_setprio(0);
    }
  }

  // ---- epilogue: + bias (fp32), one rounding, 16-byte (V16) or 8-byte stores ----
  f32x4 bv[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    bv[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (BIAS) {
      const T16* bp = reinterpret_cast<const T16*>(p.bias) + n0 + CF::WN * wn + 16 * nt + 4 * g;
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[nt][e] = (float)bp[e];
    }
  }
  T16* cp = reinterpret_cast<T16*>(p.C);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = m0 + CF::WM * wm + 16 * mt + l15;
    if (m < p.M) {
      if constexpr (V16) {
        // two 16x16 tiles (nt = 2i, 2i+1) paired by v_permlane16_swap: lane group g then holds 8
        // consecutive columns, 16 (g & 1) + 8 (g >> 1) into the 32-column strip -- 16-byte stores
#pragma unroll
        for (int i = 0; i < NT / 2; ++i) {
          const f32x4 x = (acc[mt][2 * i] + bv[2 * i]) * p.alpha, y = (acc[mt][2 * i + 1] + bv[2 * i + 1]) * p.alpha;
          uint32_t X0 = fa::pack2<DT>(x[0], x[1]), X1 = fa::pack2<DT>(x[2], x[3]);
          uint32_t Y0 = fa::pack2<DT>(y[0], y[1]), Y1 = fa::pack2<DT>(y[2], y[3]);
          gp::swap16(X0, Y0);
          gp::swap16(X1, Y1);
          *reinterpret_cast<u32x4*>(cp + (int64_t)m * p.ldc + n0 + CF::WN * wn + 32 * i + 16 * (g & 1) + 8 * (g >> 1)) =
              u32x4{X0, X1, Y0, Y1};
        }
      } else {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const f32x4 v = (acc[mt][nt] + bv[nt]) * p.alpha;
          u32x2 w;
          w[0] = fa::pack2<DT>(v[0], v[1]);
          w[1] = fa::pack2<DT>(v[2], v[3]);
          *reinterpret_cast<u32x2*>(cp + (int64_t)m * p.ldc + n0 + CF::WN * wn + 16 * nt + 4 * g) = w;
        }
      }
    }
  }
}

}  // namespace xdot

// Tile choice: the largest tile that still puts >= 2 workgroups on every CU of the 256
// (NN needs BN = 128).  Returns -3 when the shape / layout is not eligible, or (force = 0) when
// the library GEMM is measured faster for the shape; the caller then runs that.
// force: 0 auto (kernel or library), 1 kernel with the automatic tile, 2.. one tile configuration
// (A/B: 2 = 64x64, 3 = 64x128, 4 = 128x128, 5 = 128x128 with a 3-stage ring, 6 = 256x128,
// 7 = 128x128 with the 3-stage A ring beside a 2-stage B ring).
extern "C" int xdot_gemm_proj_launch(const xdot::ProjArgs* a, int dt, int nn, int force, hipStream_t st) {
  using namespace xdot;
  if (dt != DT_BF16 && dt != DT_F16) return -3;
  if (a->M < 1 || a->K < gp::BK || a->K % gp::BK || a->N % 64 || a->lda % 8 || a->ldb % 8 || a->ldc % 4) return -3;
  if ((reinterpret_cast<uintptr_t>(a->A) | reinterpret_cast<uintptr_t>(a->B)) & 15) return -3;
  if (reinterpret_cast<uintptr_t>(a->C) & 7) return -3;
  if (nn && a->N % 128) return -3;
  auto tiles = [&](int bm, int bn) { return (int64_t)((a->M + bm - 1) / bm) * (a->N / bn); };
  int cfg;  // 2..6 as force
  if (force >= 2) {
    cfg = force;
    if (cfg > 7 || (cfg == 2 && nn) || (cfg >= 3 && a->N % 128)) return -3;
  } else {
    if (GP_HUGE && a->N % 128 == 0 && tiles(256, 128) >= 1024) cfg = 6;
    else if (GP_BIG && a->N % 128 == 0 && tiles(128, 128) >= 512) cfg = 4;
    else if (a->N % 128 == 0 && (nn || tiles(64, 128) >= 512)) cfg = 3;
    else cfg = 2;
  }
  const int bm = cfg == 6 ? 256 : (cfg >= 4 ? 128 : 64), bn = cfg == 2 ? 64 : 128;  // (cfg 7: 128x128)
  const int64_t grid = tiles(bm, bn);
  if (grid > 0x7FFFFFFF) return -3;
  const bool bias = a->bias != nullptr;
  // 16-byte output stores (paired tiles) when C's rows are 16-byte aligned
  const bool v16 = a->ldc % 8 == 0 && (reinterpret_cast<uintptr_t>(a->C) & 15) == 0;
#define GPL(DTV, BMV, BNV, NNV, NSV, BV, VV)                                                                      \
  hipLaunchKernelGGL((gemm_proj_kernel<DTV, BMV, BNV, NNV, BV, NSV, VV>), dim3((unsigned)grid),                   \
                     dim3(gp::Cfg<BMV, BNV, NNV, NSV>::NTH), (gp::Cfg<BMV, BNV, NNV, NSV>::LDS), st, *a)
#define GPV(DTV, BMV, BNV, NNV, NSV, BV) \
  if (v16) GPL(DTV, BMV, BNV, NNV, NSV, BV, true); else GPL(DTV, BMV, BNV, NNV, NSV, BV, false)
#define GPB(DTV, BMV, BNV, NNV, NSV) \
  if (bias) { GPV(DTV, BMV, BNV, NNV, NSV, true); } else { GPV(DTV, BMV, BNV, NNV, NSV, false); }
#define GPD(BMV, BNV, NNV, NSV) \
  if (dt == DT_BF16) { GPB(DT_BF16, BMV, BNV, NNV, NSV); } else { GPB(DT_F16, BMV, BNV, NNV, NSV); }
  if (nn) {
    if (cfg == 7) { GPD(128, 128, true, 32); }
    else if (cfg == 6) { GPD(256, 128, true, 2); }
    else if (cfg == 5) { GPD(128, 128, true, 3); }
    else if (cfg == 4) { GPD(128, 128, true, 2); }
    else { GPD(64, 128, true, 2); }
  } else {
    if (cfg == 7) { GPD(128, 128, false, 32); }
    else if (cfg == 6) { GPD(256, 128, false, 2); }
    else if (cfg == 5) { GPD(128, 128, false, 3); }
    else if (cfg == 4) { GPD(128, 128, false, 2); }
    else if (cfg == 3) { GPD(64, 128, false, 2); }
    else { GPD(64, 64, false, 2); }
  }
#undef GPD
#undef GPB
#undef GPV
#undef GPL
  return (int)hipGetLastError();
}
