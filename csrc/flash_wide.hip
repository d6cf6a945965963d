// xdot — flash attention for WIDE head dims (D = 160, 192, 256, 384) on gfx950 (MI355X),
// 16-bit (v_mfma_f32_32x32x16) and exact fp32 (v_mfma_f32_32x32x2_f32).
//
// The reference's own configurations use heads wider than the tuned D <= 128 families
// (flash_fwd.hip / flash_bwd.hip / flash_f32.hip) take: example.py:20 builds 768 features over
// 2 heads (D = 384) and tests/test_gradient.py:45 runs num_heads = 1 at 256 features (D = 256);
// any key_dim / num_heads > 128 does (module.py:28,35).  Without these kernels such shapes fall
// back to materialised (B, H, R, T) scores: 80 GB per head in bf16 at T = 200000.
//
// Same decomposition, layouts, masks and partial / combine protocol as the narrow families
// (rows = this rank's R query-side rows, cols = the T gathered rows, head-interleaved (B, ., H*D)
// tensors, packed masks from mask_pack.hip), re-balanced for a wide head:
//   * one wave per SIMD (launch_bounds(256, 1)): a wave's 32-row fragment of the stationary side
//     (D/4 VGPRs in 16-bit, D/2 in fp32) and its output accumulators (D/2) need up to ~430 of the
//     512 unified VGPR+AGPR registers (the 16-bit forward at D <= 256 fits two: fwd_occ);
//   * 32-row tiles of the streamed side arrive by LDS-DMA (global_load_lds_dwordx4: no staging
//     registers), double-buffered, one barrier per tile; where two fp32 D = 384 images per stage
//     would not fit LDS twice, the image used second is single-buffered and refilled mid-tile;
//   * 16-bit images use the narrow kernels' XOR-swizzled rows (flash_common.h Img<D>, widened so
//     ROW/4 = 16 or 48 mod 64 dwords: both ds_read_b128 row reads and ds_read_b64_tr_b16
//     transposed reads stay conflict-free); fp32 images are rows of D + 4 floats (b128 row reads
//     and b32 transposed reads conflict-free);
//   * the backward splits the gathered side into a dV pass and a dQ pass (the three D-wide
//     register sets a single pass needs do not fit); exact fp32 D = 384 takes S from the score
//     buffer (flash_f32.hip "score-buffer mode") in both passes and dS in the row kernel.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "flash_common.h"

namespace xdot {
namespace faw {

using fa::BwdArgs;
using fa::FwdArgs;
using fa::LN2;
using fa::LOG2E;
using fa::pair_max;
using fa::pair_sum;
using fa::wait_vm;
using fa::raw_barrier;
using fa::pin_agpr;
using fa::tidx;
using fa::flag_at;
using fa::blk_store;
using fa::blk_load;


// Output accumulators are pinned to AGPRs (fa::pin_agpr): a wide head's D/2 accumulator
// registers plus its D/4..D/2 fragment registers exceed the 256 VGPRs; left alone the allocator
// keeps the accumulators in VGPRs (the online-softmax rescale is VALU work on them) and spills.
// the first NA elements of a fragment array to AGPRs too (MFMA reads A/B operands from AGPRs):
// what the accumulators leave of the 256 AGPRs takes the fragments' overflow past the VGPRs
template <int NA, class F, int N>
__device__ __forceinline__ void pin_first(F (&f)[N]) {
#pragma unroll
  for (int i = 0; i < (NA < N ? NA : N); ++i) asm volatile("" : "+a"(f[i]));
}
// fragment elements one kernel may park in AGPRs next to `acc` accumulator registers
template <class Pl, int ACC> constexpr int agpr_frag_room() {  // (32 left for the S / dP tiles)
  return (256 - ACC - 32) / (int)(sizeof(typename Pl::Frag) / 4);
}
// online-softmax rescale of AGPR-pinned accumulators, register by register in inline asm (read
// to one VGPR, multiply, write back): in plain C++ the compiler hoists every AGPR read of the
// rare rescale branch above it and keeps a full VGPR copy of the accumulators live, which spills
template <int N>
__device__ __forceinline__ void scale_pinned(f32x16 (&x)[N], float s) {
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float t;
      asm volatile("v_accvgpr_read_b32 %1, %0\n\tv_mul_f32 %1, %1, %2\n\tv_accvgpr_write_b32 %0, %1"
                   : "+a"(x[i][r]), "=&v"(t)
                   : "v"(s));
    }
}

// ---- operand policies ------------------------------------------------------------------------
// operand reads ahead of the MFMAs in the one-workgroup-per-CU kernels (16-bit)
#ifndef XDOT_WIDE_LA
#define XDOT_WIDE_LA 2
#endif
constexpr int WIDE_LA = XDOT_WIDE_LA;

template <int DT, int D> struct Pol {  // 16-bit
  using T = typename dt_traits<DT>::T;
  using Frag = u32x4;
  static constexpr int ROW = fa::Img<D>::ROW;  // bytes per image row (swizzled)
  static constexpr int VALID = D / 8;          // 16-byte chunks holding data
  static constexpr bool SWZ = true;
  static constexpr int NF = D / 16;            // k-steps over the head dim
  static constexpr float RESCALE = 8.f;        // deferred running-max rescale (log2 units)
  struct Lanes {
    fa::Lanes L;
  };
  static __device__ __forceinline__ Lanes lanes(int lane) { return Lanes{fa::make_lanes<D>(lane)}; }
  static __device__ __forceinline__ void load_frag(Frag (&f)[NF], const T* p, bool ok, int hf) {
#pragma unroll
    for (int s = 0; s < NF; ++s) f[s] = ok ? *reinterpret_cast<const u32x4*>(p + 16 * s + 8 * hf) : u32x4{0, 0, 0, 0};
  }
  // acc += image rows (lane & 31) . fragᵀ over the head dim.  Operand reads run two MFMAs ahead
  // and sched_barrier keeps them there: unfenced, the compiler hoists all D/16 reads (4 VGPRs
  // each) to the top and a wide head spills.
  // LA: operand reads in flight ahead of the MFMA that consumes them (a ring of LA + 1 fragments,
  // compile-time indices): 1 for a kernel whose registers are two workgroups' share, more where
  // one wave per SIMD leaves LDS latency in front of every MFMA
  template <int LA = 2>
  static __device__ __forceinline__ f32x16 rowprod(const char* img, const Frag (&f)[NF], f32x16 acc, const Lanes& L) {
    constexpr int RL = LA + 1;
    u32x4 buf[RL];
#pragma unroll
    for (int s = 0; s < LA && s < NF; ++s) buf[s] = fa::row_frag<D>(img, 0, s, L.L);
#pragma unroll
    for (int s = 0; s < NF; ++s) {
      if (s + LA < NF) buf[(s + LA) % RL] = fa::row_frag<D>(img, 0, s + LA, L.L);
      acc = fa::mfma32<DT>::run(buf[s % RL], f[s], acc);
      __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
  }
  // out[db] += imageᵀ (d x tile row) . x (tile row x lane), x an accumulator tile
  template <int LA = 2>
  static __device__ __forceinline__ void trprod(const char* img, const f32x16& x, f32x16 (&out)[D / 32], const Lanes& L) {
    constexpr int DB = D / 32, N = 2 * DB, RL = LA + 1;
    const u32x4 pf[2] = {fa::acc_to_frag<DT>(x, 0), fa::acc_to_frag<DT>(x, 1)};
    u32x4 buf[RL];
#pragma unroll
    for (int i = 0; i < LA && i < N; ++i) buf[i] = fa::tr_frag<D>(img, 16 * (i / DB), 32 * (i % DB), L.L);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if (i + LA < N) buf[(i + LA) % RL] = fa::tr_frag<D>(img, 16 * ((i + LA) / DB), 32 * ((i + LA) % DB), L.L);
      out[i % DB] = fa::mfma32<DT>::run(buf[i % RL], pf[i / DB], out[i % DB]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // 4 consecutive outputs of one row, o[4g..4g+3] * k, to global memory
  static __device__ __forceinline__ void store4(T* p, float x0, float x1, float x2, float x3) {
    u32x2 w;
    w[0] = fa::pack2<DT>(x0, x1);
    w[1] = fa::pack2<DT>(x2, x3);
    *reinterpret_cast<u32x2*>(p) = w;
  }
};

template <int D> struct Pol<DT_F32, D> {
  using T = float;
  using Frag = float;
  static constexpr int ROW = 4 * (D + 4);  // padded rows, no swizzle
  static constexpr int VALID = D / 4;
  static constexpr bool SWZ = false;
  static constexpr int NF = D / 2;         // f[4g + t] = X[8g + 4h + t]
  static constexpr float RESCALE = 0.f;    // exact: rescale whenever the max grows (as flash_f32.hip)
  struct Lanes {
    int lane;
  };
  static __device__ __forceinline__ Lanes lanes(int lane) { return Lanes{lane}; }
  static __device__ __forceinline__ f32x16 mm(float a, float b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ void load_frag(Frag (&f)[NF], const float* p, bool ok, int hf) {
#pragma unroll
    for (int g = 0; g < D / 8; ++g) {
      const f32x4 v = ok ? *reinterpret_cast<const f32x4*>(p + 8 * g + 4 * hf) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 4; ++t) f[4 * g + t] = v[t];
    }
  }
  // (operand reads one group ahead, fenced as in the 16-bit policy; LA unused)
  template <int LA = 2>
  static __device__ __forceinline__ f32x16 rowprod(const char* img, const Frag (&f)[NF], f32x16 acc, const Lanes& L) {
    const float* p = reinterpret_cast<const float*>(img + (L.lane & 31) * ROW) + 4 * (L.lane >> 5);
    f32x4 a0 = *reinterpret_cast<const f32x4*>(p);
#pragma unroll
    for (int g = 0; g < D / 8; ++g) {
      f32x4 a1 = a0;
      if (g + 1 < D / 8) a1 = *reinterpret_cast<const f32x4*>(p + 8 * (g + 1));
#pragma unroll
      for (int t = 0; t < 4; ++t) acc = mm(a0[t], f[4 * g + t], acc);
      __builtin_amdgcn_sched_barrier(0);
      a0 = a1;
    }
    return acc;
  }
  template <int LA = 2>
  static __device__ __forceinline__ void trprod(const char* img, const f32x16& x, f32x16 (&out)[D / 32], const Lanes& L) {
    constexpr int DB = D / 32;
    const int hf = L.lane >> 5;
    float r0[DB];
    {
      const float* row = reinterpret_cast<const float*>(img + tidx(0, hf) * ROW) + (L.lane & 31);
#pragma unroll
      for (int db = 0; db < DB; ++db) r0[db] = row[db * 32];
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      float r1[DB];
      if (s + 1 < 16) {
        const float* row = reinterpret_cast<const float*>(img + tidx(s + 1, hf) * ROW) + (L.lane & 31);
#pragma unroll
        for (int db = 0; db < DB; ++db) r1[db] = row[db * 32];
      }
#pragma unroll
      for (int db = 0; db < DB; ++db) out[db] = mm(r0[db], x[s], out[db]);
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < 16) {
#pragma unroll
        for (int db = 0; db < DB; ++db) r0[db] = r1[db];
      }
    }
  }
  static __device__ __forceinline__ void store4(float* p, float x0, float x1, float x2, float x3) {
    *reinterpret_cast<f32x4*>(p) = f32x4{x0, x1, x2, x3};
  }
};

// ---- LDS-DMA of one 32-row image -------------------------------------------------------------
// The image occupies NPC 1-KiB pieces (a multiple of 4: every wave issues PPW of them).  Position
// p of the image holds chunk (p % ROW) / 16 of image row p / ROW (swizzled for 16-bit); padding
// chunks and the slack rows past 32 load a valid dummy address.
template <class Pl> struct Dma32 {
  static constexpr int BYTES = 32 * Pl::ROW;
  static constexpr int NPC = (BYTES + 4095) / 4096 * 4;
  static constexpr int PPW = NPC / 4;
  static constexpr int SLOT = NPC * 1024;
  static_assert(Pl::ROW <= 2048, "16 x the 16-byte chunk index must fit 11 bits");
  int wave, lane;
  // per piece of this lane: image row r (5 bits) | 16 x chunk (11 bits) << 5, two pieces per
  // register, computed once: an issue then costs 4 VALU per piece (2 bfe, min, mad) instead of the
  // ~16 of the division / swizzle / clamp arithmetic
  uint32_t pk[(PPW + 1) / 2];
  __device__ __forceinline__ void init(int w, int l, int) {
    wave = w;
    lane = l;
#pragma unroll
    for (int i = 0; i < (PPW + 1) / 2; ++i) pk[i] = 0;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = (wave * PPW + i) * 1024 + lane * 16;
      const int r = min(p / Pl::ROW, 31);
      int c = (p % Pl::ROW) >> 4;
      if (Pl::SWZ) c ^= (r >> 2) & 3;
      if (c >= Pl::VALID || p >= BYTES) c = 0;
      pk[i / 2] |= (uint32_t)(r | ((16 * c) << 5)) << (16 * (i & 1));
    }
  }
  // tile rows past rmax (past T / R) re-read row rmax: callers mask them; padding chunks and the
  // slack rows past 32 load a valid dummy address.
  // SKIP: pieces wholly past the image are not loaded (their LDS stays free for other data; the
  // waves then issue different counts, so only callers that drain with vmcnt(0) may use it)
  template <bool SKIP = false>
  __device__ __forceinline__ void issue(const char* base, int stride_bytes, int rmax, char* img, int) const {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      // (SKIP: the piece index through readfirstlane keeps the LDS address an SGPR operand)
      const int pc = SKIP ? __builtin_amdgcn_readfirstlane(wave * PPW + i) : wave * PPW + i;
      if (SKIP && pc * 1024 >= BYTES) continue;  // wave-uniform
      const uint32_t r = __builtin_amdgcn_ubfe(pk[i / 2], 16 * (i & 1), 5);
      const uint32_t c16 = __builtin_amdgcn_ubfe(pk[i / 2], 16 * (i & 1) + 5, 11);
      fa::glds16(base, (uint32_t)min((int)r, rmax) * (uint32_t)stride_bytes + c16, img + pc * 1024);
    }
  }
};

// two images per stage fit LDS twice (double-buffered) unless fp32 D = 384
template <class Pl> constexpr bool dbl2() { return 4 * Dma32<Pl>::SLOT + 1024 <= 160 * 1024; }

// ------------------------------------------------------------------------------------------
// forward: 4 waves x 32 rows of one (b, h); sweeps 32-column tiles of its column split.
// Stage: [Q image][V image]; SS: store the raw scores into a.sbuf (exact fp32).
// backward softmax: the mask select in a wave-uniform branch taken by partial tiles only, softmax
// logits in place (a per-score test on every tile cost the 16-bit D = 160-256 column side 1.3x,
// profiles/r5_wide_long.md).  K: 0 row side, 1 dV pass, 2 dQ pass.  The instantiations whose
// registers this would spill (two D-wide sets and D = 384 / fp32 D = 256) keep the per-score form.
template <int DT, int D, int K> constexpr bool SELB() {
  return K == 1 || !(D == 384 || (DT == DT_F32 && D == 256));
}
// The 16-bit D = 256 dV pass at two workgroups per CU: 128 accumulator AGPRs + the Q fragment
// in 128 VGPRs (operand reads one ahead), and its four 20-KiB images fill 80 KiB exactly, so the
// lse2 / δ rows move into the dO slots' 2 KiB of slack (aux_in_slack)
template <int DT, int D, bool DQ, bool LS> constexpr int cols_occ() {
  return (DT != DT_F32 && D == 256 && !DQ && !LS) ? 2 : 1;
}
template <int DT, int D, bool DQ, bool LS> constexpr bool aux_in_slack() { return cols_occ<DT, D, DQ, LS>() == 2; }
// 16-bit D <= 256: 128 accumulator AGPRs + the K fragment fit 256 registers, so two workgroups
// share a CU and one wave's softmax VALU runs beside the other's MFMAs (LDS: 2 x 80 KB at D = 256)
template <int DT, int D> constexpr int fwd_occ() {
  return (DT != DT_F32 && D <= 256) ? 2 : 1;
}
template <int DT, int D, bool SS>
__global__ __launch_bounds__(256, (fwd_occ<DT, D>())) void fwd_kernel(FwdArgs a) {
  using Pl = Pol<DT, D>;
  using T = typename Pl::T;
  using DM = Dma32<Pl>;
  constexpr int DB = D / 32, SLOT = DM::SLOT;
  constexpr bool DBL = dbl2<Pl>();
  constexpr int LA = fwd_occ<DT, D>() == 2 ? (D >= 256 ? 1 : 2) : WIDE_LA;  // operand reads ahead
  char* const sm = fa::smem;
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const auto L = Pl::lanes(lane);
  const int nrb = (a.R + 127) / 128;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int rb = lin % nrb, bhs = lin / nrb;
  const int bh = bhs % (a.B * a.H), sp = bhs / (a.B * a.H);
  const int b = bh / a.H, h = bh % a.H;
  const int C = a.H * D;
  const int NKT64 = (a.T + 63) / 64, NKT32 = (a.T + 31) / 32;
  const int kt_beg = 2 * (int)((int64_t)sp * NKT64 / a.nsplit);
  const int kt_end = min(NKT32, 2 * (int)((int64_t)(sp + 1) * NKT64 / a.nsplit));
  const int r0 = rb * 128 + wave * 32, row = r0 + (lane & 31);
  const bool row_ok = row < a.R;
  const int NKT4 = (NKT64 + 3) & ~3, NRB32 = (a.R + 31) / 32;

  typename Pl::Frag kf[Pl::NF];
  Pl::load_frag(kf, reinterpret_cast<const T*>(a.rows) + ((int64_t)b * a.R + (row_ok ? row : 0)) * C + h * D, row_ok, hf);
  // VGPRs past ~200 of fragment: the head of kf goes to the AGPRs o leaves free
  constexpr int KFA = (Pl::NF * (int)sizeof(typename Pl::Frag) / 4 > 96) ? agpr_frag_room<Pl, D / 2>() : 0;
  pin_first<KFA>(kf);
  const int ldb = (int)(a.ldkv * sizeof(T));
  const char* qb = reinterpret_cast<const char*>(reinterpret_cast<const T*>(a.kc) + (int64_t)b * a.T * a.ldkv + h * D);
  const char* vb = reinterpret_cast<const char*>(reinterpret_cast<const T*>(a.vc) + (int64_t)b * a.T * a.ldkv + h * D);
  DM dm;
  dm.init(wave, lane, ldb);
  // LDS: Q images at [0, 2 SLOT), V images after (one of them when !DBL)
  auto qimg = [&](int t) { return sm + ((t - kt_beg) & 1) * SLOT; };
  auto vimg = [&](int t) { return sm + 2 * SLOT + (DBL ? ((t - kt_beg) & 1) * SLOT : 0); };
  const float c2 = a.prescaled ? 1.f : a.scale * LOG2E, NEG_INF = -__builtin_inff();
  float m_run = NEG_INF, l_run = 0.f;
  f32x16 o[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) o[i] = f32x16{};
  pin_agpr(o);
  float* sbw = SS ? a.sbuf + ((int64_t)bh * NRB32 + (r0 >> 5)) * NKT32 * 1024 : nullptr;

  if (kt_beg < kt_end) {
    dm.issue(qb + (int64_t)kt_beg * 32 * ldb, ldb, a.T - 1 - kt_beg * 32, qimg(kt_beg), wave);
    dm.issue(vb + (int64_t)kt_beg * 32 * ldb, ldb, a.T - 1 - kt_beg * 32, vimg(kt_beg), wave);
    wait_vm<0>();
    raw_barrier();
  }
  for (int kt = kt_beg; kt < kt_end; ++kt) {
    const bool more = kt + 1 < kt_end;
    const int64_t nx = (int64_t)(kt + 1) * 32 * ldb;
    if (more) {
      dm.issue(qb + nx, ldb, a.T - 1 - (kt + 1) * 32, qimg(kt + 1), wave);
      if (DBL) dm.issue(vb + nx, ldb, a.T - 1 - (kt + 1) * 32, vimg(kt + 1), wave);
    }
    int flag = r0 >= a.R ? 1 : (a.mflags ? flag_at(a.mflags, b, NRB32, NKT4, r0 >> 5, kt >> 1) : 0);
    flag = __builtin_amdgcn_readfirstlane(flag);
    f32x16 s;
    if (flag != 1) {
      s = Pl::template rowprod<LA>(qimg(kt), kf, f32x16{}, L);  // Sᵀ: col (register) x row (lane)
      pin_first<KFA>(kf);
      if constexpr (SS) blk_store(sbw + (int64_t)kt * 1024, s, lane);
      const int valid = a.T - kt * 32;
      if (flag == 2 || valid < 32) {  // bit tidx(r, hf) of the word (or column >= valid) -> -inf
        uint32_t w = 0;
        if (flag == 2 && row_ok) w = fa::settle((uint32_t)(a.mbits[((int64_t)b * NKT64 + (kt >> 1)) * a.R + row] >> (32 * (kt & 1))));
        fa::sel_bits16(s, (uint32_t)fa::tile_bits(w, valid, hf), fa::NINF_BITS);
      }
      float mx = NEG_INF;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[r]);
      mx = pair_max(mx) * c2;
      const float m_new = fmaxf(m_run, mx);
      if (__any(m_new > m_run + Pl::RESCALE)) {
        const float alpha = __builtin_amdgcn_exp2f(m_run - (m_new == NEG_INF ? 0.f : m_new));  // m_run = -inf: 0
        l_run *= alpha;
        scale_pinned(o, alpha);
        m_run = m_new;
      }
      const float m_use = m_run == NEG_INF ? 0.f : m_run;
      float ls = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[r] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[r], c2, -m_use));
        ls += s[r];
      }
      l_run += ls;
    }
    if (!DBL) {  // V(kt) was DMA'd after the previous tile's PV: complete and visible first
      wait_vm<0>();
      raw_barrier();
    }
    if (flag != 1) Pl::template trprod<LA>(vimg(kt), s, o, L);  // Oᵀ += Vᵀ · Pᵀ
    pin_agpr(o);
    if (!DBL && more) {
      raw_barrier();  // every wave is done with the single V image
      dm.issue(vb + nx, ldb, a.T - 1 - (kt + 1) * 32, vimg(kt + 1), wave);
      wait_vm<DM::PPW>();  // Q(kt+1) landed (V(kt+1) may still fly: waited above next tile)
    } else {
      wait_vm<0>();
    }
    raw_barrier();
  }

  const float l_tot = pair_sum(l_run);
  const float inv = 1.f / l_tot;
  if (!row_ok) return;
  const float lse = (m_run + __log2f(l_tot)) * LN2;
  if (a.nsplit == 1 && !a.force_partial) {
    T* op = reinterpret_cast<T*>(a.out) + ((int64_t)b * a.R + row) * C + h * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        Pl::store4(op + db * 32 + 8 * g + 4 * hf, o[db][4 * g] * inv, o[db][4 * g + 1] * inv, o[db][4 * g + 2] * inv,
                   o[db][4 * g + 3] * inv);
    if (hf == 0) a.lse[((int64_t)b * a.H + h) * a.R + row] = lse;
  } else {
    float* op = a.opart + (((int64_t)(a.sp0 + sp) * a.B + b) * a.R + row) * C + h * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(op + db * 32 + 8 * g + 4 * hf) =
            f32x4{o[db][4 * g] * inv, o[db][4 * g + 1] * inv, o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv};
    if (hf == 0) a.lpart[(((int64_t)(a.sp0 + sp) * a.B + b) * a.H + h) * a.R + row] = lse;
  }
}

// ------------------------------------------------------------------------------------------
// backward, row side: dK = scale · Σ_cols dS · Q_cols.  4 waves x 32 rows, column split.
// LD: dS from the score buffer (one product per tile, Q image only); else S and dP are
// recomputed from register-resident K / dO fragments (stage [Q image][V image]).
// 16-bit D = 160 row side (recomputed S): K / dO fragments + dK accumulators fit two waves'
// share of the registers (operand reads one ahead); its four images fit LDS twice.  D = 160 h = 4
// row side 2.63 -> 2.29 ms (r5s56)
template <int DT, int D, bool LD> constexpr int rows_occ() {
  return (DT != DT_F32 && D <= 160 && !LD) ? 2 : 1;  // D = 192 would spill 84 registers
}
template <int DT, int D, bool LD>
__global__ __launch_bounds__(256, (rows_occ<DT, D, LD>())) void bwd_rows_kernel(BwdArgs a) {
  using Pl = Pol<DT, D>;
  using T = typename Pl::T;
  using DM = Dma32<Pl>;
  constexpr int DB = D / 32, SLOT = DM::SLOT, NIMG = LD ? 1 : 2;
  char* const sm = fa::smem;
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const auto L = Pl::lanes(lane);
  const int nrb = (a.R + 127) / 128;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int rb = lin % nrb, bhs = lin / nrb;
  const int bh = bhs % (a.B * a.H), sp = bhs / (a.B * a.H);
  const int b = bh / a.H, h = bh % a.H;
  const int C = a.H * D;
  const int NKT64 = (a.T + 63) / 64, NKT32 = (a.T + 31) / 32;
  const int kt_beg = 2 * (int)((int64_t)sp * NKT64 / a.nsplit);
  const int kt_end = min(NKT32, 2 * (int)((int64_t)(sp + 1) * NKT64 / a.nsplit));
  const int r0 = rb * 128 + wave * 32, row = r0 + (lane & 31);
  const bool row_ok = row < a.R, wave_ok = r0 < a.R;
  const int NKT4 = (NKT64 + 3) & ~3, NRB32 = (a.R + 31) / 32;

  typename Pl::Frag kf[LD ? 1 : Pl::NF], df[LD ? 1 : Pl::NF];
  if constexpr (!LD) {
    const int64_t off = ((int64_t)b * a.R + (row_ok ? row : 0)) * C + h * D;
    Pl::load_frag(kf, reinterpret_cast<const T*>(a.rows) + off, row_ok, hf);
    Pl::load_frag(df, reinterpret_cast<const T*>(a.dout) + off, row_ok, hf);
  }
  const int64_t li = ((int64_t)b * a.H + h) * a.R + (row_ok ? row : 0);
  const float lse2 = row_ok ? a.lse[li] * LOG2E : 0.f, dlt = row_ok ? a.delta[li] : 0.f;
  const int ldb = (int)(a.ldkv * sizeof(T));
  const char* qb = reinterpret_cast<const char*>(reinterpret_cast<const T*>(a.kc) + (int64_t)b * a.T * a.ldkv + h * D);
  const char* vb = reinterpret_cast<const char*>(reinterpret_cast<const T*>(a.vc) + (int64_t)b * a.T * a.ldkv + h * D);
  DM dm;
  dm.init(wave, lane, ldb);
  auto stage = [&](int t) { return sm + ((t - kt_beg) & 1) * NIMG * SLOT; };
  const float c2 = a.prescaled ? 1.f : a.scale * LOG2E, NEG_INF = -__builtin_inff();
  const float* sbr = LD ? (a.dsbuf ? a.dsbuf : a.sbuf) + ((int64_t)bh * NRB32 + (wave_ok ? r0 >> 5 : 0)) * NKT32 * 1024 : nullptr;
  f32x16 dk[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) dk[i] = f32x16{};
  pin_agpr(dk);

  auto issue = [&](int t) {
    const int64_t o_ = (int64_t)t * 32 * ldb;
    dm.issue(qb + o_, ldb, a.T - 1 - t * 32, stage(t), wave);
    if (!LD) dm.issue(vb + o_, ldb, a.T - 1 - t * 32, stage(t) + SLOT, wave);
  };
  f32x16 dnext{};
  if (kt_beg < kt_end) {
    issue(kt_beg);
    if (LD && wave_ok) dnext = blk_load(sbr + (int64_t)kt_beg * 1024, lane);
    wait_vm<0>();
    raw_barrier();
  }
  for (int kt = kt_beg; kt < kt_end; ++kt) {
    const bool more = kt + 1 < kt_end;
    f32x16 ds = dnext;
    if (more) {
      issue(kt + 1);
      if (LD && wave_ok) dnext = blk_load(sbr + (int64_t)(kt + 1) * 1024, lane);
    }
    const char* qi = stage(kt);
    int flag = !wave_ok ? 1 : (a.mflags ? flag_at(a.mflags, b, NRB32, NKT4, r0 >> 5, kt >> 1) : 0);
    flag = __builtin_amdgcn_readfirstlane(flag);
    if (flag != 1) {
      const int valid = a.T - kt * 32;
      if constexpr (LD) {
        if (valid < 32) {  // the column kernel's values past T are not gradients
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (tidx(r, hf) >= valid) ds[r] = 0.f;
        }
      } else {
        constexpr int RLA = rows_occ<DT, D, LD>() == 2 ? 1 : WIDE_LA;
        f32x16 s = Pl::template rowprod<RLA>(qi, kf, f32x16{}, L);          // Sᵀ  (col x row)
        f32x16 dp = Pl::template rowprod<RLA>(qi + SLOT, df, f32x16{}, L);  // dPᵀ (col x row)
        if constexpr (SELB<DT, D, 0>()) {
#pragma unroll
          for (int r = 0; r < 16; ++r) s[r] = __builtin_fmaf(s[r], c2, -lse2);  // in place
          if (flag == 2 || valid < 32) {  // partial tiles only: masked bits / columns past T -> -inf
            uint32_t w = 0;
            if (flag == 2 && row_ok) w = fa::settle((uint32_t)(a.mbits[((int64_t)b * NKT64 + (kt >> 1)) * a.R + row] >> (32 * (kt & 1))));
            fa::sel_bits16(s, (uint32_t)fa::tile_bits(w, valid, hf), fa::NINF_BITS);
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) ds[r] = __builtin_amdgcn_exp2f(s[r]) * (dp[r] - dlt);  // dSᵀ / scale
        } else {
          uint32_t w = 0;
          const bool chk = flag == 2 || valid < 32;
          if (flag == 2 && row_ok) w = fa::settle((uint32_t)(a.mbits[((int64_t)b * NKT64 + (kt >> 1)) * a.R + row] >> (32 * (kt & 1))));
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float x = __builtin_fmaf(s[r], c2, -lse2);
            if (chk) {
              const int c = tidx(r, hf);
              if (((w >> c) & 1u) || c >= valid) x = NEG_INF;
            }
            ds[r] = __builtin_amdgcn_exp2f(x) * (dp[r] - dlt);  // dSᵀ / scale
          }
        }
      }
      Pl::template trprod<(rows_occ<DT, D, LD>() == 2 ? 1 : WIDE_LA)>(qi, ds, dk, L);  // dKᵀ += Q_colsᵀ · dSᵀ
    }
    pin_agpr(dk);
    wait_vm<0>();
    raw_barrier();
  }
  if (!row_ok) return;
  const float sc = a.scale;
  if (a.nsplit > 1 || a.force_partial) {
    float* op = a.dpart + (((int64_t)(a.sp0 + sp) * a.B + b) * a.R + row) * C + h * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(op + db * 32 + 8 * g + 4 * hf) =
            f32x4{dk[db][4 * g] * sc, dk[db][4 * g + 1] * sc, dk[db][4 * g + 2] * sc, dk[db][4 * g + 3] * sc};
  } else {
    T* op = reinterpret_cast<T*>(a.drows) + ((int64_t)b * a.R + row) * C + h * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        Pl::store4(op + db * 32 + 8 * g + 4 * hf, dk[db][4 * g] * sc, dk[db][4 * g + 1] * sc, dk[db][4 * g + 2] * sc,
                   dk[db][4 * g + 3] * sc);
  }
}

// ------------------------------------------------------------------------------------------
// backward, gathered side, one of two passes (4 waves x 32 columns of one (b, h), sweeping
// 32-row tiles of K_rows / dO and their lse2 / δ):
//   DQ = false: dV_cols = Σ_rows Pᵀ · dO           (needs S, the dO image)
//   DQ = true:  dQ_cols = scale · Σ_rows dSᵀ · K   (needs S, dP = dO · V_colsᵀ, the K image)
// LS: S from the score buffer (DQ: each block then overwritten with dS / scale for the row
// kernel); else S = K · Q_colsᵀ from register-resident Q fragments and the K image.
// Stage: [dO image][K image][lse2 | δ, 256 B]; images a pass does not read are not loaded.
template <int DT, int D, bool DQ, bool LS>
__global__ __launch_bounds__(256, (cols_occ<DT, D, DQ, LS>())) void bwd_cols_kernel(BwdArgs a) {
  using Pl = Pol<DT, D>;
  using T = typename Pl::T;
  using DM = Dma32<Pl>;
  constexpr int DB = D / 32, SLOT = DM::SLOT;
  constexpr bool NEED_K = DQ || !LS, NEED_DO = true;
  // the image used second in the tile (K for dQ) is single-buffered when two per stage do not fit
  constexpr bool DBL = !(NEED_K && NEED_DO) || dbl2<Pl>();
  constexpr int AUX = 1024;  // lse2[32], δ[32] at the start of a 1-KiB slot
  constexpr int CLA = cols_occ<DT, D, DQ, LS>() == 2 ? 1 : WIDE_LA;  // operand reads ahead
  char* const sm = fa::smem;
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const auto L = Pl::lanes(lane);
  const int ncb = (a.T + 127) / 128;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int cb = lin % ncb, bhs = lin / ncb;
  // row split sp of ns (BwdArgs::csq for the dQ pass, csv for the dV pass): row tiles [rt_beg, rt_end)
  const int ns = DQ ? (a.csq > 1 ? a.csq : 1) : (a.csv > 1 ? a.csv : 1);
  const int bh = bhs % (a.B * a.H), sp = bhs / (a.B * a.H);
  const int b = bh / a.H, h = bh % a.H;
  const int C = a.H * D;
  const int c0 = cb * 128 + wave * 32, col = c0 + (lane & 31);
  const bool col_ok = col < a.T;
  const int NKT64 = (a.T + 63) / 64, NKT4 = (NKT64 + 3) & ~3, NRB32 = (a.R + 31) / 32;
  const int NRT64 = (a.R + 63) / 64, TPAD = (a.T + 127) / 128 * 128;
  const int NRT = (a.R + 31) / 32, NKT32 = (a.T + 31) / 32;
  const int rt_beg = (int)((int64_t)sp * NRT / ns), rt_end = (int)((int64_t)(sp + 1) * NRT / ns);

  typename Pl::Frag qf[LS ? 1 : Pl::NF], vf[DQ ? Pl::NF : 1];
  {
    const int64_t off = ((int64_t)b * a.T + (col_ok ? col : 0)) * a.ldkv + h * D;
    if constexpr (!LS) Pl::load_frag(qf, reinterpret_cast<const T*>(a.kc) + off, col_ok, hf);
    if constexpr (DQ) Pl::load_frag(vf, reinterpret_cast<const T*>(a.vc) + off, col_ok, hf);
  }
  // the dQ pass holds two fragments + D/2 accumulators: Q's (else V's) head goes to free AGPRs
  constexpr int FRA = DQ ? agpr_frag_room<Pl, D / 2>() : 0;
  auto pin_frags = [&]() {
    if constexpr (!LS) pin_first<FRA>(qf);
    else pin_first<FRA>(vf);
  };
  pin_frags();
  const int ldb = (int)(C * sizeof(T));  // rows / dO are (B, R, C)
  const char* kb = reinterpret_cast<const char*>(reinterpret_cast<const T*>(a.rows) + (int64_t)b * a.R * C + h * D);
  const char* db_ = reinterpret_cast<const char*>(reinterpret_cast<const T*>(a.dout) + (int64_t)b * a.R * C + h * D);
  const float* lse2 = a.lse2 + ((int64_t)b * a.H + h) * a.R;
  const float* dlt = a.delta + ((int64_t)b * a.H + h) * a.R;
  DM dm;
  dm.init(wave, lane, ldb);
  // LDS: [dO 0][dO 1][aux 0][aux 1][K 0][K 1 (DBL)]
  // AUXS (two workgroups per CU): lse2 / δ in the dO slots' slack past the image, so the
  // four images alone fill the workgroup's 80 KiB
  constexpr bool AUXS = aux_in_slack<DT, D, DQ, LS>();
  static_assert(!AUXS || (DM::BYTES % 1024 == 0 && DM::SLOT - DM::BYTES >= 512), "lse2 / δ need 512 B of whole-piece slack");
  auto doimg = [&](int t) { return sm + (t & 1) * SLOT; };
  auto aux = [&](int t) { return AUXS ? doimg(t) + DM::BYTES : sm + 2 * SLOT + (t & 1) * AUX; };
  auto kimg = [&](int t) { return sm + 2 * SLOT + (AUXS ? 0 : 2 * AUX) + (DBL ? (t & 1) * SLOT : 0); };
  const float c2 = a.prescaled ? 1.f : a.scale * LOG2E, NEG_INF = -__builtin_inff();
  f32x16 acc[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) acc[i] = f32x16{};
  pin_agpr(acc);
  const bool sown = LS && c0 < a.T;
  float* sbc = LS ? a.sbuf + ((int64_t)bh * NRB32 * NKT32 + (c0 >> 5)) * 1024 : nullptr;
  float* dsc = LS ? (a.dsbuf ? a.dsbuf : a.sbuf) + ((int64_t)bh * NRB32 * NKT32 + (c0 >> 5)) * 1024 : nullptr;
  const int64_t sstep = (int64_t)NKT32 * 1024;

  // first-used image(s) + the row constants of tile t (rows past R clamp: masked below): lse2 of
  // the tile's rows at aux floats [0, 32), δ at [64, 96) (two 256-byte DMAs, lanes >= 32 load
  // duplicates into the unused halves)
  auto issue_a = [&](int t) {
    dm.template issue<AUXS>(db_ + (int64_t)t * 32 * ldb, ldb, a.R - 1 - t * 32, doimg(t), wave);
    const uint32_t rr = (uint32_t)min(t * 32 + (lane & 31), a.R - 1) * 4;
    fa::glds4(lse2, rr, aux(t));
    fa::glds4(dlt, rr, aux(t) + 256);
    if (NEED_K && DBL) dm.issue(kb + (int64_t)t * 32 * ldb, ldb, a.R - 1 - t * 32, kimg(t), wave);
  };
  auto issue_k = [&](int t) { dm.issue(kb + (int64_t)t * 32 * ldb, ldb, a.R - 1 - t * 32, kimg(t), wave); };
  f32x16 snext{};
  if (rt_beg < rt_end) {
    issue_a(rt_beg);
    if (NEED_K && !DBL) issue_k(rt_beg);
    if (sown) snext = blk_load(sbc + rt_beg * sstep, lane);
    wait_vm<0>();
    raw_barrier();
  }
  for (int rt = rt_beg; rt < rt_end; ++rt) {
    const bool more = rt + 1 < rt_end;
    f32x16 s = snext;
    if (more) {
      issue_a(rt + 1);
      if (sown) snext = blk_load(sbc + (rt + 1) * sstep, lane);
    }
    const float* ls = reinterpret_cast<const float*>(aux(rt));  // lse2 at [0, 32), δ at [64, 96)
    int flag = c0 >= a.T ? 1 : (a.mflags ? flag_at(a.mflags, b, NRB32, NKT4, rt, c0 >> 6) : 0);
    flag = __builtin_amdgcn_readfirstlane(flag);
    f32x16 dp;
    if (flag != 1) {
      if constexpr (!LS) s = Pl::template rowprod<CLA>(kimg(rt), qf, f32x16{}, L);  // S (row x col)
      if constexpr (DQ) dp = Pl::template rowprod<CLA>(doimg(rt), vf, f32x16{}, L);  // dP (row x col)
      pin_frags();
      if constexpr (SELB<DT, D, DQ ? 2 : 1>()) {
        const int vr = a.R - rt * 32;  // valid rows of this tile
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = __builtin_fmaf(s[r], c2, -ls[tidx(r, hf)]);  // in place
        // partial tiles only (wave-uniform branch): masked bits / rows past R -> -inf
        if (flag == 2 || vr < 32) {
          uint32_t w = 0;
          if (flag == 2 && col_ok) w = fa::settle((uint32_t)(a.mbits[((int64_t)b * NRT64 + (rt >> 1)) * TPAD + col] >> (32 * (rt & 1))));
          fa::sel_bits16(s, (uint32_t)fa::tile_bits(w, vr, hf), fa::NINF_BITS);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(s[r]);
          if constexpr (DQ) dp[r] = p * (dp[r] - ls[64 + tidx(r, hf)]);  // dS / scale
          else s[r] = p;
        }
      } else {
        uint32_t w = 0;
        if (flag == 2 && col_ok) w = fa::settle((uint32_t)(a.mbits[((int64_t)b * NRT64 + (rt >> 1)) * TPAD + col] >> (32 * (rt & 1))));
        const int vr = a.R - rt * 32;  // valid rows of this tile
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int i = tidx(r, hf);
          float x = __builtin_fmaf(s[r], c2, -ls[i]);
          if ((flag == 2 && ((w >> i) & 1u)) || i >= vr) x = NEG_INF;
          const float p = __builtin_amdgcn_exp2f(x);
          if constexpr (DQ) dp[r] = p * (dp[r] - ls[64 + i]);  // dS / scale
          else s[r] = p;
        }
      }
      if constexpr (DQ && LS) blk_store(dsc + rt * sstep, dp, lane);  // dS over S or apart (row-kernel order)
      if constexpr (!DQ) Pl::template trprod<CLA>(doimg(rt), s, acc, L);  // dVᵀ += dOᵀ · P
    }
    if constexpr (DQ) {
      if (!DBL) {  // K(rt) was DMA'd after the previous tile's dQ: complete and visible first
        wait_vm<0>();
        raw_barrier();
      }
      if (flag != 1) Pl::template trprod<CLA>(kimg(rt), dp, acc, L);  // dQᵀ += Kᵀ · dS
      if (!DBL && more) {
        raw_barrier();
        issue_k(rt + 1);
        wait_vm<DM::PPW>();
      } else {
        wait_vm<0>();
      }
    } else {
      wait_vm<0>();
    }
    pin_agpr(acc);
    raw_barrier();
  }
  if (!col_ok) return;
  // dQ = scale · Σ dSᵀ K; a pre-scaled K image holds K · scale · log2 e, so that factor is 1 / log2 e
  const float sc = DQ ? (a.prescaled ? LN2 : a.scale) : 1.f;
  char* base = reinterpret_cast<char*>(DQ ? a.dkc : a.dvc);
  const int64_t eo = ((int64_t)b * a.T + col) * a.ldg + h * D;
  float* const part = ns > 1 ? (DQ ? a.cpq : a.cpv) + (((int64_t)sp * a.B + b) * a.T + col) * C + h * D : nullptr;
#pragma unroll
  for (int d = 0; d < DB; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float x0 = acc[d][4 * g] * sc, x1 = acc[d][4 * g + 1] * sc, x2 = acc[d][4 * g + 2] * sc, x3 = acc[d][4 * g + 3] * sc;
      if (part) *reinterpret_cast<f32x4*>(part + d * 32 + 8 * g + 4 * hf) = f32x4{x0, x1, x2, x3};  // fp32 split partial
      else if (a.dkv16) Pl::store4(reinterpret_cast<T*>(base) + eo + d * 32 + 8 * g + 4 * hf, x0, x1, x2, x3);
      else *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(base) + eo + d * 32 + 8 * g + 4 * hf) = f32x4{x0, x1, x2, x3};
    }
}

template <class Pl> constexpr int fwd_lds() { return (2 + (dbl2<Pl>() ? 2 : 1)) * Dma32<Pl>::SLOT; }
template <class Pl, bool LD> constexpr int rows_lds() { return 2 * (LD ? 1 : 2) * Dma32<Pl>::SLOT; }
template <class Pl, bool DQ, bool LS, bool AUXS = false> constexpr int cols_lds() {
  constexpr bool NEED_K = DQ || !LS;
  constexpr bool DBL = !NEED_K || dbl2<Pl>();
  return 2 * Dma32<Pl>::SLOT + (AUXS ? 0 : 2 * 1024) + (NEED_K ? (DBL ? 2 : 1) * Dma32<Pl>::SLOT : 0);
}

}  // namespace faw
}  // namespace xdot

// ---- launchers ------------------------------------------------------------------------------
// D dispatch of the wide family; -1 = not a wide (dtype, D) this file instantiates
#define XW_DISPATCH(CALL)                                                   \
  switch (dt * 1000 + D) {                                                  \
    case xdot::DT_BF16 * 1000 + 160: CALL(xdot::DT_BF16, 160); return 0;   \
    case xdot::DT_BF16 * 1000 + 192: CALL(xdot::DT_BF16, 192); return 0;   \
    case xdot::DT_BF16 * 1000 + 256: CALL(xdot::DT_BF16, 256); return 0;   \
    case xdot::DT_BF16 * 1000 + 384: CALL(xdot::DT_BF16, 384); return 0;   \
    case xdot::DT_F16 * 1000 + 160: CALL(xdot::DT_F16, 160); return 0;     \
    case xdot::DT_F16 * 1000 + 192: CALL(xdot::DT_F16, 192); return 0;     \
    case xdot::DT_F16 * 1000 + 256: CALL(xdot::DT_F16, 256); return 0;     \
    case xdot::DT_F16 * 1000 + 384: CALL(xdot::DT_F16, 384); return 0;     \
    case xdot::DT_F32 * 1000 + 160: CALL(xdot::DT_F32, 160); return 0;     \
    case xdot::DT_F32 * 1000 + 192: CALL(xdot::DT_F32, 192); return 0;     \
    case xdot::DT_F32 * 1000 + 256: CALL(xdot::DT_F32, 256); return 0;     \
    case xdot::DT_F32 * 1000 + 384: CALL(xdot::DT_F32, 384); return 0;     \
    default: return -1;                                                     \
  }

namespace {
template <int DT, int D>
void wide_fwd(const xdot::fa::FwdArgs* a, hipStream_t st) {
  using namespace xdot::faw;
  using Pl = Pol<DT, D>;
  const dim3 grid(((a->R + 127) / 128) * a->B * a->H * a->nsplit);
  if constexpr (DT == xdot::DT_F32) {
    if (a->sbuf) {
      hipLaunchKernelGGL((fwd_kernel<DT, D, true>), grid, dim3(256), fwd_lds<Pl>(), st, *a);
      return;
    }
  }
  hipLaunchKernelGGL((fwd_kernel<DT, D, false>), grid, dim3(256), fwd_lds<Pl>(), st, *a);
}

// fp32 D > 256 has no recompute variant (three D-wide register sets): it needs the score buffer
template <int DT, int D> constexpr bool recompute_ok() { return DT != xdot::DT_F32 || D <= 256; }

template <int DT, int D>
int wide_rows(const xdot::fa::BwdArgs* a, hipStream_t st) {
  using namespace xdot::faw;
  using Pl = Pol<DT, D>;
  const dim3 grid(((a->R + 127) / 128) * a->B * a->H * a->nsplit);
  if constexpr (DT == xdot::DT_F32) {
    if (a->sbuf) {
      hipLaunchKernelGGL((bwd_rows_kernel<DT, D, true>), grid, dim3(256), (rows_lds<Pl, true>()), st, *a);
      return 0;
    }
  }
  if constexpr (recompute_ok<DT, D>()) {
    hipLaunchKernelGGL((bwd_rows_kernel<DT, D, false>), grid, dim3(256), (rows_lds<Pl, false>()), st, *a);
    return 0;
  }
  return -2;
}

template <int DT, int D>
int wide_cols(const xdot::fa::BwdArgs* a, hipStream_t st) {
  using namespace xdot::faw;
  using Pl = Pol<DT, D>;
  const int W = ((a->T + 127) / 128) * a->B * a->H, sq = a->csq > 1 ? a->csq : 1, sv = a->csv > 1 ? a->csv : 1;
  if ((sq > 1 && !a->cpq) || (sv > 1 && !a->cpv)) return -1;
  const int odt = a->dkv16 ? DT : (int)xdot::DT_F32;
  const int64_t rows = (int64_t)a->B * a->T;
  // split partials of a pass summed into its grad half (output dtype)
  auto fin = [&](bool dq) {
    const int s = dq ? sq : sv;
    if (s > 1) xdot_flash_cols_sum_launch(dq ? a->cpq : a->cpv, dq ? a->dkc : a->dvc, s, rows, a->H * D, a->ldg, odt, st);
  };
  auto dvp = [&](auto LSC) {
    constexpr bool LSV = decltype(LSC)::value;
    hipLaunchKernelGGL((bwd_cols_kernel<DT, D, false, LSV>), dim3(W * sv), dim3(256), (cols_lds<Pl, false, LSV, aux_in_slack<DT, D, false, LSV>()>()), st, *a);
    fin(false);
  };
  auto dqp = [&](auto LSC) {
    constexpr bool LSV = decltype(LSC)::value;
    hipLaunchKernelGGL((bwd_cols_kernel<DT, D, true, LSV>), dim3(W * sq), dim3(256), (cols_lds<Pl, true, LSV>()), st, *a);
    fin(true);
  };
  if constexpr (DT == xdot::DT_F32) {
    if (a->sbuf) {  // in place: dV first (the dQ pass overwrites S with dS); with a dS buffer dQ first
      const int ps = a->sb_passes ? a->sb_passes : 3;
      const bool dv_first = !a->dsbuf;
      if ((ps & 1) && dv_first) dvp(std::true_type{});
      if (ps & 2) dqp(std::true_type{});
      if ((ps & 1) && !dv_first) dvp(std::true_type{});
      return 0;
    }
  }
  if constexpr (recompute_ok<DT, D>()) {
    dvp(std::false_type{});
    dqp(std::false_type{});
    return 0;
  }
  return -2;
}

// occupancy (workgroups per CU) of a wide instantiation: kernel 0 forward, 1 row side, 2 / 3
// the column side's dQ / dV pass
template <int DT, int D>
int wide_occ(int kernel, bool sbuf) {
  using namespace xdot::faw;
  using xdot::fa::wg_per_cu;
  using Pl = Pol<DT, D>;
  const bool sb = DT == xdot::DT_F32 && sbuf;
  if constexpr (DT == xdot::DT_F32) {
    if (sb) {
      if (kernel == 0) return wg_per_cu(fwd_kernel<DT, D, true>, fwd_lds<Pl>());
      if (kernel == 1) return wg_per_cu(bwd_rows_kernel<DT, D, true>, rows_lds<Pl, true>());
      if (kernel == 2) return wg_per_cu(bwd_cols_kernel<DT, D, true, true>, cols_lds<Pl, true, true>());
      return wg_per_cu(bwd_cols_kernel<DT, D, false, true>, cols_lds<Pl, false, true>());
    }
  }
  if constexpr (recompute_ok<DT, D>()) {
    if (kernel == 0) return wg_per_cu(fwd_kernel<DT, D, false>, fwd_lds<Pl>());
    if (kernel == 1) return wg_per_cu(bwd_rows_kernel<DT, D, false>, rows_lds<Pl, false>());
    if (kernel == 2) return wg_per_cu(bwd_cols_kernel<DT, D, true, false>, cols_lds<Pl, true, false>());
    return wg_per_cu(bwd_cols_kernel<DT, D, false, false>, cols_lds<Pl, false, false, aux_in_slack<DT, D, false, false>()>());
  }
  return 0;
}
}  // namespace

extern "C" int xdot_flash_wide_fwd_launch(const xdot::fa::FwdArgs* a, int dt, int D, hipStream_t st) {
  if (a->R == 0 || a->B == 0 || a->H == 0) return 0;
#define L(DTV, DV) wide_fwd<DTV, DV>(a, st)
  XW_DISPATCH(L)
#undef L
}

extern "C" int xdot_flash_wide_rows_launch(const xdot::fa::BwdArgs* a, int dt, int D, hipStream_t st) {
  if (a->R == 0 || a->B == 0 || a->H == 0 || a->T == 0) return 0;
#define L(DTV, DV) return wide_rows<DTV, DV>(a, st)
  XW_DISPATCH(L)
#undef L
}

extern "C" int xdot_flash_wide_cols_launch(const xdot::fa::BwdArgs* a, int dt, int D, hipStream_t st) {
  if (a->R == 0 || a->B == 0 || a->H == 0 || a->T == 0) return 0;
#define L(DTV, DV) return wide_cols<DTV, DV>(a, st)
  XW_DISPATCH(L)
#undef L
}

namespace {
int wide_split_env() {  // XDOT_WIDE_SPLIT: unset / auto = the round model, 0 = the caller's old model, n = forced
  const char* e = std::getenv("XDOT_WIDE_SPLIT");
  if (!e || !*e || !std::strcmp(e, "auto")) return -1;
  return std::max(0, std::atoi(e));
}
}  // namespace

// Split counts of the wide kernels from their own occupancy (one workgroup per CU at these
// widths): kernel 0 / 1 column splits of the forward / row side (0: the caller's model), kernel
// 2 / 3 row splits of the column side's dQ / dV pass.  W = unsplit workgroups, n = tiles (32 wide)
// of the split dimension.
extern "C" int xdot_flash_wide_splits(int kernel, int dt, int D, bool sbuf, int64_t W, int64_t n) {
  const int e = wide_split_env();
  if (e == 0) return kernel >= 2 ? 1 : 0;
  if (e > 0) return (int)std::min<int64_t>(e, n);
  int occ = 0;
#define L(DTV, DV) occ = wide_occ<DTV, DV>(kernel, sbuf); break
  switch (dt * 1000 + D) {
    case xdot::DT_BF16 * 1000 + 160: L(xdot::DT_BF16, 160);
    case xdot::DT_BF16 * 1000 + 192: L(xdot::DT_BF16, 192);
    case xdot::DT_BF16 * 1000 + 256: L(xdot::DT_BF16, 256);
    case xdot::DT_BF16 * 1000 + 384: L(xdot::DT_BF16, 384);
    case xdot::DT_F16 * 1000 + 160: L(xdot::DT_F16, 160);
    case xdot::DT_F16 * 1000 + 192: L(xdot::DT_F16, 192);
    case xdot::DT_F16 * 1000 + 256: L(xdot::DT_F16, 256);
    case xdot::DT_F16 * 1000 + 384: L(xdot::DT_F16, 384);
    case xdot::DT_F32 * 1000 + 160: L(xdot::DT_F32, 160);
    case xdot::DT_F32 * 1000 + 192: L(xdot::DT_F32, 192);
    case xdot::DT_F32 * 1000 + 256: L(xdot::DT_F32, 256);
    case xdot::DT_F32 * 1000 + 384: L(xdot::DT_F32, 384);
    default: break;
  }
#undef L
  if (occ <= 0) return kernel >= 2 ? 1 : 0;
  // forward / row side: partials of a wide 16-bit kernel cost ~1 % per split; the column side's
  // row splits are capped at 4 (fp32 partials of the whole D-wide gradient per split)
  return kernel >= 2 ? xdot::fa::pick_csplit(W, (int)n, occ * xdot_num_cus(), 4, 0.02)
                     : xdot::fa::pick_csplit(W, (int)n, occ * xdot_num_cus(), 8, 0.01);
}

