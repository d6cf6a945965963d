// xdot — fp32 flash attention on the bf16 matrix pipe ("split-bf16", opt-in fp32 mode).
//
// The exact-fp32 family (csrc/flash_f32.hip) runs every product on v_mfma_f32_32x32x2_f32:
// 64 FLOP/clk/SIMD, 1/16 of the bf16 rate, so an fp32 step costs ~10x a bf16 one.  Here every
// fp32 operand x is split into two bf16 values, hi = bf16(x) and lo = bf16(x - hi) (x = hi + lo
// up to ~2^-17 |x|), and a product a·b is three bf16 MFMAs accumulated in fp32:
//     a·b ≈ a_lo·b_hi + a_hi·b_lo + a_hi·b_hi      (a_lo·b_lo ~ 2^-16 |a·b| dropped)
// = 3 x 32x32x16 bf16 MFMAs per 16-deep K step instead of 8 x 32x32x2 f32 ones: 5.3x fewer
// matrix-pipe cycles.  Softmax, LSE, δ and every accumulation stay fp32; measured against fp64
// the relative error is 6e-6..9e-6 (exact fp32: 3e-7..6e-7), profiles/r3_fp32_split.md.  The
// default fp32 family (``XDOT_FP32_MODE=split``, per call ``fp32_mode=1``); ``exact`` keeps
// flash_f32.hip.
//
// Same decomposition, layouts, masks and partial/combine protocol as flash_f32.hip (same
// reference semantics, distributed_dot_product/module.py:60-71): 4 waves x 32 rows (columns
// for the gathered-side kernel), 32-row tiles staged global -> VGPR (one tile ahead) -> LDS.
// The staging step splits each fp32 tile ONCE per workgroup into the bf16 images the MFMAs
// read:
//   * row-major  [row][d] hi / lo, stride D + 8 (16-byte pad: the 16-lane ds_read_b128 groups
//     hit 16 distinct bank quads) — A operand of products over the head dim;
//   * transposed [d][slot] hi / lo, stride 40 — A operand of products over the tile index,
//     slots permuted so that lane half h of K step j reads tile rows tidx(8j + t, h), t = 0..7,
//     i.e. the accumulator registers 8j..8j+7 of the previous product (B operand straight from
//     the accumulator, split in registers).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "flash_common.h"

namespace xdot {
namespace fa3 {

using fa::BwdArgs;
using fa::FwdArgs;
using fa::LN2;
using fa::LOG2E;
using fa::pair_max;
using fa::pair_sum;
using fa::tidx;
using fa::flag_at;
using fa::blk_store_lds;
using fa::blk_load;

typedef __attribute__((ext_vector_type(2))) __bf16 bf2;

__device__ __forceinline__ f32x16 mm(const u32x4& a, const u32x4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
// a·b of one 16-deep K step from split operands (small terms first)
__device__ __forceinline__ f32x16 mm3(const u32x4& ah, const u32x4& al, const u32x4& bh, const u32x4& bl, f32x16 c) {
  c = mm(al, bh, c);
  c = mm(ah, bl, c);
  return mm(ah, bh, c);
}
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

// two floats -> packed hi pair and packed lo pair
__device__ __forceinline__ void split2(float x, float y, uint32_t& hi, uint32_t& lo) {
  const bf2 h = {(__bf16)x, (__bf16)y};
  const uint32_t hb = __builtin_bit_cast(uint32_t, h);
  const float xh = __builtin_bit_cast(float, hb << 16), yh = __builtin_bit_cast(float, hb & 0xffff0000u);
  const bf2 l = {(__bf16)(x - xh), (__bf16)(y - yh)};
  hi = hb;
  lo = __builtin_bit_cast(uint32_t, l);
}
__device__ __forceinline__ void split8(const float* x, u32x4& hi, u32x4& lo) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    uint32_t h, l;
    split2(x[2 * t], x[2 * t + 1], h, l);
    hi[t] = h;
    lo[t] = l;
  }
}

template <int D> struct Cfg {
  static constexpr int ROW = fa::Img<D>::ROW;  // image row stride (bytes): the bf16 kernels' layout
  static constexpr int KS = D / 16;            // 16-deep K steps over the head dim
  static constexpr int DB = D / 32;            // 32-wide output blocks
  static constexpr int NC = D / 32;            // f32x4 per thread per 32-row fp32 tile (256 threads)
};

// One staged 32-row tile: a hi and a lo bf16 image, row-major in the bf16 kernels' swizzled
// layout (fa::Img / fa::img_off: rows of ROW bytes, 16-byte chunks XOR (row >> 2) & 3).  Products
// over the head dim read it with ds_read_b128 (fa::row_frag), products over the tile index with
// the hardware transpose ds_read_b64_tr_b16 (fa::tr_frag), whose key order (k0 + 8 (j >> 2) + 4h
// + (j & 3)) is the accumulator-register order the B operands come in: one image serves both
// (the flags say which reads a kernel makes; the layout is the same).
template <int D, bool RMF, bool TRF> struct Img {
  static constexpr int H = 0, L = 32 * Cfg<D>::ROW;
  static constexpr int BYTES = (RMF || TRF) ? 64 * Cfg<D>::ROW : 0;
};

// one 32-row fp32 tile global -> registers (rows row0.., clamped to row0 + rmax) -> split images
template <int D> struct Tile {
  using CF = Cfg<D>;
  f32x4 r[CF::NC];
  __device__ __forceinline__ void load(const float* base, int64_t ld, int64_t row0, int rmax, int tid) {
#pragma unroll
    for (int i = 0; i < CF::NC; ++i) {
      const int q = tid + 256 * i, row = q / (D / 4), c = q % (D / 4);
      r[i] = *reinterpret_cast<const f32x4*>(base + (row0 + min(row, rmax)) * ld + 4 * c);
    }
  }
  template <bool RMF, bool TRF>
  __device__ __forceinline__ void store(char* img, int tid) const {
    using IL = Img<D, RMF, TRF>;
#pragma unroll
    for (int i = 0; i < CF::NC; ++i) {
      const int q = tid + 256 * i, row = q / (D / 4), c = q % (D / 4);
      uint32_t h0, l0, h1, l1;
      split2(r[i][0], r[i][1], h0, l0);
      split2(r[i][2], r[i][3], h1, l1);
      const int o = fa::img_off<D>(row, c >> 1) + 8 * (c & 1);  // 4 bf16 = half a 16-byte chunk
      *reinterpret_cast<u32x2*>(img + IL::H + o) = u32x2{h0, h1};
      *reinterpret_cast<u32x2*>(img + IL::L + o) = u32x2{l0, l1};
    }
  }
};

// register-resident split fragments of one 32-row block (B operand of row products):
// fh/fl[m] = X[row][16m + 8h .. +7]; p points at X[row][8h]
template <int D>
__device__ __forceinline__ void load_frag(u32x4 (&fh)[D / 16], u32x4 (&fl)[D / 16], const float* p, bool ok) {
#pragma unroll
  for (int m = 0; m < D / 16; ++m) {
    float x[8];
    const f32x4 a = ok ? *reinterpret_cast<const f32x4*>(p + 16 * m) : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 b = ok ? *reinterpret_cast<const f32x4*>(p + 16 * m + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      x[t] = a[t];
      x[4 + t] = b[t];
    }
    split8(x, fh[m], fl[m]);
  }
}

// acc[c][j] += Σ_d img[c][d] · frag[j][d]  (c = tile row: register, j = frag row: lane)
template <int D, bool RMF, bool TRF>
__device__ __forceinline__ f32x16 rowprod(const char* img, const u32x4 (&fh)[D / 16], const u32x4 (&fl)[D / 16],
                                          f32x16 acc, int lane) {
  using IL = Img<D, RMF, TRF>;
  const fa::Lanes Ln = fa::make_lanes<D>(lane);
#pragma unroll
  for (int m = 0; m < D / 16; ++m) {
    const u32x4 ah = fa::row_frag<D>(img + IL::H, 0, m, Ln);
    const u32x4 al = fa::row_frag<D>(img + IL::L, 0, m, Ln);
    acc = mm3(ah, al, fh[m], fl[m], acc);
  }
  return acc;
}

// out[db][d][j] += Σ_c img[c][d] · x[c][j]  (x: an accumulator tile, c its register rows)
template <int D, bool RMF, bool TRF>
__device__ __forceinline__ void trprod(const char* img, const f32x16& x, f32x16 (&out)[D / 32], int lane) {
  using CF = Cfg<D>;
  using IL = Img<D, RMF, TRF>;
  u32x4 bh[2], bl[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = x[8 * j + t];
    split8(v, bh[j], bl[j]);
  }
  const fa::Lanes Ln = fa::make_lanes<D>(lane);
#pragma unroll
  for (int db = 0; db < D / 32; ++db)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const u32x4 ah = fa::tr_frag<D>(img + IL::H, 16 * j, 32 * db, Ln);
      const u32x4 al = fa::tr_frag<D>(img + IL::L, 16 * j, 32 * db, Ln);
      out[db] = mm3(ah, al, bh[j], bl[j], out[db]);
    }
}


// ------------------------------------------------------------------------------------------
// forward: 4 waves x 32 rows of one (b, h); sweeps 32-column tiles of its column split
template <int D> struct FwdL {
  using Q = Img<D, true, false>;
  using V = Img<D, false, true>;
  static constexpr int STAGE = Q::BYTES + V::BYTES;
  static constexpr int LDS = 2 * STAGE;
  static constexpr int LDS_SB = LDS + 4 * 4096;  // + a 4-KiB transpose tile per wave (blk_store_lds)
};

// SS: store the raw scores into a.sbuf (score-buffer mode, same block format as flash_f32.hip)
template <int D, bool SS>
__global__ __launch_bounds__(256, 2) void fwd_kernel(FwdArgs a) {
  using CF = Cfg<D>;
  using FL = FwdL<D>;
  constexpr int DB = CF::DB;
  using fa::smem;
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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

  u32x4 kh[CF::KS], kl[CF::KS];
  load_frag<D>(kh, kl, reinterpret_cast<const float*>(a.rows) + ((int64_t)b * a.R + (row_ok ? row : 0)) * C + h * D + 8 * hf,
               row_ok);
  const float* qb = reinterpret_cast<const float*>(a.kc) + (int64_t)b * a.T * a.ldkv + h * D;
  const float* vb = reinterpret_cast<const float*>(a.vc) + (int64_t)b * a.T * a.ldkv + h * D;
  const float c2 = a.scale * LOG2E, NEG_INF = -__builtin_inff();
  float m_run = NEG_INF, l_run = 0.f;
  f32x16 o[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) o[i] = f32x16{};
  // score buffer: this wave's row of 32x32 blocks (r0 < R: waves past R never store)
  // (waves past R write the dump block: uniform store counts keep the compiler's vmcnt waits exact)
  float* sbw = SS ? a.sbuf + (r0 < a.R ? ((int64_t)bh * NRB32 + (r0 >> 5)) * NKT32 * 1024 : fa::sb_dump(a.B, a.H, a.R, a.T))
                  : nullptr;
  const int sbw_step = r0 < a.R ? 1024 : 0;

  Tile<D> tq, tv;
  if (kt_beg < kt_end) {
    tq.load(qb, a.ldkv, (int64_t)kt_beg * 32, a.T - 1 - kt_beg * 32, tid);
    tv.load(vb, a.ldkv, (int64_t)kt_beg * 32, a.T - 1 - kt_beg * 32, tid);
    tq.template store<true, false>(smem, tid);
    tv.template store<false, true>(smem + FL::Q::BYTES, tid);
    __syncthreads();
  }
  for (int kt = kt_beg; kt < kt_end; ++kt) {
    const bool more = kt + 1 < kt_end;
    if (more) {
      tq.load(qb, a.ldkv, (int64_t)(kt + 1) * 32, a.T - 1 - (kt + 1) * 32, tid);
      tv.load(vb, a.ldkv, (int64_t)(kt + 1) * 32, a.T - 1 - (kt + 1) * 32, tid);
    }
    const char* qi = smem + ((kt - kt_beg) & 1) * FL::STAGE;
    const char* vi = qi + FL::Q::BYTES;
    int flag = r0 >= a.R ? 1 : (a.mflags ? flag_at(a.mflags, b, NRB32, NKT4, r0 >> 5, kt >> 1) : 0);
    flag = __builtin_amdgcn_readfirstlane(flag);
    f32x16 s{};
    if (flag != 1) s = rowprod<D, true, false>(qi, kh, kl, f32x16{}, lane);  // Sᵀ: col (register) x row (lane)
    // raw S, every tile (skipped tiles store zeros nobody reads): LDS writes here, the transposed
    // global stores after the PV product
    float* swl = reinterpret_cast<float*>(smem + FL::LDS) + wave * 1024;
    if constexpr (SS) fa::blk_put_lds(swl, s, lane);
    if (flag != 1) {
      const int valid = a.T - kt * 32;
      if (flag == 2 || valid < 32) {
        uint32_t w = 0;
        if (flag == 2 && row_ok) w = fa::settle((uint32_t)(a.mbits[((int64_t)b * NKT64 + (kt >> 1)) * a.R + row] >> (32 * (kt & 1))));
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int c = tidx(r, hf);
          if (((w >> c) & 1u) || c >= valid) s[r] = NEG_INF;
        }
      }
      float mx = NEG_INF;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[r]);
      mx = pair_max(mx) * c2;
      const float m_new = fmaxf(m_run, mx);
      if (m_new > m_run) {
        const float alpha = ex2(m_run - m_new);  // m_run = -inf: 0
        l_run *= alpha;
#pragma unroll
        for (int i = 0; i < DB; ++i) o[i] *= alpha;
        m_run = m_new;
      }
      const float m_use = m_run == NEG_INF ? 0.f : m_run;
      float ls = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[r] = ex2(__builtin_fmaf(s[r], c2, -m_use));
        ls += s[r];
      }
      l_run += ls;
      trprod<D, false, true>(vi, s, o, lane);  // Oᵀ += Vᵀ · Pᵀ
    }
    if constexpr (SS) fa::blk_flush_lds(sbw + kt * sbw_step, swl, lane);
    if (more) {
      char* nx = smem + ((kt + 1 - kt_beg) & 1) * FL::STAGE;
      tq.template store<true, false>(nx, tid);
      tv.template store<false, true>(nx + FL::Q::BYTES, tid);
    }
    __syncthreads();
  }

  const float l_tot = pair_sum(l_run);
  const float inv = 1.f / l_tot;
  if (!row_ok) return;
  const float lse = (m_run + __log2f(l_tot)) * LN2;
  float* op;
  if (a.nsplit == 1 && !a.force_partial) {
    op = reinterpret_cast<float*>(a.out) + ((int64_t)b * a.R + row) * C + h * D;
    if (hf == 0) a.lse[((int64_t)b * a.H + h) * a.R + row] = lse;
  } else {
    op = a.opart + (((int64_t)(a.sp0 + sp) * a.B + b) * a.R + row) * C + h * D;
    if (hf == 0) a.lpart[(((int64_t)(a.sp0 + sp) * a.B + b) * a.H + h) * a.R + row] = lse;
  }
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<f32x4*>(op + db * 32 + 8 * g + 4 * hf) =
          f32x4{o[db][4 * g] * inv, o[db][4 * g + 1] * inv, o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv};
}

// ------------------------------------------------------------------------------------------
// backward, row side: dK = scale · Σ_cols dS · Q_cols.  4 waves x 32 rows, column split.
// Two LDS stages (the next tile is stored while the current one is read: one barrier per tile).
template <int D> struct RowsL {
  using Q = Img<D, true, true>;
  using V = Img<D, true, false>;
  static constexpr int STAGE = Q::BYTES + V::BYTES;
  static constexpr int LDS = 2 * STAGE;
};

template <int D>
__global__ __launch_bounds__(256, D <= 64 ? 2 : 1) void bwd_rows_kernel(BwdArgs a) {
  using CF = Cfg<D>;
  using RL = RowsL<D>;
  constexpr int DB = CF::DB;
  using fa::smem;
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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

  u32x4 kh[CF::KS], kl[CF::KS], dh[CF::KS], dl[CF::KS];
  {
    const int64_t off = ((int64_t)b * a.R + (row_ok ? row : 0)) * C + h * D + 8 * hf;
    load_frag<D>(kh, kl, reinterpret_cast<const float*>(a.rows) + off, row_ok);
    load_frag<D>(dh, dl, reinterpret_cast<const float*>(a.dout) + off, row_ok);
  }
  const int64_t li = ((int64_t)b * a.H + h) * a.R + (row_ok ? row : 0);
  const float lse2 = row_ok ? a.lse[li] * LOG2E : 0.f, dlt = row_ok ? a.delta[li] : 0.f;
  const float* qb = reinterpret_cast<const float*>(a.kc) + (int64_t)b * a.T * a.ldkv + h * D;
  const float* vb = reinterpret_cast<const float*>(a.vc) + (int64_t)b * a.T * a.ldkv + h * D;
  const float c2 = a.scale * LOG2E, NEG_INF = -__builtin_inff();
  f32x16 dk[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) dk[i] = f32x16{};
  fa::pin_agpr(dk);  // loop-carried: AGPR-resident, no per-product copies

  Tile<D> tq, tv;
  if (kt_beg < kt_end) {
    tq.load(qb, a.ldkv, (int64_t)kt_beg * 32, a.T - 1 - kt_beg * 32, tid);
    tv.load(vb, a.ldkv, (int64_t)kt_beg * 32, a.T - 1 - kt_beg * 32, tid);
    tq.template store<true, true>(smem, tid);
    tv.template store<true, false>(smem + RL::Q::BYTES, tid);
    __syncthreads();
  }
  for (int kt = kt_beg; kt < kt_end; ++kt) {
    const bool more = kt + 1 < kt_end;
    if (more) {
      tq.load(qb, a.ldkv, (int64_t)(kt + 1) * 32, a.T - 1 - (kt + 1) * 32, tid);
      tv.load(vb, a.ldkv, (int64_t)(kt + 1) * 32, a.T - 1 - (kt + 1) * 32, tid);
    }
    const char* qi = smem + ((kt - kt_beg) & 1) * RL::STAGE;
    const char* vi = qi + RL::Q::BYTES;
    int flag = r0 >= a.R ? 1 : (a.mflags ? flag_at(a.mflags, b, NRB32, NKT4, r0 >> 5, kt >> 1) : 0);
    flag = __builtin_amdgcn_readfirstlane(flag);
    if (flag != 1) {
      f32x16 s = rowprod<D, true, true>(qi, kh, kl, f32x16{}, lane);    // Sᵀ  (col x row)
      f32x16 dp = rowprod<D, true, false>(vi, dh, dl, f32x16{}, lane);  // dPᵀ (col x row)
      const int valid = a.T - kt * 32;
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
        s[r] = ex2(x) * (dp[r] - dlt);  // dSᵀ / scale
      }
      trprod<D, true, true>(qi, s, dk, lane);  // dKᵀ += Q_colsᵀ · dSᵀ
      fa::pin_agpr(dk);
    }
    if (more) {
      char* nx = smem + ((kt + 1 - kt_beg) & 1) * RL::STAGE;
      tq.template store<true, true>(nx, tid);
      tv.template store<true, false>(nx + RL::Q::BYTES, tid);
    }
    __syncthreads();
  }
  if (!row_ok) return;
  float* op = (a.nsplit > 1 || a.force_partial) ? a.dpart + (((int64_t)(a.sp0 + sp) * a.B + b) * a.R + row) * C + h * D
                                                : reinterpret_cast<float*>(a.drows) + ((int64_t)b * a.R + row) * C + h * D;
  const float sc = a.scale;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<f32x4*>(op + db * 32 + 8 * g + 4 * hf) =
          f32x4{dk[db][4 * g] * sc, dk[db][4 * g + 1] * sc, dk[db][4 * g + 2] * sc, dk[db][4 * g + 3] * sc};
}

// ------------------------------------------------------------------------------------------
// backward, gathered side: dQ_cols = scale · Σ_rows dSᵀ · K_rows, dV_cols = Σ_rows Pᵀ · dO.
// 4 waves x 32 columns of one (b, h); sweeps 32-row tiles of K_rows / dO + their lse2 / δ.
// LS (score-buffer mode): S comes from a.sbuf (prefetched one tile ahead) instead of the K·Qᵀ
// product, each block is overwritten with dS / scale for bwd_rows_ds_kernel, and dV is left to
// bwd_cols_dv_kernel (run first).  K then needs only its transposed image, dO its row-major one.
// DS (dS-only buffer mode, recompute kernel): S recomputed as without a buffer, dS stored into
// a.dsbuf for bwd_rows_ds_kernel (40 GB of score traffic per step instead of the 100 GB of the
// S + dS mode, which bounds this family's kernels)
template <int D, bool LS, bool DS = LS> struct ColsL {
  using K = Img<D, !LS, true>;
  using DO = Img<D, true, !LS>;
  static constexpr int AUX = 256;  // lse2[32], δ[32] (fp32)
  static constexpr int STAGE = K::BYTES + DO::BYTES + AUX;
  static constexpr int LDS = 2 * STAGE + (DS ? 4 * 4096 : 0);
};

template <int D, bool LS, bool DS = LS>
__global__ __launch_bounds__(256, LS && D <= 96 ? 2 : 1) void bwd_cols_kernel(BwdArgs a) {
  using CF = Cfg<D>;
  using KL = ColsL<D, LS, DS>;
  constexpr int DB = CF::DB;
  using fa::smem;
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ncb = (a.T + 127) / 128;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int cb = lin % ncb, bhs = lin / ncb;
  const int bh = bhs % (a.B * a.H), sp = bhs / (a.B * a.H), ns = a.csq > 1 ? a.csq : 1;
  const int b = bh / a.H, h = bh % a.H;
  const int C = a.H * D;
  const int c0 = cb * 128 + wave * 32, col = c0 + (lane & 31);
  const bool col_ok = col < a.T;
  const int NKT64 = (a.T + 63) / 64, NKT4 = (NKT64 + 3) & ~3, NRB32 = (a.R + 31) / 32;
  const int NRT64 = (a.R + 63) / 64, TPAD = (a.T + 127) / 128 * 128;
  const int NRT = (a.R + 31) / 32;
  // row split sp of ns (BwdArgs::csq): row tiles [rt_beg, rt_end)
  const int rt_beg = (int)((int64_t)sp * NRT / ns), rt_end = (int)((int64_t)(sp + 1) * NRT / ns);

  constexpr int QS = LS ? 1 : CF::KS;
  u32x4 qh[QS], ql[QS], vh[CF::KS], vl[CF::KS];
  {
    const int64_t off = ((int64_t)b * a.T + (col_ok ? col : 0)) * a.ldkv + h * D + 8 * hf;
    if constexpr (!LS) load_frag<D>(qh, ql, reinterpret_cast<const float*>(a.kc) + off, col_ok);
    load_frag<D>(vh, vl, reinterpret_cast<const float*>(a.vc) + off, col_ok);
  }
  const int NKT32 = (a.T + 31) / 32;
  const bool sown = DS && c0 < a.T;
  // every wave loads and stores every tile (waves past T: a valid block / the dump block)
  float* sbc = LS ? a.sbuf + ((int64_t)bh * NRB32 * NKT32 + min(c0 >> 5, NKT32 - 1)) * 1024 : nullptr;
  float* dsc = DS ? (a.dsbuf ? a.dsbuf : a.sbuf) +
                        (sown ? ((int64_t)bh * NRB32 * NKT32 + (c0 >> 5)) * 1024 : fa::sb_dump(a.B, a.H, a.R, a.T))
                  : nullptr;
  const int64_t dstep = sown ? (int64_t)NKT32 * 1024 : 0;
  const int64_t sstep = (int64_t)NKT32 * 1024;
  f32x16 snext{};
  if (LS && rt_beg < rt_end) snext = blk_load(sbc + rt_beg * sstep, lane);
  const float* kb = reinterpret_cast<const float*>(a.rows) + (int64_t)b * a.R * C + h * D;
  const float* db_ = reinterpret_cast<const float*>(a.dout) + (int64_t)b * a.R * C + h * D;
  const float* lse2 = a.lse2 + ((int64_t)b * a.H + h) * a.R;
  const float* dlt = a.delta + ((int64_t)b * a.H + h) * a.R;
  const float c2 = a.scale * LOG2E, NEG_INF = -__builtin_inff();
  f32x16 dq[DB], dv[LS ? 1 : DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) dq[i] = f32x16{};
  if constexpr (!LS) {
#pragma unroll
    for (int i = 0; i < DB; ++i) dv[i] = f32x16{};
    fa::pin_agpr(dq);  // loop-carried: AGPR-resident, no per-product copies
    fa::pin_agpr(dv);
  }

  // row constants of a tile: lse2 (+inf past R: P = 0) and δ, by threads 0..63
  auto aux_load = [&](int rt) -> float {
    const int rr = rt * 32 + (tid & 31);
    if (tid < 32) return rr < a.R ? lse2[rr] : __builtin_inff();
    if (tid < 64) return rr < a.R ? dlt[rr] : 0.f;
    return 0.f;
  };
  auto put = [&](char* st, const Tile<D>& tk, const Tile<D>& td, float ax) {
    tk.template store<!LS, true>(st, tid);
    td.template store<true, !LS>(st + KL::K::BYTES, tid);
    if (tid < 64) reinterpret_cast<float*>(st + KL::K::BYTES + KL::DO::BYTES)[tid] = ax;
  };
  Tile<D> tk, td;
  float ax = 0.f;
  if (rt_beg < rt_end) {
    tk.load(kb, C, (int64_t)rt_beg * 32, a.R - 1 - rt_beg * 32, tid);
    td.load(db_, C, (int64_t)rt_beg * 32, a.R - 1 - rt_beg * 32, tid);
    ax = aux_load(rt_beg);
    put(smem, tk, td, ax);
    __syncthreads();
  }
  for (int rt = rt_beg; rt < rt_end; ++rt) {
    const bool more = rt + 1 < rt_end;
    f32x16 scur;
    if constexpr (LS) scur = snext;
    if (more) {
      tk.load(kb, C, (int64_t)(rt + 1) * 32, a.R - 1 - (rt + 1) * 32, tid);
      td.load(db_, C, (int64_t)(rt + 1) * 32, a.R - 1 - (rt + 1) * 32, tid);
      ax = aux_load(rt + 1);
      if constexpr (LS)
        snext = blk_load(sbc + (rt + 1) * sstep, lane);
    }
    const char* ki = smem + ((rt - rt_beg) & 1) * KL::STAGE;
    const char* di = ki + KL::K::BYTES;
    const float* ls = reinterpret_cast<const float*>(di + KL::DO::BYTES);  // lse2[32], δ[32]
    int flag = c0 >= a.T ? 1 : (a.mflags ? flag_at(a.mflags, b, NRB32, NKT4, rt, c0 >> 6) : 0);
    flag = __builtin_amdgcn_readfirstlane(flag);
    f32x16 s, dp;  // (skipped tiles store whatever dp holds: nobody reads those blocks)
    if (flag != 1) {
      if constexpr (LS) s = scur;                                     // S  (row x col), stored by the forward
      else s = rowprod<D, !LS, true>(ki, qh, ql, f32x16{}, lane);     // S  (row x col)
      dp = rowprod<D, true, !LS>(di, vh, vl, f32x16{}, lane);         // dP (row x col)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = tidx(r, hf);
        const float p = ex2(__builtin_fmaf(s[r], c2, -ls[i]));
        s[r] = p;
        dp[r] = p * (dp[r] - ls[32 + i]);  // dS / scale
      }
      if (flag == 2) {  // masked entries: P = dS = 0 (the unmasked loop stays select-free)
        const uint32_t w = col_ok ? fa::settle((uint32_t)(a.mbits[((int64_t)b * NRT64 + (rt >> 1)) * TPAD + col] >> (32 * (rt & 1)))) : 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if ((w >> tidx(r, hf)) & 1u) s[r] = dp[r] = 0.f;
      }
    }
    // dS, every tile: uniform store counts keep the compiler's vmcnt waits exact (LDS writes
    // before the products, the transposed global stores after them)
    float* dwl = reinterpret_cast<float*>(smem + 2 * KL::STAGE) + wave * 1024;
    if constexpr (DS) fa::blk_put_lds(dwl, dp, lane);
    if (flag != 1) {
      if constexpr (LS) {
        trprod<D, false, true>(ki, dp, dq, lane);  // dQᵀ += Kᵀ · dS
      } else {
        trprod<D, true, true>(di, s, dv, lane);   // dVᵀ += dOᵀ · P
        trprod<D, true, true>(ki, dp, dq, lane);  // dQᵀ += Kᵀ · dS
        fa::pin_agpr(dq);
        fa::pin_agpr(dv);
      }
    }
    if constexpr (DS) fa::blk_flush_lds(dsc + rt * dstep, dwl, lane);
    if (more) put(smem + ((rt + 1 - rt_beg) & 1) * KL::STAGE, tk, td, ax);
    __syncthreads();
  }
  if (!col_ok) return;
  const int64_t prow = ((int64_t)sp * a.B + b) * a.T + col;  // row of the split partials
  float* pq = ns > 1 ? a.cpq + prow * C + h * D : reinterpret_cast<float*>(a.dkc) + ((int64_t)b * a.T + col) * a.ldg + h * D;
  float* pv = ns > 1 ? a.cpv + prow * C + h * D : reinterpret_cast<float*>(a.dvc) + ((int64_t)b * a.T + col) * a.ldg + h * D;
  const float sc = a.scale;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      *reinterpret_cast<f32x4*>(pq + db * 32 + 8 * g + 4 * hf) =
          f32x4{dq[db][4 * g] * sc, dq[db][4 * g + 1] * sc, dq[db][4 * g + 2] * sc, dq[db][4 * g + 3] * sc};
      if constexpr (!LS)
        *reinterpret_cast<f32x4*>(pv + db * 32 + 8 * g + 4 * hf) =
            f32x4{dv[db][4 * g], dv[db][4 * g + 1], dv[db][4 * g + 2], dv[db][4 * g + 3]};
    }
}

// ------------------------------------------------------------------------------------------
// Score-buffer mode, gathered side pass 1 of 2: dV_cols = Σ_rows Pᵀ · dO with P recomputed
// elementwise from the stored S (one product per tile, dO's transposed image only).  Runs BEFORE
// bwd_cols_kernel<D, true>, which overwrites S with dS.  Stage = dO image + lse2[32].
template <int D> struct DvL {
  using DO = Img<D, false, true>;
  static constexpr int STAGE = DO::BYTES + 128;
  static constexpr int LDS = 2 * STAGE;
};

template <int D>
__global__ __launch_bounds__(256, 2) void bwd_cols_dv_kernel(BwdArgs a) {
  using CF = Cfg<D>;
  using VL = DvL<D>;
  constexpr int DB = CF::DB;
  using fa::smem;
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ncb = (a.T + 127) / 128;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int cb = lin % ncb, bhs = lin / ncb;
  const int bh = bhs % (a.B * a.H), sp = bhs / (a.B * a.H), ns = a.csv > 1 ? a.csv : 1;
  const int b = bh / a.H, h = bh % a.H;
  const int C = a.H * D;
  const int c0 = cb * 128 + wave * 32, col = c0 + (lane & 31);
  const bool col_ok = col < a.T, sown = c0 < a.T;
  const int NKT64 = (a.T + 63) / 64, NKT4 = (NKT64 + 3) & ~3, NRB32 = (a.R + 31) / 32;
  const int NRT64 = (a.R + 63) / 64, TPAD = (a.T + 127) / 128 * 128;
  const int NRT = (a.R + 31) / 32, NKT32 = (a.T + 31) / 32;
  const int rt_beg = (int)((int64_t)sp * NRT / ns), rt_end = (int)((int64_t)(sp + 1) * NRT / ns);
  const float* sbc = a.sbuf + ((int64_t)bh * NRB32 * NKT32 + min(c0 >> 5, NKT32 - 1)) * 1024;  // valid for every wave
  const int64_t sstep = (int64_t)NKT32 * 1024;
  const float* db_ = reinterpret_cast<const float*>(a.dout) + (int64_t)b * a.R * C + h * D;
  const float* lse2 = a.lse2 + ((int64_t)b * a.H + h) * a.R;
  const float c2 = a.scale * LOG2E, NEG_INF = -__builtin_inff();
  f32x16 dv[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) dv[i] = f32x16{};
  auto aux_load = [&](int rt) -> float {  // lse2 (+inf past R: P = 0), threads 0..31
    const int rr = rt * 32 + tid;
    return tid < 32 && rr < a.R ? lse2[rr] : __builtin_inff();
  };
  constexpr int PF = fa::SB_PF;
  Tile<D> td;
  f32x16 q[PF];
  float ax = 0.f;
  if (rt_beg < rt_end) {
    td.load(db_, C, (int64_t)rt_beg * 32, a.R - 1 - rt_beg * 32, tid);
    ax = aux_load(rt_beg);
#pragma unroll
    for (int j = 0; j < PF; ++j)
      if (rt_beg + j < rt_end) q[j] = blk_load(sbc + (rt_beg + j) * sstep, lane);
    td.template store<false, true>(smem, tid);
    if (tid < 32) reinterpret_cast<float*>(smem + VL::DO::BYTES)[tid] = ax;
    __syncthreads();
  }
  fa::ring_loop<PF>(rt_beg, rt_end, [&](int rt, auto J) {
    constexpr int j = decltype(J)::value;
    const bool more = rt + 1 < rt_end;
    f32x16 s = q[j];
    if (more) {
      td.load(db_, C, (int64_t)(rt + 1) * 32, a.R - 1 - (rt + 1) * 32, tid);
      ax = aux_load(rt + 1);
    }
    if (rt + PF < rt_end) q[j] = blk_load(sbc + (rt + PF) * sstep, lane);  // every wave: uniform vmcnt
    const char* di = smem + ((rt - rt_beg) & 1) * VL::STAGE;
    const float* ls = reinterpret_cast<const float*>(di + VL::DO::BYTES);
    int flag = !sown ? 1 : (a.mflags ? flag_at(a.mflags, b, NRB32, NKT4, rt, c0 >> 6) : 0);
    flag = __builtin_amdgcn_readfirstlane(flag);
    if (flag != 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = ex2(__builtin_fmaf(s[r], c2, -ls[tidx(r, hf)]));
      if (flag == 2) {  // masked entries: P = 0
        const uint32_t w = col_ok ? fa::settle((uint32_t)(a.mbits[((int64_t)b * NRT64 + (rt >> 1)) * TPAD + col] >> (32 * (rt & 1)))) : 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if ((w >> tidx(r, hf)) & 1u) s[r] = 0.f;
      }
      trprod<D, false, true>(di, s, dv, lane);  // dVᵀ += dOᵀ · P
    }
    if (more) {
      char* nx = smem + ((rt + 1 - rt_beg) & 1) * VL::STAGE;
      td.template store<false, true>(nx, tid);
      if (tid < 32) reinterpret_cast<float*>(nx + VL::DO::BYTES)[tid] = ax;
    }
    __syncthreads();
  });
  if (!col_ok) return;
  float* pv = ns > 1 ? a.cpv + (((int64_t)sp * a.B + b) * a.T + col) * C + h * D
                     : reinterpret_cast<float*>(a.dvc) + ((int64_t)b * a.T + col) * a.ldg + h * D;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<f32x4*>(pv + db * 32 + 8 * g + 4 * hf) =
          f32x4{dv[db][4 * g], dv[db][4 * g + 1], dv[db][4 * g + 2], dv[db][4 * g + 3]};
}

// ------------------------------------------------------------------------------------------
// Score-buffer mode, row side: dK = scale · Σ_cols dS · Q_cols with dS from the buffer the
// column kernel wrote (one product per tile; Q's transposed image only).  Same grid, column split
// and partial protocol as bwd_rows_kernel.
template <int D> struct RowsDsL {
  using Q = Img<D, false, true>;
  static constexpr int LDS = 2 * Q::BYTES;
};

template <int D>
__global__ __launch_bounds__(256, 2) void bwd_rows_ds_kernel(BwdArgs a) {
  using CF = Cfg<D>;
  using RL = RowsDsL<D>;
  constexpr int DB = CF::DB;
  using fa::smem;
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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
  const float* qb = reinterpret_cast<const float*>(a.kc) + (int64_t)b * a.T * a.ldkv + h * D;
  const float* sbr = (a.dsbuf ? a.dsbuf : a.sbuf) + ((int64_t)bh * NRB32 + (wave_ok ? r0 >> 5 : 0)) * NKT32 * 1024;
  f32x16 dk[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) dk[i] = f32x16{};

  constexpr int PF = fa::SB_PF;
  Tile<D> tq;
  f32x16 q[PF];
  if (kt_beg < kt_end) {
    tq.load(qb, a.ldkv, (int64_t)kt_beg * 32, a.T - 1 - kt_beg * 32, tid);
#pragma unroll
    for (int j = 0; j < PF; ++j)
      if (kt_beg + j < kt_end) q[j] = blk_load(sbr + (int64_t)(kt_beg + j) * 1024, lane);
    tq.template store<false, true>(smem, tid);
    __syncthreads();
  }
  fa::ring_loop<PF>(kt_beg, kt_end, [&](int kt, auto J) {
    constexpr int j = decltype(J)::value;
    const bool more = kt + 1 < kt_end;
    f32x16 ds = q[j];
    if (more) tq.load(qb, a.ldkv, (int64_t)(kt + 1) * 32, a.T - 1 - (kt + 1) * 32, tid);
    if (kt + PF < kt_end) q[j] = blk_load(sbr + (int64_t)(kt + PF) * 1024, lane);  // every wave: uniform vmcnt
    const char* qi = smem + ((kt - kt_beg) & 1) * RL::Q::BYTES;
    int flag = !wave_ok ? 1 : (a.mflags ? flag_at(a.mflags, b, NRB32, NKT4, r0 >> 5, kt >> 1) : 0);
    flag = __builtin_amdgcn_readfirstlane(flag);
    if (flag != 1) {
      const int valid = a.T - kt * 32;
      if (valid < 32) {  // columns past T: the column kernel's values there are not gradients
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (tidx(r, hf) >= valid) ds[r] = 0.f;
      }
      trprod<D, false, true>(qi, ds, dk, lane);  // dKᵀ += Q_colsᵀ · dSᵀ
    }
    if (more) tq.template store<false, true>(smem + ((kt + 1 - kt_beg) & 1) * RL::Q::BYTES, tid);
    __syncthreads();
  });
  if (!row_ok) return;
  float* op = (a.nsplit > 1 || a.force_partial) ? a.dpart + (((int64_t)(a.sp0 + sp) * a.B + b) * a.R + row) * C + h * D
                                                : reinterpret_cast<float*>(a.drows) + ((int64_t)b * a.R + row) * C + h * D;
  const float sc = a.scale;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<f32x4*>(op + db * 32 + 8 * g + 4 * hf) =
          f32x4{dk[db][4 * g] * sc, dk[db][4 * g + 1] * sc, dk[db][4 * g + 2] * sc, dk[db][4 * g + 3] * sc};
}

}  // namespace fa3
}  // namespace xdot

#define X3_DISPATCH(CALL)              \
  switch (D) {                         \
    case 32: CALL(32); return 0;       \
    case 64: CALL(64); return 0;       \
    case 96: CALL(96); return 0;       \
    case 128: CALL(128); return 0;     \
    default: return -1;                \
  }

extern "C" int xdot_flash_fwd_x3_launch(const xdot::fa::FwdArgs* a, int D, hipStream_t st) {
  using namespace xdot::fa3;
  if (a->R == 0 || a->B == 0 || a->H == 0 || a->prescaled) return a->prescaled ? -1 : 0;
  const dim3 grid(((a->R + 127) / 128) * a->B * a->H * a->nsplit);
  if (a->sbuf) {
#define L(DV) hipLaunchKernelGGL((fwd_kernel<DV, true>), grid, dim3(256), FwdL<DV>::LDS_SB, st, *a)
    X3_DISPATCH(L)
#undef L
  }
#define L(DV) hipLaunchKernelGGL((fwd_kernel<DV, false>), grid, dim3(256), FwdL<DV>::LDS, st, *a)
  X3_DISPATCH(L)
#undef L
}

extern "C" int xdot_flash_bwd_rows_x3_launch(const xdot::fa::BwdArgs* a, int D, hipStream_t st) {
  using namespace xdot::fa3;
  if (a->R == 0 || a->B == 0 || a->H == 0 || a->T == 0) return 0;
  if (a->prescaled) return -1;
  const dim3 grid(((a->R + 127) / 128) * a->B * a->H * a->nsplit);
  if (a->sbuf || a->dsbuf) {  // score-buffer modes: dS from the column kernel, Q image only
#define L(DV) hipLaunchKernelGGL(bwd_rows_ds_kernel<DV>, grid, dim3(256), RowsDsL<DV>::LDS, st, *a)
    X3_DISPATCH(L)
#undef L
  }
#define L(DV) hipLaunchKernelGGL(bwd_rows_kernel<DV>, grid, dim3(256), RowsL<DV>::LDS, st, *a)
  X3_DISPATCH(L)
#undef L
}

namespace {
// dS-only column launch: the recompute kernel's two-image stages plus the transpose tiles exceed
// the 160 KiB of LDS at D = 128 (refused: -1)
template <int D> int launch_cols_ds(const xdot::fa::BwdArgs& a, dim3 grid, hipStream_t st) {
  using namespace xdot::fa3;
  if constexpr (ColsL<D, false, true>::LDS > 160 * 1024) {
    (void)a; (void)grid; (void)st;
    return -1;
  } else {
    hipLaunchKernelGGL((bwd_cols_kernel<D, false, true>), grid, dim3(256), (ColsL<D, false, true>::LDS), st, a);
    return 0;
  }
}
}  // namespace

extern "C" int xdot_flash_bwd_cols_x3_launch(const xdot::fa::BwdArgs* a, int D, hipStream_t st) {
  using namespace xdot::fa3;
  if (a->R == 0 || a->B == 0 || a->H == 0 || a->T == 0) return 0;
  if (a->prescaled || a->dkv16) return -1;
  const int W = ((a->T + 127) / 128) * a->B * a->H, sq = a->csq > 1 ? a->csq : 1, sv = a->csv > 1 ? a->csv : 1;
  if ((sq > 1 && (!a->cpq || (!a->sbuf && !a->cpv))) || (sv > 1 && !a->cpv) || (D & 3)) return -1;
  const int64_t rows = (int64_t)a->B * a->T;
  const int C = a->H * D;
  auto sum_q = [&] {  // split partials of a pass summed into its grad half (BwdArgs::csq / csv)
    if (sq > 1) xdot_flash_cols_sum_launch(a->cpq, a->dkc, sq, rows, C, a->ldg, xdot::DT_F32, st);
  };
  auto sum_v = [&](int s) {
    if (s > 1) xdot_flash_cols_sum_launch(a->cpv, a->dvc, s, rows, C, a->ldg, xdot::DT_F32, st);
  };
  if (a->sbuf) {  // in place: dV from S first, then dQ (S -> dS); with a dS buffer dQ first
    const int ps = a->sb_passes ? a->sb_passes : 3;
    const bool dv_first = !a->dsbuf;
#define LDV(DV) hipLaunchKernelGGL(bwd_cols_dv_kernel<DV>, dim3(W * sv), dim3(256), DvL<DV>::LDS, st, *a)
#define LDQ(DV) hipLaunchKernelGGL((bwd_cols_kernel<DV, true>), dim3(W * sq), dim3(256), (ColsL<DV, true>::LDS), st, *a)
#define L(DV)                            \
  if ((ps & 1) && dv_first) {            \
    LDV(DV);                             \
    sum_v(sv);                           \
  }                                      \
  if (ps & 2) {                          \
    LDQ(DV);                             \
    sum_q();                             \
  }                                      \
  if ((ps & 1) && !dv_first) {           \
    LDV(DV);                             \
    sum_v(sv);                           \
  }
    X3_DISPATCH(L)
#undef L
#undef LDQ
#undef LDV
  }
  if (a->dsbuf) {  // dS-only buffer: recompute S, store dS for the row kernel (D <= 96: LDS)
    int rc = -1;
    switch (D) {
      case 32: rc = launch_cols_ds<32>(*a, dim3(W * sq), st); break;
      case 64: rc = launch_cols_ds<64>(*a, dim3(W * sq), st); break;
      case 96: rc = launch_cols_ds<96>(*a, dim3(W * sq), st); break;
      case 128: rc = launch_cols_ds<128>(*a, dim3(W * sq), st); break;
      default: break;
    }
    if (rc) return rc;
    sum_q();
    sum_v(sq);
    return 0;
  }
#define L(DV)                                                                                                          \
  hipLaunchKernelGGL((bwd_cols_kernel<DV, false>), dim3(W * sq), dim3(256), (ColsL<DV, false>::LDS), st, *a); \
  sum_q();                                                                                                             \
  sum_v(sq)
  X3_DISPATCH(L)
#undef L
}

namespace {
int x3_csplit_env() {  // XDOT_CSPLIT, as in flash_f32.hip
  const char* e = std::getenv("XDOT_CSPLIT");  // read per call (tests switch it)
  return (!e || !*e || !std::strcmp(e, "auto")) ? -1 : std::max(1, std::min(4, std::atoi(e)));
}
template <int D> void x3_splits(const xdot::fa::BwdArgs* a, int* sq, int* sv) {
  using namespace xdot::fa3;
  const int64_t W = (int64_t)((a->T + 127) / 128) * a->B * a->H;
  const int NRT = (a->R + 31) / 32, cus = xdot_num_cus();
  if (a->sbuf) {
    *sq = xdot::fa::pick_csplit(W, NRT, cus * xdot::fa::wg_per_cu(bwd_cols_kernel<D, true>, ColsL<D, true>::LDS));
    *sv = xdot::fa::pick_csplit(W, NRT, cus * xdot::fa::wg_per_cu(bwd_cols_dv_kernel<D>, DvL<D>::LDS));
  } else if (a->dsbuf) {
    *sq = *sv =
        xdot::fa::pick_csplit(W, NRT, cus * xdot::fa::wg_per_cu(bwd_cols_kernel<D, false, true>, ColsL<D, false, true>::LDS));
  } else {
    *sq = *sv = xdot::fa::pick_csplit(W, NRT, cus * xdot::fa::wg_per_cu(bwd_cols_kernel<D, false>, ColsL<D, false>::LDS));
  }
}
}  // namespace

extern "C" int xdot_flash_cols_splits_x3(const xdot::fa::BwdArgs* a, int D, int* sq, int* sv) {
  *sq = *sv = 1;
  const int e = x3_csplit_env();
  if (e >= 0) {
    *sq = *sv = (a->R + 31) / 32 / e >= 1 ? e : 1;
    return 0;
  }
  switch (D) {
    case 32: x3_splits<32>(a, sq, sv); break;
    case 64: x3_splits<64>(a, sq, sv); break;
    case 96: x3_splits<96>(a, sq, sv); break;
    case 128: x3_splits<128>(a, sq, sv); break;
    default: return -1;
  }
  return 0;
}

// column splits of the split-bf16 forward (kernel 0) / row-side backward (1), see kernels.h
extern "C" int xdot_flash_f32_row_splits_x3(int kernel, int D, bool sbuf, int64_t W, int64_t T) {
  using namespace xdot::fa3;
  int occ = 0;
#define OC(DV)                                                                                                   \
  if (D == DV)                                                                                                   \
    occ = kernel == 0 ? (sbuf ? xdot::fa::wg_per_cu(fwd_kernel<DV, true>, FwdL<DV>::LDS_SB)                    \
                              : xdot::fa::wg_per_cu(fwd_kernel<DV, false>, FwdL<DV>::LDS))                     \
                      : (sbuf ? xdot::fa::wg_per_cu(bwd_rows_ds_kernel<DV>, RowsDsL<DV>::LDS)                  \
                              : xdot::fa::wg_per_cu(bwd_rows_kernel<DV>, RowsL<DV>::LDS));
  OC(32) OC(64) OC(96) OC(128)
#undef OC
  if (!occ) return 0;
  return xdot::fa::pick_csplit(W, (int)((T + 31) / 32), occ * xdot_num_cus(), 8, 0.004);
}
