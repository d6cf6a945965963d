// xdot — sequence-parallel flash-attention BACKWARD for gfx950 (MI355X).
//
// Reference backward of the module (distributed_dot_product/multiplication/ops.py:29-37 and
// :49-54, driven by module.py:60-71): 2x distributed_matmul_nt + 2x distributed_matmul_tn +
// 1x distributed_matmul_all + ATen softmax/masked_fill/div backward, each a full pass over a
// materialised (B, H, R, T) tensor and each re-gathering K/V over the network.
//
// Here the probabilities are recomputed per tile from the forward's LSE and three kernels
// run back to back, no score-sized tensor ever exists:
//   flash_bwd_prep  δ[row] = Σ_d dO·O                                   (memory-bound, tiny)
//   flash_bwd_rows  per 128 local rows: sweep all T gathered columns,
//                   Sᵀ, dPᵀ by MFMA, dSᵀ = Pᵀ ⊙ (dPᵀ − δ), dK += dS · Q_cols
//                   -> grad of the row side (this rank's `keys`), no atomics
//   flash_bwd_cols  per 128 gathered columns: sweep all R local rows,
//                   S, dP by MFMA, P, dS, dV_cols += Pᵀ · dO, dQ_cols += dSᵀ · K_rows
//                   -> fp32 partials for ALL T columns in the gathered (rank-major)
//                   layout, which the host reduce-scatters over RCCL (the `tn` pattern).
// Splitting the row-side and column-side sums into two kernels costs two extra MFMA
// products (S and dP are recomputed once more) but removes every cross-workgroup float
// atomic: with 256-column blocks those would move ≈7.5 GB of atomic traffic per step at
// T=25000 — ≈5.8 ms at MI355X's ≈1.3 TB/s atomic rate, more than the MFMA work they save.
// Accumulator-as-operand orientation (see flash_fwd.hip): each product is arranged so the
// following MFMA sums over the accumulator's ROW index, so P and dS feed the next MFMA as
// packed registers; the one operand that must be transposed is read with ds_read_b64_tr_b16.
#include "flash_common.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include <type_traits>

namespace xdot {
namespace fa {

// ---------------------------------------------------------------------------------------
// δ = rowsum(dO ⊙ O) per (b, h, row); one thread per (b, row, h)
// (and lse2 = lse * log2 e when a.lse2 is set; delta == nullptr: lse2 only)
template <int DT, int D>
__global__ __launch_bounds__(256) void flash_bwd_prep_kernel(BwdArgs a, const void* out_, float* delta) {
  using T16 = typename dt_traits<DT>::T;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)a.B * a.R * a.H;
  if (idx >= total) return;
  const int h = (int)(idx % a.H);
  const int64_t br = idx / a.H;
  const int row = (int)(br % a.R), b = (int)(br / a.R);
  const int64_t li = ((int64_t)b * a.H + h) * a.R + row;
  if (a.lse2) a.lse2[li] = a.lse[li] * LOG2E;
  if (!delta) return;
  const int64_t off = br * (a.H * D) + h * D;
  const T16* o = reinterpret_cast<const T16*>(out_) + off;
  const T16* d = reinterpret_cast<const T16*>(a.dout) + off;
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < D / 8; ++c) {
    union { u32x4 u; T16 e[8]; } x, y;
    x.u = *reinterpret_cast<const u32x4*>(o + 8 * c);
    y.u = *reinterpret_cast<const u32x4*>(d + 8 * c);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += (float)x.e[e] * (float)y.e[e];
  }
  delta[li] = acc;
}

// ---------------------------------------------------------------------------------------
// grad of the row side.  4 waves x 32 rows; 64-column tiles of Q_cols / V_cols arrive by
// LDS-DMA into the same ring as the forward's (RowsCfg).
//
// Software-pipelined tile body.  Per 64-column tile the wave runs
//   A0: Sᵀ/dPᵀ chains of sub-tile 0 (12 MFMAs, operand reads two ahead)
//   A1 ∥ V0: the chains of sub-tile 1, each MFMA followed by its share of sub-tile 0's
//            softmax gradient (v_exp, multiply)
//   K0 ∥ V1: dk += Q·dSᵀ of sub-tile 0, each MFMA followed by a share of sub-tile 1's VALU
//   K1:      dk of sub-tile 1
// so nearly all the VALU work issues between this wave's own MFMAs (a plain S/dP -> VALU -> dk
// body leaves the matrix pipe to the partner wave during the VALU block: 1.5 % slower).
// Masks never reach the VALU: a masked (or past-T) column seeds its Sᵀ accumulator with -inf
// (pre-scaled: P = 2^acc = 0; otherwise P = 2^(acc·c2 - lse2) = 0), so masked and unmasked
// tiles run the same body and only the seeds differ.
template <int DT, int D, bool PS = false>
__global__ __launch_bounds__(256, 2) void flash_bwd_rows_kernel(BwdArgs a) {
  using T16 = typename dt_traits<DT>::T;
  using CF = RowsCfg<D>;
  constexpr int IMG = CF::IMG, NG = CF::NG, PF = CF::PF, NBUF = CF::NBUF;
  constexpr int KS = D / 16, DB = D / 32;

  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: keeps wave-derived flags in SGPRs
  const Lanes L = make_lanes<D>(lane);
  const int nrb = (a.R + 127) / 128;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int rb = lin % nrb, bhs = lin / nrb;
  const int bh = bhs % (a.B * a.H), sp = bhs / (a.B * a.H);
  const int b = bh / a.H, h = bh % a.H;
  const int C = a.H * D;
  const int NKT = (a.T + 63) / 64;
  const int kt_beg = (int)((int64_t)sp * NKT / a.nsplit), kt_end = (int)((int64_t)(sp + 1) * NKT / a.nsplit);
  const int r0 = rb * 128 + wave * 32;
  const int row = r0 + (lane & 31);
  const bool row_ok = row < a.R;

  u32x4 kf[KS], df[KS];
  {
    const int64_t off = ((int64_t)b * a.R + row) * C + h * D + 8 * hf;
    const T16* pk = reinterpret_cast<const T16*>(a.rows) + off;
    const T16* pd = reinterpret_cast<const T16*>(a.dout) + off;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      kf[s] = row_ok ? *reinterpret_cast<const u32x4*>(pk + 16 * s) : u32x4{0, 0, 0, 0};
      df[s] = row_ok ? *reinterpret_cast<const u32x4*>(pd + 16 * s) : u32x4{0, 0, 0, 0};
    }
  }
  const int64_t lrow = ((int64_t)b * a.H + h) * a.R + (row_ok ? row : 0);
  float lse2 = row_ok ? a.lse[lrow] * LOG2E : 0.f;
  float dlt = row_ok ? a.delta[lrow] : 0.f;
  // retire these loads here, before the first DMA (else: vmcnt(0) inside the loop)
#pragma unroll
  for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(kf[s]), "+v"(df[s]));
  asm volatile("" : "+v"(lse2), "+v"(dlt));
  const float c2 = a.scale * LOG2E;
  const float NEG_INF = -__builtin_inff();
  // -dO fragments + a δ-filled seed (loop-invariant): the dPᵀ accumulator ends at δ - dP, so
  // dSᵀ' = Pᵀ ⊙ acc = -dSᵀ with no per-element subtract; the dk epilogue scales by -scale
#pragma unroll
  for (int s = 0; s < KS; ++s) df[s] ^= u32x4{0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
  f32x16 dseed;
#pragma unroll
  for (int r = 0; r < 16; ++r) dseed[r] = dlt;
  // PS: K rows pre-multiplied by scale*log2 e on the host (the forward's buffer) and the Sᵀ
  // accumulator seeded with -lse2, so P = 2^acc: no per-element FMA
  f32x16 sseed;
#pragma unroll
  for (int r = 0; r < 16; ++r) sseed[r] = PS ? -lse2 : 0.f;

  const int ldb = a.ldkv * 2;
  ImgDma<D> dma;
  dma.init(wave, lane, ldb);
  const char* kcb = reinterpret_cast<const char*>(reinterpret_cast<const T16*>(a.kc) + h * D + (int64_t)b * a.T * a.ldkv);
  const char* vcb = reinterpret_cast<const char*>(reinterpret_cast<const T16*>(a.vc) + h * D + (int64_t)b * a.T * a.ldkv);
  const uint64_t* mwg = a.mbits ? a.mbits + (int64_t)b * NKT * a.R + rb * 128 : nullptr;  // + kt * R per tile
  const uint32_t moff = (uint32_t)(min((wave & 1) * 64 + lane, a.R - 1 - rb * 128) * 8 + (wave >> 1) * 4);
  const int NKT4 = (NKT + 3) & ~3;
  const int NRB32 = (a.R + 31) / 32;
  const uint8_t* fwg = a.mflags ? a.mflags + ((int64_t)b * NRB32 + rb * 4) * NKT4 : nullptr;
  const int fn = min(4, NRB32 - rb * 4);
  auto issue = [&](int kt) {
    char* st = smem + ((kt - kt_beg) % NBUF) * CF::STAGE;
    const int64_t t0 = (int64_t)kt * 64;
    const int rmax = a.T - 1 - (int)t0;
    dma.issue(kcb + t0 * ldb, ldb, rmax, st, wave);
    dma.issue(vcb + t0 * ldb, ldb, rmax, st + IMG, wave);
    if (mwg) {
      glds4(mwg + (int64_t)kt * a.R, moff, st + CF::OFF_W + (wave >> 1) * 512 + (wave & 1) * 256);
      glds_flags(fwg, NKT4, fn, kt >> 2, st + CF::OFF_F);
    } else {  // keeps NG DMAs per wave per tile
      glds4(kcb, (uint32_t)lane * 4, st + CF::OFF_X);
      glds4(kcb, (uint32_t)lane * 4, st + CF::OFF_X);
    }
  };

  f32x16 dk[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) dk[i][r] = 0.f;
  // seed of sub-tile tt with the masked columns (bits of w, MFMA C/D order) at -inf
  auto masked_seed = [&](uint64_t w, int tt) {
    f32x16 sd = sseed;
    sel_bits16(sd, (uint32_t)(w >> (32 * tt)), NINF_BITS);
    return sd;
  };
  auto pipe_body = [&](const char* qs, const char* vs, const f32x16& sd0, bool masked, uint64_t w) __attribute__((always_inline)) {
    constexpr int NA = 2 * KS, NK = 2 * DB;
    auto elem = [&](f32x16& sc, const f32x16& dc, int r) {
      const float x = PS ? sc[r] : __builtin_fmaf(sc[r], c2, -lse2);
      float y = fast_exp2(x) * dc[r];  // -dSᵀ (unscaled)
      asm volatile("" : "+v"(y));      // keeps it in this MFMA gap (LLVM would sink it to its use)
      sc[r] = y;
    };
    // operand i of a sub-tile's interleaved S (even i) / dP (odd i) chains
    auto opnd = [&](int tt, int i) { return (i & 1) ? row_frag<D>(vs, tt * 32, i >> 1, L) : row_frag<D>(qs, tt * 32, i >> 1, L); };
    f32x16 s0, d0, s1, d1;
    // sub-tile 1's seed, built under A0's MFMAs
    const f32x16 sd1 = masked ? masked_seed(w, 1) : sseed;
    {
      // A0: operand reads two MFMAs ahead (s1/d1 are not live yet)
      u32x4 ow[NA];
      ow[0] = opnd(0, 0);
      ow[1] = opnd(0, 1);
      __builtin_amdgcn_iglp_opt(1);  // MFMA / DS interleave (-2 % at N=1)
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        if (i + 2 < NA) ow[i + 2] = opnd(0, i + 2);
        const int ks = i >> 1;
        if (i & 1) d0 = mfma32<DT>::run(ow[i], df[ks], ks == 0 ? dseed : d0);
        else s0 = mfma32<DT>::run(ow[i], kf[ks], ks == 0 ? sd0 : s0);
      }
    }
    {
      u32x4 o0 = opnd(1, 0), o1 = opnd(1, 1);
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        u32x4 o2 = o1;
        if (i + 2 < NA) o2 = opnd(1, i + 2);
        const int ks = i >> 1;
        if (i & 1) d1 = mfma32<DT>::run(o0, df[ks], ks == 0 ? dseed : d1);
        else s1 = mfma32<DT>::run(o0, kf[ks], ks == 0 ? sd1 : s1);
#pragma unroll
        for (int j = (i * 16) / NA; j < ((i + 1) * 16) / NA; ++j) elem(s0, d0, j);
        __builtin_amdgcn_sched_barrier(0);  // pins the MFMA / VALU issue order
        o0 = o1;
        o1 = o2;
      }
    }
    const u32x4 p00 = acc_to_frag<DT>(s0, 0), p01 = acc_to_frag<DT>(s0, 1);
    {
      u32x4 t0 = tr_frag<D>(qs, 0, 0, L), t1 = tr_frag<D>(qs, 16, 0, L);
#pragma unroll
      for (int i = 0; i < NK; ++i) {
        u32x4 t2 = t1;
        if (i + 2 < NK) t2 = tr_frag<D>(qs, ((i + 2) & 1) * 16, ((i + 2) >> 1) * 32, L);
        dk[i >> 1] = mfma32<DT>::run(t0, (i & 1) ? p01 : p00, dk[i >> 1]);
#pragma unroll
        for (int j = (i * 16) / NK; j < ((i + 1) * 16) / NK; ++j) elem(s1, d1, j);
        __builtin_amdgcn_sched_barrier(0);
        t0 = t1;
        t1 = t2;
      }
    }
    const u32x4 p10 = acc_to_frag<DT>(s1, 0), p11 = acc_to_frag<DT>(s1, 1);
#pragma unroll
    for (int db = 0; db < DB; ++db) {
      dk[db] = mfma32<DT>::run(tr_frag<D>(qs, 32, db * 32, L), p10, dk[db]);
      dk[db] = mfma32<DT>::run(tr_frag<D>(qs, 48, db * 32, L), p11, dk[db]);
    }
  };

  auto tile = [&](auto bufc, int kt) {
    constexpr int BUF = decltype(bufc)::value;
    if (kt + PF < kt_end) issue(kt + PF);
    const char* qs = smem + BUF * CF::STAGE;
    const char* vs = qs + IMG;
    const int flag = r0 >= a.R ? 1 : (fwg ? staged_flag(qs + CF::OFF_F, wave, kt & 3) : 0);
    const bool tail = (kt + 1) * 64 > a.T;
    if (flag != 1) {
      if (flag == 2 || tail) {
        const uint64_t w = tile_bits(flag == 2 ? staged_word(qs + CF::OFF_W, wave * 32 + (lane & 31)) : 0ull,
                                     a.T - kt * 64, hf);
        pipe_body(qs, vs, masked_seed(w, 0), true, w);
      } else {
        pipe_body(qs, vs, sseed, false, 0ull);
      }
    }
    if (kt + PF < kt_end) wait_vm<NG * (PF - 1)>();
    else wait_vm<0>();
    raw_barrier();
  };

#pragma unroll
  for (int t = 0; t < PF; ++t)
    if (kt_beg + t < kt_end) issue(kt_beg + t);
  if (PF > 1 && kt_beg + 1 < kt_end) wait_vm<NG * (PF - 1)>();
  else wait_vm<0>();
  raw_barrier();
  for (int kt = kt_beg; kt < kt_end; kt += NBUF) {
    tile(std::integral_constant<int, 0>{}, kt);
    if (kt + 1 < kt_end) tile(std::integral_constant<int, 1>{}, kt + 1);
    if constexpr (NBUF > 2) {
      if (kt + 2 < kt_end) tile(std::integral_constant<int, 2>{}, kt + 2);
    }
  }
  const float nscale = -a.scale;  // dk was accumulated from -dS
  if (row_ok && (a.nsplit > 1 || a.force_partial)) {
    float* op = a.dpart + (((int64_t)(a.sp0 + sp) * a.B + b) * a.R + row) * C + h * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 v = {dk[db][4 * g] * nscale, dk[db][4 * g + 1] * nscale, dk[db][4 * g + 2] * nscale, dk[db][4 * g + 3] * nscale};
        *reinterpret_cast<f32x4*>(op + db * 32 + 8 * g + 4 * hf) = v;
      }
  } else if (row_ok) {
    T16* op = reinterpret_cast<T16*>(a.drows) + ((int64_t)b * a.R + row) * C + h * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2 wv;
        wv[0] = pack2<DT>(dk[db][4 * g + 0] * nscale, dk[db][4 * g + 1] * nscale);
        wv[1] = pack2<DT>(dk[db][4 * g + 2] * nscale, dk[db][4 * g + 3] * nscale);
        *reinterpret_cast<u32x2*>(op + db * 32 + 8 * g + 4 * hf) = wv;
      }
  }
}

// ---------------------------------------------------------------------------------------
// grads of the gathered side.  4 waves x 32 columns; 64-row tiles of K_rows / dO.
//
// Staging is LDS-DMA (global_load_lds_dwordx4): no VGPRs hold a tile in flight, which is
// what lets this kernel (qf/vf 48 + dq/dv 96 + S/dP 32 registers) keep its LDS fragment
// reads ahead of the MFMAs instead of spilling.  The DMA destination is lane-linear, so the
// swizzled image is produced by permuting the per-lane SOURCE addresses (position p of the
// image holds chunk (p's chunk) ^ swizzle(row) of row p / ROW).  Per tile every wave issues
// exactly NG DMAs (its share of the two images + one 256 B/1 KiB row-constant piece), so a
// counted `s_waitcnt vmcnt(NG)` retires tile rt+1 while tile rt+2 stays in flight across the
// raw barrier (3-deep ring; 2-deep when three stages do not fit twice in 160 KiB).
template <int D, int NB = 0> struct ColsCfg {
  static constexpr int IMG = Img<D>::BYTES;
  static constexpr int IPW = IMG / 4096;  // 1 KiB DMA pieces per wave per image
  static constexpr int OFF_L = 2 * IMG, OFF_D = OFF_L + 256, OFF_W = OFF_D + 256, OFF_X = OFF_W + 1024;
  static constexpr int OFF_F = OFF_X + 256;  // tile flags of the two 32-row halves (glds_flags)
  static constexpr int STAGE = OFF_F + 256;
  static constexpr int NBUF = NB ? NB : ((2 * 3 * STAGE <= 160 * 1024) ? 3 : 2);
  static constexpr int PF = NBUF - 1;     // tiles in flight ahead of the one being computed
  static constexpr int NG = 2 * IPW + 2;  // DMAs per wave per tile
};

template <int DT, int D, int WPS = 2, int NB = 0, bool PS = false>
__global__ __launch_bounds__(256, WPS) void flash_bwd_cols_kernel(BwdArgs a) {
  using T16 = typename dt_traits<DT>::T;
  using CF = ColsCfg<D, NB>;
  constexpr int ROW = Img<D>::ROW, IMG = CF::IMG, IPW = CF::IPW, NG = CF::NG, PF = CF::PF, NBUF = CF::NBUF;
  constexpr int KS = D / 16, DB = D / 32;

  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Lanes L = make_lanes<D>(lane);
  const int ncb = (a.T + 127) / 128;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int cb = lin % ncb, bh = lin / ncb;
  const int b = bh / a.H, h = bh % a.H;
  const int C = a.H * D;
  const int NKT = (a.T + 63) / 64;
  const int NRB32 = (a.R + 31) / 32;
  const int NKT4 = (NKT + 3) & ~3;
  const int c0 = cb * 128 + wave * 32;
  const int col = c0 + (lane & 31);
  const bool col_ok = col < a.T;
  const int kt_w = c0 >> 6;           // this wave's 64-column mask tile

  u32x4 qf[KS], vf[KS];
  {
    const int64_t off = col_off(col_ok ? col : 0, b, a.T, a.ldkv) + h * D + 8 * hf;
    const T16* pq = reinterpret_cast<const T16*>(a.kc) + off;
    const T16* pv = reinterpret_cast<const T16*>(a.vc) + off;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      qf[s] = col_ok ? *reinterpret_cast<const u32x4*>(pq + 16 * s) : u32x4{0, 0, 0, 0};
      vf[s] = col_ok ? *reinterpret_cast<const u32x4*>(pv + 16 * s) : u32x4{0, 0, 0, 0};
    }
    // consume the fragments here: the compiler's vmcnt bookkeeping then retires these loads
    // before the first DMA instead of waiting vmcnt(0) (all DMAs in flight) inside the loop
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(qf[s]), "+v"(vf[s]));
    // -V: the dP accumulator then starts at δ and ends at δ - dP, so dS' = P ⊙ acc = -dS with
    // no per-element subtraction; the sign comes back in the dq epilogue (scale -> -scale)
#pragma unroll
    for (int s = 0; s < KS; ++s) vf[s] ^= u32x4{0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
  }
  const float c2 = a.scale * LOG2E;
  // PS: the K-row images hold K * scale * log2 e (host pre-scaled, the forward's buffer) and the
  // S accumulator is seeded with -lse2 of its rows, so P = 2^acc (no per-element FMA in
  // softmax_grad); dq = Σ dS'·K' then carries the factor -ln 2 instead of -scale
  const float NEG_INF = -__builtin_inff();
  const int NRT = (a.R + 63) / 64;

  ImgDma<D> dma;
  dma.init(wave, lane, C * 2);
  const char* rows_b = reinterpret_cast<const char*>(reinterpret_cast<const T16*>(a.rows) + (int64_t)b * a.R * C + h * D);
  const char* dout_b = reinterpret_cast<const char*>(reinterpret_cast<const T16*>(a.dout) + (int64_t)b * a.R * C + h * D);
  const float* lse = a.lse2 + ((int64_t)b * a.H + h) * a.R;  // log2-domain LSE
  const float* dlt = a.delta + ((int64_t)b * a.H + h) * a.R;
  // column-major mask words (mask_pack's bits_t): one u64 per (64-row tile, column)
  const int NRT64 = (a.R + 63) / 64, TPAD = (a.T + 127) / 128 * 128;
  const uint64_t* mb = a.mbits ? a.mbits + (int64_t)b * NRT64 * TPAD + cb * 128 : nullptr;

  auto issue = [&](int rt) {
    char* st = smem + (rt % NBUF) * CF::STAGE;
    const int r0 = rt * 64;
    const int rmax = a.R - 1 - r0;  // rows past R re-read row R-1; the compute masks them
    dma.issue(rows_b + (int64_t)r0 * C * 2, C * 2, rmax, st, wave);
    dma.issue(dout_b + (int64_t)r0 * C * 2, C * 2, rmax, st + IMG, wave);
    const uint32_t ro = (uint32_t)min(lane, rmax);  // offsets stay tile-relative (32-bit)
    if (wave == 0) glds4(lse + r0, ro * 4, st + CF::OFF_L);
    else if (wave == 1) glds4(dlt + r0, ro * 4, st + CF::OFF_D);
    else if (wave == 2 && mb) glds16(mb + (int64_t)rt * TPAD, (uint32_t)lane * 16, st + CF::OFF_W);
    else glds4(lse + r0, ro * 4, st + CF::OFF_X);  // keeps NG DMAs per wave per tile
    if (a.mflags) glds_flags(a.mflags + ((int64_t)b * NRB32 + 2 * rt) * NKT4, NKT4, min(2, NRB32 - 2 * rt), cb >> 1,
                             st + CF::OFF_F);
    else glds4(lse + r0, ro * 4, st + CF::OFF_X);
  };

  f32x16 dq[DB], dv[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dq[i][r] = 0.f; dv[i][r] = 0.f; }

#pragma unroll
  for (int t = 0; t < PF; ++t)
    if (t < NRT) issue(t);
  if (PF > 1 && NRT > 1) wait_vm<NG * (PF - 1)>();
  else wait_vm<0>();
  raw_barrier();
  // P and dS of one 32-row half tile in place (s <- P, dp <- dS); rows of register r:
  // tt*32 + (r&3) + 8*(r>>2) + 4*hf.  Rows past R carry lse = +inf (patched below), so the
  // unmasked path has no per-element test at all.
  // (dp holds δ - dP on entry: see the -V fragments above; leaves -dS)
  auto softmax_grad = [&](f32x16& s, f32x16& dp, const float* ls, const uint64_t* ws, int tt, bool masked) {
    // masked: this lane's column word over the tile's 64 rows, shifted to its row half
    const uint32_t hw = masked ? (uint32_t)(ws[wave * 32 + (lane & 31)] >> (tt * 32)) >> (4 * hf) : 0u;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int rbase = tt * 32 + 8 * g + 4 * hf;
      f32x4 l4 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (!PS) l4 = *reinterpret_cast<const f32x4*>(ls + rbase);  // lse * log2 e
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * g + e;
        float x = PS ? s[r] : __builtin_fmaf(s[r], c2, -l4[e]);
        if (masked && ((hw >> (8 * g + e)) & 1u)) x = NEG_INF;
        const float p = fast_exp2(x);
        s[r] = p;
        dp[r] = p * dp[r];
      }
    }
  };
  // dP accumulator seed: δ of the half tile's rows in the accumulator's row order
  auto delta_seed = [&](const float* dls, int tt) {
    f32x16 d;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 d4 = *reinterpret_cast<const f32x4*>(dls + tt * 32 + 8 * g + 4 * hf);
#pragma unroll
      for (int e = 0; e < 4; ++e) d[4 * g + e] = d4[e];
    }
    return d;
  };

  // S accumulator seed (PS): -lse2 of the half tile's rows in the accumulator's row order
  auto lse_seed = [&](const float* ls, int tt) {
    f32x16 d;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 l4 = *reinterpret_cast<const f32x4*>(ls + tt * 32 + 8 * g + 4 * hf);
#pragma unroll
      for (int e = 0; e < 4; ++e) d[4 * g + e] = -l4[e];
    }
    return d;
  };

  // one row tile from ring stage BUF (a compile-time constant: every LDS address is a lane
  // base + immediate, no per-read address arithmetic)
  auto tile = [&](auto bufc, int rt) {
    constexpr int BUF = decltype(bufc)::value;
    if (rt + PF < NRT) issue(rt + PF);
    char* ks = smem + BUF * CF::STAGE;
    const char* ds = ks + IMG;
    float* ls = reinterpret_cast<float*>(ks + CF::OFF_L);
    const float* dls = reinterpret_cast<const float*>(ks + CF::OFF_D);
    const uint64_t* ws = reinterpret_cast<const uint64_t*>(ks + CF::OFF_W);
    if (rt * 64 + 64 > a.R) {  // last tile, partial: rows past R get lse = +inf -> P = dS = 0
      if (wave == 0 && rt * 64 + lane >= a.R) ls[lane] = __builtin_inff();
      __syncthreads();
    }
    int flag = 0;
    if (a.mflags && c0 < a.T) {
      const int f0 = staged_flag(ks + CF::OFF_F, 0, kt_w & 3);
      const int f1 = (2 * rt + 1 < NRB32) ? staged_flag(ks + CF::OFF_F, 1, kt_w & 3) : 1;
      flag = __builtin_amdgcn_readfirstlane((f0 == 1 && f1 == 1) ? 1 : ((f0 == 0 && (f1 == 0 || 2 * rt + 1 >= NRB32)) ? 0 : 2));
    }
    if (flag != 1 && c0 < a.T) {
      __builtin_amdgcn_iglp_opt(0);  // -1 % (iglp_opt(1): +0.6 %)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        f32x16 s = mfma32<DT>::run(row_frag<D>(ks, tt * 32, 0, L), qf[0], PS ? lse_seed(ls, tt) : f32x16{});
        f32x16 dp = mfma32<DT>::run(row_frag<D>(ds, tt * 32, 0, L), vf[0], delta_seed(dls, tt));
#pragma unroll
        for (int kk = 1; kk < KS; ++kk) {
          s = mfma32<DT>::run(row_frag<D>(ks, tt * 32, kk, L), qf[kk], s);
          dp = mfma32<DT>::run(row_frag<D>(ds, tt * 32, kk, L), vf[kk], dp);
        }
        if (flag == 2) softmax_grad(s, dp, ls, ws, tt, true);
        else softmax_grad(s, dp, ls, ws, tt, false);
        // one 16-row k-step at a time: only 2 packed operand fragments live
#pragma unroll
        for (int sh = 0; sh < 2; ++sh) {
          const u32x4 pf = acc_to_frag<DT>(s, sh), gf = acc_to_frag<DT>(dp, sh);
#pragma unroll
          for (int db = 0; db < DB; ++db) {
            dv[db] = mfma32<DT>::run(tr_frag<D>(ds, tt * 32 + 16 * sh, db * 32, L), pf, dv[db]);
            dq[db] = mfma32<DT>::run(tr_frag<D>(ks, tt * 32 + 16 * sh, db * 32, L), gf, dq[db]);
          }
        }
      }
    }
    // tile rt+1 complete (this wave's DMAs), everyone done with tile rt, then rotate
    if (rt + PF < NRT) wait_vm<NG * (PF - 1)>();
    else wait_vm<0>();
    raw_barrier();
  };
  for (int rt = 0; rt < NRT; rt += NBUF) {
    tile(std::integral_constant<int, 0>{}, rt);
    if (rt + 1 < NRT) tile(std::integral_constant<int, 1>{}, rt + 1);
    if constexpr (NBUF > 2) {
      if (rt + 2 < NRT) tile(std::integral_constant<int, 2>{}, rt + 2);
    }
  }
  const float nscale = PS ? -LN2 : -a.scale;  // dq was accumulated from -dS (and K' = K * scale * log2 e)
  if (col_ok && a.dkv16) {  // input dtype: half the store (and reduce-scatter) bytes
    const int64_t off = col_off(col, b, a.T, a.ldg) + h * D;
    T16* pq = reinterpret_cast<T16*>(a.dkc) + off;
    T16* pv = reinterpret_cast<T16*>(a.dvc) + off;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2 q2, v2;
        q2[0] = pack2<DT>(dq[db][4 * g] * nscale, dq[db][4 * g + 1] * nscale);
        q2[1] = pack2<DT>(dq[db][4 * g + 2] * nscale, dq[db][4 * g + 3] * nscale);
        v2[0] = pack2<DT>(dv[db][4 * g], dv[db][4 * g + 1]);
        v2[1] = pack2<DT>(dv[db][4 * g + 2], dv[db][4 * g + 3]);
        *reinterpret_cast<u32x2*>(pq + db * 32 + 8 * g + 4 * hf) = q2;
        *reinterpret_cast<u32x2*>(pv + db * 32 + 8 * g + 4 * hf) = v2;
      }
  } else if (col_ok) {
    const int64_t off = col_off(col, b, a.T, a.ldg) + h * D;
    float* pq = reinterpret_cast<float*>(a.dkc) + off;
    float* pv = reinterpret_cast<float*>(a.dvc) + off;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 q4 = {dq[db][4 * g] * nscale, dq[db][4 * g + 1] * nscale, dq[db][4 * g + 2] * nscale, dq[db][4 * g + 3] * nscale};
        f32x4 v4 = {dv[db][4 * g], dv[db][4 * g + 1], dv[db][4 * g + 2], dv[db][4 * g + 3]};
        *reinterpret_cast<f32x4*>(pq + db * 32 + 8 * g + 4 * hf) = q4;
        *reinterpret_cast<f32x4*>(pv + db * 32 + 8 * g + 4 * hf) = v4;
      }
  }
}

// sum column-split partials of the row-side gradient -> output dtype
template <int DT, int D>
__global__ __launch_bounds__(256) void flash_bwd_rows_sum(BwdArgs a) {
  using T16 = typename dt_traits<DT>::T;
  const int64_t total4 = (int64_t)a.B * a.R * a.H * D / 4;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total4) return;
  const int64_t stride = total4 * 4;
  f32x4 acc = *reinterpret_cast<const f32x4*>(a.dpart + idx * 4);
  for (int s = 1; s < a.nsplit; ++s) acc += *reinterpret_cast<const f32x4*>(a.dpart + s * stride + idx * 4);
  u32x2 w;
  w[0] = pack2<DT>(acc[0], acc[1]);
  w[1] = pack2<DT>(acc[2], acc[3]);
  *reinterpret_cast<u32x2*>(reinterpret_cast<T16*>(a.drows) + idx * 4) = w;
}

// column-side row-split partials (BwdArgs::csq / csv): out[r * ldo + c] = Σ_s part[(s * rows + r) * C + c],
// in split order (deterministic), fp32 partials -> output dtype
// One 16-byte chunk per thread; every split's chunk is loaded before any is added (up to 4 splits in
// flight per thread) and the chunk index splits with 32-bit math where it fits
template <int DT>
__global__ __launch_bounds__(256) void cols_sum_kernel(const float* __restrict__ part, void* __restrict__ out_, int S,
                                                        int64_t rows, int C, int64_t ldo) {
  const uint32_t c4 = (uint32_t)C / 4;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = rows * c4;
  if (idx >= total) return;
  int64_t r;
  int c;
  if (total <= 0xFFFFFFFFll) {  // (uniform) 32-bit division
    const uint32_t i32 = (uint32_t)idx, r32 = i32 / c4;
    r = r32;
    c = (int)(i32 - r32 * c4) * 4;
  } else {
    r = idx / c4;
    c = (int)(idx - r * c4) * 4;
  }
  const int64_t sl = rows * C;
  const float* p = part + r * C + c;
  f32x4 v[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    if (s < S) v[s] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + s * sl));
  f32x4 acc = v[0];
#pragma unroll
  for (int s = 1; s < 4; ++s)
    if (s < S) acc += v[s];
  for (int s = 4; s < S; ++s) acc += *reinterpret_cast<const f32x4*>(p + s * sl);  // (more than 4 splits)
  if constexpr (DT == DT_F32) {
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(out_) + r * ldo + c) = acc;
  } else {
    using T16 = typename dt_traits<DT>::T;
    u32x2 w;
    w[0] = pack2<DT>(acc[0], acc[1]);
    w[1] = pack2<DT>(acc[2], acc[3]);
    *reinterpret_cast<u32x2*>(reinterpret_cast<T16*>(out_) + r * ldo + c) = w;
  }
}

// δ (+ lse2) with 8 lanes per (b, row, h): lane `sub` reads D / 8 contiguous elements of O and dO
// in 8-byte pieces (a wave covers 8 heads' rows contiguously), a 3-step xor sum, lane 0 writes.
// The one-thread-per-row kernel above streams 2 x D x 2 bytes alone per thread: 27 us at T = R =
// 25000, H = 8 (2.8 TB/s).
template <int DT, int D>
__global__ __launch_bounds__(256) void flash_bwd_prep8_kernel(BwdArgs a, const void* out_, float* delta) {
  static_assert(D % 32 == 0, "prep8: D / 8 elements per lane in 4-element pieces");
  using T16 = typename dt_traits<DT>::T;
  constexpr int NP = D / 32;  // 4-element (8-byte) pieces per lane
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t pr = idx >> 3;  // (b, row, h), h fastest: the (B, R, H*D) layout
  const int sub = (int)(idx & 7);
  const bool ok = pr < (int64_t)a.B * a.R * a.H;
  float acc = 0.f;
  if (ok && delta) {
    const int64_t off = pr * D + sub * (D / 8);
    const u32x2* o = reinterpret_cast<const u32x2*>(reinterpret_cast<const T16*>(out_) + off);
    const u32x2* d = reinterpret_cast<const u32x2*>(reinterpret_cast<const T16*>(a.dout) + off);
    union P { u32x2 u; T16 e[4]; } x[NP], y[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      x[i].u = o[i];
      y[i].u = d[i];
    }
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc += (float)x[i].e[e] * (float)y[i].e[e];
  }
  acc += __shfl_xor(acc, 1);
  acc += __shfl_xor(acc, 2);
  acc += __shfl_xor(acc, 4);
  if (!ok || sub) return;
  const int h = (int)(pr % a.H);
  const int64_t br = pr / a.H;
  const int row = (int)(br % a.R), b = (int)(br / a.R);
  const int64_t li = ((int64_t)b * a.H + h) * a.R + row;
  if (a.lse2) a.lse2[li] = a.lse[li] * LOG2E;
  if (delta) delta[li] = acc;
}

template <int DT, int D>
static void launch_bwd_delta(const BwdArgs& a, const void* out, float* delta, hipStream_t st) {
  const int64_t n0 = (int64_t)a.B * a.R * a.H;
  if constexpr (D % 32 == 0 && D <= 128) {
    hipLaunchKernelGGL((flash_bwd_prep8_kernel<DT, D>), dim3((unsigned)((8 * n0 + 255) / 256)), dim3(256), 0, st, a, out,
                       delta);
    return;
  }
  hipLaunchKernelGGL((flash_bwd_prep_kernel<DT, D>), dim3((unsigned)((n0 + 255) / 256)), dim3(256), 0, st, a, out, delta);
}

// Pre-scaled D <= 96 runs the software-pipelined column kernel (csrc/flash_cols.hip: 7 % faster
// standalone, profiles/r3_cols_pipe.md); D = 128 and non-pre-scaled inputs run the plain kernel below.
// The plain column kernel runs 2 ring stages: 3 stages spilled 9 VGPRs inside the tile loop at
// D = 96 (every scratch reload's vmcnt drained the DMA prefetch): 4.36 vs 4.62 ms at T = R =
// 25000, 0.60 vs 0.64 ms at R = 3125 on MI355X.
template <int DT, int D>
static void launch_bwd_cols(const BwdArgs& a, hipStream_t st) {
  if (D <= 96 && a.prescaled && xdot_flash_bwd_cols2_launch(&a, DT, D, st) == 0) return;
  const int ncb = (a.T + 127) / 128;
  constexpr int LDS2 = 2 * ColsCfg<D, 2>::STAGE;
  const dim3 grid(ncb * a.B * a.H);
  if (a.prescaled) hipLaunchKernelGGL((flash_bwd_cols_kernel<DT, D, 2, 2, true>), grid, dim3(256), LDS2, st, a);
  else hipLaunchKernelGGL((flash_bwd_cols_kernel<DT, D, 2, 2>), grid, dim3(256), LDS2, st, a);
}

template <int DT, int D>
static void launch_rows_sum(const BwdArgs& a, hipStream_t st) {
  const int64_t n4 = (int64_t)a.B * a.R * a.H * D / 4;
  hipLaunchKernelGGL((flash_bwd_rows_sum<DT, D>), dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, a);
}

template <int DT, int D>
static void launch_bwd_rows(const BwdArgs& a, hipStream_t st) {
  const int nrb = (a.R + 127) / 128;
  constexpr int LDS = RowsCfg<D>::NBUF * RowsCfg<D>::STAGE;
  const dim3 grid(nrb * a.B * a.H * a.nsplit);
  if (a.prescaled) hipLaunchKernelGGL((flash_bwd_rows_kernel<DT, D, true>), grid, dim3(256), LDS, st, a);
  else hipLaunchKernelGGL((flash_bwd_rows_kernel<DT, D, false>), grid, dim3(256), LDS, st, a);
  if (a.nsplit > 1 && !a.force_partial) launch_rows_sum<DT, D>(a, st);
}

}  // namespace fa
}  // namespace xdot

#define XB_DISPATCH(CALL)                                                                        \
  if (dt == DT_BF16 && D == 32) { CALL(DT_BF16, 32); return 0; }                                 \
  if (dt == DT_BF16 && D == 64) { CALL(DT_BF16, 64); return 0; }                                 \
  if (dt == DT_BF16 && D == 96) { CALL(DT_BF16, 96); return 0; }                                 \
  if (dt == DT_BF16 && D == 128) { CALL(DT_BF16, 128); return 0; }                               \
  if (dt == DT_F16 && D == 32) { CALL(DT_F16, 32); return 0; }                                   \
  if (dt == DT_F16 && D == 64) { CALL(DT_F16, 64); return 0; }                                   \
  if (dt == DT_F16 && D == 96) { CALL(DT_F16, 96); return 0; }                                   \
  if (dt == DT_F16 && D == 128) { CALL(DT_F16, 128); return 0; }                                 \
  return -1;

// the D-templated helpers (prep, row-partial sum) also for the wide heads of flash_wide.hip
#define XB_DISPATCH_W(CALL)                                                                      \
  if (dt == DT_BF16 && D == 160) { CALL(DT_BF16, 160); return 0; }                               \
  if (dt == DT_BF16 && D == 192) { CALL(DT_BF16, 192); return 0; }                               \
  if (dt == DT_BF16 && D == 256) { CALL(DT_BF16, 256); return 0; }                               \
  if (dt == DT_BF16 && D == 384) { CALL(DT_BF16, 384); return 0; }                               \
  if (dt == DT_F16 && D == 160) { CALL(DT_F16, 160); return 0; }                                 \
  if (dt == DT_F16 && D == 192) { CALL(DT_F16, 192); return 0; }                                 \
  if (dt == DT_F16 && D == 256) { CALL(DT_F16, 256); return 0; }                                 \
  if (dt == DT_F16 && D == 384) { CALL(DT_F16, 384); return 0; }                                 \
  XB_DISPATCH(CALL)

extern "C" int xdot_flash_bwd_delta_launch(const xdot::fa::BwdArgs* a, const void* out, float* delta, int dt, int D,
                                           hipStream_t st) {
  using namespace xdot;
  using namespace xdot::fa;
  if (a->R == 0 || a->B == 0 || a->H == 0) return 0;
  if (dt == DT_F32) return xdot_flash_bwd_prep_f32_launch(a, out, delta, D, st);
#define XP(DTV, DV) launch_bwd_delta<DTV, DV>(*a, out, delta, st)
  XB_DISPATCH_W(XP)
#undef XP
}

extern "C" int xdot_flash_bwd_cols_launch(const xdot::fa::BwdArgs* a, int dt, int D, hipStream_t st) {
  using namespace xdot;
  using namespace xdot::fa;
  if (a->R == 0 || a->B == 0 || a->H == 0 || a->T == 0) return 0;
  if (D > 128) return xdot_flash_wide_cols_launch(a, dt, D, st);  // dV pass + dQ pass
  if (dt == DT_F32) return a->fp32_mode ? xdot_flash_bwd_cols_x3_launch(a, D, st) : xdot_flash_bwd_cols_f32_launch(a, D, st);
#define XC(DTV, DV) launch_bwd_cols<DTV, DV>(*a, st)
  XB_DISPATCH(XC)
#undef XC
}

extern "C" int xdot_flash_cols_splits(const xdot::fa::BwdArgs* a, int dt, int D, int* sq, int* sv) {
  *sq = *sv = 1;
  if (a->R == 0 || a->B == 0 || a->H == 0 || a->T == 0) return 0;
  if (D > 128) {  // the wide family's two passes, each from its own occupancy
    const int64_t W = (int64_t)((a->T + 127) / 128) * a->B * a->H, nrt = (a->R + 31) / 32;
    *sq = std::max(1, xdot_flash_wide_splits(2, dt, D, a->sbuf != nullptr, W, nrt));
    *sv = std::max(1, xdot_flash_wide_splits(3, dt, D, a->sbuf != nullptr, W, nrt));
    return 0;
  }
  if (dt != xdot::DT_F32) {  // the pipelined 16-bit column kernel (pre-scaled, D <= 96) only
    if (D > 96 || !a->prescaled) return 0;
    const int r = xdot_flash_cols_splits_cols2(a, dt, D, sq);
    *sv = *sq;
    return r;
  }
  return a->fp32_mode ? xdot_flash_cols_splits_x3(a, D, sq, sv) : xdot_flash_cols_splits_f32(a, D, sq, sv);
}

// XDOT_F32_SPLIT: unset / "auto" = the occupancy round model for the fp32 forward and row-side
// backward (measured r5s20: step 55.99 -> 55.23 ms, forward 16.61 -> 16.05, rows 8.63 -> 8.46);
// "fwd" = the model for the forward only; "old" = the 16-bit model (pick_split / rows_split) for
// both; n = n splits for both.  Returns 0 when the caller should use its own model.
extern "C" int xdot_flash_f32_row_splits(int kernel, int fp32_mode, int D, bool sbuf, int64_t W, int64_t T) {
  if (D > 128 || W <= 0 || T <= 0) return 0;
  const char* e = std::getenv("XDOT_F32_SPLIT");
  const bool dflt = !e || !*e || !std::strcmp(e, "auto");
  if (!dflt && !std::strcmp(e, "old")) return 0;
  if (!dflt && !std::strcmp(e, "fwd")) {
    if (kernel == 1) return 0;
  } else if (!dflt) {
    const int n = std::atoi(e);
    return n > 0 ? std::min<int64_t>(n, (T + 31) / 32) : 0;
  }
  return fp32_mode ? xdot_flash_f32_row_splits_x3(kernel, D, sbuf, W, T)
                   : xdot_flash_f32_row_splits_exact(kernel, D, sbuf, W, T);
}

extern "C" int xdot_flash_cols_sum_launch(const float* part, void* out, int S, int64_t rows, int C, int64_t ldo, int dt,
                                          hipStream_t st) {
  using namespace xdot;
  if (rows == 0 || C == 0) return 0;
  if (C & 3) return -1;
  const dim3 grid((unsigned)((rows * (C / 4) + 255) / 256));
  switch (dt) {
    case DT_F32: hipLaunchKernelGGL(fa::cols_sum_kernel<DT_F32>, grid, dim3(256), 0, st, part, out, S, rows, C, ldo); return 0;
    case DT_BF16: hipLaunchKernelGGL(fa::cols_sum_kernel<DT_BF16>, grid, dim3(256), 0, st, part, out, S, rows, C, ldo); return 0;
    case DT_F16: hipLaunchKernelGGL(fa::cols_sum_kernel<DT_F16>, grid, dim3(256), 0, st, part, out, S, rows, C, ldo); return 0;
    default: return -1;
  }
}

// sum a->nsplit slots of dpart into drows (input dtype)
extern "C" int xdot_flash_bwd_rows_sum_launch(const xdot::fa::BwdArgs* a, int dt, int D, hipStream_t st) {
  using namespace xdot;
  using namespace xdot::fa;
  if (a->R == 0 || a->B == 0 || a->H == 0) return 0;
  if (dt == DT_F32) return xdot_flash_rows_sum_f32_launch(a, D, st);
#define XS(DTV, DV) launch_rows_sum<DTV, DV>(*a, st)
  XB_DISPATCH_W(XS)
#undef XS
}

extern "C" int xdot_flash_bwd_rows_launch(const xdot::fa::BwdArgs* a, int dt, int D, hipStream_t st) {
  using namespace xdot;
  using namespace xdot::fa;
  if (a->R == 0 || a->B == 0 || a->H == 0 || a->T == 0) return 0;
  if (D > 128) {
    const int rc = xdot_flash_wide_rows_launch(a, dt, D, st);
    if (rc == 0 && a->nsplit > 1 && !a->force_partial) return xdot_flash_bwd_rows_sum_launch(a, dt, D, st);
    return rc;
  }
  if (dt == DT_F32) {
    const int rc = a->fp32_mode ? xdot_flash_bwd_rows_x3_launch(a, D, st) : xdot_flash_bwd_rows_f32_launch(a, D, st);
    if (rc == 0 && a->nsplit > 1 && !a->force_partial) return xdot_flash_rows_sum_f32_launch(a, D, st);
    return rc;
  }
#define XR(DTV, DV) launch_bwd_rows<DTV, DV>(*a, st)
  XB_DISPATCH(XR)
#undef XR
}
