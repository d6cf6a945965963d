// xdot — sequence-parallel flash-attention FORWARD for gfx950 (MI355X).
//
// Per rank: O = softmax(scale * K_rows · Q_colsᵀ, bool mask) · V_cols, where the columns are
// the all-gathered T rows of the module's `queries`/`values` projections and the rows are
// this rank's R rows of `keys` (reference: distributed_dot_product/module.py:60-71 — there
// the (B, H, R, T) scores are materialised by distributed_matmul_nt, scaled, masked,
// softmaxed and multiplied by distributed_matmul_all; here they only ever exist as MFMA
// accumulators).
//
// Structure (one workgroup = 4 waves = 128 rows of one (batch, head); 2 workgroups/CU):
//   * each wave owns 32 rows; their K-fragments stay in VGPRs for the whole sweep;
//   * the workgroup streams 64-column tiles of Q_cols / V_cols HBM -> VGPR -> LDS, double
//     buffered: tile t+1's global loads are issued before tile t's MFMAs and written to LDS
//     after them (one barrier per tile);
//   * S is computed TRANSPOSED (Sᵀ = Q_cols · K_rowsᵀ, v_mfma_f32_32x32x16) so that every
//     lane holds 32 scores of ONE row: the online-softmax max/sum are lane-local plus a
//     single cross-half exchange — no LDS round trip, no serial lanes;
//   * the probabilities are packed to bf16 straight from the accumulators and used as the B
//     operand of Oᵀ += V_colsᵀ · Pᵀ, with V_cols read through ds_read_b64_tr_b16 (hardware
//     transpose) from a bank-conflict-free LDS image;
//   * the boolean mask arrives pre-packed (csrc/mask_pack.hip): fully masked tiles are
//     skipped, unmasked tiles pay nothing, partial tiles test one 64-bit word per row;
//   * output O is written in the head-interleaved (B, R, H*D) layout the output projection
//     consumes, plus the natural-log LSE per row for the backward recomputation.
// Workgroup ids are XCD-remapped so the row blocks that stream the same (b, h) columns share
// an XCD L2.
#include "flash_common.h"

#include <type_traits>

namespace xdot {
namespace fa {

template <int DT, int D, int WPS = 2>
__global__ __launch_bounds__(256, WPS) void flash_fwd_kernel(FwdArgs a) {
  using T16 = typename dt_traits<DT>::T;
  using CF = RowsCfg<D>;
  constexpr int IMG = CF::IMG, NG = CF::NG, PF = CF::PF, NBUF = CF::NBUF;
  constexpr int KS = D / 16;      // k-steps over the head dim
  constexpr int DB = D / 32;      // 32-wide d blocks of the output

  extern __shared__ __attribute__((aligned(16))) char smem[];

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

  const T16* rows = reinterpret_cast<const T16*>(a.rows);

  // row-side fragments (B operand of Sᵀ): lane -> row, d = 16s + 8hf .. +7
  u32x4 kf[KS];
  {
    const T16* p = rows + ((int64_t)b * a.R + row) * C + h * D + 8 * hf;
#pragma unroll
    for (int s = 0; s < KS; ++s) kf[s] = row_ok ? *reinterpret_cast<const u32x4*>(p + 16 * s) : u32x4{0, 0, 0, 0};
    // retire these loads here, before the first DMA (else: vmcnt(0) inside the loop)
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(kf[s]));
  }

  // ---- LDS-DMA ring: Q_cols / V_cols images + the workgroup rows' mask words ----
  ImgDma<D> dma;
  dma.init(wave, lane);
  const int ldb = a.ldkv * 2;  // gathered row stride, bytes
  const char* kcb = reinterpret_cast<const char*>(reinterpret_cast<const T16*>(a.kc) + h * D + (int64_t)b * a.T * a.ldkv);
  const char* vcb = reinterpret_cast<const char*>(reinterpret_cast<const T16*>(a.vc) + h * D + (int64_t)b * a.T * a.ldkv);
  const uint64_t* mwg = a.mbits ? a.mbits + ((int64_t)b * a.R + rb * 128) * NKT : nullptr;
  const uint32_t moff = (uint32_t)(min((wave & 1) * 64 + lane, a.R - 1 - rb * 128) * NKT * 8 + (wave >> 1) * 4);
  auto issue = [&](int kt) {
    char* st = smem + ((kt - kt_beg) % NBUF) * CF::STAGE;
    const int64_t t0 = (int64_t)kt * 64;
    const int rmax = a.T - 1 - (int)t0;  // columns past T re-read column T-1 (masked in compute)
    dma.issue(kcb + t0 * ldb, ldb, rmax, st, wave);
    dma.issue(vcb + t0 * ldb, ldb, rmax, st + IMG, wave);
    if (mwg) glds4(mwg + kt, moff, st + CF::OFF_W + (wave >> 1) * 512 + (wave & 1) * 256);
    else glds4(kcb, (uint32_t)lane * 4, st + CF::OFF_X);  // keeps NG DMAs per wave per tile
  };

  const float c2 = a.scale * LOG2E;
  const float NEG_INF = -__builtin_inff();
  float m_run = NEG_INF, l_run = 0.f;
  f32x16 o[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;

  const int NKT4 = (NKT + 3) & ~3;
  const uint8_t* flags = a.mflags ? a.mflags + ((int64_t)b * ((a.R + 31) / 32) + __builtin_amdgcn_readfirstlane(r0 >> 5)) * NKT4 : nullptr;

  // one column tile from ring stage BUF (compile-time: LDS addresses = lane base + immediate)
  auto tile = [&](auto bufc, int kt) {
    constexpr int BUF = decltype(bufc)::value;
    if (kt + PF < kt_end) issue(kt + PF);
    const char* qs = smem + BUF * CF::STAGE;
    const char* vs = qs + IMG;
    const int flag = (flags && r0 < a.R) ? tile_flag(flags, kt) : 0;
    const bool tail = (kt + 1) * 64 > a.T;
    if (flag != 1 && r0 < a.R) {
      // ---- Sᵀ = Q_cols · K_rowsᵀ : two 32x32 tiles (cols 0-31, 32-63) ----
      f32x16 s[2];
      {
        u32x4 qa = row_frag<D>(qs, 0, 0, L);
#pragma unroll
        for (int i = 0; i < 2 * KS; ++i) {
          const int tt = i / KS, ks = i % KS;
          u32x4 qn = qa;
          if (i + 1 < 2 * KS) qn = row_frag<D>(qs, ((i + 1) / KS) * 32, (i + 1) % KS, L);
          s[tt] = mfma32<DT>::run(qa, kf[ks], ks == 0 ? f32x16{} : s[tt]);
          qa = qn;
        }
      }
      // ---- online softmax (lane-local row, partner lane = lane ^ 32) ----
      // max over raw scores (scale > 0), exponent as one FMA: p = 2^(s*c2 - m)
      float mx = NEG_INF;
      if (flag == 2 || tail) {
        const uint64_t w = flag == 2 ? staged_word(qs + CF::OFF_W, wave * 32 + (lane & 31)) : 0ull;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int kk = tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
            if (((w >> kk) & 1ull) || kt * 64 + kk >= a.T) s[tt][r] = NEG_INF;
            mx = fmaxf(mx, s[tt][r]);
          }
      } else {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[tt][r]);
      }
      mx = pair_max(mx) * c2;
      const float m_new = fmaxf(m_run, mx);
      const float m_use = (m_new == NEG_INF) ? 0.f : m_new;
      // rescale the running output only when some row of the wave raised its max
      if (__any(m_new > m_run)) {
        const float alpha = fast_exp2(m_run - m_use);
        l_run *= alpha;
#pragma unroll
        for (int i = 0; i < DB; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
      }
      m_run = m_new;
      float ls = 0.f;
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fast_exp2(__builtin_fmaf(s[tt][r], c2, -m_use));
          s[tt][r] = p;
          ls += p;
        }
      l_run += ls;
      // ---- Oᵀ += V_colsᵀ · Pᵀ ----
      u32x4 pf[4];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int sh = 0; sh < 2; ++sh) pf[tt * 2 + sh] = acc_to_frag<DT>(s[tt], sh);
      // operand reads run one MFMA ahead of their use
      u32x4 va = tr_frag<D>(vs, 0, 0, L);
#pragma unroll
      for (int i = 0; i < 4 * DB; ++i) {
        const int db = i >> 2, k4 = i & 3;
        u32x4 vn = va;
        if (i + 1 < 4 * DB) vn = tr_frag<D>(vs, ((i + 1) & 3) * 16, ((i + 1) >> 2) * 32, L);
        o[db] = mfma32<DT>::run(va, pf[k4], o[db]);
        va = vn;
      }
    }
    // tile kt+1 complete (this wave's DMAs), everyone done with tile kt, then rotate
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

  // ---- epilogue ----
  const float l_tot = pair_sum(l_run);
  const float inv = 1.f / l_tot;
  if (row_ok && a.nsplit == 1) {
    T16* op = reinterpret_cast<T16*>(a.out) + ((int64_t)b * a.R + row) * C + h * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2 w;
        w[0] = pack2<DT>(o[db][4 * g + 0] * inv, o[db][4 * g + 1] * inv);
        w[1] = pack2<DT>(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv);
        *reinterpret_cast<u32x2*>(op + db * 32 + 8 * g + 4 * hf) = w;
      }
    if (hf == 0) a.lse[((int64_t)b * a.H + h) * a.R + row] = (m_run + __log2f(l_tot)) * LN2;
  } else if (row_ok) {
    // split partial: normalised fp32 output + its LSE; merged by flash_fwd_combine
    float* op = a.opart + (((int64_t)sp * a.B + b) * a.R + row) * C + h * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 v = {o[db][4 * g] * inv, o[db][4 * g + 1] * inv, o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv};
        *reinterpret_cast<f32x4*>(op + db * 32 + 8 * g + 4 * hf) = v;
      }
    if (hf == 0) a.lpart[(((int64_t)sp * a.B + b) * a.H + h) * a.R + row] = (m_run + __log2f(l_tot)) * LN2;
  }
}

// merge column-split partials: lse = log Σ_s e^{lse_s}, O = Σ_s e^{lse_s - lse} O_s.
// A split that saw only masked columns has lse_s = -inf and contributes nothing; a row with
// every split -inf is fully masked and yields NaN like the unsplit kernel.
template <int DT, int D>
__global__ __launch_bounds__(256) void flash_fwd_combine(FwdArgs a) {
  using T16 = typename dt_traits<DT>::T;
  const int C = a.H * D;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)a.B * a.R * (C / 4);
  if (idx >= total) return;
  const int c4 = (int)(idx % (C / 4));
  const int64_t br = idx / (C / 4);
  const int row = (int)(br % a.R), b = (int)(br / a.R);
  const int h = (c4 * 4) / D;
  const int64_t lstride = (int64_t)a.B * a.H * a.R;
  const float* lp = a.lpart + ((int64_t)b * a.H + h) * a.R + row;
  float mx = -__builtin_inff();
  for (int s = 0; s < a.nsplit; ++s) mx = fmaxf(mx, lp[s * lstride]);
  float sum = 0.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int64_t ostride = (int64_t)a.B * a.R * C;
  const float* opp = a.opart + br * C + c4 * 4;
  for (int s = 0; s < a.nsplit; ++s) {
    const float l = lp[s * lstride];
    if (l == -__builtin_inff()) continue;
    const float wgt = __expf(l - mx);
    sum += wgt;
    const f32x4 v = *reinterpret_cast<const f32x4*>(opp + s * ostride);
    acc += wgt * v;
  }
  const float inv = 1.f / sum;  // sum == 0 (fully masked row) -> NaN output, -inf lse
  T16* op = reinterpret_cast<T16*>(a.out) + br * C + c4 * 4;
  u32x2 w;
  w[0] = pack2<DT>(acc[0] * inv, acc[1] * inv);
  w[1] = pack2<DT>(acc[2] * inv, acc[3] * inv);
  if (sum == 0.f) { w[0] = pack2<DT>(__builtin_nanf(""), __builtin_nanf("")); w[1] = w[0]; }
  *reinterpret_cast<u32x2*>(op) = w;
  if ((c4 * 4) % D == 0) a.lse[((int64_t)b * a.H + h) * a.R + row] = mx + __logf(sum);
}

template <int DT, int D>
static void launch_fwd(const FwdArgs& a, hipStream_t st) {
  constexpr int LDS = RowsCfg<D>::NBUF * RowsCfg<D>::STAGE;
  const int nrb = (a.R + 127) / 128;
  if (fa_wps() == 1) hipLaunchKernelGGL((flash_fwd_kernel<DT, D, 1>), dim3(nrb * a.B * a.H * a.nsplit), dim3(256), LDS, st, a);
  else hipLaunchKernelGGL((flash_fwd_kernel<DT, D, 2>), dim3(nrb * a.B * a.H * a.nsplit), dim3(256), LDS, st, a);
  if (a.nsplit > 1) {
    const int64_t n = (int64_t)a.B * a.R * (a.H * D / 4);
    hipLaunchKernelGGL((flash_fwd_combine<DT, D>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
  }
}

}  // namespace fa
}  // namespace xdot

extern "C" int xdot_flash_fwd_launch(const xdot::fa::FwdArgs* a, int dt, int D, hipStream_t st) {
  using namespace xdot;
  using namespace xdot::fa;
  if (a->R == 0 || a->B == 0 || a->H == 0) return 0;
#define XF(DTV, DV) if (dt == DTV && D == DV) { launch_fwd<DTV, DV>(*a, st); return 0; }
  XF(DT_BF16, 32) XF(DT_BF16, 64) XF(DT_BF16, 96) XF(DT_BF16, 128)
  XF(DT_F16, 32) XF(DT_F16, 64) XF(DT_F16, 96) XF(DT_F16, 128)
#undef XF
  return -1;
}
