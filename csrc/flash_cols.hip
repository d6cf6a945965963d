// xdot — software-pipelined gathered-side flash backward kernel for gfx950 (MI355X).
// (Split from csrc/flash_bwd.hip: that file holds the plain column kernel, the row kernel and
// the prep / sum kernels; flash_bwd.hip's launcher routes pre-scaled D <= 96 launches here.)
#include "flash_common.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace xdot {
namespace fa {

// ring-stage layout shared with the plain column kernel (flash_bwd.hip: ColsCfg)
template <int D> struct ColsStage {
  static constexpr int IMG = Img<D>::BYTES;
  static constexpr int IPW = IMG / 4096;
  static constexpr int OFF_L = 2 * IMG, OFF_D = OFF_L + 256, OFF_W = OFF_D + 256, OFF_X = OFF_W + 1024;
  static constexpr int OFF_F = OFF_X + 256;
  static constexpr int STAGE = OFF_F + 256;
  static constexpr int NG = 2 * IPW + 2;
};

// ---------------------------------------------------------------------------------------
// Software-pipelined gathered-side kernel (pre-scaled row side, D <= 96).  Same grid, tiles and
// LDS-DMA ring as flash_bwd_cols_kernel; per 64-row tile every wave runs
//   A0:       S / dP chains of half 0 (12 MFMAs, operand reads two ahead)
//   A1 || E0: the chains of half 1, each MFMA followed by its share of half 0's softmax
//             gradient (v_exp + multiply), then half 0 packed to bf16 fragments
//   K0 || E1: dV += dOᵀ·P and dQ += Kᵀ·dS of half 0, each MFMA followed by a share of half 1's
//             softmax gradient
//   K1:       dV / dQ of half 1
// so the VALU work issues between this wave's own MFMAs instead of leaving the matrix pipe to
// the partner wave (the plain body runs S/dP -> VALU -> dV/dQ back to back).  The registers
// this needs (a second S/dP pair) come from V: the workgroup's 128 columns of V live in LDS (one
// swizzled image, 24 KiB at D = 96: two workgroups per CU still fit) and the dP chains read their
// B operand there instead of from 24 VGPRs.  Signs: q is negated at load and the S accumulator
// is seeded with +lse2 (read straight from the staged row constants), so acc = lse2 - S' and
// P = 2^-acc (the negation is a free source modifier of v_exp_f32); -V and the δ seed give
// dS' = P ⊙ acc = -dS as in the plain kernel.
template <int D> struct Cols2Cfg {
  using B = ColsStage<D>;
  static constexpr int NBUF = 2, PF = 1, STAGE = B::STAGE;
  static constexpr int OFF_V = NBUF * STAGE;               // V image of the workgroup's 128 columns
  static constexpr int LDS = OFF_V + 128 * Img<D>::ROW;
};

template <int DT, int D>
__global__ __launch_bounds__(256, 2) void flash_bwd_cols2_kernel(BwdArgs a) {
  using T16 = typename dt_traits<DT>::T;
  using CB = ColsStage<D>;
  using CF = Cols2Cfg<D>;
  constexpr int ROW = Img<D>::ROW, IMG = CB::IMG, NG = CB::NG;
  constexpr int KS = D / 16, DB = D / 32;
  static_assert(D <= 96, "cols2: two workgroups per CU need D <= 96");

  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Lanes L = make_lanes<D>(lane);
  const int ncb = (a.T + 127) / 128;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int cb = lin % ncb, bhs = lin / ncb;
  const int bh = bhs % (a.B * a.H), sp = bhs / (a.B * a.H), ns = a.csq > 1 ? a.csq : 1;
  const int b = bh / a.H, h = bh % a.H;
  const int C = a.H * D;
  const int NKT = (a.T + 63) / 64;
  const int NRB32 = (a.R + 31) / 32;
  const int NKT4 = (NKT + 3) & ~3;
  const int c0 = cb * 128 + wave * 32;
  const int col = c0 + (lane & 31);
  const bool col_ok = col < a.T;
  const int kt_w = c0 >> 6;
  constexpr uint32_t SGN = 0x80008000u;

  // -q fragments in VGPRs; -V of the workgroup's columns -> LDS image rows wave*32 + (lane & 31)
  char* vimg = smem + CF::OFF_V;
  u32x4 qf[KS];
  {
    const int64_t off = col_off(col_ok ? col : 0, b, a.T, a.ldkv) + h * D + 8 * hf;
    const T16* pq = reinterpret_cast<const T16*>(a.kc) + off;
    const T16* pv = reinterpret_cast<const T16*>(a.vc) + off;
    const int vr = wave * 32 + (lane & 31), f = (vr >> 2) & 3;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      qf[s] = (col_ok ? *reinterpret_cast<const u32x4*>(pq + 16 * s) : u32x4{0, 0, 0, 0}) ^ u32x4{SGN, SGN, SGN, SGN};
      const u32x4 v = (col_ok ? *reinterpret_cast<const u32x4*>(pv + 16 * s) : u32x4{0, 0, 0, 0}) ^ u32x4{SGN, SGN, SGN, SGN};
      *reinterpret_cast<u32x4*>(vimg + vr * ROW + (((2 * s + hf) ^ f) << 4)) = v;
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(qf[s]));
  }
  const char* vw = vimg + wave * 32 * ROW;  // this wave's 32 V rows (row_frag base, r0 = 0)

  // row split sp of ns (BwdArgs::csq, against the last-round tail): 64-row tiles [rt_beg, rt_end),
  // rt_beg even (ring stage = tile parity)
  const int NRT = (a.R + 63) / 64, NRT2 = (NRT + 1) / 2;
  const int rt_beg = 2 * (int)((int64_t)sp * NRT2 / ns), rt_end = min(NRT, 2 * (int)((int64_t)(sp + 1) * NRT2 / ns));
  ImgDma<D> dma;
  dma.init(wave, lane, C * 2);
  const char* rows_b = reinterpret_cast<const char*>(reinterpret_cast<const T16*>(a.rows) + (int64_t)b * a.R * C + h * D);
  const char* dout_b = reinterpret_cast<const char*>(reinterpret_cast<const T16*>(a.dout) + (int64_t)b * a.R * C + h * D);
  const float* lse = a.lse2 + ((int64_t)b * a.H + h) * a.R;  // log2-domain LSE
  const float* dlt = a.delta + ((int64_t)b * a.H + h) * a.R;
  const int NRT64 = (a.R + 63) / 64, TPAD = (a.T + 127) / 128 * 128;
  const uint64_t* mb = a.mbits ? a.mbits + (int64_t)b * NRT64 * TPAD + cb * 128 : nullptr;

  auto issue = [&](int rt) {
    char* st = smem + (rt & 1) * CF::STAGE;
    const int r0 = rt * 64;
    const int rmax = a.R - 1 - r0;
    dma.issue(rows_b + (int64_t)r0 * C * 2, C * 2, rmax, st, wave);
    dma.issue(dout_b + (int64_t)r0 * C * 2, C * 2, rmax, st + IMG, wave);
    const uint32_t ro = (uint32_t)min(lane, rmax);
    if (wave == 0) glds4(lse + r0, ro * 4, st + CB::OFF_L);
    else if (wave == 1) glds4(dlt + r0, ro * 4, st + CB::OFF_D);
    else if (wave == 2 && mb) glds16(mb + (int64_t)rt * TPAD, (uint32_t)lane * 16, st + CB::OFF_W);
    else glds4(lse + r0, ro * 4, st + CB::OFF_X);
    if (a.mflags) glds_flags(a.mflags + ((int64_t)b * NRB32 + 2 * rt) * NKT4, NKT4, min(2, NRB32 - 2 * rt), cb >> 1,
                             st + CB::OFF_F);
    else glds4(lse + r0, ro * 4, st + CB::OFF_X);
  };

  f32x16 dq[DB], dv[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dq[i][r] = 0.f; dv[i][r] = 0.f; }

  // row constants of half tt in the accumulator's row order (lse2 -> S seed, δ -> dP seed)
  auto seed = [&](const float* c, int tt) {
    f32x16 d;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(c + tt * 32 + 8 * g + 4 * hf);
#pragma unroll
      for (int e = 0; e < 4; ++e) d[4 * g + e] = v[e];
    }
    return d;
  };

  // S seed of half tt with the mask folded in: +inf where (row, col) is masked (or past R), so the
  // accumulator ends at +inf and P = 2^-acc = 0 with no per-element test in the pipelined body
  auto seed_masked = [&](const float* c, int tt, uint32_t hw) {
    f32x16 d = seed(c, tt);
    sel_bits16(d, hw, PINF_BITS);
    return d;
  };

  auto body = [&](const char* ks, const char* ds, const float* ls, const float* dls, const uint64_t* ws,
                  bool masked) __attribute__((always_inline)) {
    constexpr int NA = 2 * KS, NK = 4 * DB;
    // this lane's column word over the tile's 64 rows, at its row half (masked tiles only)
    const uint64_t cw = masked ? ws[wave * 32 + (lane & 31)] >> (4 * hf) : 0ull;
    auto elem = [&](f32x16& sc, f32x16& dc, int r) {
      const float p = fast_exp2(-sc[r]);
      float y = p * dc[r];  // -dS (unscaled)
      asm volatile("" : "+v"(y));  // keeps it in this MFMA gap
      sc[r] = p;
      dc[r] = y;
    };
    // operand i of half tt's interleaved S (even i) / dP (odd i) chains: A from the K / dO tile
    auto opa = [&](int tt, int i) { return (i & 1) ? row_frag<D>(ds, tt * 32, i >> 1, L) : row_frag<D>(ks, tt * 32, i >> 1, L); };
    auto opb = [&](int i) { return (i & 1) ? row_frag<D>(vw, 0, i >> 1, L) : qf[i >> 1]; };
    f32x16 s0 = masked ? seed_masked(ls, 0, (uint32_t)cw) : seed(ls, 0), d0 = seed(dls, 0), s1, d1;
    // ---- A0 (operand reads one MFMA ahead) ----
    {
      u32x4 a0 = opa(0, 0), b0 = opb(0);
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        u32x4 a1 = a0, b1 = b0;
        if (i + 1 < NA) { a1 = opa(0, i + 1); b1 = opb(i + 1); }
        if (i & 1) d0 = mfma32<DT>::run(a0, b0, d0);
        else s0 = mfma32<DT>::run(a0, b0, s0);
        a0 = a1; b0 = b1;
      }
    }
    // half 1's seeds are built under A0's MFMAs (no barrier between: the mask select VALU fills
    // A0's gaps instead of stalling A1's first MFMA)
    s1 = masked ? seed_masked(ls, 1, (uint32_t)(cw >> 32)) : seed(ls, 1);
    d1 = seed(dls, 1);
    __builtin_amdgcn_sched_barrier(0);
    // ---- A1 || E0 ----
    {
      u32x4 a0 = opa(1, 0), b0 = opb(0);
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        u32x4 a1 = a0, b1 = b0;
        if (i + 1 < NA) { a1 = opa(1, i + 1); b1 = opb(i + 1); }
        if (i & 1) d1 = mfma32<DT>::run(a0, b0, d1);
        else s1 = mfma32<DT>::run(a0, b0, s1);
#pragma unroll
        for (int j = (i * 16) / NA; j < ((i + 1) * 16) / NA; ++j) elem(s0, d0, j);
        __builtin_amdgcn_sched_barrier(0);
        a0 = a1; b0 = b1;
      }
    }
    const u32x4 p00 = acc_to_frag<DT>(s0, 0), p01 = acc_to_frag<DT>(s0, 1);
    const u32x4 g00 = acc_to_frag<DT>(d0, 0), g01 = acc_to_frag<DT>(d0, 1);
    __builtin_amdgcn_sched_barrier(0);
    // ---- K0 || E1: MFMA i -> (sh = i / (2 DB), db = (i / 2) % DB, dV for even i, dQ for odd i) ----
    auto opk = [&](int tt, int i) {
      const int sh = i / (2 * DB), db = (i >> 1) % DB;
      return (i & 1) ? tr_frag<D>(ks, tt * 32 + 16 * sh, db * 32, L) : tr_frag<D>(ds, tt * 32 + 16 * sh, db * 32, L);
    };
    {
      u32x4 t0 = opk(0, 0), t1 = opk(0, 1);
#pragma unroll
      for (int i = 0; i < NK; ++i) {
        u32x4 t2 = t1;
        if (i + 2 < NK) t2 = opk(0, i + 2);
        const int sh = i / (2 * DB), db = (i >> 1) % DB;
        if (i & 1) dq[db] = mfma32<DT>::run(t0, sh ? g01 : g00, dq[db]);
        else dv[db] = mfma32<DT>::run(t0, sh ? p01 : p00, dv[db]);
#pragma unroll
        for (int j = (i * 16) / NK; j < ((i + 1) * 16) / NK; ++j) elem(s1, d1, j);
        __builtin_amdgcn_sched_barrier(0);
        t0 = t1; t1 = t2;
      }
    }
    const u32x4 p10 = acc_to_frag<DT>(s1, 0), p11 = acc_to_frag<DT>(s1, 1);
    const u32x4 g10 = acc_to_frag<DT>(d1, 0), g11 = acc_to_frag<DT>(d1, 1);
    __builtin_amdgcn_sched_barrier(0);
    // ---- K1 ----
    {
      u32x4 t0 = opk(1, 0), t1 = opk(1, 1);
#pragma unroll
      for (int i = 0; i < NK; ++i) {
        u32x4 t2 = t1;
        if (i + 2 < NK) t2 = opk(1, i + 2);
        const int sh = i / (2 * DB), db = (i >> 1) % DB;
        if (i & 1) dq[db] = mfma32<DT>::run(t0, sh ? g11 : g10, dq[db]);
        else dv[db] = mfma32<DT>::run(t0, sh ? p11 : p10, dv[db]);
        t0 = t1; t1 = t2;
      }
    }
  };

  if (rt_beg < rt_end) issue(rt_beg);
  wait_vm<0>();
  __syncthreads();  // also publishes the V image (drains its LDS stores)
  auto tile = [&](auto bufc, int rt) {
    constexpr int BUF = decltype(bufc)::value;
    if (rt + 1 < rt_end) issue(rt + 1);
    char* ks = smem + BUF * CF::STAGE;
    const char* ds = ks + IMG;
    float* ls = reinterpret_cast<float*>(ks + CB::OFF_L);
    const float* dls = reinterpret_cast<const float*>(ks + CB::OFF_D);
    const uint64_t* ws = reinterpret_cast<const uint64_t*>(ks + CB::OFF_W);
    if (rt * 64 + 64 > a.R) {  // last tile, partial: rows past R get lse2 = +inf -> P = dS = 0
      if (wave == 0 && rt * 64 + lane >= a.R) ls[lane] = __builtin_inff();
      __syncthreads();
    }
    int flag = 0;
    if (a.mflags && c0 < a.T) {
      const int f0 = staged_flag(ks + CB::OFF_F, 0, kt_w & 3);
      const int f1 = (2 * rt + 1 < NRB32) ? staged_flag(ks + CB::OFF_F, 1, kt_w & 3) : 1;
      flag = __builtin_amdgcn_readfirstlane((f0 == 1 && f1 == 1) ? 1 : ((f0 == 0 && (f1 == 0 || 2 * rt + 1 >= NRB32)) ? 0 : 2));
    }
    if (flag != 1 && c0 < a.T) body(ks, ds, ls, dls, ws, flag == 2);
    wait_vm<0>();  // tile rt+1 landed (the only DMAs in flight)
    raw_barrier();
  };
  for (int rt = rt_beg; rt < rt_end; rt += 2) {
    tile(std::integral_constant<int, 0>{}, rt);
    if (rt + 1 < rt_end) tile(std::integral_constant<int, 1>{}, rt + 1);
  }
  const float nscale = -LN2;  // dq was accumulated from -dS and K' = K * scale * log2 e
  if (col_ok && ns > 1) {  // fp32 partials of split sp, (ns, B*T, C) per half
    const int64_t off = (((int64_t)sp * a.B + b) * a.T + col) * C + h * D;
    float* pq = a.cpq + off;
    float* pv = a.cpv + off;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 q4 = {dq[db][4 * g] * nscale, dq[db][4 * g + 1] * nscale, dq[db][4 * g + 2] * nscale, dq[db][4 * g + 3] * nscale};
        f32x4 v4 = {dv[db][4 * g], dv[db][4 * g + 1], dv[db][4 * g + 2], dv[db][4 * g + 3]};
        *reinterpret_cast<f32x4*>(pq + db * 32 + 8 * g + 4 * hf) = q4;
        *reinterpret_cast<f32x4*>(pv + db * 32 + 8 * g + 4 * hf) = v4;
      }
  } else if (col_ok && a.dkv16) {
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


}  // namespace fa
}  // namespace xdot

extern "C" int xdot_flash_bwd_cols2_launch(const xdot::fa::BwdArgs* a, int dt, int D, hipStream_t st) {
  using namespace xdot;
  using namespace xdot::fa;
  const int ns = a->csq > 1 ? a->csq : 1;
  if (ns > 1 && (!a->cpq || !a->cpv || (D & 3))) return -1;
  const dim3 grid(((a->T + 127) / 128) * a->B * a->H * ns);
  const int odt = a->dkv16 ? dt : (int)DT_F32;
  const int64_t rows = (int64_t)a->B * a->T;
#define XC2(DTV, DV)                                                                                   \
  if (dt == DTV && D == DV) {                                                                          \
    hipLaunchKernelGGL((flash_bwd_cols2_kernel<DTV, DV>), grid, dim3(256), Cols2Cfg<DV>::LDS, st, *a); \
    if (ns > 1) {                                                                                      \
      xdot_flash_cols_sum_launch(a->cpq, a->dkc, ns, rows, a->H * D, a->ldg, odt, st);                 \
      xdot_flash_cols_sum_launch(a->cpv, a->dvc, ns, rows, a->H * D, a->ldg, odt, st);                 \
    }                                                                                                  \
    return 0;                                                                                          \
  }
  XC2(DT_BF16, 32) XC2(DT_BF16, 64) XC2(DT_BF16, 96) XC2(DT_F16, 32) XC2(DT_F16, 64) XC2(DT_F16, 96)
#undef XC2
  return -1;
}

namespace {
int cols2_csplit_env() {  // XDOT_CSPLIT, as in flash_f32.hip
  const char* e = std::getenv("XDOT_CSPLIT");
  return (!e || !*e || !std::strcmp(e, "auto")) ? -1 : std::max(1, std::min(4, std::atoi(e)));
}
}  // namespace

// row splits of the pipelined column kernel: XDOT_CSPLIT=n only (opt-in)
extern "C" int xdot_flash_cols_splits_cols2(const xdot::fa::BwdArgs* a, int dt, int D, int* sq) {
  using namespace xdot;
  using namespace xdot::fa;
  *sq = 1;
  const int NRT = (a->R + 63) / 64;
  const int e = cols2_csplit_env();
  if (e >= 0) {
    *sq = (NRT + 1) / 2 / e >= 1 ? e : 1;
    return 0;
  }
  // automatic choice: none.  Measured on MI355X (profiles/r5_fp32.md §2b): T = R = 25000, h = 8
  // 3.68 -> 3.49 ms for the kernel, but the fp32 partials (3 x 154 MB written and read back)
  // cost more than that in the step (7.84 -> 8.08 ms); at the N=8 rank shape 0.51 -> 0.71 ms.
  // The tail workgroups of this short kernel run faster alone than the round model assumes.
  (void)dt;
  (void)D;
  return 0;
}
