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

// The launch may carry a packed mask; without one every wave still issues the two per-tile mask
// DMAs as placeholders (a mask-less instantiation without them measured 5 % slower:
// profiles/r2_fwd_issue_budget.md).
template <int DT, int D, bool PS = false>
__global__ __launch_bounds__(256, 2) void flash_fwd_kernel(FwdArgs a) {
  constexpr bool MK = true;
  using T16 = typename dt_traits<DT>::T;
  using CF = RowsCfg<D>;
  constexpr int IMG = CF::IMG;  // ring of 3 stages (the pipelined loop reads two of them)
  constexpr int KS = D / 16;      // k-steps over the head dim
  constexpr int DB = D / 32;      // 32-wide d blocks of the output


  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: keeps wave-derived flags in SGPRs
  const Lanes L = make_lanes<D>(lane);
  const int nrb = (a.R + 127) / 128;
  int rbl, sp, ns, tail = -1;  // linear row block (bh * nrb + rb), column piece, pieces of this block
  if (a.xrbs > 0) {
    // head-heavy grid: XCD x runs its row blocks whole, then its last xrem split in nsplit
    // column pieces (compact partial index `tail`), so its last round of 64 slots is full
    const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
    if (k < a.xwhole) {
      rbl = x * a.xrbs + k;
      sp = 0;
      ns = 1;
    } else {
      const int p = k - a.xwhole, j = p / a.nsplit;
      rbl = x * a.xrbs + a.xwhole + j;
      sp = p - j * a.nsplit;
      ns = a.nsplit;
      tail = x * a.xrem + j;
    }
  } else {
    const int lin = xcd_remap(blockIdx.x, gridDim.x);
    rbl = lin % (nrb * a.B * a.H);
    sp = lin / (nrb * a.B * a.H);
    ns = a.nsplit;
  }
  const int rb = rbl % nrb, bh = rbl / nrb;
  const int b = bh / a.H, h = bh % a.H;
  const int C = a.H * D;
  const int NKT = (a.T + 63) / 64;
  const int kt_beg = (int)((int64_t)sp * NKT / ns), kt_end = (int)((int64_t)(sp + 1) * NKT / ns);
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
  const int ldb = a.ldkv * 2;  // gathered row stride, bytes
  ImgDma<D> dma;
  dma.init(wave, lane, ldb);
  const char* kcb = reinterpret_cast<const char*>(reinterpret_cast<const T16*>(a.kc) + h * D + (int64_t)b * a.T * a.ldkv);
  const char* vcb = reinterpret_cast<const char*>(reinterpret_cast<const T16*>(a.vc) + h * D + (int64_t)b * a.T * a.ldkv);
  const uint64_t* mwg = a.mbits ? a.mbits + (int64_t)b * NKT * a.R + rb * 128 : nullptr;  // + kt * R per tile
  const uint32_t moff = (uint32_t)(min((wave & 1) * 64 + lane, a.R - 1 - rb * 128) * 8 + (wave >> 1) * 4);
  // two rings over the same 3 stages: Q(t) + mask words(t) and V(t) go to stage (t - kt_beg) % 3,
  // but Q/mask are DMA'd one tile earlier than V (Q(kt+1) is read in iteration kt)
  constexpr int NQ = ImgDma<D>::IPW + (MK ? 2 : 0), NV = ImgDma<D>::IPW;  // DMAs per wave
  const int NKT4 = (NKT + 3) & ~3;
  const int NRB32 = (a.R + 31) / 32;
  const uint8_t* fwg = (MK && a.mflags) ? a.mflags + ((int64_t)b * NRB32 + rb * 4) * NKT4 : nullptr;
  const int fn = min(4, NRB32 - rb * 4);
  // Q and V tiles are issued strictly in order: running byte offsets (no per-tile 64-bit
  // products) and ring stages that are compile-time constants at every call site
  int64_t q_off = (int64_t)kt_beg * 64 * ldb, v_off = q_off;
  const uint64_t* mw_next = mwg ? mwg + (int64_t)kt_beg * a.R : nullptr;
  auto issue_q = [&](int kt, auto stc) {
    char* st = smem + decltype(stc)::value * CF::STAGE;
    dma.issue(kcb + q_off, ldb, a.T - 1 - kt * 64, st, wave);  // columns past T re-read T-1 (masked)
    q_off += (int64_t)64 * ldb;
    if constexpr (MK) {
      if (mwg) {
        glds4(mw_next, moff, st + CF::OFF_W + (wave >> 1) * 512 + (wave & 1) * 256);
        mw_next += a.R;
        glds_flags(fwg, NKT4, fn, kt >> 2, st + CF::OFF_F);
      } else {  // same DMA count with or without a mask
        glds4(kcb, (uint32_t)lane * 4, st + CF::OFF_X);
        glds4(kcb, (uint32_t)lane * 4, st + CF::OFF_X);
      }
    }
  };
  auto issue_v = [&](int kt, auto stc) {
    char* st = smem + decltype(stc)::value * CF::STAGE;
    dma.issue(vcb + v_off, ldb, a.T - 1 - kt * 64, st + IMG, wave);
    v_off += (int64_t)64 * ldb;
  };

  const float c2 = a.scale * LOG2E;
  const float NEG_INF = -__builtin_inff();
  float m_run = NEG_INF, l_run = 0.f;
  // PS: K rows pre-multiplied by scale*log2 e on the host (FwdArgs::prescaled; one bf16
  // rounding, the same buffer the backward reads) and every score chain seeded
  // with -m (the running max it will be exponentiated against), so P = 2^acc with no per-score
  // FMA.  m_seed is the m encoded in mseed; a (rare, deferred) max update corrects the pending
  // tile by m_seed - m_new and re-seeds.
  f32x16 mseed;
#pragma unroll
  for (int r = 0; r < 16; ++r) mseed[r] = 0.f;
  float m_seed = 0.f;
  f32x16 o[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;


  // ---- software-pipelined sweep ----------------------------------------------------
  // Iteration kt overlaps the MFMAs of one tile with the VALU work of another:
  //   block A: Sᵀ(kt+1) = Q(kt+1)·Kᵀ (12 MFMAs)   ||  P(kt) = 2^(S(kt)·c2 - m), packed to bf16
  //   block B: Oᵀ += V(kt)ᵀ·P(kt)ᵀ (12 MFMAs)     ||  row sums of P(kt)
  // then the row max of S(kt+1) and the (rare, deferred) rescale for tile kt+1 (moving the max
  // into block B's MFMA gaps measured 1.5 % slower: profiles/r2_sched_variants.md).  The score registers alternate between
  // two sets (PAR) and the ring stage rotates over three (BUF): the loop is unrolled by 6 so
  // both are compile-time.  Iteration kt DMAs Q(kt+3) and V(kt+2): each has one full
  // iteration in flight before the wait at the bottom of the next one.
  constexpr float RESCALE_LOG2 = 8.f;  // deferred max: p <= 2^8 between rescales (exact in fp32 / bf16)
  f32x16 sv[2][2];
  // flag of tile kt from the stage holding Q(kt) (1 = skip: wave past R / past the split)
  auto flag_of = [&](int kt, const char* st) -> int {
    if (r0 >= a.R || kt >= kt_end) return 1;
    return fwg ? staged_flag(st + CF::OFF_F, wave, kt & 3) : 0;
  };
  auto s_tile = [&](f32x16 (&s)[2], const char* qs) {
    u32x4 qa = row_frag<D>(qs, 0, 0, L);
#pragma unroll
    for (int i = 0; i < 2 * KS; ++i) {
      const int tt = i / KS, ks = i % KS;
      u32x4 qn = qa;
      if (i + 1 < 2 * KS) qn = row_frag<D>(qs, ((i + 1) / KS) * 32, (i + 1) % KS, L);
      s[tt] = mfma32<DT>::run(qa, kf[ks], ks == 0 ? (PS ? mseed : f32x16{}) : s[tt]);
      qa = qn;
    }
  };
  // mask (partial words / tail columns) or blank (fully masked) a score tile in place
  auto mask_tile = [&](f32x16 (&s)[2], int kt, int flag, const char* st) {
    if (flag == 1) {
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int r = 0; r < 16; ++r) s[tt][r] = NEG_INF;
      return;
    }
    const uint64_t w = tile_bits(flag == 2 ? staged_word(st + CF::OFF_W, wave * 32 + (lane & 31)) : 0ull,
                                 a.T - kt * 64, hf);
    sel_bits16(s[0], (uint32_t)w, NINF_BITS);
    sel_bits16(s[1], (uint32_t)(w >> 32), NINF_BITS);
  };
  // four independent v_max3 chains of 8 scores, then their max: dependency depth 6 instead of
  // one 16-deep chain (this runs between the PV MFMAs and the tile barrier, outside any MFMA gap)
  auto row_max = [&](const f32x16 (&s)[2]) {
    float mc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const f32x16& v = s[c >> 1];
      const int o = (c & 1) * 8;
      float m = fmaxf(fmaxf(v[o], v[o + 1]), v[o + 2]);
      m = fmaxf(fmaxf(m, v[o + 3]), v[o + 4]);
      m = fmaxf(fmaxf(m, v[o + 5]), v[o + 6]);
      mc[c] = fmaxf(m, v[o + 7]);
    }
    const float mx = fmaxf(fmaxf(mc[0], mc[1]), fmaxf(mc[2], mc[3]));
    return PS ? pair_max(mx) + m_seed : pair_max(mx) * c2;
  };
  // s: the tile whose max is mx (exponentiated next; PS: corrected to the new m)
  auto rescale_to = [&](float mx, f32x16 (&s)[2]) {
    const float m_new = fmaxf(m_run, mx);
    if (__any(m_new > m_run + RESCALE_LOG2)) {
      const float alpha = fast_exp2(m_run - ((m_new == NEG_INF) ? 0.f : m_new));
      l_run *= alpha;
#pragma unroll
      for (int i = 0; i < DB; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
      m_run = m_new;
      if constexpr (PS) {
        const float mu = (m_run == NEG_INF) ? 0.f : m_run;
        const float corr = m_seed - mu;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 16; ++r) s[tt][r] += corr;
        m_seed = mu;
#pragma unroll
        for (int r = 0; r < 16; ++r) mseed[r] = -mu;
      }
    }
  };

  int flag_cur = 1;
  auto iter = [&](auto bufc, auto parc, int kt) {
    constexpr int BUF = decltype(bufc)::value, PAR = decltype(parc)::value;
    f32x16 (&sc)[2] = sv[PAR];
    f32x16 (&sn)[2] = sv[PAR ^ 1];
    const bool dq = kt + 3 < kt_end, dv = kt + 2 < kt_end;
    if (dq) issue_q(kt + 3, std::integral_constant<int, BUF>{});            // stage (BUF + 3) % 3
    if (dv) issue_v(kt + 2, std::integral_constant<int, (BUF + 2) % 3>{});
    const char* cur = smem + BUF * CF::STAGE;             // V(kt)
    const char* nxt = smem + ((BUF + 1) % 3) * CF::STAGE; // Q(kt+1), mask words (kt+1)
    // flag(kt) was read one iteration ago (its stage is being refilled with Q(kt+3) now)
    const int flag_c = flag_cur, flag_n = flag_of(kt + 1, nxt);
    flag_cur = flag_n;
    if (flag_c != 1 || flag_n != 1) {
      const float m_use = (m_run == NEG_INF) ? 0.f : m_run;
      // ---- block A: S(kt+1) MFMAs, each followed by its share of P(kt) = 2^(S·c2 - m) ----
      // Written in issue order and fenced with sched_barrier so the compiler keeps the MFMA /
      // VALU interleave (it otherwise clusters the MFMAs); operand reads run two MFMAs ahead.
      constexpr int NA = 2 * KS, NB = 4 * DB;
      // D >= 96: block A's gaps cannot hold all 32 exps (2.67 v_exp + 1.33 cvt + a row read per
      // 32-cycle MFMA gap is ~39 issue cycles): the exps of P's last 8 columns (pf[3]) move into
      // block B, whose MFMAs run k-step-major so pf[3] is first needed at MFMA 3*DB >= 9
      constexpr int NX = DB >= 3 ? 8 : 0, JA = 32 - NX;
      // blocks A and B at raised issue priority, the row-max / rescale tail below at 0: a partner
      // wave's MFMA blocks then win the SIMD over this wave's tail (step -0.5 %, profiles/r6_fp32.md)
      __builtin_amdgcn_s_setprio(1);
      u32x4 pf[4];
      auto p_of = [&](int j) {
        sc[j >> 4][j & 15] = PS ? fast_exp2(sc[j >> 4][j & 15]) : fast_exp2(__builtin_fmaf(sc[j >> 4][j & 15], c2, -m_use));
        if ((j & 7) == 7) pf[j >> 3] = acc_to_frag<DT>(sc[j >> 4], (j >> 3) & 1);
      };
      {
        u32x4 q0 = row_frag<D>(nxt, 0, 0, L), q1 = row_frag<D>(nxt, (1 / KS) * 32, 1 % KS, L);
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const int tt = i / KS, ks = i % KS;
          u32x4 q2 = q1;
          if (i + 2 < NA) q2 = row_frag<D>(nxt, ((i + 2) / KS) * 32, (i + 2) % KS, L);
          sn[tt] = mfma32<DT>::run(q0, kf[ks], ks == 0 ? (PS ? mseed : f32x16{}) : sn[tt]);
#pragma unroll
          for (int j = (i * JA) / NA; j < ((i + 1) * JA) / NA; ++j) p_of(j);
          __builtin_amdgcn_sched_barrier(0);
          q0 = q1;
          q1 = q2;
        }
      }
      // ---- block B: P(kt)·V(kt) MFMAs, each followed by its share of the row sums (scalar
      // adds: packed v_pk_add_f32 pairs measured 0.5-3 % slower beside the MFMAs) ----
      float ls = 0.f;
      {
        // MFMA i of block B: (k-step, d block) = d-block-major, or k-step-major when NX > 0
        auto kb_of = [&](int i) { return NX ? i / DB : (i & 3); };
        auto db_of = [&](int i) { return NX ? i % DB : (i >> 2); };
        u32x4 v0 = tr_frag<D>(cur + IMG, kb_of(0) * 16, db_of(0) * 32, L);
        u32x4 v1 = tr_frag<D>(cur + IMG, kb_of(1) * 16, db_of(1) * 32, L);
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const int db = db_of(i), k4 = kb_of(i);
          u32x4 v2 = v1;
          if (i + 2 < NB) v2 = tr_frag<D>(cur + IMG, kb_of(i + 2) * 16, db_of(i + 2) * 32, L);
          o[db] = mfma32<DT>::run(v0, pf[k4], o[db]);
          if (i < NX) p_of(JA + i);
          // row sums: columns < JA spread over every gap, the moved ones after their exps
#pragma unroll
          for (int j = (i * JA) / NB; j < ((i + 1) * JA) / NB; ++j) ls += sc[j >> 4][j & 15];
          if (NX && i >= NX) {
#pragma unroll
            for (int j = JA + ((i - NX) * NX) / (NB - NX); j < JA + ((i - NX + 1) * NX) / (NB - NX); ++j)
              ls += sc[j >> 4][j & 15];
          }
          asm volatile("" : "+v"(ls));  // keeps the adds here (LLVM would sink them past the branch)
          __builtin_amdgcn_sched_barrier(0);
          v0 = v1;
          v1 = v2;
        }
      }
      l_run += ls;
      __builtin_amdgcn_s_setprio(0);
      if (flag_n != 0 || (kt + 2) * 64 > a.T) mask_tile(sn, kt + 1, flag_n, nxt);
      rescale_to(row_max(sn), sn);
    } else {
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int r = 0; r < 16; ++r) sn[tt][r] = NEG_INF;
    }
    // Q(kt+2) and V(kt+1) (issued one iteration ago) complete; this iteration's DMAs fly on
    if (dq) wait_vm<NQ + NV>();
    else if (dv) wait_vm<NV>();
    else wait_vm<0>();
    raw_barrier();
  };

  if (kt_beg < kt_end) {
    issue_q(kt_beg, std::integral_constant<int, 0>{});
    issue_v(kt_beg, std::integral_constant<int, 0>{});
    if (kt_beg + 1 < kt_end) {
      issue_q(kt_beg + 1, std::integral_constant<int, 1>{});
      issue_v(kt_beg + 1, std::integral_constant<int, 1>{});
    }
    if (kt_beg + 2 < kt_end) issue_q(kt_beg + 2, std::integral_constant<int, 2>{});
    wait_vm<0>();
    raw_barrier();
    // prologue: S of the first tile, masked, its max sets m
    const int f0 = flag_of(kt_beg, smem);
    flag_cur = f0;
    if (f0 != 1) s_tile(sv[0], smem);
    if (f0 != 0 || (kt_beg + 1) * 64 > a.T) mask_tile(sv[0], kt_beg, f0, smem);
    rescale_to(row_max(sv[0]), sv[0]);
  }
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  for (int kt = kt_beg; kt < kt_end; kt += 6) {
    iter(I0{}, I0{}, kt);
    if (kt + 1 < kt_end) iter(I1{}, I1{}, kt + 1);
    if (kt + 2 < kt_end) iter(I2{}, I0{}, kt + 2);
    if (kt + 3 < kt_end) iter(I0{}, I1{}, kt + 3);
    if (kt + 4 < kt_end) iter(I1{}, I0{}, kt + 4);
    if (kt + 5 < kt_end) iter(I2{}, I1{}, kt + 5);
  }

  // ---- epilogue ----
  const float l_tot = pair_sum(l_run);
  const float inv = 1.f / l_tot;
  if (row_ok && ns == 1 && !a.force_partial) {
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
  } else if (row_ok && tail >= 0) {
    // head-heavy tail piece: compact partial, merged by flash_fwd_combine_tail
    const int64_t pi = ((int64_t)sp * 8 * a.xrem + tail) * 128 + (row - rb * 128);
    float* op = a.opart + pi * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 v = {o[db][4 * g] * inv, o[db][4 * g + 1] * inv, o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv};
        *reinterpret_cast<f32x4*>(op + db * 32 + 8 * g + 4 * hf) = v;
      }
    if (hf == 0) a.lpart[pi] = (m_run + __log2f(l_tot)) * LN2;
  } else if (row_ok) {
    // split partial: normalised fp32 output + its LSE; merged by flash_fwd_combine
    float* op = a.opart + (((int64_t)(a.sp0 + sp) * a.B + b) * a.R + row) * C + h * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 v = {o[db][4 * g] * inv, o[db][4 * g + 1] * inv, o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv};
        *reinterpret_cast<f32x4*>(op + db * 32 + 8 * g + 4 * hf) = v;
      }
    if (hf == 0) a.lpart[(((int64_t)(a.sp0 + sp) * a.B + b) * a.H + h) * a.R + row] = (m_run + __log2f(l_tot)) * LN2;
  }
}

// merge column-split partials: lse = log Σ_s e^{lse_s}, O = Σ_s e^{lse_s - lse} O_s.
// A split that saw only masked columns has lse_s = -inf and contributes nothing; a row with
// every split -inf is fully masked and yields NaN like the unsplit kernel.
constexpr int CMB_MAX = 16;  // slots merged with all loads in flight (more: a per-slot loop)

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
  const int64_t ostride = (int64_t)a.B * a.R * C;
  const float* opp = a.opart + br * C + c4 * 4;
  float mx = -__builtin_inff(), sum = 0.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (a.nsplit <= CMB_MAX) {
    // every slot's LSE and 16-byte partial in flight at once (the loop below waits per slot)
    float l[CMB_MAX];
    f32x4 v[CMB_MAX];
#pragma unroll
    for (int s = 0; s < CMB_MAX; ++s) {
      l[s] = s < a.nsplit ? lp[s * lstride] : -__builtin_inff();
      v[s] = s < a.nsplit ? *reinterpret_cast<const f32x4*>(opp + s * ostride) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int s = 0; s < CMB_MAX; ++s) mx = fmaxf(mx, l[s]);
#pragma unroll
    for (int s = 0; s < CMB_MAX; ++s) {
      // a split that saw only masked columns wrote NaN (0 / 0): selected out, not multiplied by 0
      const bool live = l[s] != -__builtin_inff();
      const float wgt = live ? __expf(l[s] - mx) : 0.f;
      const f32x4 t = wgt * v[s];
      sum += wgt;
      acc += live ? t : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  } else {
    for (int s = 0; s < a.nsplit; ++s) mx = fmaxf(mx, lp[s * lstride]);
    for (int s = 0; s < a.nsplit; ++s) {
      const float l = lp[s * lstride];
      if (l == -__builtin_inff()) continue;
      const float wgt = __expf(l - mx);
      sum += wgt;
      const f32x4 v = *reinterpret_cast<const f32x4*>(opp + s * ostride);
      acc += wgt * v;
    }
  }
  const float inv = 1.f / sum;  // sum == 0 (fully masked row) -> NaN output, -inf lse
  if (a.out32) {  // running fp32 merge (ring attention): masked-so-far rows stay 0 / -inf
    *reinterpret_cast<f32x4*>(a.out32 + br * C + c4 * 4) = sum == 0.f ? f32x4{0.f, 0.f, 0.f, 0.f} : acc * inv;
    if ((c4 * 4) % D == 0) a.lse[((int64_t)b * a.H + h) * a.R + row] = sum == 0.f ? -__builtin_inff() : mx + __logf(sum);
    return;
  }
  T16* op = reinterpret_cast<T16*>(a.out) + br * C + c4 * 4;
  u32x2 w;
  w[0] = pack2<DT>(acc[0] * inv, acc[1] * inv);
  w[1] = pack2<DT>(acc[2] * inv, acc[3] * inv);
  if (sum == 0.f) { w[0] = pack2<DT>(__builtin_nanf(""), __builtin_nanf("")); w[1] = w[0]; }
  *reinterpret_cast<u32x2*>(op) = w;
  if ((c4 * 4) % D == 0) a.lse[((int64_t)b * a.H + h) * a.R + row] = mx + __logf(sum);
}

// merge the head-heavy grid's split tail blocks (compact partials) into out / lse
template <int DT, int D>
__global__ __launch_bounds__(256) void flash_fwd_combine_tail(FwdArgs a) {
  using T16 = typename dt_traits<DT>::T;
  const int ntail = 8 * a.xrem;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)ntail * 128 * (D / 4)) return;
  const int c4 = (int)(idx % (D / 4));
  const int tr = (int)(idx / (D / 4));
  const int rloc = tr & 127, t = tr >> 7;
  const int nrb = (a.R + 127) / 128;
  const int rbl = (t / a.xrem) * a.xrbs + a.xwhole + t % a.xrem;
  const int rb = rbl % nrb, bh = rbl / nrb, b = bh / a.H, h = bh % a.H;
  const int row = rb * 128 + rloc;
  if (row >= a.R) return;
  const int64_t pstride = (int64_t)ntail * 128, p0 = (int64_t)t * 128 + rloc;
  float mx = -__builtin_inff(), sum = 0.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float l[16];
  f32x4 v[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    l[s] = s < a.nsplit ? a.lpart[s * pstride + p0] : -__builtin_inff();
    v[s] = s < a.nsplit ? *reinterpret_cast<const f32x4*>(a.opart + (s * pstride + p0) * D + 4 * c4)
                        : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int s = 0; s < 16; ++s) mx = fmaxf(mx, l[s]);
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const bool live = l[s] != -__builtin_inff();
    const float wgt = live ? __expf(l[s] - mx) : 0.f;
    const f32x4 tv = wgt * v[s];
    sum += wgt;
    acc += live ? tv : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const float inv = 1.f / sum;  // fully masked row: NaN output, -inf lse
  T16* op = reinterpret_cast<T16*>(a.out) + ((int64_t)b * a.R + row) * (a.H * D) + h * D + 4 * c4;
  u32x2 w;
  w[0] = pack2<DT>(acc[0] * inv, acc[1] * inv);
  w[1] = pack2<DT>(acc[2] * inv, acc[3] * inv);
  if (sum == 0.f) { w[0] = pack2<DT>(__builtin_nanf(""), __builtin_nanf("")); w[1] = w[0]; }
  *reinterpret_cast<u32x2*>(op) = w;
  if (c4 == 0) a.lse[((int64_t)b * a.H + h) * a.R + row] = mx + __logf(sum);
}

template <int DT, int D>
static void launch_combine(const FwdArgs& a, hipStream_t st) {
  const int64_t n = (int64_t)a.B * a.R * (a.H * D / 4);
  hipLaunchKernelGGL((flash_fwd_combine<DT, D>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
}

// 32 rows per wave: a 64-row-per-wave variant (two sub-blocks sharing every operand read)
// measured 2 % faster at R = 25000 and 6 % slower at R = 3125 (256-row blocks leave more of
// the last block empty), so the pipelined 32-row kernel is the one kept.
template <int DT, int D>
static void launch_fwd(const FwdArgs& a, hipStream_t st) {
  constexpr int LDS = 3 * RowsCfg<D>::STAGE;
  const int nrb = (a.R + 127) / 128;
  const dim3 grid(a.xrbs > 0 ? 8 * (a.xwhole + a.xrem * a.nsplit) : nrb * a.B * a.H * a.nsplit);
  if (a.prescaled) hipLaunchKernelGGL((flash_fwd_kernel<DT, D, true>), grid, dim3(256), LDS, st, a);
  else hipLaunchKernelGGL((flash_fwd_kernel<DT, D>), grid, dim3(256), LDS, st, a);
  if (a.xrbs > 0) {
    const int64_t n = (int64_t)8 * a.xrem * 128 * (D / 4);
    if (a.xrem > 0) hipLaunchKernelGGL((flash_fwd_combine_tail<DT, D>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
  } else if (a.nsplit > 1 && !a.force_partial) {
    launch_combine<DT, D>(a, st);
  }
}

}  // namespace fa
}  // namespace xdot

// rows per workgroup of the forward kernel (grid / split planning on the host)
extern "C" int xdot_flash_fwd_rows_per_wg() { return 128; }

// merge a->nsplit partial slots of opart/lpart into out/lse
extern "C" int xdot_flash_fwd_combine_launch(const xdot::fa::FwdArgs* a, int dt, int D, hipStream_t st) {
  using namespace xdot;
  using namespace xdot::fa;
  if (a->R == 0 || a->B == 0 || a->H == 0) return 0;
  if (dt == DT_F32 && !a->out32) return xdot_flash_combine_f32_launch(a, D, st);
#define XF(DTV, DV) if (dt == DTV && D == DV) { launch_combine<DTV, DV>(*a, st); return 0; }
  XF(DT_BF16, 32) XF(DT_BF16, 64) XF(DT_BF16, 96) XF(DT_BF16, 128)
  XF(DT_F16, 32) XF(DT_F16, 64) XF(DT_F16, 96) XF(DT_F16, 128)
  XF(DT_BF16, 160) XF(DT_BF16, 192) XF(DT_BF16, 256) XF(DT_BF16, 384)  // wide heads (flash_wide.hip)
  XF(DT_F16, 160) XF(DT_F16, 192) XF(DT_F16, 256) XF(DT_F16, 384)
#undef XF
  return -1;
}

extern "C" int xdot_flash_fwd_launch(const xdot::fa::FwdArgs* a, int dt, int D, hipStream_t st) {
  using namespace xdot;
  using namespace xdot::fa;
  if (a->R == 0 || a->B == 0 || a->H == 0) return 0;
  if (D > 128) {  // wide heads: csrc/flash_wide.hip (fp32: always exact)
    const int rc = xdot_flash_wide_fwd_launch(a, dt, D, st);
    if (rc == 0 && a->nsplit > 1 && !a->force_partial) {
      if (dt == DT_F32) return xdot_flash_combine_f32_launch(a, D, st);
      return xdot_flash_fwd_combine_launch(a, dt, D, st);
    }
    return rc;
  }
  if (dt == DT_F32) {
    const int rc = a->fp32_mode ? xdot_flash_fwd_x3_launch(a, D, st) : xdot_flash_fwd_f32_launch(a, D, st);
    if (rc == 0 && a->nsplit > 1 && !a->force_partial) return xdot_flash_combine_f32_launch(a, D, st);
    return rc;
  }
#define XF(DTV, DV) if (dt == DTV && D == DV) { launch_fwd<DTV, DV>(*a, st); return 0; }
  XF(DT_BF16, 32) XF(DT_BF16, 64) XF(DT_BF16, 96) XF(DT_BF16, 128)
  XF(DT_F16, 32) XF(DT_F16, 64) XF(DT_F16, 96) XF(DT_F16, 128)
#undef XF
  return -1;
}
