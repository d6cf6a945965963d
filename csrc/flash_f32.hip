// xdot — fp32 flash attention (forward + both backward kernels) for gfx950 (MI355X).
//
// The reference computes the module in fp32 only (distributed_dot_product/module.py:60-71 on
// the fp32 buffers of multiplication/functions.py:86,198).  The 16-bit kernels in
// flash_fwd.hip / flash_bwd.hip would round fp32 operands to 8 significant bits; these kernels
// keep every product exact in fp32 with v_mfma_f32_32x32x2_f32 (an fmaf chain, 64 FLOP/clk/SIMD
// = the fp32 vector rate, 1/16 of bf16), so an fp32 module never falls back to materialising
// the (B, H, R, T) scores (20 GB per tensor at T = 25000, impossible at T = 200000).
//
// Same decomposition, layouts, masks and partial/combine protocol as the 16-bit kernels
// (rows = this rank's R query-side rows, cols = the T gathered key/value rows, head-interleaved
// (B, ·, H*D) tensors, packed masks from mask_pack.hip), restructured for the f32 MFMA:
//   * 32x32x2: lane l of the A operand holds A[l&31][l>>5], of B B[l>>5][l&31]; the C/D map
//     is the 32x32x16 one (lane = column l&31, register r = row (r&3)+8(r>>2)+4(l>>5)), so the
//     transposed-score trick of the 16-bit kernels carries over: softmax rows stay lane-local;
//   * the K index of a product over the head dim is permuted so that every lane fetches four
//     consecutive floats with ONE ds_read_b128 per four MFMAs (MFMA 4g+t, lane half h, uses
//     d = 8g + 4h + t, for the LDS image AND the register-resident fragments);
//   * a product over a 32-row/column tile index takes its B operand straight from the previous
//     product's accumulator register (MFMA s uses tile index (s&3)+8(s>>2)+4h = register s's
//     row) and its A operand with one ds_read_b32 from the image, read "transposed";
//   * images are 32 rows x (D + 4) floats: the 4-float pad makes the 16-lane ds_read_b128
//     groups conflict-free ((D+4)/4 odd);
//   * 32-row tiles staged global -> VGPR -> LDS one tile ahead (double-buffered LDS, one
//     barrier per tile): at 64+ MFMA cycles per 64-bit of operand this kernel family is MFMA
//     bound, so the simple staging costs nothing measurable.
//
// Score-buffer mode (FwdArgs/BwdArgs::sbuf).  In fp32 a product costs 2*D FLOP per score at the
// fp32 matrix rate (~131 TF/s): 1.47 ps per score at D = 96, while writing and re-reading the
// score costs 8 bytes of HBM traffic (~1.6 ps at 5 TB/s) that the MFMA-bound kernels leave idle.
// So the backward reads what the forward already computed instead of recomputing it:
//   forward      stores the raw S of every computed 32x32 tile (1 extra store pass, 0 products)
//   column side  loads S (no S product), computes dP, dV, dQ and overwrites the block with dS
//   row side     loads dS: dK = dS · Q is its ONLY product (no S, no dP recompute)
// 6 products per step instead of 9; the S / dS values are bit-identical to the recomputed ones
// (same MFMA chains), so results do not change.  Blocks are (B*H, ceil(R/32), ceil(T/32)) x
// 1024 floats; within a block a tile sits in the READER's accumulator order (16 floats per lane,
// 4 x b128 loads), the writer scatters (blk_store).  Tiles the mask flags skip are neither
// written nor read.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "flash_common.h"

namespace xdot {
namespace fa32 {

using fa::FwdArgs;
using fa::BwdArgs;
using fa::LOG2E;
using fa::LN2;
using fa::pair_max;
using fa::pair_sum;
using fa::tidx;
using fa::flag_at;
using fa::blk_store;
using fa::blk_store_lds;
using fa::blk_load;

__device__ __forceinline__ f32x16 mm(float a, float b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

template <int D> struct Cfg {
  static constexpr int P = D + 4;       // image row stride (floats)
  static constexpr int NPC = (32 * P * 4 + 1023) / 1024;  // 1-KiB LDS-DMA pieces of one image
  static constexpr int IMG = NPC * 256; // one 32-row image region (floats; >= 32 P, DMA slack at the end)
  static constexpr int KG = D / 8;      // b128 groups over the head dim (4 MFMAs each)
  static constexpr int DB = D / 32;     // 32-wide output blocks
  static constexpr int NC = D / 32;     // f32x4 chunks per thread per image (256 threads)
  static constexpr int AUX = 64;        // per-stage row constants (lse2, delta) of the column kernel
  static constexpr int STAGE = 2 * IMG + AUX;
};

// LDS-DMA staging of NI 32-row fp32 images with the same global row stride (HBM -> LDS with no
// VGPR round trip, no per-element LDS writes).  The padded image (rows of P floats) is filled
// linearly by 1-KiB pieces, wave w taking a contiguous run of them; each lane's 16 bytes map to
// (row, 16-byte chunk) of the image, the pad chunks and the slack past the last row load a valid
// dummy.  The kernels wait for the pieces (vmcnt(0)) before the tile's barrier.
template <int D, int NI> struct DmaStager {
  using CF = Cfg<D>;
  static constexpr int RB = CF::P * 4, NPC = CF::NPC, Q4 = NPC / 4, R4 = NPC % 4;
  static constexpr int MAXP = Q4 + (R4 ? 1 : 0);
  int off[MAXP], row[MAXP];
  int start, cnt;  // wave-uniform
  __device__ __forceinline__ void init(int wave, int lane, int ld_bytes) {
    cnt = Q4 + (wave < R4 ? 1 : 0);
    start = wave * Q4 + min(wave, R4);
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      const int p = (start + i) * 1024 + lane * 16;
      int r = p / RB, c = (p % RB) >> 4;
      if (r >= 32 || c >= D / 4) r = c = 0;
      row[i] = r;
      off[i] = r * ld_bytes + c * 16;
    }
  }
  // images k = 0..NI-1 of tile rows row0.. (rows past rmax re-read row rmax) from b[k] into
  // img + k * img_stride (floats)
  __device__ __forceinline__ void issue(const float* const* b, int64_t ld, int64_t row0, int rmax, float* img,
                                        int img_stride) const {
    uint32_t o[MAXP];
#pragma unroll
    for (int i = 0; i < MAXP; ++i) o[i] = (uint32_t)off[i];
    if (rmax < 31) {
#pragma unroll
      for (int i = 0; i < MAXP; ++i) o[i] = (uint32_t)(off[i] - (row[i] - min(row[i], rmax)) * (int)(ld * 4));
    }
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const char* base = reinterpret_cast<const char*>(b[k] + row0 * ld);
      const uint32_t lds =
          __builtin_amdgcn_readfirstlane(fa::lds_addr(reinterpret_cast<char*>(img + k * img_stride) + start * 1024));
      if constexpr (R4 == 0) {
        fa::GldsRun<Q4>::run(base, o, lds);
      } else {
        if (cnt == MAXP) fa::GldsRun<MAXP>::run(base, o, lds);
        else fa::GldsRun<MAXP - 1>::run(base, o, lds);
      }
    }
  }
};

// register-resident fragments of one 32-row block: f[4g + t] = X[row][8g + 4h + t]
template <int D>
__device__ __forceinline__ void load_frag(float (&f)[D / 2], const float* p, bool ok) {
#pragma unroll
  for (int g = 0; g < D / 8; ++g) {
    const f32x4 v = ok ? *reinterpret_cast<const f32x4*>(p + 8 * g) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) f[4 * g + t] = v[t];
  }
}

// acc += img rows (lane&31) · fragᵀ over the head dim (A from the image, B from registers).
// The image reads run one 4-MFMA group ahead, fenced by sched_barrier: with one wave per SIMD a
// read issued right before its MFMAs exposes the whole LDS latency.
template <int D>
__device__ __forceinline__ f32x16 rowprod(const float* img, const float (&f)[D / 2], f32x16 acc, int lane) {
  const float* p = img + (lane & 31) * Cfg<D>::P + 4 * (lane >> 5);
  __builtin_amdgcn_s_setprio(1);  // the MFMA block at raised priority (step -0.2 ms, profiles/r6_fp32.md)
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
  __builtin_amdgcn_s_setprio(0);
  return acc;
}

#ifndef XDOT_F32_TRPD
#define XDOT_F32_TRPD 1  // trprod operand read distance (tile indices ahead; A/B knob)
#endif
// out[db] += imgᵀ (d x tile index) · x (tile index x lane column), x = an accumulator tile
// (the A operands of tile index s+1 are read while the MFMAs of s issue)
template <int D>
__device__ __forceinline__ void trprod(const float* img, const f32x16& x, f32x16 (&out)[D / 32], int lane) {
  const int hf = lane >> 5;
  constexpr int DB = D / 32;
  // ring of PD + 1 operand sets: tile index s + PD is read while the MFMAs of s issue (the loop
  // is fully unrolled, so every ring slot is a compile-time register set)
  constexpr int PD = XDOT_F32_TRPD;
  __builtin_amdgcn_s_setprio(1);  // the MFMA block at raised priority (step -0.2 ms, profiles/r6_fp32.md)
  float rr[PD + 1][DB];
  auto rd = [&](int s, float (&dst)[DB]) {
    const float* row = img + ((s & 3) + 8 * (s >> 2) + 4 * hf) * Cfg<D>::P + (lane & 31);
#pragma unroll
    for (int db = 0; db < DB; ++db) dst[db] = row[db * 32];
  };
#pragma unroll
  for (int s = 0; s < PD; ++s) rd(s, rr[s]);
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    if (s + PD < 16) rd(s + PD, rr[(s + PD) % (PD + 1)]);
#pragma unroll
    for (int db = 0; db < DB; ++db) out[db] = mm(rr[s % (PD + 1)][db], x[s], out[db]);
    __builtin_amdgcn_sched_barrier(0);
  }
  __builtin_amdgcn_s_setprio(0);
}

// ------------------------------------------------------------------------------------------
// forward: 4 waves x 32 rows of one (b, h); sweeps 32-column tiles of its column split
// SS: store the raw scores into a.sbuf (score-buffer mode); SD (with SS): stored by direct 16-dword
// scatters (fa::blk_store) instead of through the wave-private LDS transpose tile: 16 KiB less LDS
// per workgroup, so three workgroups fit a CU (52.5 KiB each at D = 96) instead of two
template <int D, bool SS, bool SD = false>
__global__ __launch_bounds__(256, SD && D <= 96 ? 3 : 2) void fwd_kernel(FwdArgs a) {
  using CF = Cfg<D>;
  constexpr int DB = CF::DB;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nrb = (a.R + 127) / 128;
  int rbl, sp, ns, tail = -1;  // linear row block (bh * nrb + rb), column piece, pieces of this block
  if (a.xrbs > 0) {
    // head-heavy grid (as the 16-bit forward): XCD x = blockIdx % 8 runs its row blocks whole,
    // then splits only its last xrem blocks in nsplit column pieces (compact partials `tail`,
    // merged by combine_tail_kernel), so no uniform split pays partial writes and a full combine
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
  const int NKT64 = (a.T + 63) / 64, NKT32 = (a.T + 31) / 32;
  const int kt_beg = 2 * (int)((int64_t)sp * NKT64 / ns);
  const int kt_end = min(NKT32, 2 * (int)((int64_t)(sp + 1) * NKT64 / ns));
  const int r0 = rb * 128 + wave * 32, row = r0 + (lane & 31);
  const bool row_ok = row < a.R;
  const int NKT4 = (NKT64 + 3) & ~3, NRB32 = (a.R + 31) / 32;

  float kf[D / 2];
  load_frag<D>(kf, reinterpret_cast<const float*>(a.rows) + ((int64_t)b * a.R + (row_ok ? row : 0)) * C + h * D + 4 * hf,
               row_ok);
  const float* qb = reinterpret_cast<const float*>(a.kc) + (int64_t)b * a.T * a.ldkv + h * D;
  const float* vb = reinterpret_cast<const float*>(a.vc) + (int64_t)b * a.T * a.ldkv + h * D;
  const float c2 = a.scale * LOG2E, NEG_INF = -__builtin_inff();
  float m_run = NEG_INF, l_run = 0.f;
  f32x16 o[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) o[i] = f32x16{};
  // score buffer: this wave's row of 32x32 blocks (r0 < R: waves past R never store)
  // (waves past R write the dump block after the last one: every wave stores every tile, so the
  // store count per tile is uniform and the compiler's vmcnt waits stay exact)
  float* sbw = SS ? a.sbuf + (r0 < a.R ? ((int64_t)bh * NRB32 + (r0 >> 5)) * NKT32 * 1024 : fa::sb_dump(a.B, a.H, a.R, a.T))
                  : nullptr;
  const int64_t sbw_step = r0 < a.R ? 1024 : 0;

  DmaStager<D, 2> dm;
  dm.init(wave, lane, (int)(a.ldkv * 4));
  const float* const qvb[2] = {qb, vb};
  if (kt_beg < kt_end) {
    dm.issue(qvb, a.ldkv, (int64_t)kt_beg * 32, a.T - 1 - kt_beg * 32, sm, CF::IMG);
    fa::wait_vm<0>();
    __syncthreads();
  }
  float* const swl = sm + 2 * CF::STAGE + wave * 1024;  // S transpose tile (score buffer)
  for (int kt = kt_beg; kt < kt_end; ++kt) {
    const bool more = kt + 1 < kt_end;
    // the previous tile's S leaves first: its global stores then complete under this tile's
    // products instead of in the wait before its barrier (vmcnt counts stores too)
    if constexpr (SS && !SD) {
      if (kt > kt_beg) fa::blk_flush_lds(sbw + (int64_t)(kt - 1) * sbw_step, swl, lane);
    }
    if (more)  // into the stage the previous tile used (all reads of it ended at its barrier)
      dm.issue(qvb, a.ldkv, (int64_t)(kt + 1) * 32, a.T - 1 - (kt + 1) * 32, sm + ((kt + 1 - kt_beg) & 1) * CF::STAGE,
               CF::IMG);
    const float* qi = sm + ((kt - kt_beg) & 1) * CF::STAGE;
    const float* vi = qi + CF::IMG;
    int flag = r0 >= a.R ? 1 : (a.mflags ? flag_at(a.mflags, b, NRB32, NKT4, r0 >> 5, kt >> 1) : 0);
    flag = __builtin_amdgcn_readfirstlane(flag);
    f32x16 s{};
    if (flag != 1) s = rowprod<D>(qi, kf, f32x16{}, lane);  // Sᵀ: col (register) x row (lane)
    // raw S, every tile (skipped tiles store zeros nobody reads): LDS writes here, the transposed
    // global stores at the start of the next tile
    if constexpr (SS && !SD) fa::blk_put_lds(swl, s, lane);
    if constexpr (SS && SD) fa::blk_store(sbw + (int64_t)kt * sbw_step, s, lane);
    if (flag != 1) {
      const int valid = a.T - kt * 32;
      if (flag == 2 || valid < 32) {
        uint32_t w = 0;
        if (flag == 2 && row_ok) w = fa::settle((uint32_t)(a.mbits[((int64_t)b * NKT64 + (kt >> 1)) * a.R + row] >> (32 * (kt & 1))));
        // lane-half offset applied once: constant shifts / compares per register
        const uint32_t wh = w >> (4 * hf);
        const int vh = valid - 4 * hf;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int c = tidx(r, 0);
          if (((wh >> c) & 1u) || c >= vh) s[r] = NEG_INF;
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
      trprod<D>(vi, s, o, lane);  // Oᵀ += Vᵀ · Pᵀ
    }
    fa::wait_vm<0>();  // the next tile's pieces landed
    __syncthreads();
  }
  if constexpr (SS && !SD) {
    if (kt_end > kt_beg) fa::blk_flush_lds(sbw + (int64_t)(kt_end - 1) * sbw_step, swl, lane);
  }

  const float l_tot = pair_sum(l_run);
  const float inv = 1.f / l_tot;
  if (!row_ok) return;
  const float lse = (m_run + __log2f(l_tot)) * LN2;
  float* op;
  if (ns == 1 && !a.force_partial) {
    op = reinterpret_cast<float*>(a.out) + ((int64_t)b * a.R + row) * C + h * D;
    if (hf == 0) a.lse[((int64_t)b * a.H + h) * a.R + row] = lse;
  } else if (tail >= 0) {  // head-heavy tail piece: compact partial
    const int64_t pi = ((int64_t)sp * 8 * a.xrem + tail) * 128 + (row - rb * 128);
    op = a.opart + pi * D;
    if (hf == 0) a.lpart[pi] = lse;
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

// merge the head-heavy grid's split tail blocks (compact partials, fp32 out); see
// flash_fwd_combine_tail.  One thread per (tail row, 4 output columns).
__global__ __launch_bounds__(256) void combine_tail_kernel(FwdArgs a, int D) {
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
  for (int s = 0; s < a.nsplit; ++s) mx = fmaxf(mx, a.lpart[s * pstride + p0]);
  for (int s = 0; s < a.nsplit; ++s) {
    const float l = a.lpart[s * pstride + p0];
    if (l == -__builtin_inff()) continue;  // a piece that saw only masked columns (0 / 0 output)
    const float wgt = __expf(l - mx);
    sum += wgt;
    acc += wgt * *reinterpret_cast<const f32x4*>(a.opart + (s * pstride + p0) * D + 4 * c4);
  }
  const float inv = 1.f / sum;  // fully masked row: NaN output, -inf lse
  float* op = reinterpret_cast<float*>(a.out) + ((int64_t)b * a.R + row) * (a.H * D) + h * D + 4 * c4;
  *reinterpret_cast<f32x4*>(op) = sum == 0.f ? f32x4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""),
                                                     __builtin_nanf("")}
                                             : acc * inv;
  if (c4 == 0) a.lse[((int64_t)b * a.H + h) * a.R + row] = mx + __logf(sum);
}

// merge split partials (fp32 out); see flash_fwd_combine
__global__ __launch_bounds__(256) void combine_kernel(FwdArgs a, int D) {
  const int C = a.H * D;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)a.B * a.R * (C / 4);
  if (idx >= total) return;
  const int c4 = (int)(idx % (C / 4));
  const int64_t br = idx / (C / 4);
  const int row = (int)(br % a.R), b = (int)(br / a.R);
  const int h = (c4 * 4) / D;
  const int64_t lstride = (int64_t)a.B * a.H * a.R, ostride = (int64_t)a.B * a.R * C;
  const float* lp = a.lpart + ((int64_t)b * a.H + h) * a.R + row;
  float mx = -__builtin_inff();
  for (int s = 0; s < a.nsplit; ++s) mx = fmaxf(mx, lp[s * lstride]);
  float sum = 0.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* opp = a.opart + br * C + c4 * 4;
  for (int s = 0; s < a.nsplit; ++s) {
    const float l = lp[s * lstride];
    if (l == -__builtin_inff()) continue;
    const float wgt = __expf(l - mx);
    sum += wgt;
    acc += wgt * *reinterpret_cast<const f32x4*>(opp + s * ostride);
  }
  const float inv = 1.f / sum;  // fully masked row: NaN output, -inf lse (as the reference)
  f32x4 v = acc * inv;
  if (sum == 0.f) v = f32x4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
  *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.out) + br * C + c4 * 4) = v;
  if ((c4 * 4) % D == 0) a.lse[((int64_t)b * a.H + h) * a.R + row] = mx + __logf(sum);
}

// δ = rowsum(dO ⊙ O) (unless delta == nullptr) and lse2 = lse * log2 e, per (b, h, row)
__global__ __launch_bounds__(256) void prep_kernel(BwdArgs a, const float* out, float* delta, int D) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)a.B * a.R * a.H) return;
  const int h = (int)(idx % a.H);
  const int64_t br = idx / a.H;
  const int row = (int)(br % a.R), b = (int)(br / a.R);
  const int64_t li = ((int64_t)b * a.H + h) * a.R + row;
  if (a.lse2) a.lse2[li] = a.lse[li] * LOG2E;
  if (!delta) return;
  const float* o = out + br * (int64_t)(a.H * D) + h * D;
  const float* d = reinterpret_cast<const float*>(a.dout) + br * (int64_t)(a.H * D) + h * D;
  float acc = 0.f;
  for (int c = 0; c < D; c += 4) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(o + c), y = *reinterpret_cast<const f32x4*>(d + c);
    acc += x[0] * y[0] + x[1] * y[1] + x[2] * y[2] + x[3] * y[3];
  }
  delta[li] = acc;
}

// the same, 8 lanes per (b, row, h): each lane a contiguous D / 8 floats of O and dO (the wave reads
// 8 heads' rows contiguously), a 3-step xor reduction, lane 0 of the 8 writes (the one-thread-per-row
// form ran 170 us at T = R = 25000, H = 8: one thread streamed 2 x 384 B alone)
template <int D>
__global__ __launch_bounds__(256) void prep8_kernel(BwdArgs a, const float* out, float* delta) {
  constexpr int NV = D / 32;  // float4 per lane
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t pr = idx >> 3;  // (b, row, h) pair, h fastest
  const int sub = (int)(idx & 7);
  const int64_t npairs = (int64_t)a.B * a.R * a.H;
  const bool ok = pr < npairs;
  float acc = 0.f;
  if (ok) {
    const int64_t off = pr * D + sub * (D / 8);
    const f32x4* o = reinterpret_cast<const f32x4*>(out + off);
    const f32x4* d = reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(a.dout) + off);
    f32x4 x[NV], y[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      x[i] = o[i];
      y[i] = d[i];
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) acc += x[i][0] * y[i][0] + x[i][1] * y[i][1] + x[i][2] * y[i][2] + x[i][3] * y[i][3];
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
  delta[li] = acc;
}

// ------------------------------------------------------------------------------------------
// backward, row side: dK = scale · Σ_cols dS · Q_cols.  4 waves x 32 rows, column split.
template <int D>
__global__ __launch_bounds__(256, D >= 128 ? 1 : 2) void bwd_rows_kernel(BwdArgs a) {
  using CF = Cfg<D>;
  constexpr int DB = CF::DB;
  extern __shared__ __attribute__((aligned(16))) float sm[];
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

  float kf[D / 2], df[D / 2];
  {
    const int64_t off = ((int64_t)b * a.R + (row_ok ? row : 0)) * C + h * D + 4 * hf;
    load_frag<D>(kf, reinterpret_cast<const float*>(a.rows) + off, row_ok);
    load_frag<D>(df, reinterpret_cast<const float*>(a.dout) + off, row_ok);
  }
  const int64_t li = ((int64_t)b * a.H + h) * a.R + (row_ok ? row : 0);
  const float lse2 = row_ok ? a.lse[li] * LOG2E : 0.f, dlt = row_ok ? a.delta[li] : 0.f;
  const float* qb = reinterpret_cast<const float*>(a.kc) + (int64_t)b * a.T * a.ldkv + h * D;
  const float* vb = reinterpret_cast<const float*>(a.vc) + (int64_t)b * a.T * a.ldkv + h * D;
  const float c2 = a.scale * LOG2E, NEG_INF = -__builtin_inff();
  f32x16 dk[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) dk[i] = f32x16{};
  if constexpr (D >= 128) fa::pin_agpr(dk);  // one wave per SIMD: accumulators in AGPRs

  DmaStager<D, 2> dm;
  dm.init(wave, lane, (int)(a.ldkv * 4));
  const float* const qvb[2] = {qb, vb};
  if (kt_beg < kt_end) {
    dm.issue(qvb, a.ldkv, (int64_t)kt_beg * 32, a.T - 1 - kt_beg * 32, sm, CF::IMG);
    fa::wait_vm<0>();
    __syncthreads();
  }
  for (int kt = kt_beg; kt < kt_end; ++kt) {
    const bool more = kt + 1 < kt_end;
    if (more)  // into the stage the previous tile used (all reads of it ended at its barrier)
      dm.issue(qvb, a.ldkv, (int64_t)(kt + 1) * 32, a.T - 1 - (kt + 1) * 32, sm + ((kt + 1 - kt_beg) & 1) * CF::STAGE,
               CF::IMG);
    const float* qi = sm + ((kt - kt_beg) & 1) * CF::STAGE;
    const float* vi = qi + CF::IMG;
    int flag = r0 >= a.R ? 1 : (a.mflags ? flag_at(a.mflags, b, NRB32, NKT4, r0 >> 5, kt >> 1) : 0);
    flag = __builtin_amdgcn_readfirstlane(flag);
    if (flag != 1) {
      f32x16 s = rowprod<D>(qi, kf, f32x16{}, lane);   // Sᵀ  (col x row)
      f32x16 dp = rowprod<D>(vi, df, f32x16{}, lane);  // dPᵀ (col x row)
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
      trprod<D>(qi, s, dk, lane);  // dKᵀ += Q_colsᵀ · dSᵀ
      if constexpr (D >= 128) fa::pin_agpr(dk);
    }
    fa::wait_vm<0>();  // the next tile's pieces landed
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
// LS (score-buffer mode): S comes from a.sbuf (prefetched one tile ahead) instead of the
// K·Qᵀ product, each block is overwritten with dS / scale for the row kernel, and dV is left to
// bwd_cols_dv_kernel (run first): without the dV accumulators this dQ pass fits two waves per
// SIMD at D <= 96 (one wave per SIMD exposed every LDS / barrier stall: MFMA 54 % busy with both).
// DS (dS-only buffer mode, recompute kernel): S recomputed as without a buffer, dS stored into
// a.dsbuf for the row kernel (the split family's memory-bound mode: 40 GB of score traffic per
// step instead of 100)
// DV (with LS: the fused column pass, BwdArgs::sb_passes == 4): dV = Σ_rows Pᵀ · dO is accumulated here
// too, from the P this pass computes anyway -- three products per tile, S read once, no dV pass
template <int D, bool LS, bool DS = LS, bool DV = !LS>
__global__ __launch_bounds__(256, LS && D <= 96 ? 2 : 1) void bwd_cols_kernel(BwdArgs a) {
  using CF = Cfg<D>;
  constexpr int DB = CF::DB;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ncb = (a.T + 127) / 128;
  int cbl, sp, ns, tail = -1;  // linear column block (bh * ncb + cb), row piece, pieces of this block
  if (a.xcb > 0) {  // head-heavy grid (BwdArgs::xcb): whole blocks first, the XCD's last ones split
    const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
    if (k < a.xwhole) {
      cbl = x * a.xcb + k;
      sp = 0;
      ns = 1;
    } else {
      const int p = k - a.xwhole, j = p / a.csq;
      cbl = x * a.xcb + a.xwhole + j;
      sp = p - j * a.csq;
      ns = a.csq;
      tail = x * a.xrem + j;
    }
  } else {
    const int lin = xcd_remap(blockIdx.x, gridDim.x);
    cbl = lin % (ncb * a.B * a.H);
    sp = lin / (ncb * a.B * a.H);
    ns = a.csq > 1 ? a.csq : 1;
  }
  const int cb = cbl % ncb, bh = cbl / ncb;
  const int b = bh / a.H, h = bh % a.H;
  const int C = a.H * D;
  const int c0 = cb * 128 + wave * 32, col = c0 + (lane & 31);
  const bool col_ok = col < a.T;
  const int NKT64 = (a.T + 63) / 64, NKT4 = (NKT64 + 3) & ~3, NRB32 = (a.R + 31) / 32;
  const int NRT64 = (a.R + 63) / 64, TPAD = (a.T + 127) / 128 * 128;
  const int NRT = (a.R + 31) / 32, NKT32 = (a.T + 31) / 32;
  // row split sp of ns: row tiles [rt_beg, rt_end)
  const int rt_beg = (int)((int64_t)sp * NRT / ns), rt_end = (int)((int64_t)(sp + 1) * NRT / ns);

  float qf[LS ? 1 : D / 2], vf[D / 2];
  {
    const int64_t off = ((int64_t)b * a.T + (col_ok ? col : 0)) * a.ldkv + h * D + 4 * hf;
    if constexpr (!LS) load_frag<D>(qf, reinterpret_cast<const float*>(a.kc) + off, col_ok);
    load_frag<D>(vf, reinterpret_cast<const float*>(a.vc) + off, col_ok);
  }
  // score buffer column of this wave: block (bh, rt, c0/32) at sbc + rt * NKT32 * 1024
  const bool sown = DS && c0 < a.T;
  // loads of waves past T read a valid block, their dS stores go to the dump block: every wave
  // loads and stores every tile (uniform counts keep the compiler's vmcnt waits exact)
  float* sbc = LS ? a.sbuf + ((int64_t)bh * NRB32 * NKT32 + min(c0 >> 5, NKT32 - 1)) * 1024 : nullptr;
  float* dsc = DS ? (sown ? (a.dsbuf ? a.dsbuf : a.sbuf) + ((int64_t)bh * NRB32 * NKT32 + (c0 >> 5)) * 1024
                          : (a.dsbuf ? a.dsbuf : a.sbuf) + fa::sb_dump(a.B, a.H, a.R, a.T))
                  : nullptr;
  const int64_t dstep = sown ? (int64_t)NKT32 * 1024 : 0;
  const int64_t sstep = (int64_t)NKT32 * 1024;
  // S of the next tile prefetched into registers (the fused pass has no room for the second set:
  // it loads each tile's S at the tile's top, issued last, landing under the dP product)
  constexpr bool PF = LS && !DV;
  f32x16 snext{};
  if (PF && rt_beg < rt_end) snext = blk_load(sbc + rt_beg * sstep, lane);
  const float* kb = reinterpret_cast<const float*>(a.rows) + (int64_t)b * a.R * C + h * D;
  const float* db_ = reinterpret_cast<const float*>(a.dout) + (int64_t)b * a.R * C + h * D;
  const float* lse2 = a.lse2 + ((int64_t)b * a.H + h) * a.R;
  const float* dlt = a.delta + ((int64_t)b * a.H + h) * a.R;
  const float c2 = a.scale * LOG2E, NEG_INF = -__builtin_inff();
  f32x16 dq[DB], dv[DV ? DB : 1];
#pragma unroll
  for (int i = 0; i < DB; ++i) dq[i] = f32x16{};
  if constexpr (DV) {
#pragma unroll
    for (int i = 0; i < DB; ++i) dv[i] = f32x16{};
    // loop-carried accumulators live in AGPRs (unpinned they sit in VGPRs and are copied into
    // AGPRs and back around every trprod: ~4 VALU moves per MFMA, VALU/MFMA 4.3 measured)
    if constexpr (!LS) {  // (the fused pass at two waves per SIMD leaves the split to the allocator)
      fa::pin_agpr(dq);
      fa::pin_agpr(dv);
    }
  }

  // row constants of a tile: lse2 (+inf past R: P = 0) and δ, by threads 0..63
  auto aux_load = [&](int rt) -> float {
    const int rr = rt * 32 + (tid & 31);
    if (tid < 32) return rr < a.R ? lse2[rr] : __builtin_inff();
    if (tid < 64) return rr < a.R ? dlt[rr] : 0.f;
    return 0.f;
  };
  DmaStager<D, 2> dm;
  dm.init(wave, lane, C * 4);
  const float* const kdb[2] = {kb, db_};
  float ax = 0.f;
  if (rt_beg < rt_end) {
    dm.issue(kdb, C, (int64_t)rt_beg * 32, a.R - 1 - rt_beg * 32, sm, CF::IMG);
    ax = aux_load(rt_beg);
    if (tid < 64) sm[2 * CF::IMG + tid] = ax;
    fa::wait_vm<0>();
    __syncthreads();
  }
  for (int rt = rt_beg; rt < rt_end; ++rt) {
    const bool more = rt + 1 < rt_end;
    f32x16 scur;
    if constexpr (PF) scur = snext;
    if (more) {
      dm.issue(kdb, C, (int64_t)(rt + 1) * 32, a.R - 1 - (rt + 1) * 32, sm + ((rt + 1 - rt_beg) & 1) * CF::STAGE, CF::IMG);
      ax = aux_load(rt + 1);
      if constexpr (PF) snext = blk_load(sbc + (rt + 1) * sstep, lane);
    }
    if constexpr (LS && !PF) scur = blk_load(sbc + rt * sstep, lane);
    const float* ki = sm + ((rt - rt_beg) & 1) * CF::STAGE;
    const float* di = ki + CF::IMG;
    const float* ls = ki + 2 * CF::IMG;  // lse2[32], δ[32]
    int flag = c0 >= a.T ? 1 : (a.mflags ? flag_at(a.mflags, b, NRB32, NKT4, rt, c0 >> 6) : 0);
    flag = __builtin_amdgcn_readfirstlane(flag);
    f32x16 s{}, dp{};
    if (flag != 1) {
      if constexpr (LS) s = scur;                        // S  (row x col), stored by the forward
      else s = rowprod<D>(ki, qf, f32x16{}, lane);      // S  (row x col)
      dp = rowprod<D>(di, vf, f32x16{}, lane);          // dP (row x col)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = tidx(r, hf);
        const float p = ex2(__builtin_fmaf(s[r], c2, -ls[i]));
        s[r] = p;
        dp[r] = p * (dp[r] - ls[32 + i]);  // dS / scale
      }
      if (flag == 2) {  // masked entries: P = dS = 0 (the unmasked loop stays select-free)
        const uint32_t w = col_ok ? fa::settle((uint32_t)(a.mbits[((int64_t)b * NRT64 + (rt >> 1)) * TPAD + col] >> (32 * (rt & 1)))) : 0u;
        const uint32_t wh = w >> (4 * hf);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if ((wh >> tidx(r, 0)) & 1u) s[r] = dp[r] = 0.f;
      }
    }
    // dS (over S or apart), every tile (skipped tiles store zeros nobody reads): 16 dword
    // scatters per lane straight into the row kernel's order, before the dQ product
    if constexpr (DS) fa::blk_store(dsc + rt * dstep, dp, lane);
    if (flag != 1) {
      if constexpr (DV) trprod<D>(di, s, dv, lane);  // dVᵀ += dOᵀ · P
      trprod<D>(ki, dp, dq, lane);                    // dQᵀ += Kᵀ · dS
      if constexpr (DV && !LS) {
        fa::pin_agpr(dq);
        fa::pin_agpr(dv);
      }
    }
    if (more) {
      float* nx = sm + ((rt + 1 - rt_beg) & 1) * CF::STAGE;
      if (tid < 64) nx[2 * CF::IMG + tid] = ax;
    }
    fa::wait_vm<0>();  // the next tile's pieces (and S) landed
    __syncthreads();
  }
  if (!col_ok) return;
  const int64_t prow = ((int64_t)sp * a.B + b) * a.T + col;  // row of the split partials
  float* pq = ns > 1 ? a.cpq + prow * C + h * D : reinterpret_cast<float*>(a.dkc) + ((int64_t)b * a.T + col) * a.ldg + h * D;
  float* pv = ns > 1 ? a.cpv + prow * C + h * D : reinterpret_cast<float*>(a.dvc) + ((int64_t)b * a.T + col) * a.ldg + h * D;
  if (tail >= 0) {  // head-heavy tail piece: compact partials
    const int64_t pi = ((int64_t)sp * 8 * a.xrem + tail) * 128 + (col - cb * 128);
    pq = a.cpq + pi * D;
    pv = a.cpv + pi * D;
  }
  const float sc = a.scale;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      *reinterpret_cast<f32x4*>(pq + db * 32 + 8 * g + 4 * hf) =
          f32x4{dq[db][4 * g] * sc, dq[db][4 * g + 1] * sc, dq[db][4 * g + 2] * sc, dq[db][4 * g + 3] * sc};
      if constexpr (DV)
        *reinterpret_cast<f32x4*>(pv + db * 32 + 8 * g + 4 * hf) =
            f32x4{dv[db][4 * g], dv[db][4 * g + 1], dv[db][4 * g + 2], dv[db][4 * g + 3]};
    }
}

// head-heavy column pass: the tail blocks' compact row-piece partials summed in piece order into
// the gathered-side gradient (fp32, row stride ldg).  One thread per (tail column, 4 values).
__global__ __launch_bounds__(256) void cols_sum_tail_kernel(BwdArgs a, const float* part, float* out, int D) {
  const int ntail = 8 * a.xrem;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)ntail * 128 * (D / 4)) return;
  const int c4 = (int)(idx % (D / 4));
  const int tc = (int)(idx / (D / 4));
  const int cloc = tc & 127, t = tc >> 7;
  const int ncb = (a.T + 127) / 128;
  const int cbl = (t / a.xrem) * a.xcb + a.xwhole + t % a.xrem;
  const int cb = cbl % ncb, bh = cbl / ncb, b = bh / a.H, h = bh % a.H;
  const int col = cb * 128 + cloc;
  if (col >= a.T) return;
  const int64_t pstride = (int64_t)ntail * 128 * D, p0 = ((int64_t)t * 128 + cloc) * D + 4 * c4;
  f32x4 acc = *reinterpret_cast<const f32x4*>(part + p0);
  for (int s = 1; s < a.csq; ++s) acc += *reinterpret_cast<const f32x4*>(part + s * pstride + p0);
  *reinterpret_cast<f32x4*>(out + ((int64_t)b * a.T + col) * a.ldg + h * D + 4 * c4) = acc;
}

// ------------------------------------------------------------------------------------------
// backward, row side in score-buffer mode: dK = scale · Σ_cols dS · Q_cols with dS read from the
// buffer the column kernel wrote (one product per tile: no S, no dP, no V / dO traffic).  Same
// grid, column split and partial protocol as bwd_rows_kernel; the only LDS image is Q.

template <int D>
__global__ __launch_bounds__(256, 2) void bwd_rows_ds_kernel(BwdArgs a) {
  using CF = Cfg<D>;
  constexpr int DB = CF::DB;
  extern __shared__ __attribute__((aligned(16))) float sm[];
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
  DmaStager<D, 1> dm;
  dm.init(wave, lane, (int)(a.ldkv * 4));
  f32x16 q[PF];
  if (kt_beg < kt_end) {
    dm.issue(&qb, a.ldkv, (int64_t)kt_beg * 32, a.T - 1 - kt_beg * 32, sm, CF::IMG);
#pragma unroll
    for (int j = 0; j < PF; ++j)
      if (kt_beg + j < kt_end) q[j] = blk_load(sbr + (int64_t)(kt_beg + j) * 1024, lane);
    fa::wait_vm<0>();
    __syncthreads();
  }
  fa::ring_loop<PF>(kt_beg, kt_end, [&](int kt, auto J) {
    constexpr int j = decltype(J)::value;
    const bool more = kt + 1 < kt_end;
    f32x16 ds = q[j];
    if (more) dm.issue(&qb, a.ldkv, (int64_t)(kt + 1) * 32, a.T - 1 - (kt + 1) * 32, sm + ((kt + 1 - kt_beg) & 1) * CF::IMG, 0);
    if (kt + PF < kt_end) q[j] = blk_load(sbr + (int64_t)(kt + PF) * 1024, lane);  // every wave: uniform vmcnt
    const float* qi = sm + ((kt - kt_beg) & 1) * CF::IMG;
    int flag = !wave_ok ? 1 : (a.mflags ? flag_at(a.mflags, b, NRB32, NKT4, r0 >> 5, kt >> 1) : 0);
    flag = __builtin_amdgcn_readfirstlane(flag);
    if (flag != 1) {
      const int valid = a.T - kt * 32;
      if (valid < 32) {  // columns past T: the column kernel's values there are not gradients
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (tidx(r, hf) >= valid) ds[r] = 0.f;
      }
      trprod<D>(qi, ds, dk, lane);  // dKᵀ += Q_colsᵀ · dSᵀ
    }
    fa::wait_vm<0>();  // the next tile's pieces landed
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

// ------------------------------------------------------------------------------------------
// backward, gathered side in score-buffer mode, pass 1 of 2: dV_cols = Σ_rows Pᵀ · dO with P
// recomputed elementwise from the stored S (the dV product is the only one: a third of the
// column work, no V / K traffic).  Runs BEFORE bwd_cols_kernel<D, true>, which overwrites S with
// dS.  Same grid as the column kernel; stage = dO image + lse2[32].
template <int D>
__global__ __launch_bounds__(256, D <= 96 ? 4 : 2) void bwd_cols_dv_kernel(BwdArgs a) {
  using CF = Cfg<D>;
  constexpr int DB = CF::DB, STG = CF::IMG + 32;
  extern __shared__ __attribute__((aligned(16))) float sm[];
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
  DmaStager<D, 1> dm;
  dm.init(wave, lane, C * 4);
  f32x16 q[PF];
  float ax = 0.f;
  if (rt_beg < rt_end) {
    dm.issue(&db_, C, (int64_t)rt_beg * 32, a.R - 1 - rt_beg * 32, sm, 0);
    ax = aux_load(rt_beg);
#pragma unroll
    for (int j = 0; j < PF; ++j)
      if (rt_beg + j < rt_end) q[j] = blk_load(sbc + (rt_beg + j) * sstep, lane);
    if (tid < 32) sm[CF::IMG + tid] = ax;
    fa::wait_vm<0>();
    __syncthreads();
  }
  fa::ring_loop<PF>(rt_beg, rt_end, [&](int rt, auto J) {
    constexpr int j = decltype(J)::value;
    const bool more = rt + 1 < rt_end;
    f32x16 s = q[j];
    if (more) {
      dm.issue(&db_, C, (int64_t)(rt + 1) * 32, a.R - 1 - (rt + 1) * 32, sm + ((rt + 1 - rt_beg) & 1) * STG, 0);
      ax = aux_load(rt + 1);
    }
    if (rt + PF < rt_end) q[j] = blk_load(sbc + (rt + PF) * sstep, lane);  // every wave: uniform vmcnt
    const float* di = sm + ((rt - rt_beg) & 1) * STG;
    const float* ls = di + CF::IMG;
    int flag = !sown ? 1 : (a.mflags ? flag_at(a.mflags, b, NRB32, NKT4, rt, c0 >> 6) : 0);
    flag = __builtin_amdgcn_readfirstlane(flag);
    if (flag != 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = ex2(__builtin_fmaf(s[r], c2, -ls[tidx(r, hf)]));
      if (flag == 2) {  // masked entries: P = 0 (the lane-half shift once, then constant shifts:
                        // no per-register shift amounts held across the loop)
        const uint32_t w = col_ok ? fa::settle((uint32_t)(a.mbits[((int64_t)b * NRT64 + (rt >> 1)) * TPAD + col] >> (32 * (rt & 1)))) : 0u;
        const uint32_t wh = w >> (4 * hf);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if ((wh >> tidx(r, 0)) & 1u) s[r] = 0.f;
      }
      trprod<D>(di, s, dv, lane);  // dVᵀ += dOᵀ · P
    }
    if (more) {
      float* nx = sm + ((rt + 1 - rt_beg) & 1) * STG;
      if (tid < 32) nx[CF::IMG + tid] = ax;
    }
    fa::wait_vm<0>();  // the next tile's pieces landed
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

// sum a.nsplit slots of a.dpart into the fp32 row-side grad
__global__ __launch_bounds__(256) void rows_sum_kernel(BwdArgs a, int D) {
  const int64_t total4 = (int64_t)a.B * a.R * a.H * D / 4;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total4) return;
  f32x4 acc = *reinterpret_cast<const f32x4*>(a.dpart + idx * 4);
  for (int s = 1; s < a.nsplit; ++s) acc += *reinterpret_cast<const f32x4*>(a.dpart + s * total4 * 4 + idx * 4);
  *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.drows) + idx * 4) = acc;
}

template <int D> constexpr int lds_bytes() { return 2 * Cfg<D>::STAGE * 4; }
// + one 4-KiB transpose tile per wave for the score-buffer stores (blk_store_lds)
template <int D> constexpr int lds_bytes_sb() { return lds_bytes<D>() + 4 * 4096; }
// the column kernels that store dS scatter it directly (no transpose tile): exact fp32 step
// 52.9 -> 51.9 ms on one box (the LDS-transposed store and its 12.5 % bank conflicts measured
// slower; profiles/r6_fp32.md)
template <int D> constexpr int lds_bytes_ds() { return lds_bytes<D>(); }

}  // namespace fa32
}  // namespace xdot

#define XF32_DISPATCH(CALL)            \
  switch (D) {                         \
    case 32: CALL(32); return 0;       \
    case 64: CALL(64); return 0;       \
    case 96: CALL(96); return 0;       \
    case 128: CALL(128); return 0;     \
    default: return -1;                \
  }

namespace {
// The score-storing forward scatters S directly (three workgroups per CU at D <= 96): exact fp32
// step 54.6-55.0 -> 53.6-54.0 ms on one box (profiles/r6_fp32.md).  XDOT_F32_FWD_DIRECT=0: the
// LDS-transposed store at two workgroups per CU.
bool fwd_direct_store() {
  const char* e = std::getenv("XDOT_F32_FWD_DIRECT");  // read per call (A/B in one process)
  return !(e && *e == '0');
}
}  // namespace

extern "C" int xdot_flash_fwd_f32_launch(const xdot::fa::FwdArgs* a, int D, hipStream_t st) {
  using namespace xdot::fa32;
  if (a->R == 0 || a->B == 0 || a->H == 0 || a->prescaled) return a->prescaled ? -1 : 0;
  const int nrb = (a->R + 127) / 128;
  const dim3 grid(a->xrbs > 0 ? 8 * (a->xwhole + a->xrem * a->nsplit) : nrb * a->B * a->H * a->nsplit);
  if (a->sbuf) {
    if (fwd_direct_store()) {
#define L(DV) hipLaunchKernelGGL((fwd_kernel<DV, true, true>), grid, dim3(256), lds_bytes<DV>(), st, *a)
      XF32_DISPATCH(L)
#undef L
    }
#define L(DV) hipLaunchKernelGGL((fwd_kernel<DV, true>), grid, dim3(256), lds_bytes_sb<DV>(), st, *a)
    XF32_DISPATCH(L)
#undef L
  }
#define L(DV) hipLaunchKernelGGL((fwd_kernel<DV, false>), grid, dim3(256), lds_bytes<DV>(), st, *a)
  XF32_DISPATCH(L)
#undef L
}

extern "C" int xdot_flash_combine_f32_launch(const xdot::fa::FwdArgs* a, int D, hipStream_t st) {
  if (a->R == 0 || a->B == 0 || a->H == 0) return 0;
  if (a->xrbs > 0) {  // head-heavy grid: only the tail blocks' compact partials
    if (a->xrem <= 0) return 0;
    const int64_t n = (int64_t)8 * a->xrem * 128 * (D / 4);
    hipLaunchKernelGGL(xdot::fa32::combine_tail_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, *a, D);
    return 0;
  }
  const int64_t n = (int64_t)a->B * a->R * (a->H * D / 4);
  hipLaunchKernelGGL(xdot::fa32::combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, *a, D);
  return 0;
}

extern "C" int xdot_flash_bwd_prep_f32_launch(const xdot::fa::BwdArgs* a, const void* out, float* delta, int D,
                                              hipStream_t st) {
  if (a->R == 0 || a->B == 0 || a->H == 0) return 0;
  const int64_t n = (int64_t)a->B * a->R * a->H;
  if (delta && (D == 32 || D == 64 || D == 96 || D == 128)) {
    const dim3 grid((unsigned)((8 * n + 255) / 256));
    const float* o = reinterpret_cast<const float*>(out);
    switch (D) {
      case 32: hipLaunchKernelGGL(xdot::fa32::prep8_kernel<32>, grid, dim3(256), 0, st, *a, o, delta); break;
      case 64: hipLaunchKernelGGL(xdot::fa32::prep8_kernel<64>, grid, dim3(256), 0, st, *a, o, delta); break;
      case 96: hipLaunchKernelGGL(xdot::fa32::prep8_kernel<96>, grid, dim3(256), 0, st, *a, o, delta); break;
      default: hipLaunchKernelGGL(xdot::fa32::prep8_kernel<128>, grid, dim3(256), 0, st, *a, o, delta); break;
    }
    return 0;
  }
  hipLaunchKernelGGL(xdot::fa32::prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, *a,
                     reinterpret_cast<const float*>(out), delta, D);
  return 0;
}

extern "C" int xdot_flash_bwd_rows_f32_launch(const xdot::fa::BwdArgs* a, int D, hipStream_t st) {
  using namespace xdot::fa32;
  if (a->R == 0 || a->B == 0 || a->H == 0 || a->T == 0) return 0;
  if (a->prescaled) return -1;
  const int nrb = (a->R + 127) / 128;
  const dim3 grid(nrb * a->B * a->H * a->nsplit);
  if (a->sbuf || a->dsbuf) {  // score-buffer modes: dS from the column kernel, Q image only
#define L(DV) hipLaunchKernelGGL(bwd_rows_ds_kernel<DV>, grid, dim3(256), 2 * Cfg<DV>::IMG * 4, st, *a)
    XF32_DISPATCH(L)
#undef L
  }
#define L(DV) hipLaunchKernelGGL(bwd_rows_kernel<DV>, grid, dim3(256), lds_bytes<DV>(), st, *a)
  XF32_DISPATCH(L)
#undef L
}

extern "C" int xdot_flash_bwd_cols_f32_launch(const xdot::fa::BwdArgs* a, int D, hipStream_t st) {
  using namespace xdot::fa32;
  if (a->R == 0 || a->B == 0 || a->H == 0 || a->T == 0) return 0;
  if (a->prescaled || a->dkv16) return -1;
  const int W = ((a->T + 127) / 128) * a->B * a->H, sq = a->csq > 1 ? a->csq : 1, sv = a->csv > 1 ? a->csv : 1;
  if ((sq > 1 && (!a->cpq || (!a->sbuf && !a->cpv))) || (sv > 1 && !a->cpv) || (D & 3)) return -1;
  const int64_t rows = (int64_t)a->B * a->T;
  const int C = a->H * D;
  // the split partials of one pass, summed into its grad half (fp32, ldg-strided)
  auto sum_q = [&] {
    if (sq > 1) xdot_flash_cols_sum_launch(a->cpq, a->dkc, sq, rows, C, a->ldg, xdot::DT_F32, st);
  };
  auto sum_v = [&](int s) {
    if (s > 1) xdot_flash_cols_sum_launch(a->cpv, a->dvc, s, rows, C, a->ldg, xdot::DT_F32, st);
  };
  if (a->sbuf && a->sb_passes == 4 && a->xcb > 0) {  // fused pass on the head-heavy grid
    if (sq < 2 || !a->cpq || !a->cpv || 8 * a->xcb != W) return -1;
    const dim3 grid(8 * (a->xwhole + a->xrem * sq));
    const int64_t nt = (int64_t)8 * a->xrem * 128 * (D / 4);
#define L(DV)                                                                                                  \
  hipLaunchKernelGGL((bwd_cols_kernel<DV, true, true, true>), grid, dim3(256), lds_bytes_ds<DV>(), st, *a);     \
  if (nt > 0) {                                                                                                  \
    hipLaunchKernelGGL(cols_sum_tail_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, *a, a->cpq,   \
                       reinterpret_cast<float*>(a->dkc), DV);                                                    \
    hipLaunchKernelGGL(cols_sum_tail_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, *a, a->cpv,   \
                       reinterpret_cast<float*>(a->dvc), DV);                                                    \
  }                                                                                                              \
  return 0;
    XF32_DISPATCH(L)
#undef L
  }
  if (a->sbuf && a->sb_passes == 4) {  // fused: dP, dQ and dV in one pass (S -> dS)
#define L(DV)                                                                                                  \
  hipLaunchKernelGGL((bwd_cols_kernel<DV, true, true, true>), dim3(W * sq), dim3(256), lds_bytes_ds<DV>(), st, *a); \
  sum_q();                                                                                                       \
  sum_v(sq)
    XF32_DISPATCH(L)
#undef L
  }
  if (a->sbuf) {  // in place: dV from S first, then dQ (S -> dS); with a dS buffer dQ first
    const int ps = a->sb_passes ? a->sb_passes : 3;
    const bool dv_first = !a->dsbuf;
#define LDV(DV) hipLaunchKernelGGL(bwd_cols_dv_kernel<DV>, dim3(W * sv), dim3(256), 2 * (Cfg<DV>::IMG + 32) * 4, st, *a)
#define LDQ(DV) hipLaunchKernelGGL((bwd_cols_kernel<DV, true>), dim3(W * sq), dim3(256), lds_bytes_ds<DV>(), st, *a)
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
    XF32_DISPATCH(L)
#undef L
#undef LDQ
#undef LDV
  }
  if (a->dsbuf) {  // dS-only buffer: recompute S, store dS for the row kernel
#define L(DV)                                                                                                     \
  hipLaunchKernelGGL((bwd_cols_kernel<DV, false, true>), dim3(W * sq), dim3(256), lds_bytes_ds<DV>(), st, *a); \
  sum_q();                                                                                                        \
  sum_v(sq)
    XF32_DISPATCH(L)
#undef L
  }
#define L(DV)                                                                                                \
  hipLaunchKernelGGL((bwd_cols_kernel<DV, false>), dim3(W * sq), dim3(256), lds_bytes<DV>(), st, *a); \
  sum_q();                                                                                                   \
  sum_v(sq)
  XF32_DISPATCH(L)
#undef L
}

namespace {
// XDOT_CSPLIT: unset / "auto" = occupancy round model, "0" / "1" = no split, n = n splits (<= 8)
int csplit_env() {
  const char* e = std::getenv("XDOT_CSPLIT");  // read per call (tests switch it)
  return (!e || !*e || !std::strcmp(e, "auto")) ? -1 : std::max(1, std::min(8, std::atoi(e)));
}
template <int D> void f32_splits(const xdot::fa::BwdArgs* a, int* sq, int* sv) {
  using namespace xdot::fa32;
  const int64_t W = (int64_t)((a->T + 127) / 128) * a->B * a->H;
  const int NRT = (a->R + 31) / 32, cus = xdot_num_cus();
  if (a->sbuf && a->sb_passes == 4) {
    // up to 8 splits priced at 0.4 % each (as the fp32 forward): a split costs the fused pass two
    // fp32 partial copies of the gathered-side gradient (~0.06 ms at T = 25000), its last-round
    // tail ~1.4 ms at 4 splits
    *sq = *sv = xdot::fa::pick_csplit(W, NRT, cus * xdot::fa::wg_per_cu(bwd_cols_kernel<D, true, true, true>, lds_bytes_ds<D>()),
                                      8, 0.004);
  } else if (a->sbuf) {
    *sq = xdot::fa::pick_csplit(W, NRT, cus * xdot::fa::wg_per_cu(bwd_cols_kernel<D, true>, lds_bytes_ds<D>()));
    *sv = xdot::fa::pick_csplit(W, NRT, cus * xdot::fa::wg_per_cu(bwd_cols_dv_kernel<D>, 2 * (Cfg<D>::IMG + 32) * 4));
  } else if (a->dsbuf) {
    *sq = *sv = xdot::fa::pick_csplit(W, NRT, cus * xdot::fa::wg_per_cu(bwd_cols_kernel<D, false, true>, lds_bytes_ds<D>()));
  } else {
    *sq = *sv = xdot::fa::pick_csplit(W, NRT, cus * xdot::fa::wg_per_cu(bwd_cols_kernel<D, false>, lds_bytes<D>()));
  }
}
}  // namespace

extern "C" int xdot_flash_cols_splits_f32(const xdot::fa::BwdArgs* a, int D, int* sq, int* sv) {
  *sq = *sv = 1;
  const int e = csplit_env();
  if (e >= 0) {
    const int NRT = (a->R + 31) / 32;
    *sq = *sv = NRT / e >= 1 ? e : 1;
    return 0;
  }
  switch (D) {
    case 32: f32_splits<32>(a, sq, sv); break;
    case 64: f32_splits<64>(a, sq, sv); break;
    case 96: f32_splits<96>(a, sq, sv); break;
    case 128: f32_splits<128>(a, sq, sv); break;
    default: return -1;
  }
  return 0;
}

extern "C" int xdot_flash_rows_sum_f32_launch(const xdot::fa::BwdArgs* a, int D, hipStream_t st) {
  if (a->R == 0 || a->B == 0 || a->H == 0) return 0;
  const int64_t n4 = (int64_t)a->B * a->R * a->H * D / 4;
  hipLaunchKernelGGL(xdot::fa32::rows_sum_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, *a, D);
  return 0;
}

// column splits of the exact-fp32 forward (kernel 0) / row-side backward (1), see kernels.h
extern "C" int xdot_flash_f32_cols_heavy(const xdot::fa::BwdArgs* a, int D, int sq, int* whole, int* rem, int* split) {
  using namespace xdot::fa32;
  if (!xdot_flash_f32_heavy() || !a->sbuf || a->sb_passes != 4 || a->fp32_mode || D > 128) return 0;
  int occ = 0;
#define OC(DV) \
  if (D == DV) occ = xdot::fa::wg_per_cu(bwd_cols_kernel<DV, true, true, true>, lds_bytes_ds<DV>());
  OC(32) OC(64) OC(96) OC(128)
#undef OC
  const int64_t W = (int64_t)((a->T + 127) / 128) * a->B * a->H, S = (int64_t)occ * (xdot_num_cus() / 8);
  if (occ <= 0 || S <= 0 || W % 8) return 0;
  // the forward's round model (bindings.cpp head_heavy_plan) over 64-row tiles of the row sweep
  const int64_t m = W / 8, n = (a->R + 63) / 64, full = m / S, r = m % S;
  if (r == 0 || full == 0) return 0;
  const int su = sq > 1 ? sq : 1;
  const double cu = (double)((W * su + 8 * S - 1) / (8 * S)) * ((double)n / su + 8.0);
  double best = 1e300;
  int bs = 0;
  for (int s = 1; s <= 16; ++s) {
    if (s > 1 && n / s < 8) break;
    const double c = (double)full * ((double)n + 8.0) + (double)((r * s + S - 1) / S) * ((double)n / s + 8.0);
    if (c < best * 0.985) { best = c; bs = s; }
  }
  if (bs < 2 || best >= cu * 0.97) return 0;
  *whole = (int)(full * S);
  *rem = (int)r;
  *split = bs;
  return 1;
}

extern "C" int xdot_flash_f32_heavy() {
  static const int v = [] {
    const char* e = std::getenv("XDOT_F32_HEAVY");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v;
}

// resident forward workgroups per CU of the exact-fp32 forward the launcher would pick (0: none)
extern "C" int xdot_flash_f32_fwd_occ(int D, bool sbuf) {
  using namespace xdot::fa32;
  int occ = 0;
#define OC(DV)                                                                                               \
  if (D == DV)                                                                                               \
    occ = sbuf ? (fwd_direct_store() ? xdot::fa::wg_per_cu(fwd_kernel<DV, true, true>, lds_bytes<DV>())      \
                                     : xdot::fa::wg_per_cu(fwd_kernel<DV, true>, lds_bytes_sb<DV>()))        \
               : xdot::fa::wg_per_cu(fwd_kernel<DV, false>, lds_bytes<DV>());
  OC(32) OC(64) OC(96) OC(128)
#undef OC
  return occ;
}

extern "C" int xdot_flash_f32_row_splits_exact(int kernel, int D, bool sbuf, int64_t W, int64_t T) {
  using namespace xdot::fa32;
  int occ = 0;
#define OC(DV)                                                                                                   \
  if (D == DV)                                                                                                   \
    occ = kernel == 0 ? (sbuf ? (fwd_direct_store() ? xdot::fa::wg_per_cu(fwd_kernel<DV, true, true>, lds_bytes<DV>()) \
                                                    : xdot::fa::wg_per_cu(fwd_kernel<DV, true>, lds_bytes_sb<DV>())) \
                              : xdot::fa::wg_per_cu(fwd_kernel<DV, false>, lds_bytes<DV>()))                   \
                      : (sbuf ? xdot::fa::wg_per_cu(bwd_rows_ds_kernel<DV>, 2 * Cfg<DV>::IMG * 4)              \
                              : xdot::fa::wg_per_cu(bwd_rows_kernel<DV>, lds_bytes<DV>()));
  OC(32) OC(64) OC(96) OC(128)
#undef OC
  if (!occ) return 0;
  // the forward's workgroups are long (a 32-column fp32 tile is ~16x a 16-bit one), so a split
  // costs little beside a part-full last round: up to 32 splits at 0.1 % each (the N=8 rank's 200
  // row blocks: 23 splits fill six rounds of 768 slots instead of 7 splits in two part-full ones)
  if (kernel == 0) return xdot::fa::pick_csplit(W, (int)((T + 31) / 32), occ * xdot_num_cus(), 32, 0.001);
  return xdot::fa::pick_csplit(W, (int)((T + 31) / 32), occ * xdot_num_cus(), 8, 0.004);
}
