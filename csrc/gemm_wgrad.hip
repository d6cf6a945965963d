// xdot — weight-gradient GEMM for gfx950: dW = dYᵀ · X of the module's Linear layers
// (reference: distributed_dot_product/module.py:43-45, :75 — autograd's
// Linear backward there), K = the rank's rows.
//
//   part[s](m, n) = sum_{k in slab s} A[k][m] · B[k][n]      A = dY (K, M), B = X (K, N),
//                                                            both row-major: mn-contiguous
//
// The output is small (768 x 768 .. 1536 x 768: 36-72 tiles of 128 x 128) and K long (3125 rows at
// an N=8 rank, 25000 at N=1), so the reduction is split into S slabs of whole 64-row k-tiles
// (tiles x S ~ 2 workgroups per CU) whose fp32 partials one ordered pass sums and casts
// (csrc/reduce.hip: deterministic).  Per workgroup (4 waves, 2 x 2, 64 x 64 each):
//   * k-tiles of 64 rows through a 2-stage LDS ring; both operand images are mn-contiguous
//     [64 k][256 B] (gemm3's swizzle) filled by buffer_load ... lds whose buffer ends at the slab's
//     last row: rows past K read as zeros, so the tail k-tile needs no special path;
//   * fragments through ds_read_b64_tr_b16 (hardware transpose) for both operands;
//   * v_mfma_f32_16x16x32 on the Cᵀ tile (each lane ends with 4 consecutive output columns):
//     16-byte fp32 stores of the partial.
// Eligibility: 16-bit, M % 128 == 0, N % 128 == 0, lda / ldb % 8 == 0, 16-byte aligned bases.
// One launch may carry two independent products (dWk and dW[q|v], both due at the end of the
// fused backward): their blocks share the GPU instead of running one after the other.
#include "flash_common.h"

namespace xdot {
namespace gw {

constexpr int BM = 128, BN = 128, BK = 64, NTH = 256;
constexpr int IMG = BK * 256;        // one operand image: 64 k rows x 128 mn x 2 B
constexpr int STAGE = 2 * IMG;       // [A | B]
constexpr int LDS = 2 * STAGE;       // 64 KiB: two workgroups per CU

template <int DT> __device__ __forceinline__ f32x4 mfma16(u32x4 a, u32x4 b, f32x4 c) {
  if constexpr (DT == DT_BF16)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

typedef __attribute__((ext_vector_type(4))) int i32x4;
// raw buffer descriptor over [base, base + bytes): loads at offsets >= bytes return zeros
__device__ __forceinline__ i32x4 rsrc(const void* base, uint32_t bytes) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  i32x4 r;
  r[0] = (int)__builtin_amdgcn_readfirstlane((uint32_t)b);
  r[1] = (int)(__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) & 0xFFFFu);
  r[2] = (int)__builtin_amdgcn_readfirstlane(bytes);
  r[3] = 0x00020000;
  return r;
}
// four consecutive 1 KiB LDS-DMA pieces of one wave through buffer_load ... lds
__device__ __forceinline__ void bdma4(i32x4 rs, const uint32_t* o, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %5\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %6, 0 offen lds\n\t"
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %6, 0 offen lds\n\t"
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tbuffer_load_dwordx4 %3, %6, 0 offen lds\n\t"
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tbuffer_load_dwordx4 %4, %6, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]), "s"(lds), "s"(rs) : "memory", "scc");
}

struct Prob {
  const void* A;  // (K, M) row-major, row stride lda
  const void* B;  // (K, N) row-major, row stride ldb
  float* part;    // (S, M, N) fp32
  int M, N, K, S;
  int64_t lda, ldb;
};
// one or two independent products in one launch (the module's dWk and dW[q|v] at the end of the
// backward: each alone fills only part of the GPU); problem 1's blocks start at wg1 (a multiple of
// 8, so the XCD remap of either problem sees its own blocks in dispatch order)
struct Args {
  Prob q0, q1;
  int np, wg1;
};

}  // namespace gw

template <int DT>
__global__ __launch_bounds__(256, 2) void gemm_wgrad_kernel(gw::Args pa) {
  using namespace gw;
  using fa::smem;
  using fa::lds_addr;
  // this block's problem (wave-uniform selects: no dynamic indexing of the kernel arguments)
  const int bx = blockIdx.x;
  const bool q1 = pa.np > 1 && bx >= pa.wg1;
  Prob p;
  p.A = q1 ? pa.q1.A : pa.q0.A;
  p.B = q1 ? pa.q1.B : pa.q0.B;
  p.part = q1 ? pa.q1.part : pa.q0.part;
  p.M = q1 ? pa.q1.M : pa.q0.M;
  p.N = q1 ? pa.q1.N : pa.q0.N;
  p.K = q1 ? pa.q1.K : pa.q0.K;
  p.S = q1 ? pa.q1.S : pa.q0.S;
  p.lda = q1 ? pa.q1.lda : pa.q0.lda;
  p.ldb = q1 ? pa.q1.ldb : pa.q0.ldb;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4;
  const int tiles_n = p.N / BN, tiles = (p.M / BM) * tiles_n;
  const int span = q1 ? (int)gridDim.x - pa.wg1 : (pa.np > 1 ? pa.wg1 : (int)gridDim.x);
  const int lin = xcd_remap(q1 ? bx - pa.wg1 : bx, span);  // slab-major: one slab's tiles share an XCD
  if (lin >= tiles * p.S) return;  // problem 0's padding to a multiple of 8 blocks (before any barrier)
  const int s = lin / tiles, t = lin % tiles;
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  const int KT = (p.K + BK - 1) / BK;
  const int kt0 = (int)((int64_t)s * KT / p.S), kt1 = (int)((int64_t)(s + 1) * KT / p.S);
  const int k0 = kt0 * BK, k1 = min(p.K, kt1 * BK);
  const int64_t lda2 = p.lda * 2, ldb2 = p.ldb * 2;

  // operand bases at (k0, m0 / n0); the descriptors end at row k1 (zeros past it)
  const char* abase = reinterpret_cast<const char*>(p.A) + (int64_t)k0 * lda2 + (int64_t)m0 * 2;
  const char* bbase = reinterpret_cast<const char*>(p.B) + (int64_t)k0 * ldb2 + (int64_t)n0 * 2;
  // per-lane offsets of the wave's four 1 KiB pieces of a k-tile image: image row k (0..63) holds
  // chunk c of k row k at 16 * (c ^ (2 (k & 3) + 8 ((k >> 3) & 1))) (gemm3's mn-contiguous layout)
  uint32_t oa[4], ob[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int pc = wave * 4 + i;
    const int k = 4 * pc + (lane >> 4), c = (lane & 15) ^ (2 * (k & 3) + 8 * ((k >> 3) & 1));
    oa[i] = (uint32_t)(k * lda2 + 16 * c);
    ob[i] = (uint32_t)(k * ldb2 + 16 * c);
  }
  auto issue = [&](int kt, int st) __attribute__((always_inline)) {
    char* sb = smem + st * STAGE;
    const int kr = (kt - kt0) * BK;  // first row of this k-tile inside the slab
    const uint32_t rows_left = (uint32_t)(k1 - k0 - kr);  // > 0
    bdma4(rsrc(abase + (int64_t)kr * lda2, rows_left * (uint32_t)lda2), oa, lds_addr(sb + wave * 4096));
    bdma4(rsrc(bbase + (int64_t)kr * ldb2, rows_left * (uint32_t)ldb2), ob, lds_addr(sb + IMG + wave * 4096));
  };

  // transposed fragment reads (16x16x32 operand: lane l holds mn = base + (l & 15), k = 8 (l >> 4) .. +7)
  typedef const __attribute__((address_space(3))) char lds_char;
  const int tq = (lane & 15) >> 2, tp = lane & 3;
  auto mc_base = [&](int cb) __attribute__((always_inline)) {
    const int c = (tp >> 1) | ((cb ^ (2 * tq + 8 * (g & 1))) & 14);
    return (8 * g + tq) * 256 + 16 * c + 8 * (tp & 1);
  };
  int mca[4], mcb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    mca[i] = mc_base((64 * wm + 16 * i) / 8);
    mcb[i] = mc_base((64 * wn + 16 * i) / 8);
  }
  auto frag = [&](const char* img, int mci, int ks) __attribute__((always_inline)) -> u32x4 {
    lds_char* b = (lds_char*)img + mci + ks * 32 * 256;
    fa::s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((fa::lds_s16x4*)(b));
    fa::s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((fa::lds_s16x4*)(b + 4 * 256));
    union { struct { fa::s16x4 a, b; } s; u32x4 u; } r;
    r.s.a = lo;
    r.s.b = hi;
    return r.u;
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1) issue(kt0, 0);
  for (int kt = kt0; kt < kt1; ++kt) {
    const int st = (kt - kt0) & 1;
    fa::wait_vm<0>();   // k-tile kt landed
    fa::raw_barrier();  // ... for every wave; every wave is done with the other stage
    if (kt + 1 < kt1) issue(kt + 1, st ^ 1);
    const char* ai = smem + st * STAGE;
    const char* bi = ai + IMG;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      u32x4 fa_[4], fb_[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa_[i] = frag(ai, mca[i], ks);
        fb_[i] = frag(bi, mcb[i], ks);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16<DT>(fb_[j], fa_[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  }

  // acc[i][j]: rows m0 + 64 wm + 16 i + (l & 15), columns n0 + 64 wn + 16 j + 4 g .. +3
  float* pp = p.part + (int64_t)s * p.M * p.N;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + 64 * wm + 16 * i + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<f32x4*>(pp + (int64_t)m * p.N + n0 + 64 * wn + 16 * j + 4 * g) = acc[i][j];
  }
}

}  // namespace xdot

namespace {
bool wgrad_ok(const xdot::gw::Prob& q) {
  using namespace xdot;
  if (q.M % gw::BM || q.N % gw::BN || q.K < 1 || q.S < 1 || q.lda % 8 || q.ldb % 8) return false;
  if ((reinterpret_cast<uintptr_t>(q.A) | reinterpret_cast<uintptr_t>(q.B)) & 15) return false;
  const int KT = (q.K + gw::BK - 1) / gw::BK;
  if (q.S > KT) return false;
  // every slab's descriptor spans at most 2^32 - 1 bytes
  const int64_t ld = q.lda > q.ldb ? q.lda : q.ldb;
  return (int64_t)((KT + q.S - 1) / q.S) * gw::BK * 2 * ld < (int64_t)0xFFFFFFFF;
}
}  // namespace

// np (1 or 2) products {A, B, part, M, N, K, S, lda, ldb} in one launch; each part must hold
// S * M * N fp32; returns -3 when a shape / layout is not eligible
extern "C" int xdot_gemm_wgrad_launch(int np, const void* const* A, const void* const* B, float* const* part,
                                      const int* M, const int* N, const int* K, const int* S, const int64_t* lda,
                                      const int64_t* ldb, int dt, hipStream_t st) {
  using namespace xdot;
  if (dt != DT_BF16 && dt != DT_F16) return -3;
  if (np < 1 || np > 2) return -3;
  gw::Args a{};
  gw::Prob* qs[2] = {&a.q0, &a.q1};
  int64_t grid = 0;
  for (int i = 0; i < np; ++i) {
    *qs[i] = gw::Prob{A[i], B[i], part[i], M[i], N[i], K[i], S[i], lda[i], ldb[i]};
    if (!wgrad_ok(*qs[i])) return -3;
    const int64_t blocks = (int64_t)(M[i] / gw::BM) * (N[i] / gw::BN) * S[i];
    if (i == 0 && np > 1) {
      a.wg1 = (int)((blocks + 7) / 8 * 8);
      grid = a.wg1;
    } else {
      grid += blocks;
    }
  }
  a.np = np;
  if (grid > 0x7FFFFFFF) return -3;
  if (dt == DT_BF16) hipLaunchKernelGGL(gemm_wgrad_kernel<DT_BF16>, dim3((unsigned)grid), dim3(gw::NTH), gw::LDS, st, a);
  else hipLaunchKernelGGL(gemm_wgrad_kernel<DT_F16>, dim3((unsigned)grid), dim3(gw::NTH), gw::LDS, st, a);
  return (int)hipGetLastError();
}
