// xdot — generic batched, K-segmented MFMA GEMM for gfx950.
//
//   C[z](m, n) = alpha * sum_{s < nseg} sum_{k < K} opA_s[z](m, k) * opB_s[z](k, n)
//
// This one kernel family carries the three distributed products of the reference
// (reference: distributed_dot_product/multiplication/functions.py:89-97 [nt GEMM],
// :140-147 [tn GEMM], :202-211 [all GEMM + sum over ranks]):
//   * nt : out[p, :, j*R:(j+1)*R] = left[p] @ gathered[j, p]^T   (2-level batch (j, p),
//          written straight into the final (P, R, T) layout: no permute copy);
//   * all: out[p] = sum_j left[p, :, j*R:(j+1)*R] @ gathered[j, p]   (K-segments = ranks,
//          the reference's stack copy and sum(dim=0) are folded into the K loop);
//   * tn : send[j, p] = left[p, :, j*R:(j+1)*R]^T @ right[p]          (A read transposed
//          in place, output is the reduce-scatter send buffer).
//
// Operand storage (chosen per operand by template flag):
//   A_MC = 0 : A(m, k) = A[m*lda + k]   (k contiguous)      A_MC = 1 : A(m, k) = A[k*lda + m]
//   B_MC = 0 : B(k, n) = B[n*ldb + k]   (k contiguous)      B_MC = 1 : B(k, n) = B[k*ldb + n]
//
// Tiling (CDNA4): 128x128 output tile per 256-thread workgroup, 4 waves in 2x2, each wave
// owns 64x64 = 4x4 MFMA tiles.  bf16/fp16 use v_mfma_f32_16x16x32_{bf16,f16} (BK = 32);
// fp32 uses the exact-f32 v_mfma_f32_16x16x4_f32 (BK = 16).  Operands are register-staged
// into a double-buffered LDS image (one barrier per K tile, loads for tile t+1 issued before
// the MFMAs of tile t, LDS writes after them).  LDS images:
//   k-contiguous operand : [128 rows][6 x 16 B]  (4 data slots + 2 pad: ds_read_b128 conflict-free)
//   mn-contiguous operand: [BK rows][128 + pad]  read with ds_read_b64_tr_b16 (bf16/f16) or
//                          ds_read_b32 (fp32) -- the hardware transpose read replaces the
//                          reference's .transpose(-1,-2).contiguous() copies.
// The epilogue stages each wave's fp32 accumulators through LDS and writes whole rows with
// 16-byte stores.  Workgroup ids are XCD-remapped so tiles sharing an A panel share an L2.
#include "common.h"

namespace xdot {


namespace gemm {

constexpr int BM = 128, BN = 128, NT = 256;
constexpr int KC_ROW = 96;                  // bytes per row of a k-contiguous image
constexpr int KC_BYTES = 128 * KC_ROW;      // 12288
template <int ES> struct MCGeom {           // mn-contiguous image geometry
  static constexpr int BK = (ES == 2) ? 32 : 16;
  static constexpr int ROW = (ES == 2) ? (128 + 8) * 2 : 132 * 4;  // bytes
  static constexpr int BYTES = BK * ROW;
};
constexpr int IMG_BYTES = 12288;            // >= KC_BYTES and >= MCGeom<*>::BYTES
constexpr int STAGE_BYTES = 2 * IMG_BYTES;  // A image + B image
constexpr int LDS_BYTES = 2 * STAGE_BYTES;  // double buffer = 48 KiB
constexpr int EPI_ROW = 68 * 4;             // fp32 epilogue staging row (64 + 4 pad floats)
static_assert(MCGeom<2>::BYTES <= IMG_BYTES && MCGeom<4>::BYTES <= IMG_BYTES, "img");
static_assert(4 * 16 * EPI_ROW <= LDS_BYTES, "epilogue");

typedef __attribute__((address_space(3))) short lds_short;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// ---- global -> register staging ------------------------------------------------------
// Each thread stages 2 x 16 B per operand per K tile.
template <typename T, bool MC, bool VEC>
__device__ __forceinline__ void load_operand(u32x4 (&r)[2], const T* __restrict__ base,
                                             int64_t ld, int mn0, int MN, int k0, int K,
                                             int tid) {
  constexpr int ES = sizeof(T);
  constexpr int EPS = 16 / ES;             // elements per 16-byte slot
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + NT * i;
    int mn, k;
    if (!MC) { mn = v >> 2; k = (v & 3) * EPS; }          // [128 rows][4 slots]
    else     { constexpr int VPR = 128 / EPS; k = v / VPR; mn = (v % VPR) * EPS; }
    const int gm = mn0 + mn, gk = k0 + k;
    union { u32x4 u; T e[EPS]; } buf;
    if (!MC) {
      const T* p = base + (int64_t)gm * ld + gk;
      if (VEC && gm < MN && gk + EPS <= K) {
        buf.u = *reinterpret_cast<const u32x4*>(p);
      } else {
#pragma unroll
        for (int e = 0; e < EPS; ++e)
          buf.e[e] = (gm < MN && gk + e < K) ? p[e] : (T)0.0f;
      }
    } else {
      const T* p = base + (int64_t)gk * ld + gm;
      if (VEC && gk < K && gm + EPS <= MN) {
        buf.u = *reinterpret_cast<const u32x4*>(p);
      } else {
#pragma unroll
        for (int e = 0; e < EPS; ++e)
          buf.e[e] = (gk < K && gm + e < MN) ? p[e] : (T)0.0f;
      }
    }
    r[i] = buf.u;
  }
}

template <int ES, bool MC>
__device__ __forceinline__ void store_operand(char* img, const u32x4 (&r)[2], int tid) {
  constexpr int EPS = 16 / ES;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + NT * i;
    int off;
    if (!MC) off = (v >> 2) * KC_ROW + (v & 3) * 16;
    else { constexpr int VPR = 128 / EPS; off = (v / VPR) * MCGeom<ES>::ROW + (v % VPR) * 16; }
    *reinterpret_cast<u32x4*>(img + off) = r[i];
  }
}

// ---- LDS -> MFMA fragments -------------------------------------------------------------
// 16-bit types: fragment = 8 elements, element j <-> tile-k 8*(lane>>4) + j.
template <bool MC>
__device__ __forceinline__ u32x4 frag16(const char* img, int mn, int lane) {
  if (!MC) {
    return *reinterpret_cast<const u32x4*>(img + (mn + (lane & 15)) * KC_ROW + (lane >> 4) * 16);
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const char* a0 = img + (8 * g + q) * MCGeom<2>::ROW + (mn + 4 * p) * 2;
    const char* a1 = a0 + 4 * MCGeom<2>::ROW;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
    union { struct { s16x4 a, b; } s; u32x4 u; } cvt;
    cvt.s.a = lo; cvt.s.b = hi;
    return cvt.u;
  }
}
// fp32: fragment = 4 floats, element s <-> tile-k 4*(lane>>4) + s (MFMA s uses element s).
template <bool MC>
__device__ __forceinline__ f32x4 frag32(const char* img, int mn, int lane) {
  if (!MC) {
    return *reinterpret_cast<const f32x4*>(img + (mn + (lane & 15)) * KC_ROW + (lane >> 4) * 16);
  } else {
    f32x4 r;
    const char* a = img + (4 * (lane >> 4)) * MCGeom<4>::ROW + (mn + (lane & 15)) * 4;
#pragma unroll
    for (int s = 0; s < 4; ++s) r[s] = *reinterpret_cast<const float*>(a + s * MCGeom<4>::ROW);
    return r;
  }
}

template <int DTI> struct mfma16;
template <> struct mfma16<DT_BF16> {
  static __device__ __forceinline__ f32x4 run(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};
template <> struct mfma16<DT_F16> {
  static __device__ __forceinline__ f32x4 run(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
};

}  // namespace gemm

template <int DTI, int DTO, bool A_MC, bool B_MC, bool VEC>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs p) {
  using namespace gemm;
  using TI = typename dt_traits<DTI>::T;
  using TO = typename dt_traits<DTO>::T;
  constexpr int ES = sizeof(TI);
  constexpr int BK = (ES == 2) ? 32 : 16;

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // tile coordinates: XCD-aware remap, row-major over (tile_m, tile_n)
  const int ntile = p.tiles_m * p.tiles_n;
  const int t_lin = xcd_remap(blockIdx.x, gridDim.x);
  if (t_lin >= ntile) return;
  const int tile_m = t_lin / p.tiles_n, tile_n = t_lin % p.tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int z = blockIdx.y, z1 = z / p.nb2, z2 = z % p.nb2;

  const TI* A = reinterpret_cast<const TI*>(p.A) + z1 * p.sA1 + z2 * p.sA2;
  const TI* B = reinterpret_cast<const TI*>(p.B) + z1 * p.sB1 + z2 * p.sB2;
  TO* C = reinterpret_cast<TO*>(p.C) + z1 * p.sC1 + z2 * p.sC2;

  const int ktiles = (p.K + BK - 1) / BK;
  const int ntiles = ktiles * p.nseg;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[2], rb[2];
  auto load_tile = [&](int t) {
    const int seg = t / ktiles, k0 = (t % ktiles) * BK;
    load_operand<TI, A_MC, VEC>(ra, A + seg * p.sAseg, p.lda, m0, p.M, k0, p.K, tid);
    load_operand<TI, B_MC, VEC>(rb, B + seg * p.sBseg, p.ldb, n0, p.N, k0, p.K, tid);
  };
  auto store_tile = [&](int buf) {
    char* s = smem + buf * STAGE_BYTES;
    store_operand<ES, A_MC>(s, ra, tid);
    store_operand<ES, B_MC>(s + IMG_BYTES, rb, tid);
  };

  if (ntiles > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) load_tile(t + 1);  // global loads in flight under the MFMAs
    const char* sa = smem + cur * STAGE_BYTES;
    const char* sb = sa + IMG_BYTES;
    if constexpr (ES == 2) {
      u32x4 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag16<A_MC>(sa, wm * 64 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag16<B_MC>(sb, wn * 64 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16<DTI>::run(fa[i], fb[j], acc[i][j]);
    } else {
      f32x4 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag32<A_MC>(sa, wm * 64 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag32<B_MC>(sb, wn * 64 + j * 16, lane);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < ntiles) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: per wave, 4 passes of 16 rows x 64 cols through LDS ----
  char* ep = smem + wave * 16 * EPI_ROW;
  constexpr int EO = 16 / sizeof(TO);  // output elements per 16-byte store
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *reinterpret_cast<float*>(ep + ((lane >> 4) * 4 + r) * EPI_ROW + (j * 16 + (lane & 15)) * 4) =
            acc[i][j][r] * p.alpha;
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-private region, no barrier needed
    __builtin_amdgcn_wave_barrier();
    const int row = lane >> 2, c0 = (lane & 3) * 16;
    const int gm = m0 + wm * 64 + i * 16 + row;
    const int gn = n0 + wn * 64 + c0;
    const float* src = reinterpret_cast<const float*>(ep + row * EPI_ROW + c0 * 4);
    if (gm < p.M) {
      TO* dst = C + (int64_t)gm * p.ldc + gn;
      if (gn + 16 <= p.N) {  // 16-byte stores at any element-aligned address (u32x4_ua)
#pragma unroll
        for (int v = 0; v < 16 / EO; ++v) {
          union { u32x4 u; TO e[EO]; } o;
          if (p.beta != 0.f) {
            o.u = *reinterpret_cast<const u32x4_ua*>(dst + v * EO);
#pragma unroll
            for (int e = 0; e < EO; ++e) o.e[e] = (TO)(src[v * EO + e] + p.beta * (float)o.e[e]);
          } else {
#pragma unroll
            for (int e = 0; e < EO; ++e) o.e[e] = (TO)src[v * EO + e];
          }
          *reinterpret_cast<u32x4_ua*>(dst + v * EO) = o.u;
        }
      } else {
        for (int e = 0; e < 16; ++e)
          if (gn + e < p.N) dst[e] = (TO)(p.beta != 0.f ? src[e] + p.beta * (float)dst[e] : src[e]);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  }
}

// ----------------------------------------------------------------------------------------
template <int DTI, int DTO, bool AMC, bool BMC, bool VEC>
static void launch_t(const GemmArgs& a, int batches, hipStream_t st) {
  dim3 grid(a.tiles_m * a.tiles_n, batches);
  hipLaunchKernelGGL((gemm_kernel<DTI, DTO, AMC, BMC, VEC>), grid, dim3(256), gemm::LDS_BYTES, st, a);
}

template <int DTI, int DTO>
static void launch_d(const GemmArgs& a, int batches, bool amc, bool bmc, bool vec, hipStream_t st) {
#define G1_CASE(AM, BM_, V) \
  if (amc == AM && bmc == BM_ && vec == V) return launch_t<DTI, DTO, AM, BM_, V>(a, batches, st);
  G1_CASE(false, false, true) G1_CASE(false, true, true) G1_CASE(true, false, true) G1_CASE(true, true, true)
  G1_CASE(false, false, false) G1_CASE(false, true, false) G1_CASE(true, false, false) G1_CASE(true, true, false)
#undef G1_CASE
}

}  // namespace xdot

// C ABI launcher used by the torch binding.  Returns 0 on success, <0 on bad dtype combo.
extern "C" int xdot_gemm_launch(const xdot::GemmArgs* a, int batches, int dt_in, int dt_out,
                                int a_mc, int b_mc, int vec, hipStream_t st) {
  using namespace xdot;
  GemmArgs g = *a;
  g.tiles_m = (g.M + gemm::BM - 1) / gemm::BM;
  g.tiles_n = (g.N + gemm::BN - 1) / gemm::BN;
  if (g.tiles_m == 0 || g.tiles_n == 0 || batches == 0) return 0;
#define G1_DT(I, O) \
  if (dt_in == I && dt_out == O) { launch_d<I, O>(g, batches, a_mc, b_mc, vec, st); return 0; }
  G1_DT(DT_BF16, DT_BF16) G1_DT(DT_BF16, DT_F32) G1_DT(DT_F16, DT_F16) G1_DT(DT_F16, DT_F32)
  G1_DT(DT_F32, DT_F32) G1_DT(DT_F32, DT_BF16)
#undef G1_DT
  return -1;
}
