// xdot — exact-fp32 GEMM on the f32-input matrix cores of gfx950 (MI355X).
//
//   C[z](m, n) = alpha * sum_{s < nseg} sum_{k < K} opA_s[z](m, k) * opB_s[z](k, n) + beta * C[z](m, n)
//
// Same argument block and operand conventions as csrc/gemm.hip (GemmArgs: 2-level batch,
// K segments, per-operand storage order), for fp32 inputs and outputs: the reference computes
// every distributed product in fp32 (distributed_dot_product/multiplication/functions.py:96,142,
// 209 into the fp32 buffers of :86,198), so this kernel is what nt / tn / all and the module's
// projections run on at the reference's precision.  Every product is exact fp32
// (v_mfma_f32_32x32x2_f32: a k-ordered fmaf chain).
//
// Tiling: 128x128 output tile per 256-thread workgroup (4 waves 2x2, each 64x64 = 2x2 blocks of
// 32x32), K tiles of 32, staged global -> VGPR -> LDS (double-buffered, one barrier per K tile;
// the next tile's global loads fly under the current tile's 64 MFMAs = 4096 cycles per wave;
// a two-tile-ahead register ring measured no better).  Large products take the persistent
// 256x256 LDS-DMA kernel of csrc/gemm2_f32.hip; this one keeps small / unaligned ones.
// A K tile's 16 MFMA k-steps pair k = s (lane half 0) with k = 16 + s (lane half 1) for both
// operands.  Images keep the global storage order (coalesced loads, conflict-free 16-byte LDS
// writes): a k-contiguous operand as [mn][32 + 4 k] (a lane's 4 k-steps are one ds_read_b128;
// the 16-lane b128 groups are conflict-free), an mn-contiguous one as [k][128 + 4 mn] (one
// ds_read_b32 per MFMA operand: lanes read 32 consecutive mn).  The epilogue stores straight
// from the accumulators (lane = column: 128-byte row segments per half-wave).
#include "common.h"

namespace xdot {
namespace gf32 {

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;
constexpr int ROWK = BK + 4;                 // [mn][k] image row stride (floats)
constexpr int ROWM = 128 + 4;                // [k][mn] image row stride (floats)
constexpr int IMG = 128 * ROWK;              // floats per operand image (>= 32 * ROWM)
constexpr int STAGE = 2 * IMG;               // A + B
constexpr int LDS_BYTES = 2 * STAGE * 4;     // double buffer: 73,728 B
static_assert(32 * ROWM <= IMG, "image");

__device__ __forceinline__ f32x16 mm(float a, float b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// One operand tile (128 mn x 32 k) global -> registers: 4 x 16 B per thread.
//   k-contiguous (MC = false): thread loads 4 consecutive k of one mn row;
//   mn-contiguous (MC = true): thread loads 4 consecutive mn of one k row.
// Interior K tiles of 16-byte-aligned operands (VEC, k0 + BK <= K: wave-uniform) load without
// per-element predicates: mn positions past MN only feed outputs that are never stored, so they
// read a clamped valid address instead of zeros (an mn-contiguous chunk that starts below MN ends
// inside its ld row: ld % 4 == 0 under VEC).  Only the K-tail tile zero-fills element by element.
template <bool MC, bool VEC>
__device__ __forceinline__ void load_tile(f32x4 (&r)[4], const float* __restrict__ base, int64_t ld, int mn0, int MN,
                                          int k0, int K, int tid) {
  if (VEC && k0 + BK <= K) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int v = tid + NT * i;
      if (!MC) {
        const int gm = min(mn0 + (v >> 3), MN - 1);
        r[i] = *reinterpret_cast<const f32x4*>(base + (int64_t)gm * ld + k0 + (v & 7) * 4);
      } else {
        int gm = mn0 + (v & 31) * 4;
        gm = gm < MN ? gm : 0;
        r[i] = *reinterpret_cast<const f32x4*>(base + (int64_t)(k0 + (v >> 5)) * ld + gm);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int v = tid + NT * i;  // 0..1023
    int mn, k;
    if (!MC) { mn = v >> 3; k = (v & 7) * 4; }   // [128 rows][8 chunks]
    else { k = v >> 5; mn = (v & 31) * 4; }      // [32 k rows][32 chunks]
    const int gm = mn0 + mn, gk = k0 + k;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (!MC) {
      const float* p = base + (int64_t)gm * ld + gk;
      if (VEC && gm < MN && gk + 4 <= K) x = *reinterpret_cast<const f32x4*>(p);
      else {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = (gm < MN && gk + e < K) ? p[e] : 0.f;
      }
    } else {
      const float* p = base + (int64_t)gk * ld + gm;
      if (VEC && gk < K && gm + 4 <= MN) x = *reinterpret_cast<const f32x4*>(p);
      else {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = (gk < K && gm + e < MN) ? p[e] : 0.f;
      }
    }
    r[i] = x;
  }
}

template <bool MC>
__device__ __forceinline__ void store_tile(float* img, const f32x4 (&r)[4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int v = tid + NT * i;
    if (!MC) *reinterpret_cast<f32x4*>(img + (v >> 3) * ROWK + (v & 7) * 4) = r[i];
    else *reinterpret_cast<f32x4*>(img + (v >> 5) * ROWM + (v & 31) * 4) = r[i];
  }
}

// k = 16 hf + 4 g + t (t = 0..3) of fragment row `mn` (the lane's row / column of a 32-block)
template <bool MC>
__device__ __forceinline__ f32x4 frag4(const float* img, int mn, int g, int hf) {
  if (!MC) return *reinterpret_cast<const f32x4*>(img + mn * ROWK + 16 * hf + 4 * g);
  const float* p = img + (16 * hf + 4 * g) * ROWM + mn;
  return f32x4{p[0], p[ROWM], p[2 * ROWM], p[3 * ROWM]};
}

}  // namespace gf32

template <bool A_MC, bool B_MC, bool VEC>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(GemmArgs p) {
  using namespace gf32;
  extern __shared__ __attribute__((aligned(16))) float smf[];
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int ntile = p.tiles_m * p.tiles_n;
  const int t_lin = xcd_remap(blockIdx.x, gridDim.x);
  if (t_lin >= ntile) return;
  // groups of GM tile rows walked column-major: an XCD's concurrent tiles share GM A panels and
  // a few B panels in its L2 instead of streaming a fresh B panel per tile
  constexpr int GM = 8;
  const int gsz = GM * p.tiles_n, first_m = (t_lin / gsz) * GM;
  const int gm_n = min(GM, p.tiles_m - first_m);
  const int tile_m = first_m + (t_lin % gsz) % gm_n, tile_n = (t_lin % gsz) / gm_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int z = blockIdx.y, z1 = z / p.nb2, z2 = z % p.nb2;
  const float* A = reinterpret_cast<const float*>(p.A) + z1 * p.sA1 + z2 * p.sA2;
  const float* B = reinterpret_cast<const float*>(p.B) + z1 * p.sB1 + z2 * p.sB2;
  float* C = reinterpret_cast<float*>(p.C) + z1 * p.sC1 + z2 * p.sC2;
  const int ktiles = (p.K + BK - 1) / BK, ntiles = ktiles * p.nseg;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  const int ar = wm * 64 + (lane & 31), br = wn * 64 + (lane & 31);  // + 32 i: the lane's fragment rows
  // 16 k-steps of one LDS stage: 4 groups of 4, operand reads one group ahead
  auto compute = [&](int cur) {
    const float* sa = smf + cur * STAGE;
    const float* sb = sa + IMG;
    f32x4 a0[2], b0[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      a0[i] = gf32::frag4<A_MC>(sa, ar + 32 * i, 0, hf);
      b0[i] = gf32::frag4<B_MC>(sb, br + 32 * i, 0, hf);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 a1[2] = {a0[0], a0[1]}, b1[2] = {b0[0], b0[1]};
      if (g + 1 < 4) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          a1[i] = gf32::frag4<A_MC>(sa, ar + 32 * i, g + 1, hf);
          b1[i] = gf32::frag4<B_MC>(sb, br + 32 * i, g + 1, hf);
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = gf32::mm(a0[i][s], b0[j][s], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a0[i] = a1[i];
        b0[i] = b1[i];
      }
    }
  };
  struct Regs {
    f32x4 a[4], b[4];
  };
  auto load = [&](Regs& r, int t) {
    const int seg = t / ktiles, k0 = (t % ktiles) * BK;
    gf32::load_tile<A_MC, VEC>(r.a, A + seg * p.sAseg, p.lda, m0, p.M, k0, p.K, tid);
    gf32::load_tile<B_MC, VEC>(r.b, B + seg * p.sBseg, p.ldb, n0, p.N, k0, p.K, tid);
  };
  auto store = [&](const Regs& r, int buf) {
    float* s = smf + buf * STAGE;
    gf32::store_tile<A_MC>(s, r.a, tid);
    gf32::store_tile<B_MC>(s + IMG, r.b, tid);
  };
  Regs r0;
  if (ntiles > 0) {
    load(r0, 0);
    store(r0, 0);
  }
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    if (t + 1 < ntiles) load(r0, t + 1);
    compute(t & 1);
    if (t + 1 < ntiles) store(r0, (t + 1) & 1);
    __syncthreads();
  }

  // epilogue: register r of block (i, j) = row wm*64 + 32i + (r&3) + 8(r>>2) + 4hf, column
  // wn*64 + 32j + (lane & 31)
  const float alpha = p.alpha, beta = p.beta;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int gn = n0 + wn * 64 + 32 * j + (lane & 31);
      if (gn >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gm = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hf;
        if (gm < p.M) {
          float* d = C + (int64_t)gm * p.ldc + gn;
          const float v = acc[i][j][r] * alpha;
          *d = beta != 0.f ? v + beta * *d : v;
        }
      }
    }
}

namespace {
template <bool AMC, bool BMC, bool V>
void launch_gf32(const GemmArgs& a, int batches, hipStream_t st) {
  const dim3 grid(a.tiles_m * a.tiles_n, batches);
  hipLaunchKernelGGL((gemm_f32_kernel<AMC, BMC, V>), grid, dim3(256), gf32::LDS_BYTES, st, a);
}
}  // namespace

}  // namespace xdot

// fp32 in / fp32 out; vec: 16-byte aligned operand bases and leading dims / strides
extern "C" int xdot_gemm_f32_launch(const xdot::GemmArgs* a, int batches, int a_mc, int b_mc, int vec,
                                    hipStream_t st) {
  using namespace xdot;
  GemmArgs g = *a;
  g.tiles_m = (g.M + gf32::BM - 1) / gf32::BM;
  g.tiles_n = (g.N + gf32::BN - 1) / gf32::BN;
  if (g.tiles_m == 0 || g.tiles_n == 0 || batches == 0) return 0;
#define GF(AM, BM_, V) \
  if (a_mc == AM && b_mc == BM_ && (vec != 0) == V) { launch_gf32<AM, BM_, V>(g, batches, st); return 0; }
  GF(false, false, true) GF(false, true, true) GF(true, false, true) GF(true, true, true)
  GF(false, false, false) GF(false, true, false) GF(true, false, false) GF(true, true, false)
#undef GF
  return -1;
}
