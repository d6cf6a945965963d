// xdot — torch operator bindings for the gfx950 kernels (registered as torch.ops.xdot.*).
//
// The kernels themselves live in *.hip translation units that do not include any torch
// header (fast rebuilds); this file only validates arguments on the host, resolves the
// current HIP stream and calls the C-ABI launchers.  Every launch is bounds-checked on
// the host against the tensors' storage so a bad stride can never turn into a GPU fault.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include "kernels.h"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

// sha256 of csrc/* + flags, compiled in by xdot/build.py (build/xdot/build_id.cpp)
extern "C" const char xdot_build_id[];

namespace {

std::string build_id() { return std::string(xdot_build_id + 14); }  // after "XDOT_BUILD_ID="

// roctx ranges around every op (visible in rocprofv3 --marker-trace timelines); enabled by
// XDOT_ROCTX=1 so the default path pays one predictable branch.
bool roctx_on() {
  static const bool v = [] {
    const char* e = std::getenv("XDOT_ROCTX");
    return e && e[0] == '1';
  }();
  return v;
}
struct Range {
  bool on;
  explicit Range(const char* name) : on(roctx_on()) {
    if (on) roctxRangePushA(name);
  }
  ~Range() {
    if (on) roctxRangePop();
  }
};



int dt_code(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return xdot::DT_F32;
    case at::kBFloat16: return xdot::DT_BF16;
    case at::kHalf: return xdot::DT_F16;
    default: TORCH_CHECK(false, "xdot: unsupported dtype ", t);
  }
  return -1;
}

hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

// elements addressable from t.data_ptr() to the end of its storage
int64_t avail_elems(const at::Tensor& t) {
  const int64_t bytes = (int64_t)t.storage().nbytes() - t.storage_offset() * (int64_t)t.element_size();
  return bytes / (int64_t)t.element_size();
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// XDOT_GEMM_LIB: which plain large products may take the library GEMM (at::baddbmm ->
// hipBLASLt) on in-place strided views.  Default (unset / 0) = none: 16-bit products run gemm3
// (matches or beats the library), exact-fp32 products the 128x128 f32-MFMA kernel of
// csrc/gemm_f32.hip.  "fp32" = exact-fp32 plain products on the library (the round-4 default,
// kept for A/B); 1 = 16-bit products too (round-2 route).
int gemm_lib() {
  static const int v = [] {
    const char* e = std::getenv("XDOT_GEMM_LIB");
    if (e && e[0] == '1') return 2;
    if (e && (e[0] == 'f' || e[0] == 'F')) return 1;  // fp32 only
    return 0;
  }();
  return v;
}

// exact-fp32 products: the f32-MFMA kernel of csrc/gemm_f32.hip (fp32 out); anything else (an
// fp32 -> 16-bit output) the generic kernel
int gemm_exact(const xdot::GemmArgs* g, int batches, int dt_in, int dt_out, bool a_mc, bool b_mc, bool vec,
               hipStream_t st) {
  if (dt_in == xdot::DT_F32 && dt_out == xdot::DT_F32) return xdot_gemm_f32_launch(g, batches, a_mc, b_mc, vec, st);
  return xdot_gemm_launch(g, batches, dt_in, dt_out, a_mc, b_mc, vec, st);
}

// The library route of xdot.gemm: true when it ran.  opA / opB / C are expressed as strided
// views of the operands' storage (no copies; the BLAS reads leading dimensions / batch
// strides directly).  Measured (scripts/gemm_lib_ab.sh, MI355X): hipBLASLt 1.2-1.35x the
// 256x256 kernel on bf16 nt 75000^2 x 768 and all 75000 x 768 x 75000, 1.2x the 128x128 fp32
// kernel; the xdot kernels stay ahead on skinny long-K bf16 products (all3: 25000 x 768 x
// 75000, split-K: 1.4x) and own every layout a single strided batch cannot express (two batch
// levels, scattered K segments, mixed dtypes, small products).
// split-K: fewest k-slices S minimising ceil(items / CUs) / S (idle CUs of the last round),
// each slice >= 4 k-tiles of 64, with a 3 % charge per slice for the fp32 partial round trip
int64_t pick_splits(int64_t tiles, int64_t kt64) {
  const int64_t ncu = 256;
  int64_t S = 1;
  double best = 1e300;
  for (int64_t s = 1; s <= 64 && (s == 1 || kt64 / s >= 4); ++s) {
    const double cost = (double)((tiles * s + ncu - 1) / ncu) / (double)s * (1.0 + 0.03 * (s - 1));
    if (cost < best * 0.98) { best = cost; S = s; }
  }
  return S;
}

// XDOT_GEMM3: 1 (default) = the automatic path tries the 8-phase kernel first (csrc/gemm3.hip)
int gemm3_auto() {
  static const int v = [] {
    const char* e = std::getenv("XDOT_GEMM3");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v;
}

bool gemm_library(const at::Tensor& A, const at::Tensor& B, at::Tensor& C, int64_t M, int64_t N, int64_t K,
                  int64_t nseg, int64_t nb1, int64_t nb2, int64_t lda, int64_t ldb, int64_t ldc, int64_t sA1,
                  int64_t sA2, int64_t sB1, int64_t sB2, int64_t sC1, int64_t sC2, int64_t sAseg, int64_t sBseg,
                  bool a_mc, bool b_mc, double alpha, double beta) {
  if (C.scalar_type() != A.scalar_type() || K == 0) return false;
  // one batch level
  int64_t nb = nb1 * nb2, sa = 0, sb = 0, sc = 0;
  if (nb1 == 1) { sa = sA2; sb = sB2; sc = sC2; }
  else if (nb2 == 1) { sa = sA1; sb = sB1; sc = sC1; }
  else if (sA1 == nb2 * sA2 && sB1 == nb2 * sB2 && sC1 == nb2 * sC2) { sa = sA2; sb = sB2; sc = sC2; }
  else return false;
  // K segments that continue each other are one longer K
  if (nseg > 1) {
    if (sAseg != (a_mc ? K * lda : K) || sBseg != (b_mc ? K * ldb : K)) return false;
    K *= nseg;
  }
  // conservative output layouts only: every output batch its own dense matrix (no batches
  // interleaved inside one output row -- the per-rank column blocks of nt's (P, R, T) output,
  // which faulted on this route, stay on the xdot kernels); input batches may interleave or be
  // broadcast (tn's column blocks of `left` against one `right`: verified against torch in
  // tests/test_gemm2_gpu.py); 16-byte aligned bases, leading dims and batch strides
  if (nb > 1 && (sa < 0 || sb < 0 || sc < M * ldc)) return false;
  const int64_t ev = 16 / (int64_t)A.element_size();
  auto al = [&](int64_t v) { return v % ev == 0; };
  if (ldc != N) return false;  // whole output rows (no column-slice views)
  if (!aligned16(A.data_ptr()) || !aligned16(B.data_ptr()) || !aligned16(C.data_ptr()) || !al(lda) || !al(ldb) ||
      !al(ldc) || (nb > 1 && (!al(sa) || !al(sb) || !al(sc))))
    return false;
  // 16-bit: only where the output alone fills >= 2 rounds of 256x256 tiles (skinny long-K
  // products keep the split-K kernel); fp32: the library's exact-fp32 GEMM is ahead everywhere
  // measured (1.1-1.2x the 128x128 kernel), so every large plain product
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256) * nb;
  const double flop = 2.0 * (double)M * (double)N * (double)K * (double)nb;
  if (flop < 2e10 || (A.element_size() == 2 && tiles < 512)) return false;
  const int64_t oa = A.storage_offset(), ob = B.storage_offset(), oc = C.storage_offset();
  at::Tensor a = A.as_strided({nb, M, K}, {nb > 1 ? sa : M * K, a_mc ? 1 : lda, a_mc ? lda : 1}, oa);
  at::Tensor b = B.as_strided({nb, K, N}, {nb > 1 ? sb : K * N, b_mc ? ldb : 1, b_mc ? 1 : ldb}, ob);
  at::Tensor c = C.as_strided({nb, M, N}, {nb > 1 ? sc : M * N, ldc, 1}, oc);
  if (nb == 1) {
    at::Tensor c2 = c.select(0, 0);
    at::addmm_out(c2, c2, a.select(0, 0), b.select(0, 0), beta, alpha);
  } else {
    at::baddbmm_out(c, c, a, b, beta, alpha);
  }
  return true;
}

void check_launch(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "xdot: ", what, " launch failed: ", hipGetErrorString(e));
}

// ------------------------------------------------------------------------------------
void gemm(const at::Tensor& A, const at::Tensor& B, at::Tensor& C, int64_t M, int64_t N,
          int64_t K, int64_t nseg, int64_t nb1, int64_t nb2, int64_t lda, int64_t ldb,
          int64_t ldc, int64_t sA1, int64_t sA2, int64_t sB1, int64_t sB2, int64_t sC1,
          int64_t sC2, int64_t sAseg, int64_t sBseg, bool a_mc, bool b_mc, double alpha, double beta,
          int64_t path) {
  Range rr_("xdot.gemm");
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda(), "xdot.gemm: tensors must be on GPU");
  TORCH_CHECK(A.scalar_type() == B.scalar_type(), "xdot.gemm: A/B dtype mismatch");
  TORCH_CHECK(M >= 0 && N >= 0 && K >= 0 && nseg >= 1 && nb1 >= 1 && nb2 >= 1, "xdot.gemm: bad sizes");
  if (M == 0 || N == 0) return;
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31), "xdot.gemm: dim too large");
  TORCH_CHECK(nb1 * nb2 <= 65535, "xdot.gemm: too many batches");
  // host-side bounds check of the furthest element each operand touches
  auto last = [](int64_t b1, int64_t s1, int64_t b2, int64_t s2, int64_t ns, int64_t ss) {
    return (b1 - 1) * s1 + (b2 - 1) * s2 + (ns - 1) * ss;
  };
  if (K > 0) {
    const int64_t la = last(nb1, sA1, nb2, sA2, nseg, sAseg) + (a_mc ? (K - 1) * lda + (M - 1) : (M - 1) * lda + (K - 1));
    const int64_t lb = last(nb1, sB1, nb2, sB2, nseg, sBseg) + (b_mc ? (K - 1) * ldb + (N - 1) : (N - 1) * ldb + (K - 1));
    TORCH_CHECK(la < avail_elems(A), "xdot.gemm: A access out of bounds (", la, " >= ", avail_elems(A), ")");
    TORCH_CHECK(lb < avail_elems(B), "xdot.gemm: B access out of bounds (", lb, " >= ", avail_elems(B), ")");
  }
  const int64_t lc = last(nb1, sC1, nb2, sC2, 1, 0) + (M - 1) * ldc + (N - 1);
  TORCH_CHECK(lc < avail_elems(C), "xdot.gemm: C access out of bounds");

  const int eps = 16 / (int)A.element_size();
  auto mult = [&](int64_t v) { return v % eps == 0; };
  // operand loads vectorise on A/B alignment alone; the output is stored 16 bytes at a time
  // wherever the address allows, element by element elsewhere (the kernels test each strip's
  // address: an odd column block of nt's (P, R, T) output at T/N = 3125 must not turn every
  // operand load of the GEMM into element loads)
  bool vec = aligned16(A.data_ptr()) && aligned16(B.data_ptr()) &&
             mult(lda) && mult(ldb) && mult(sA1) && mult(sA2) && mult(sB1) && mult(sB2) &&
             mult(sAseg) && mult(sBseg);

  xdot::GemmArgs g{};
  g.A = A.data_ptr(); g.B = B.data_ptr(); g.C = C.data_ptr();
  g.M = (int)M; g.N = (int)N; g.K = (int)K; g.nseg = (int)nseg; g.nb2 = (int)nb2;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.sA1 = sA1; g.sA2 = sA2; g.sB1 = sB1; g.sB2 = sB2; g.sC1 = sC1; g.sC2 = sC2;
  g.sAseg = sAseg; g.sBseg = sBseg; g.alpha = (float)alpha; g.beta = (float)beta;
  c10::DeviceGuard guard(A.device());
  // v2 (256x256 tiles, LDS-DMA, csrc/gemm2.hip) for 16-bit operands whose layout meets its
  // alignment rules and whose output fills 256-wide tiles; split-K when the tiles alone would
  // leave CUs idle.  path: 0 = auto, 1 = v1, 2 = v2 whenever its layout rules hold (per call)
  int mode = (int)path;
  // fp32 operands on the bf16 matrix pipe (path 6 = automatic with split allowed, which Python
  // passes under XDOT_FP32_MODE=split; path 4 forces it): hi/lo bf16 copies, three bf16 products
  // in one gemm3 call (csrc/gemm3.hip, split3_kernel).  The mode is decided in Python only
  // (xdot.ops.gemm.strided_gemm reads FLAGS.fp32_mode per call): no second source of truth here.
  if (A.scalar_type() == at::kFloat && (mode == 4 || (mode == 6 && gemm3_auto()))) {
    const int64_t tpb = ((M + 255) / 256) * ((N + 255) / 256);
    // worth it when three bf16 products plus the operand copies (read 4 B, write 6 B per
    // element) beat one exact fp32 product: a product whose operand is far larger than its
    // output (the materialised P.V: 2.5 GB of P per head) keeps the exact kernel
    // Both sides are priced at the fraction of the 256 CUs their grid fills: the exact kernel
    // has no split-K (128x128 tiles), gemm3 splits K (pick_splits), so a product with few
    // output tiles and a long K (the K = T weight-side products of the autograd ops) goes split.
    const double flop = 2.0 * (double)M * N * K * nseg * nb1 * nb2;
    const double elems = (double)nb1 * nb2 * nseg * K * ((double)M + (double)N);
    const int64_t t128 = ((M + 127) / 128) * ((N + 127) / 128) * nb1 * nb2;
    const int64_t s3 = pick_splits(tpb * nb1 * nb2, 3 * nseg * ((K + 63) / 64));
    const double fill1 = std::min(1.0, (double)t128 / 256.0);
    const double fill3 = std::min(1.0, (double)(tpb * nb1 * nb2 * s3) / 256.0);
    const double t_split = 3.0 * flop / (1.1e15 * fill3) + 10.0 * elems / 5e12 +
                           (s3 > 1 ? 8.0 * (double)s3 * M * N * nb1 * nb2 / 5e12 : 0.0);
    const double t_exact = flop / (1.15e14 * fill1);
    // the hi/lo copies are transient HBM (6 B per operand element): never more than a quarter of
    // what is free, else the exact kernel (no extra memory) runs
    const double copy_bytes = 6.0 * elems;
    bool fits = copy_bytes < 1e9;
    if (!fits) {
      size_t fr = 0, tot = 0;
      fits = hipMemGetInfo(&fr, &tot) == hipSuccess && copy_bytes < 0.25 * (double)fr;
    }
    const bool big = flop >= 2e9 && t_split < t_exact && fits;
    const bool ok = beta == 0.0 && K > 0 && M >= 256 && N >= 256 && K % 8 == 0 && (!a_mc || M % 8 == 0) &&
                    (!b_mc || N % 8 == 0) && C.scalar_type() == at::kFloat && nb1 * nb2 * 3 * nseg <= 65535;
    TORCH_CHECK(mode != 4 || ok, "xdot.gemm: path 4 (split fp32) not eligible for this call");
    if (ok && (mode == 4 || big)) {
      const int64_t Ra = a_mc ? K : M, Ca = a_mc ? M : K, Rb = b_mc ? K : N, Cb = b_mc ? N : K;
      at::Tensor a3 = at::empty({nb1 * nb2 * 3 * nseg * Ra * Ca}, A.options().dtype(at::kBFloat16));
      at::Tensor b3 = at::empty({nb1 * nb2 * 3 * nseg * Rb * Cb}, A.options().dtype(at::kBFloat16));
      hipStream_t st = cur_stream(A);
      // A' = [hi, lo, hi], B' = [hi, hi, lo]: hi.hi + lo.hi + hi.lo
      xdot_split3_launch(A.data_ptr<float>(), a3.data_ptr(), sA1, sA2, sAseg, lda, (int)nb1, (int)nb2, (int)nseg,
                         (int)Ra, (int)Ca, 0b010, st);
      xdot_split3_launch(B.data_ptr<float>(), b3.data_ptr(), sB1, sB2, sBseg, ldb, (int)nb1, (int)nb2, (int)nseg,
                         (int)Rb, (int)Cb, 0b100, st);
      check_launch(hipGetLastError(), "split3");
      xdot::GemmArgs g3a = g;
      g3a.A = a3.data_ptr();
      g3a.B = b3.data_ptr();
      g3a.nseg = (int)(3 * nseg);
      g3a.lda = Ca;
      g3a.ldb = Cb;
      g3a.sAseg = Ra * Ca;
      g3a.sBseg = Rb * Cb;
      g3a.sA2 = 3 * nseg * Ra * Ca;
      g3a.sA1 = nb2 * g3a.sA2;
      g3a.sB2 = 3 * nseg * Rb * Cb;
      g3a.sB1 = nb2 * g3a.sB2;
      const int64_t tiles = tpb * nb1 * nb2;
      const int64_t kt64 = 3 * nseg * ((K + 63) / 64);
      const int64_t S = pick_splits(tiles, kt64);
      at::Tensor ws;
      if (S > 1) ws = at::empty({S * nb1 * nb2 * M * N}, A.options().dtype(at::kFloat));
      const int rc3 = xdot_gemm3_launch(&g3a, (int)(nb1 * nb2), xdot::DT_BF16, xdot::DT_F32, a_mc, b_mc, (int)S,
                                        S > 1 ? ws.data_ptr<float>() : nullptr, st);
      TORCH_CHECK(rc3 == 0, "xdot.gemm: split fp32 gemm3 launch declined (", rc3, ")");
      check_launch(hipGetLastError(), "gemm3 (split fp32)");
      return;
    }
  }
  if (mode == 6) mode = 0;
  if (mode == 0 && (gemm_lib() == 2 || (gemm_lib() == 1 && A.scalar_type() == at::kFloat)) &&
      gemm_library(A, B, C, M, N, K, nseg, nb1, nb2, lda, ldb, ldc, sA1, sA2, sB1, sB2, sC1, sC2, sAseg, sBseg, a_mc,
                   b_mc, alpha, beta))
    return;
  // exact fp32: the persistent 256x256 LDS-DMA kernel (csrc/gemm2_f32.hip) where its layout rules
  // hold and the output has at least one 128-wide tile in each direction; split-K
  // (pick_splits over 32-deep k-tiles, partials <= 512 MB) when the tiles alone leave CUs idle.
  // path 1 keeps the 128x128 kernel, path 2 forces this one.
  if (A.scalar_type() == at::kFloat && C.scalar_type() == at::kFloat && vec && K > 0 && mode != 1) {
    const bool ok = (a_mc || K % 4 == 0) && (b_mc || K % 4 == 0) && (!a_mc || M % 4 == 0) && (!b_mc || N % 4 == 0);
    TORCH_CHECK(mode != 2 || ok, "xdot.gemm: path 2 (fp32 v2) needs K % 4 == 0 for k-contiguous operands and "
                                 "an mn extent % 4 == 0 for mn-contiguous ones");
    const int64_t nb = nb1 * nb2;
    const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256) * nb;
    // auto: >= 2 rounds of 256x256 tiles, or a long K (split-K fills the GPU).  Short-K products
    // with few tiles (the 25000 x 768 x 768 projections: 294 tiles, K = 768) stay on the 128x128
    // kernel: 82-94 TF/s there vs 63-65 for this one split 4-6 ways (r5s9)
    if (ok && (mode == 2 || (M >= 128 && N >= 128 && (tiles >= 2 * 256 || (int64_t)K * nseg >= 4096)))) {
      int64_t S = pick_splits(tiles, nseg * ((K + 31) / 32));
      while (S > 1 && S * nb * M * N > (128LL << 20)) --S;
      at::Tensor ws;
      if (S > 1) ws = at::empty({S * nb * M * N}, A.options().dtype(at::kFloat));
      const int rc = xdot_gemm2_f32_launch(&g, (int)nb, a_mc, b_mc, (int)S, S > 1 ? ws.data_ptr<float>() : nullptr,
                                           cur_stream(A));
      if (rc == 0) {
        check_launch(hipGetLastError(), "gemm2_f32");
        return;
      }
    }
  }
  const bool half = A.element_size() == 2;
  bool v2 = half && vec && mode != 1;
  if (v2 && (!a_mc || !b_mc)) v2 = K % 8 == 0;
  if (v2 && a_mc) v2 = M % 8 == 0;
  if (v2 && b_mc) v2 = N % 8 == 0;
  if (v2 && mode != 2 && mode != 3 && mode != 5) {
    // auto: enough 256x256 tiles (>= 32 per batch entry or >= 512 overall) -- small outputs
    // batched over K slabs (the split-K weight gradients of xdot.ops.linear) keep the 128x128
    // kernel, which fills the GPU without a second split.  Skinny outputs (one side 64..191,
    // e.g. N = head dim 96 in the materialised path) still go to v2: streaming the long operand
    // through its deeper LDS-DMA ring beats v1's register staging even with 62 % of the tile
    // idle (materialised step 39.3 -> 34.2 ms at T = 25000)
    const int64_t tpb = ((M + 255) / 256) * ((N + 255) / 256);
    v2 = M >= 64 && N >= 64 && (tpb >= 32 || tpb * nb1 * nb2 >= 512);
  }
  TORCH_CHECK(mode != 3 || (v2 && K > 0), "xdot.gemm: path 3 (gemm3) needs 16-bit operands with aligned layouts");
  if (v2 && K > 0) {
    // split-K: fewest k-slices S minimising ceil(items / CUs) / S (idle CUs of the last round),
    // each slice >= 4 k-tiles of 64, with a 3 % charge per slice for the fp32 partial round trip
    const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256) * nb1 * nb2;
    const int64_t kt64 = nseg * ((K + 63) / 64);
    const int64_t ncu = 256;
    const int64_t S = pick_splits(tiles, kt64);
    at::Tensor ws;
    if (S > 1) ws = at::empty({S * nb1 * nb2 * M * N}, A.options().dtype(at::kFloat));
    // v3 (8-phase 16x16x32, csrc/gemm3.hip) first: beta = 0, M and N >= 256; it declines
    // (-3) the rest, which the v2 kernel takes
    if (mode == 3 || mode == 5 || (mode == 0 && gemm3_auto())) {
      const int rc3 = xdot_gemm3_launch(&g, (int)(nb1 * nb2), dt_code(A.scalar_type()), dt_code(C.scalar_type()),
                                        a_mc, b_mc, (int)S, S > 1 ? ws.data_ptr<float>() : nullptr, cur_stream(A));
      TORCH_CHECK(mode != 3 || rc3 == 0, "xdot.gemm: path 3 (gemm3) not eligible for this call (", rc3, ")");
      if (rc3 == 0) {
        check_launch(hipGetLastError(), "gemm3");
        return;
      }
    }
    const int rc2 = xdot_gemm2_launch(&g, (int)(nb1 * nb2), dt_code(A.scalar_type()), dt_code(C.scalar_type()),
                                      a_mc, b_mc, (int)S, S > 1 ? ws.data_ptr<float>() : nullptr, cur_stream(A));
    if (rc2 == 0) {
      check_launch(hipGetLastError(), "gemm2");
      return;
    }
  }
  // K slabs for the 128x128 kernel (the exact-fp32 path): a product with few output tiles and a
  // long K (the K = T weight-side products of the autograd ops: e.g. 1562 x 768 x 12496 = 78
  // tiles) would leave most CUs idle.  Slab s of every (batch, segment) is one outer batch entry
  // writing an fp32 partial; one ordered sum (gemm2_reduce) applies alpha / beta / the cast.
  if (mode == 0 && nb1 == 1 && K >= 1024) {
    const int64_t tiles = ((M + 127) / 128) * ((N + 127) / 128) * nb2;
    if (tiles < 384) {
      int64_t S = std::min<int64_t>(std::min<int64_t>((768 + tiles - 1) / tiles, K / 256), 32);
      S = std::min<int64_t>(S, (int64_t)(64 << 20) / std::max<int64_t>(1, nb2 * M * N));  // partials <= 256 MB
      int64_t Ks = ((K + S - 1) / S + 15) / 16 * 16;
      S = (K + Ks - 1) / Ks;
      if (S >= 2) {
        at::Tensor ws = at::empty({S * nb2 * M * N}, A.options().dtype(at::kFloat));
        xdot::GemmArgs gs = g;
        gs.C = ws.data_ptr();
        gs.ldc = N;
        gs.sC2 = M * N;
        gs.sC1 = nb2 * M * N;
        gs.alpha = 1.f;
        gs.beta = 0.f;
        gs.sA1 = a_mc ? Ks * lda : Ks;
        gs.sB1 = b_mc ? Ks * ldb : Ks;
        gs.K = (int)Ks;
        const int full = (int)(K / Ks) == S ? (int)S : (int)S - 1;
        const bool vs = vec && (Ks * (a_mc ? lda : 1)) % eps == 0 && (Ks * (b_mc ? ldb : 1)) % eps == 0;
        int rc1 = gemm_exact(&gs, full * (int)nb2, dt_code(A.scalar_type()), xdot::DT_F32, a_mc, b_mc, vs,
                             cur_stream(A));
        if (rc1 == 0 && full < S) {  // the short last slab
          xdot::GemmArgs gl = gs;
          const int64_t k0 = (int64_t)full * Ks;
          gl.A = static_cast<const char*>(A.data_ptr()) + A.element_size() * (a_mc ? k0 * lda : k0);
          gl.B = static_cast<const char*>(B.data_ptr()) + B.element_size() * (b_mc ? k0 * ldb : k0);
          gl.C = ws.data_ptr<float>() + (int64_t)full * nb2 * M * N;
          gl.K = (int)(K - k0);
          const bool vl = vs && (a_mc ? k0 * lda : k0) % eps == 0 && (b_mc ? k0 * ldb : k0) % eps == 0;
          rc1 = gemm_exact(&gl, (int)nb2, dt_code(A.scalar_type()), xdot::DT_F32, a_mc, b_mc, vl, cur_stream(A));
        }
        TORCH_CHECK(rc1 == 0, "xdot.gemm: unsupported dtype combination ", A.scalar_type(), " -> fp32 slabs");
        check_launch(hipGetLastError(), "gemm (K slabs)");
        TORCH_CHECK(xdot_gemm_reduce_launch(&g, ws.data_ptr<float>(), (int)S, (int)nb2, dt_code(C.scalar_type()),
                                            cur_stream(A)) == 0, "xdot.gemm: slab reduce dtype");
        check_launch(hipGetLastError(), "gemm slab reduce");
        return;
      }
    }
  }
  const int rc = gemm_exact(&g, (int)(nb1 * nb2), dt_code(A.scalar_type()), dt_code(C.scalar_type()), a_mc, b_mc,
                            vec, cur_stream(A));
  TORCH_CHECK(rc == 0, "xdot.gemm: unsupported dtype combination ", A.scalar_type(), " -> ", C.scalar_type());
  check_launch(hipGetLastError(), "gemm");
}

// ------------------------------------------------------------------------------------
at::Tensor softmax_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& mask, double scale,
                       int64_t mdiv, int64_t mmul, int64_t mmod) {
  Range rr_("xdot.softmax_fwd");
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "xdot.softmax_fwd: x must be a contiguous GPU tensor");
  const int64_t T = x.size(-1);
  const int64_t rows = T == 0 ? 0 : x.numel() / T;
  auto y = at::empty_like(x);
  xdot::smx::Args a{};
  a.x = x.data_ptr(); a.out = y.data_ptr(); a.rows = rows; a.T = T; a.scale = (float)scale;
  a.mdiv = mdiv; a.mmul = mmul; a.mmod = mmod; a.mask = nullptr;
  bool vec = (T % 8 == 0) && aligned16(x.data_ptr()) && aligned16(y.data_ptr());
  if (mask.has_value() && mask->defined()) {
    const auto& m = *mask;
    TORCH_CHECK(m.is_cuda() && m.is_contiguous() && m.scalar_type() == at::kBool, "xdot.softmax_fwd: mask must be contiguous bool on GPU");
    TORCH_CHECK(m.size(-1) == T, "xdot.softmax_fwd: mask last dim mismatch");
    TORCH_CHECK(mdiv > 0 && mmod > 0, "xdot.softmax_fwd: bad mask row map");
    const int64_t mrows = m.numel() / T;
    // furthest mask row touched
    const int64_t lr = ((rows - 1) / mdiv) * mmul + std::min<int64_t>(rows - 1, mmod - 1);
    TORCH_CHECK(rows == 0 || lr < mrows, "xdot.softmax_fwd: mask row map out of bounds");
    a.mask = reinterpret_cast<const uint8_t*>(m.data_ptr());
    vec = vec && ((reinterpret_cast<uintptr_t>(m.data_ptr()) & 7) == 0);
  }
  TORCH_CHECK(rows <= 0x7fffffff, "xdot.softmax_fwd: too many rows");
  c10::DeviceGuard guard(x.device());
  TORCH_CHECK(xdot_softmax_fwd_launch(&a, dt_code(x.scalar_type()), vec, cur_stream(x)) == 0, "xdot.softmax_fwd: dtype");
  check_launch(hipGetLastError(), "softmax_fwd");
  return y;
}

at::Tensor softmax_bwd(const at::Tensor& y, const at::Tensor& dy, double scale) {
  Range rr_("xdot.softmax_bwd");
  TORCH_CHECK(y.is_cuda() && y.is_contiguous() && dy.is_contiguous(), "xdot.softmax_bwd: contiguous GPU tensors required");
  TORCH_CHECK(y.sizes() == dy.sizes() && y.scalar_type() == dy.scalar_type(), "xdot.softmax_bwd: y/dy mismatch");
  const int64_t T = y.size(-1);
  const int64_t rows = T == 0 ? 0 : y.numel() / T;
  auto dx = at::empty_like(y);
  xdot::smx::Args a{};
  a.x = y.data_ptr(); a.dy = dy.data_ptr(); a.out = dx.data_ptr(); a.rows = rows; a.T = T;
  a.scale = (float)scale; a.mdiv = 1; a.mmul = 0; a.mmod = 1;
  const bool vec = (T % 8 == 0) && aligned16(y.data_ptr()) && aligned16(dy.data_ptr()) && aligned16(dx.data_ptr());
  c10::DeviceGuard guard(y.device());
  TORCH_CHECK(xdot_softmax_bwd_launch(&a, dt_code(y.scalar_type()), vec, cur_stream(y)) == 0, "xdot.softmax_bwd: dtype");
  check_launch(hipGetLastError(), "softmax_bwd");
  return dx;
}

// ------------------------------------------------------------------------------------
std::tuple<at::Tensor, at::Tensor, at::Tensor> mask_pack(const at::Tensor& mask) {
  Range rr_("xdot.mask_pack");
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == at::kBool && mask.dim() == 3, "xdot.mask_pack: (B, R, T) bool GPU mask");
  auto m = mask.contiguous();
  const int64_t B = m.size(0), R = m.size(1), T = m.size(2);
  const int64_t NKT = (T + 63) / 64, NRT = (R + 63) / 64, Tpad = (T + 127) / 128 * 128;
  auto bits = at::empty({B, NKT, R}, m.options().dtype(at::kLong));
  auto flags = at::empty({B, (R + 31) / 32, (NKT + 3) & ~3}, m.options().dtype(at::kByte));
  auto bitsT = at::empty({B, NRT, Tpad}, m.options().dtype(at::kLong));
  TORCH_CHECK(B * R * NKT < (1LL << 40) && T < (1LL << 31), "xdot.mask_pack: too large");
  c10::DeviceGuard guard(m.device());
  xdot_mask_pack_launch(reinterpret_cast<const uint8_t*>(m.data_ptr()), reinterpret_cast<uint64_t*>(bits.data_ptr()),
                        reinterpret_cast<uint64_t*>(bitsT.data_ptr()), flags.data_ptr<uint8_t>(), (int)B, (int)R, (int)T,
                        cur_stream(m));
  check_launch(hipGetLastError(), "mask_pack");
  return {bits, flags, bitsT};
}

struct FlashGeom {
  int64_t B, R, C, T, D, ld;
};

// rows: contiguous (B, R, C).  kc / vc: (B, T, C) views with unit inner stride and a common
// row stride `ld` (C for separate tensors, 2C for the two halves of a packed [q | v]).
// `bits`: the kt-major (B, NKT, R) words, or with colmajor the (B, NRT, Tpad) words of the
// backward column kernel (mask_pack's third output)
FlashGeom flash_check(const at::Tensor& rows, const at::Tensor& kc, const at::Tensor& vc, int64_t H,
                      const c10::optional<at::Tensor>& bits, const c10::optional<at::Tensor>& flags,
                      bool colmajor = false) {
  TORCH_CHECK(rows.is_cuda() && kc.is_cuda() && vc.is_cuda(), "xdot.flash: GPU tensors required");
  TORCH_CHECK(rows.is_contiguous(), "xdot.flash: rows must be contiguous");
  TORCH_CHECK(rows.scalar_type() == kc.scalar_type() && rows.scalar_type() == vc.scalar_type(), "xdot.flash: dtype mismatch");
  TORCH_CHECK(rows.scalar_type() == at::kBFloat16 || rows.scalar_type() == at::kHalf || rows.scalar_type() == at::kFloat,
              "xdot.flash: bf16/fp16/fp32 only");
  TORCH_CHECK(rows.dim() == 3 && kc.dim() == 3 && vc.sizes() == kc.sizes(), "xdot.flash: rows (B,R,C), cols (B,T,C)");
  FlashGeom g{rows.size(0), rows.size(1), rows.size(2), kc.size(1), 0, kc.stride(1)};
  TORCH_CHECK(kc.size(0) == g.B && kc.size(2) == g.C, "xdot.flash: batch / feature mismatch");
  TORCH_CHECK(g.T > 0, "xdot.flash: empty key side");
  for (const at::Tensor* t : {&kc, &vc}) {
    TORCH_CHECK(t->stride(2) == 1 && t->stride(1) == g.ld && (g.B == 1 || t->stride(0) == g.T * g.ld),
                "xdot.flash: key/value side must be (B, T, C) rows with a common row stride");
    TORCH_CHECK((g.B - 1) * g.T * g.ld + (g.T - 1) * g.ld + g.C <= avail_elems(*t), "xdot.flash: key/value out of bounds");
  }
  TORCH_CHECK(g.ld % 8 == 0 && g.ld >= g.C, "xdot.flash: row stride must be a multiple of 8 elements");
  TORCH_CHECK(H > 0 && g.C % H == 0, "xdot.flash: C not divisible by heads");
  g.D = g.C / H;
  TORCH_CHECK(g.D == 32 || g.D == 64 || g.D == 96 || g.D == 128 || g.D == 160 || g.D == 192 || g.D == 256 ||
                  g.D == 384,
              "xdot.flash: head dim must be 32/64/96/128 or (flash_wide.hip) 160/192/256/384");
  TORCH_CHECK(g.T < (1LL << 31) && g.R < (1LL << 31) && g.B * H * ((g.R + 127) / 128) * 8 < (1LL << 31), "xdot.flash: too large");
  TORCH_CHECK(aligned16(rows.data_ptr()) && aligned16(kc.data_ptr()) && aligned16(vc.data_ptr()), "xdot.flash: 16-byte alignment");
  const bool hb = bits.has_value() && bits->defined(), hf = flags.has_value() && flags->defined();
  TORCH_CHECK(hb == hf, "xdot.flash: mask bits and flags go together");
  if (hb) {
    const int64_t NKT = (g.T + 63) / 64;
    const int64_t nwords = colmajor ? g.B * ((g.R + 63) / 64) * ((g.T + 127) / 128 * 128) : g.B * g.R * NKT;
    TORCH_CHECK(bits->is_contiguous() && bits->numel() == nwords && bits->element_size() == 8,
                colmajor ? "xdot.flash_bwd_cols: mask needs the column-major bits (mask_pack output 3)"
                         : "xdot.flash: mask bits shape");
    TORCH_CHECK(flags->is_contiguous() && flags->numel() == g.B * ((g.R + 31) / 32) * ((NKT + 3) & ~3),
                "xdot.flash: mask flags shape");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(flags->data_ptr()) & 3) == 0, "xdot.flash: flags alignment");
  }
  return g;
}

// Column split of the row-block grid.  Every workgroup of a flash kernel does the same
// work, so the launch runs in ceil(workgroups / slots) equal rounds (slots = 2 per CU x 256
// CUs) and a last round that is barely occupied costs a whole round: T = 25000, H = 8 gives
// 1568 row blocks = 3.06 rounds -> 24 % idle.  Pick the split s (<= 8, >= 8 column tiles per
// split) minimising rounds(s) x (tiles / s + fixed per-workgroup cost ~ 8 tiles: prologue,
// epilogue, the combine pass); ties keep fewer splits.
int pick_split(int64_t blocks, int64_t T, int64_t slots, int64_t req) {
  const int64_t nkt = (T + 63) / 64;
  if (req > 0) return (int)std::max<int64_t>(1, std::min<int64_t>(req, nkt));
  int best = 1;
  double best_cost = 1e300;
  for (int s = 1; s <= 8; ++s) {
    if (s > 1 && nkt / s < 8) break;
    const int64_t rounds = (blocks * s + slots - 1) / slots;
    const double cost = (double)rounds * ((double)nkt / s + 8.0);
    if (cost < best_cost * 0.985) { best_cost = cost; best = s; }
  }
  return best;
}

// Column splits of the row-side backward kernel.  It runs concurrently with the gathered-side
// kernel (which has stream priority and owns the GPU while it runs): splitting the row kernel's
// column sweep until its workgroups are no longer than the column kernel's (36 vs 48 MFMAs per
// 64-tile step; R/64 tiles per column workgroup) lets it pack into that kernel's tail instead of
// running a long tail of its own.  Measured at the N = 8 rank shape (R = 3125, T = 25000, one
// MI355X, cols||rows): 2 splits 0.989, 3: 0.943, 4: 0.911, 6: 0.888 ms (profiles/r3_masked.md).
int rows_split(int64_t B, int64_t R, int64_t T, int64_t H) {
  const int64_t nkt = (T + 63) / 64, nrt = (R + 63) / 64;
  const int base = pick_split(((R + 127) / 128) * B * H, T, 512, 0);
  int64_t conc = (nkt * 36 + nrt * 48 - 1) / (nrt * 48);
  conc = std::min<int64_t>(8, std::max<int64_t>(1, std::min<int64_t>(conc, nkt / 8)));
  return std::max(base, (int)conc);
}

// Head-heavy forward grid (16-bit, whole-GPU launches).  A uniform column split makes every row
// block pay the partial writes and a combine pass, and still ends on a part-full round: at N=1
// (1568 row blocks, 512 slots) the auto split is 3 -> 10 rounds of 1/3 blocks plus a 3-slot
// combine.  Instead each XCD (64 slots: 32 CUs x 2 workgroups, blockIdx % 8) runs its row blocks
// whole and splits only its last `rem` blocks into enough column pieces to fill one more round;
// only those tail rows go through partials and the (compact) combine.  Chosen when the round
// model says it beats the uniform split; -> (whole, rem, split) per XCD, or false.
// S: resident workgroups per XCD (64: 32 CUs x 2; the exact-fp32 forward runs 3 per CU); su: the
// uniform split to beat (0: the 16-bit forward's pick_split)
bool head_heavy_plan(int64_t NB, int64_t T, int* whole, int* rem, int* split, int64_t S = 64, int su = 0) {
  if (NB % 8) return false;
  const int64_t m = NB / 8, nkt = (T + 63) / 64;
  const int64_t full = m / S, r = m % S;
  if (r == 0 || full == 0) return false;
  if (su <= 0) su = pick_split(NB, T, 8 * S, 0);
  const double cu = (double)((NB * su + 8 * S - 1) / (8 * S)) * ((double)nkt / su + 8.0);
  double best = 1e300;
  int bs = 0;
  for (int s = 1; s <= 16; ++s) {
    if (s > 1 && nkt / s < 8) break;
    const double c = (double)full * ((double)nkt + 8.0) + (double)((r * s + S - 1) / S) * ((double)nkt / s + 8.0);
    if (c < best * 0.985) { best = c; bs = s; }
  }
  if (bs < 2 || best >= cu * 0.97) return false;
  *whole = (int)(full * S);
  *rem = (int)r;
  *split = bs;
  return true;
}

// fp32 score buffer (flash_f32.hip exact, flash_x3.hip split): (B*H, ceil(R/32), ceil(T/32)) blocks
// of 1024 floats
float* sbuf_ptr(const c10::optional<at::Tensor>& sbuf, const FlashGeom& g, int64_t H, const at::Tensor& rows,
                int64_t fp32_mode, const char* what) {
  if (!sbuf.has_value() || !sbuf->defined()) return nullptr;
  const auto& t = *sbuf;
  TORCH_CHECK(rows.scalar_type() == at::kFloat && (fp32_mode == 0 || fp32_mode == 1), what,
              ": the score buffer is an fp32 (exact or split) feature");
  const int64_t need = (g.B * H * ((g.R + 31) / 32) * ((g.T + 31) / 32) + 1) * 1024;  // + the dump block
  TORCH_CHECK(t.is_cuda() && t.device() == rows.device() && t.scalar_type() == at::kFloat && t.is_contiguous() &&
                  t.numel() == need && aligned16(t.data_ptr()),
              what, ": score buffer must be a contiguous fp32 device tensor of ", need, " elements");
  return t.data_ptr<float>();
}

std::tuple<at::Tensor, at::Tensor> flash_fwd(const at::Tensor& rows, const at::Tensor& kc, const at::Tensor& vc,
                                             const c10::optional<at::Tensor>& bits, const c10::optional<at::Tensor>& flags,
                                             int64_t H, double scale, int64_t nsplit, bool prescaled, int64_t fp32_mode,
                                             const c10::optional<at::Tensor>& sbuf) {
  Range rr_("xdot.flash_fwd");
  const FlashGeom g = flash_check(rows, kc, vc, H, bits, flags);
  float* sb = sbuf_ptr(sbuf, g, H, rows, fp32_mode, "xdot.flash_fwd");
  auto out = at::empty_like(rows);
  auto lse = at::empty({g.B, H, g.R}, rows.options().dtype(at::kFloat));
  const int rpw = xdot_flash_fwd_rows_per_wg();
  const int64_t NB = ((g.R + rpw - 1) / rpw) * g.B * H;
  int hw = 0, hr = 0, hs = 0;
  bool heavy = nsplit == 0 && rows.scalar_type() != at::kFloat && g.D <= 128 && head_heavy_plan(NB, g.T, &hw, &hr, &hs);
  int ns = heavy ? hs : pick_split(NB, g.T, 512, nsplit);
  if (nsplit == 0 && rows.scalar_type() == at::kFloat) {  // fp32 kernels: their own occupancy / tile model
    const int f = xdot_flash_f32_row_splits(0, (int)fp32_mode, (int)g.D, sb != nullptr, NB, g.T);
    if (f > 0) ns = f;
    // exact fp32 (D <= 128): the head-heavy grid when the round model prefers it over that split
    const int occ = fp32_mode == 0 && g.D <= 128 && xdot_flash_f32_heavy() ? xdot_flash_f32_fwd_occ((int)g.D, sb != nullptr) : 0;
    if (occ > 0 && head_heavy_plan(NB, g.T, &hw, &hr, &hs, (int64_t)occ * (xdot_num_cus() / 8), ns)) {
      heavy = true;
      ns = hs;
    }
  }
  if (nsplit == 0 && g.D > 128) {  // wide kernels (one workgroup per CU): their own occupancy
    const int f = xdot_flash_wide_splits(0, dt_code(rows.scalar_type()), (int)g.D, sb != nullptr, NB, (g.T + 31) / 32);
    if (f > 0) ns = f;
  }
  at::Tensor opart, lpart;
  if (heavy) {  // compact partials of the split tail blocks only
    opart = at::empty({(int64_t)hs * 8 * hr * 128 * g.D}, rows.options().dtype(at::kFloat));
    lpart = at::empty({(int64_t)hs * 8 * hr * 128}, rows.options().dtype(at::kFloat));
  } else if (ns > 1) {
    opart = at::empty({ns, g.B, g.R, g.C}, rows.options().dtype(at::kFloat));
    lpart = at::empty({ns, g.B, H, g.R}, rows.options().dtype(at::kFloat));
  }
  xdot::fa::FwdArgs a{};
  if (heavy) {
    a.xrbs = (int)(NB / 8);
    a.xwhole = hw;
    a.xrem = hr;
  }
  a.rows = rows.data_ptr(); a.kc = kc.data_ptr(); a.vc = vc.data_ptr(); a.out = out.data_ptr();
  a.lse = lse.data_ptr<float>();
  const bool hb = bits.has_value() && bits->defined();
  a.mbits = hb ? reinterpret_cast<const uint64_t*>(bits->data_ptr()) : nullptr;
  a.mflags = hb ? flags->data_ptr<uint8_t>() : nullptr;
  a.B = (int)g.B; a.H = (int)H; a.R = (int)g.R; a.T = (int)g.T; a.scale = (float)scale;
  a.ldkv = g.ld;
  a.nsplit = ns;
  a.opart = ns > 1 ? opart.data_ptr<float>() : nullptr;
  a.lpart = ns > 1 ? lpart.data_ptr<float>() : nullptr;
  a.prescaled = prescaled ? 1 : 0;
  a.fp32_mode = (int)fp32_mode;
  a.sbuf = sb;
  c10::DeviceGuard guard(rows.device());
  TORCH_CHECK(xdot_flash_fwd_launch(&a, dt_code(rows.scalar_type()), (int)g.D, cur_stream(rows)) == 0, "xdot.flash_fwd: config");
  check_launch(hipGetLastError(), "flash_fwd");
  return {out, lse};
}

xdot::fa::BwdArgs bwd_args(const FlashGeom& g, const at::Tensor& dout, const at::Tensor& rows, const at::Tensor& kc,
                           const at::Tensor& vc, const at::Tensor& lse, const c10::optional<at::Tensor>& bits,
                           const c10::optional<at::Tensor>& flags, int64_t H, double scale) {
  TORCH_CHECK(dout.sizes() == rows.sizes() && dout.is_contiguous() && dout.scalar_type() == rows.scalar_type(),
              "xdot.flash_bwd: dout shape/dtype");
  TORCH_CHECK(lse.is_contiguous() && lse.scalar_type() == at::kFloat && lse.numel() == g.B * H * g.R, "xdot.flash_bwd: lse");
  xdot::fa::BwdArgs a{};
  a.rows = rows.data_ptr(); a.kc = kc.data_ptr(); a.vc = vc.data_ptr(); a.dout = dout.data_ptr();
  a.lse = lse.data_ptr<float>();
  const bool hb = bits.has_value() && bits->defined();
  a.mbits = hb ? reinterpret_cast<const uint64_t*>(bits->data_ptr()) : nullptr;
  a.mflags = hb ? flags->data_ptr<uint8_t>() : nullptr;
  a.B = (int)g.B; a.H = (int)H; a.R = (int)g.R; a.T = (int)g.T; a.scale = (float)scale;
  a.ldkv = g.ld;
  a.nsplit = 1;
  return a;
}

// gathered-side grads, packed fp32 (B, T, 2C) = [dq | dv] partials for ONE reduce-scatter,
// + δ = rowsum(dO·O)
std::tuple<at::Tensor, at::Tensor> flash_bwd_cols(const at::Tensor& dout, const at::Tensor& rows,
                                                              const at::Tensor& kc, const at::Tensor& vc,
                                                              const at::Tensor& out, const at::Tensor& lse,
                                                              const c10::optional<at::Tensor>& bits,
                                                              const c10::optional<at::Tensor>& flags, int64_t H,
                                                              double scale, const c10::optional<at::Tensor>& delta_in,
                                                              bool fp32_out, bool prescaled,
                                                              const c10::optional<at::Tensor>& lse2_in,
                                                              int64_t fp32_mode,
                                                              const c10::optional<at::Tensor>& sbuf,
                                                              const c10::optional<at::Tensor>& dsbuf, int64_t passes,
                                                              const c10::optional<at::Tensor>& dkv_out) {
  Range rr_("xdot.flash_bwd_cols");
  const FlashGeom g = flash_check(rows, kc, vc, H, bits, flags, /*colmajor=*/true);
  float* sb = sbuf_ptr(sbuf, g, H, rows, fp32_mode, "xdot.flash_bwd_cols");
  float* dsb = sbuf_ptr(dsbuf, g, H, rows, fp32_mode, "xdot.flash_bwd_cols (dS buffer)");
  // a dS buffer alone: dS-only mode (the recomputing column kernel stores dS, D <= 128)
  TORCH_CHECK(!dsb || sb || g.D <= 128, "xdot.flash_bwd_cols: a dS buffer without the score buffer needs D <= 128");
  // passes 4: the fused exact-fp32 column pass (dQ and dV in one kernel); other families run both
  // passes (3) instead
  if (passes == 4 && (!sb || fp32_mode != 0 || g.D > 128 || rows.scalar_type() != at::kFloat)) passes = 3;
  TORCH_CHECK(passes >= 1 && passes <= 4 && (passes >= 3 || (sb && dsb)),
              "xdot.flash_bwd_cols: single passes (1 = dV, 2 = dQ) need the score and dS buffers");
  TORCH_CHECK(out.sizes() == rows.sizes() && out.is_contiguous() && out.scalar_type() == rows.scalar_type(),
              "xdot.flash_bwd_cols: out shape/dtype");
  auto a = bwd_args(g, dout, rows, kc, vc, lse, bits, flags, H, scale);
  a.prescaled = prescaled ? 1 : 0;
  a.fp32_mode = (int)fp32_mode;
  at::Tensor dkv;
  if (dkv_out.has_value() && dkv_out->defined()) {  // the other pass's output, completed in place
    dkv = *dkv_out;
    TORCH_CHECK(dkv.is_contiguous() && dkv.sizes() == at::IntArrayRef({g.B, g.T, 2 * g.C}) &&
                    dkv.scalar_type() == (fp32_out ? at::kFloat : kc.scalar_type()) && dkv.device() == rows.device(),
                "xdot.flash_bwd_cols: dkv_out");
  } else {
    dkv = at::empty({g.B, g.T, 2 * g.C}, fp32_out ? kc.options().dtype(at::kFloat) : kc.options());
  }
  const bool have_delta = delta_in.has_value() && delta_in->defined();
  at::Tensor delta;
  if (have_delta) {
    delta = *delta_in;
    TORCH_CHECK(delta.is_contiguous() && delta.scalar_type() == at::kFloat && delta.numel() == g.B * H * g.R &&
                    delta.device() == rows.device(), "xdot.flash_bwd_cols: delta");
  } else {
    delta = at::empty({g.B, H, g.R}, rows.options().dtype(at::kFloat));
  }
  a.dkc = dkv.data_ptr(); a.dvc = static_cast<char*>(dkv.data_ptr()) + g.C * dkv.element_size(); a.ldg = 2 * g.C;
  a.dkv16 = (fp32_out || rows.scalar_type() == at::kFloat) ? 0 : 1;
  a.delta = delta.data_ptr<float>();
  // lse2 = lse * log2 e: given (from flash_bwd_prep, together with δ), or one prep pass here
  const bool have_lse2 = have_delta && lse2_in.has_value() && lse2_in->defined();
  at::Tensor lse2;
  if (have_lse2) {
    lse2 = *lse2_in;
    TORCH_CHECK(lse2.is_contiguous() && lse2.scalar_type() == at::kFloat && lse2.numel() == g.B * H * g.R &&
                    lse2.device() == rows.device(), "xdot.flash_bwd_cols: lse2");
  } else {
    lse2 = at::empty({g.B, H, g.R}, rows.options().dtype(at::kFloat));
  }
  a.lse2 = lse2.data_ptr<float>();
  a.sbuf = sb;
  a.dsbuf = dsb;
  a.sb_passes = (int)passes;
  c10::DeviceGuard guard(rows.device());
  const int dt = dt_code(rows.scalar_type());
  // prep: lse2 (+ δ unless given)
  if (!have_lse2)
    TORCH_CHECK(xdot_flash_bwd_delta_launch(&a, out.data_ptr(), have_delta ? nullptr : delta.data_ptr<float>(), dt,
                                            (int)g.D, cur_stream(rows)) == 0,
                "xdot.flash_bwd_cols: config");
  // column kernels: row splits against the last-round tail (fp32 partials summed in the launcher;
  // the exact / split fp32 kernels and the pipelined 16-bit kernel, else 1)
  at::Tensor cpq, cpv;
  if (dt != xdot::DT_F32 || g.D > 128 || (!a.prescaled && !a.dkv16)) {
    int sq = 1, sv = 1;  // (the single-pass recompute kernels use sq for both halves: sv == sq there)
    TORCH_CHECK(xdot_flash_cols_splits(&a, dt, (int)g.D, &sq, &sv) == 0, "xdot.flash_bwd_cols: split config");
    const bool run_q = !sb || passes == 4 || (passes & 2), run_v = !sb || passes == 4 || (passes & 1);
    int hw = 0, hr = 0, hs = 0;
    if (dt == xdot::DT_F32 && xdot_flash_f32_cols_heavy(&a, (int)g.D, sq, &hw, &hr, &hs)) {
      // head-heavy fused column pass: compact partials of the XCDs' tail blocks only
      const int64_t W = ((g.T + 127) / 128) * g.B * H;
      cpq = at::empty({(int64_t)hs * 8 * hr * 128 * g.D}, rows.options().dtype(at::kFloat));
      cpv = at::empty({(int64_t)hs * 8 * hr * 128 * g.D}, rows.options().dtype(at::kFloat));
      a.cpq = cpq.data_ptr<float>();
      a.cpv = cpv.data_ptr<float>();
      a.csq = a.csv = hs;
      a.xcb = (int)(W / 8);
      a.xwhole = hw;
      a.xrem = hr;
    }
    if (a.xcb == 0 && run_q && sq > 1) {
      cpq = at::empty({sq, g.B, g.T, g.C}, rows.options().dtype(at::kFloat));
      a.cpq = cpq.data_ptr<float>();
      a.csq = sq;
    }
    if (a.xcb == 0 && run_v && sv > 1) {
      cpv = at::empty({sv, g.B, g.T, g.C}, rows.options().dtype(at::kFloat));
      a.cpv = cpv.data_ptr<float>();
      a.csv = sv;
    }
  }
  TORCH_CHECK(xdot_flash_bwd_cols_launch(&a, dt, (int)g.D, cur_stream(rows)) == 0, "xdot.flash_bwd_cols: config");
  check_launch(hipGetLastError(), "flash_bwd_cols");
  return {dkv, delta};
}

// Σ over the leading (split) dim of fp32 partials, cast to out_dtype, one pass
at::Tensor sum_partials(const at::Tensor& part, at::ScalarType out_dtype) {
  Range rr_("xdot.sum_partials");
  TORCH_CHECK(part.is_cuda() && part.is_contiguous() && part.scalar_type() == at::kFloat && part.dim() >= 2,
              "xdot.sum_partials: contiguous fp32 (S, ...) device tensor");
  std::vector<int64_t> shape(part.sizes().begin() + 1, part.sizes().end());
  auto out = at::empty(shape, part.options().dtype(out_dtype));
  const int64_t n = out.numel();
  TORCH_CHECK(n % 4 == 0 && aligned16(part.data_ptr()), "xdot.sum_partials: numel % 4 and 16-byte alignment");
  c10::DeviceGuard guard(part.device());
  TORCH_CHECK(xdot_sum_partials_launch(part.data_ptr<float>(), out.data_ptr(), (int)part.size(0), n, dt_code(out_dtype),
                                       cur_stream(part)) == 0, "xdot.sum_partials: unsupported dtype");
  check_launch(hipGetLastError(), "sum_partials");
  return out;
}

// Projection GEMM (csrc/gemm_proj.hip): nn = false: y = x Wᵀ (+ bias), W (N, K); nn = true:
// dx = dy W, W (K, N) (the input gradient of the same Linear).  x: (..., K) with unit last
// stride; out (optional): an (M, N) row-major view to write (e.g. this rank's block of the
// all-gather buffer).  Shapes / layouts the kernel does not take, and (force = 0) products
// large enough for the library to be faster, run on the library GEMM.
at::Tensor proj(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias, bool nn,
                const c10::optional<at::Tensor>& out, int64_t force, double alpha) {
  Range rr_("xdot.proj");
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && w.dim() == 2 && x.dim() >= 1 && x.scalar_type() == w.scalar_type(),
              "xdot.proj: device tensors of one dtype, 2-D weight");
  const int64_t K = x.size(-1);
  const int64_t N = nn ? w.size(1) : w.size(0);
  TORCH_CHECK((nn ? w.size(0) : w.size(1)) == K, "xdot.proj: weight ", w.sizes(), " does not match input features ", K);
  at::Tensor a = x.dim() == 2 ? x : x.reshape({-1, K});
  if (a.stride(1) != 1) a = a.contiguous();
  const int64_t M = a.size(0);
  std::vector<int64_t> oshape(x.sizes().begin(), x.sizes().end() - 1);
  oshape.push_back(N);
  at::Tensor c;
  if (out.has_value()) {
    c = *out;
    TORCH_CHECK(c.is_cuda() && c.dim() == 2 && c.size(0) == M && c.size(1) == N && c.stride(1) == 1 &&
                    c.scalar_type() == x.scalar_type(),
                "xdot.proj: out must be an (M, N) row-major view of the input dtype");
  } else {
    c = at::empty({M, N}, x.options());
  }
  const bool has_b = bias.has_value() && bias->defined();
  TORCH_CHECK(!has_b || (!nn && bias->numel() == N && bias->is_contiguous() && bias->scalar_type() == x.scalar_type()),
              "xdot.proj: bias must be a contiguous (N,) tensor of the input dtype (forward only)");
  int rc = -3;
  if (M > 0 && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf) && w.stride(1) == 1 &&
      M <= INT32_MAX && N <= INT32_MAX && K <= INT32_MAX) {
    xdot::ProjArgs p{};
    p.A = a.data_ptr();
    p.B = w.data_ptr();
    p.bias = has_b ? bias->data_ptr() : nullptr;
    p.C = c.data_ptr();
    p.M = (int)M;
    p.N = (int)N;
    p.K = (int)K;
    p.lda = a.stride(0);
    p.ldb = w.stride(0);
    p.ldc = c.stride(0);
    p.alpha = (float)alpha;
    // every address the kernel can touch lies inside the operands' storage
    TORCH_CHECK((M - 1) * p.lda + K <= avail_elems(a) && (nn ? (K - 1) * p.ldb + N : (N - 1) * p.ldb + K) <= avail_elems(w) &&
                    (M - 1) * p.ldc + N <= avail_elems(c),
                "xdot.proj: operand extents exceed their storage");
    c10::DeviceGuard guard(x.device());
    rc = xdot_gemm_proj_launch(&p, dt_code(x.scalar_type()), nn ? 1 : 0, (int)force, cur_stream(x));
    if (rc != -3) check_launch((hipError_t)rc, "gemm_proj");
  }
  if (rc == -3) {  // library GEMM (alpha scales the bias too: C = alpha (A op(B) + bias), one rounding)
    const at::Tensor wt = nn ? w : w.t();
    if (has_b) at::addmm_out(c, *bias, a, wt, alpha, alpha);
    else if (alpha == 1.0) at::mm_out(c, a, wt);
    else at::addmm_out(c, c, a, wt, 0.0, alpha);
  }
  return out.has_value() ? c : c.view(oshape);
}

// Weight gradient of a Linear: dy (K, M), x (K, N) row-major 16-bit -> dyᵀ x (M, N) in out_dtype,
// fp32 accumulation (csrc/gemm_wgrad.hip: S slabs of K -> fp32 partials -> one ordered sum).
// splits 0: the slab count from a round / partial-traffic cost model.  Returns an undefined tensor
// when the shape is not eligible (the caller takes another route).
struct WgradProb {
  at::Tensor dy, x, part;
  int64_t K, M, N, S;
};

bool wgrad_prob(const at::Tensor& dy, const at::Tensor& x, int64_t splits, WgradProb& q) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0) &&
                  dy.scalar_type() == x.scalar_type() && dy.stride(1) == 1 && x.stride(1) == 1,
              "xdot.wgrad: (K, M) and (K, N) row-major device tensors of one dtype");
  const int64_t K = dy.size(0), M = dy.size(1), N = x.size(1);
  if (K < 1 || M % 128 || N % 128 || (dy.scalar_type() != at::kBFloat16 && dy.scalar_type() != at::kHalf) ||
      M > INT32_MAX || N > INT32_MAX || K > INT32_MAX)
    return false;
  const int64_t KT = (K + 63) / 64, tiles = (M / 128) * (N / 128);
  // slab count: rounds of 512 workgroup slots x (k-tiles per slab + a per-workgroup overhead of
  // ~4 k-tiles) + the fp32 partials' write and ordered-sum read (~0.07 k-tile per tile and slab);
  // fitted to the S sweep of benchmarks/micro/wgrad_splits.py (profiles/r4_s2.md §12)
  int64_t S = splits;
  if (S <= 0) {
    double best = 1e300;
    for (int64_t s = 1; s <= std::min<int64_t>(KT, 64); ++s) {
      const double cost = (double)((tiles * s + 511) / 512) * ((double)KT / s + 4.0) + 0.07 * (double)(tiles * s);
      if (cost < best) { best = cost; S = s; }
    }
  }
  S = std::max<int64_t>(1, std::min<int64_t>(S, KT));
  TORCH_CHECK((K - 1) * dy.stride(0) + M <= avail_elems(dy) && (K - 1) * x.stride(0) + N <= avail_elems(x),
              "xdot.wgrad: operand extents exceed their storage");
  q = WgradProb{dy, x, at::empty({S, M, N}, dy.options().dtype(at::kFloat)), K, M, N, S};
  return true;
}

// launch 1 or 2 products in one kernel, then one ordered sum per product; empty when not eligible
std::vector<at::Tensor> wgrad_run(std::vector<WgradProb>& qs, at::ScalarType out_dtype) {
  const int np = (int)qs.size();
  const void* A[2];
  const void* B[2];
  float* part[2];
  int M[2], N[2], K[2], S[2];
  int64_t lda[2], ldb[2];
  for (int i = 0; i < np; ++i) {
    A[i] = qs[i].dy.data_ptr(); B[i] = qs[i].x.data_ptr(); part[i] = qs[i].part.data_ptr<float>();
    M[i] = (int)qs[i].M; N[i] = (int)qs[i].N; K[i] = (int)qs[i].K; S[i] = (int)qs[i].S;
    lda[i] = qs[i].dy.stride(0); ldb[i] = qs[i].x.stride(0);
  }
  const at::Tensor& d0 = qs[0].dy;
  c10::DeviceGuard guard(d0.device());
  const int rc = xdot_gemm_wgrad_launch(np, A, B, part, M, N, K, S, lda, ldb, dt_code(d0.scalar_type()), cur_stream(d0));
  if (rc == -3) return {};
  check_launch((hipError_t)rc, "gemm_wgrad");
  std::vector<at::Tensor> outs;
  for (int i = 0; i < np; ++i) outs.push_back(at::empty({qs[i].M, qs[i].N}, d0.options().dtype(out_dtype)));
  if (np == 2) {  // both ordered sums in one launch
    TORCH_CHECK(xdot_sum_partials2_launch(part[0], outs[0].data_ptr(), S[0], qs[0].M * qs[0].N, part[1],
                                          outs[1].data_ptr(), S[1], qs[1].M * qs[1].N, dt_code(out_dtype),
                                          cur_stream(d0)) == 0, "xdot.wgrad2: out dtype");
    check_launch(hipGetLastError(), "wgrad2 sum");
    return outs;
  }
  for (int i = 0; i < np; ++i) {
    TORCH_CHECK(xdot_sum_partials_launch(part[i], outs[i].data_ptr(), S[i], qs[i].M * qs[i].N, dt_code(out_dtype),
                                         cur_stream(d0)) == 0, "xdot.wgrad: out dtype");
    check_launch(hipGetLastError(), "wgrad sum");
  }
  return outs;
}

at::Tensor wgrad(const at::Tensor& dy, const at::Tensor& x, at::ScalarType out_dtype, int64_t splits) {
  Range rr_("xdot.wgrad");
  std::vector<WgradProb> qs(1);
  if (!wgrad_prob(dy, x, splits, qs[0])) return at::Tensor();
  auto outs = wgrad_run(qs, out_dtype);
  return outs.empty() ? at::Tensor() : outs[0];
}

// two weight gradients in ONE launch (the fused backward's dWk and dW[q|v]); [] when either
// shape is not eligible
std::vector<at::Tensor> wgrad2(const at::Tensor& dy0, const at::Tensor& x0, const at::Tensor& dy1,
                               const at::Tensor& x1, at::ScalarType out_dtype) {
  Range rr_("xdot.wgrad2");
  TORCH_CHECK(dy0.scalar_type() == dy1.scalar_type() && dy0.device() == dy1.device(), "xdot.wgrad2: dtype / device");
  std::vector<WgradProb> qs(2);
  if (!wgrad_prob(dy0, x0, 0, qs[0]) || !wgrad_prob(dy1, x1, 0, qs[1])) return {};
  return wgrad_run(qs, out_dtype);
}

// fused MSE loss forward: (mean (y - t)^2 in y's dtype, dy = 2 (y - t) / n)
std::tuple<at::Tensor, at::Tensor> mse_fwd(const at::Tensor& y, const at::Tensor& t) {
  Range rr_("xdot.mse_fwd");
  const auto st_ = y.scalar_type();
  TORCH_CHECK(y.is_cuda() && t.is_cuda() && y.is_contiguous() && t.is_contiguous() && t.scalar_type() == st_ &&
                  y.sizes() == t.sizes() && (st_ == at::kBFloat16 || st_ == at::kHalf || st_ == at::kFloat) &&
                  aligned16(y.data_ptr()) && aligned16(t.data_ptr()) && y.numel() % (16 / y.element_size()) == 0 &&
                  y.numel() > 0,
              "xdot.mse_fwd: same-shape contiguous 16-byte aligned bf16/fp16/fp32 device tensors, numel % (16 B) == 0");
  auto dy = at::empty_like(y);
  const int64_t nv = y.numel() / (16 / y.element_size());
  const int nparts = (int)std::min<int64_t>(1024, (nv + 255) / 256);
  auto part = at::empty({nparts}, y.options().dtype(at::kFloat));
  auto loss = at::empty({}, y.options());
  c10::DeviceGuard guard(y.device());
  TORCH_CHECK(xdot_mse_fwd_launch(y.data_ptr(), t.data_ptr(), dy.data_ptr(), part.data_ptr<float>(), nparts,
                                  loss.data_ptr(), y.numel(), dt_code(st_), cur_stream(y)) == 0,
              "xdot.mse_fwd: launch rejected");
  check_launch(hipGetLastError(), "mse_fwd");
  return {loss, dy};
}

// row side of the flash kernels pre-multiplied by scale * log2(e), in the input dtype
at::Tensor flash_prescale(const at::Tensor& x, double scale) {
  Range rr_("xdot.flash_prescale");
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf) &&
                  x.numel() % 8 == 0 && aligned16(x.data_ptr()),
              "xdot.flash_prescale: contiguous 16-byte aligned bf16/fp16 device tensor, numel % 8 == 0");
  auto out = at::empty_like(x);
  c10::DeviceGuard guard(x.device());
  TORCH_CHECK(xdot_prescale_rows_launch(x.data_ptr(), out.data_ptr(), x.numel(), (float)scale, dt_code(x.scalar_type()),
                                        cur_stream(x)) == 0, "xdot.flash_prescale: dtype");
  check_launch(hipGetLastError(), "flash_prescale");
  return out;
}

// dst[i] <- src[i] converted to dst[i]'s dtype (fp32 / bf16 / fp16), every pair in one launch per
// CAST_MAX_T pairs (GradSync: 16-bit gradients <-> the fp32 buffers its all-reduce sums)
void cast_multi(at::TensorList src, at::TensorList dst) {
  Range rr_("xdot.cast_multi");
  const size_t n = src.size();
  TORCH_CHECK(dst.size() == n, "xdot.cast_multi: list sizes");
  if (n == 0) return;
  for (size_t i = 0; i < n; ++i) {
    TORCH_CHECK(src[i].is_cuda() && dst[i].is_cuda() && src[i].device() == dst[0].device() &&
                    dst[i].device() == dst[0].device(),
                "xdot.cast_multi: GPU tensors on one device");
    TORCH_CHECK(src[i].is_contiguous() && dst[i].is_contiguous() && src[i].numel() == dst[i].numel(),
                "xdot.cast_multi: contiguous tensors of equal numel");
    TORCH_CHECK(dt_code(src[i].scalar_type()) >= 0 && dt_code(dst[i].scalar_type()) >= 0,
                "xdot.cast_multi: fp32 / bf16 / fp16 only");
  }
  c10::DeviceGuard guard(dst[0].device());
  for (size_t c0 = 0; c0 < n; c0 += xdot::CAST_MAX_T) {
    xdot::CastArgs a{};
    int blk = 0;
    a.nt = (int)std::min<size_t>(xdot::CAST_MAX_T, n - c0);
    for (int i = 0; i < a.nt; ++i) {
      const size_t k = c0 + i;
      a.src[i] = src[k].data_ptr();
      a.dst[i] = dst[k].data_ptr();
      a.n[i] = src[k].numel();
      a.sdt[i] = dt_code(src[k].scalar_type());
      a.ddt[i] = dt_code(dst[k].scalar_type());
      a.blk0[i] = blk;
      const int64_t nb = (a.n[i] + xdot::CAST_BLOCK_ELEMS - 1) / xdot::CAST_BLOCK_ELEMS;
      TORCH_CHECK(blk + nb < (1LL << 31), "xdot.cast_multi: too many elements");
      blk += (int)nb;
    }
    a.blk0[a.nt] = blk;
    TORCH_CHECK(xdot_cast_multi_launch(&a, cur_stream(dst[0])) == 0, "xdot.cast_multi: dtype");
    check_launch(hipGetLastError(), "cast_multi");
  }
}

// one AdamW step for lists of same-dtype params / grads with fp32 moments (chunks of 32)
// grad_out (optional, one per parameter): the gradients are fp32 (GradSync's reduced sums of
// 16-bit parameters) and each is also written into grad_out[i] in the parameter dtype
void adamw_step(at::TensorList params, at::TensorList grads, at::TensorList exp_avg, at::TensorList exp_avg_sq,
                double lr, double beta1, double beta2, double eps, double weight_decay, int64_t step,
                at::TensorList step_ts, const c10::optional<at::Tensor>& lr_t, at::TensorList grad_out) {
  Range rr_("xdot.adamw_step");
  const size_t n = params.size();
  const bool dev_state = step_ts.size() > 0;
  if (dev_state) {
    TORCH_CHECK(step_ts.size() == n && lr_t.has_value() && lr_t->defined(),
                "xdot.adamw_step: device state needs one step tensor per parameter and lr_t");
    for (const auto& t : step_ts)
      TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.numel() == 1,
                  "xdot.adamw_step: step tensors must be one-element fp32 device tensors");
    TORCH_CHECK(lr_t->is_cuda() && lr_t->scalar_type() == at::kFloat && lr_t->numel() == 1,
                "xdot.adamw_step: lr_t must be a one-element fp32 device tensor");
  }
  TORCH_CHECK(grads.size() == n && exp_avg.size() == n && exp_avg_sq.size() == n, "xdot.adamw_step: list sizes");
  const bool g32 = grad_out.size() > 0;
  TORCH_CHECK(!g32 || grad_out.size() == n, "xdot.adamw_step: one grad_out per parameter");
  TORCH_CHECK(step >= 1, "xdot.adamw_step: step counts from 1");
  if (n == 0) return;
  const auto dtype = params[0].scalar_type();
  for (size_t i = 0; i < n; ++i) {
    TORCH_CHECK(params[i].is_cuda() && params[i].is_contiguous() && params[i].scalar_type() == dtype,
                "xdot.adamw_step: contiguous GPU params of one dtype");
    TORCH_CHECK(grads[i].sizes() == params[i].sizes() && grads[i].is_contiguous() &&
                    grads[i].scalar_type() == (g32 ? at::kFloat : dtype),
                "xdot.adamw_step: grad shape/dtype");
    if (g32)
      TORCH_CHECK(dtype != at::kFloat && grad_out[i].sizes() == params[i].sizes() && grad_out[i].is_contiguous() &&
                      grad_out[i].scalar_type() == dtype && grad_out[i].device() == params[i].device(),
                  "xdot.adamw_step: grad_out (16-bit parameters, parameter shape / dtype)");
    for (const at::Tensor* s : {&exp_avg[i], &exp_avg_sq[i]})
      TORCH_CHECK(s->numel() == params[i].numel() && s->is_contiguous() && s->scalar_type() == at::kFloat,
                  "xdot.adamw_step: fp32 moments");
  }
  const float bc1 = 1.f - (float)std::pow(beta1, (double)step);
  const float bc2 = 1.f - (float)std::pow(beta2, (double)step);
  c10::DeviceGuard guard(params[0].device());
  for (size_t c0 = 0; c0 < n; c0 += xdot::ADAM_MAX_T) {
    xdot::AdamArgs a{};
    int blk = 0;
    a.nt = (int)std::min<size_t>(xdot::ADAM_MAX_T, n - c0);
    for (int i = 0; i < a.nt; ++i) {
      const size_t k = c0 + i;
      a.p[i] = params[k].data_ptr(); a.g[i] = grads[k].data_ptr();
      a.m[i] = exp_avg[k].data_ptr<float>(); a.v[i] = exp_avg_sq[k].data_ptr<float>();
      a.n[i] = params[k].numel();
      a.step_dev[i] = dev_state ? step_ts[k].data_ptr<float>() : nullptr;
      a.gout[i] = g32 ? grad_out[k].data_ptr() : nullptr;
      a.blk0[i] = blk;
      const int64_t nb = (a.n[i] + xdot::ADAM_BLOCK_ELEMS - 1) / xdot::ADAM_BLOCK_ELEMS;
      TORCH_CHECK(blk + nb < (1LL << 31), "xdot.adamw_step: too many elements");
      blk += (int)nb;
    }
    a.blk0[a.nt] = blk;
    a.lr = (float)lr; a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.eps = (float)eps; a.wd = (float)weight_decay;
    a.bc1 = bc1; a.bc2_sqrt = std::sqrt(bc2);
    a.dev_state = dev_state ? 1 : 0;
    a.lr_dev = dev_state ? lr_t->data_ptr<float>() : nullptr;
    a.g32 = g32 ? 1 : 0;
    TORCH_CHECK(xdot_adamw_launch(&a, dt_code(dtype), cur_stream(params[0])) == 0, "xdot.adamw_step: dtype");
    check_launch(hipGetLastError(), "adamw_step");
  }
}

// δ = rowsum(dO ⊙ O) per (b, h, row), fp32 (B, H, R)
at::Tensor flash_bwd_delta(const at::Tensor& dout, const at::Tensor& out, int64_t H) {
  Range rr_("xdot.flash_bwd_delta");
  TORCH_CHECK(dout.is_cuda() && dout.dim() == 3 && dout.is_contiguous() && out.sizes() == dout.sizes() &&
                  out.is_contiguous() && out.scalar_type() == dout.scalar_type() && out.device() == dout.device(),
              "xdot.flash_bwd_delta: dout/out must be matching contiguous (B, R, H*D) device tensors");
  TORCH_CHECK(H > 0 && dout.size(2) % H == 0, "xdot.flash_bwd_delta: H");
  xdot::fa::BwdArgs a{};
  a.dout = dout.data_ptr();
  a.B = (int)dout.size(0); a.R = (int)dout.size(1); a.H = (int)H;
  auto delta = at::empty({dout.size(0), H, dout.size(1)}, dout.options().dtype(at::kFloat));
  c10::DeviceGuard guard(dout.device());
  TORCH_CHECK(xdot_flash_bwd_delta_launch(&a, out.data_ptr(), delta.data_ptr<float>(), dt_code(dout.scalar_type()),
                                          (int)(dout.size(2) / H), cur_stream(dout)) == 0,
              "xdot.flash_bwd_delta: unsupported dtype/head dim");
  check_launch(hipGetLastError(), "flash_bwd_delta");
  return delta;
}

// δ = rowsum(dO ⊙ O) and lse2 = lse * log2 e, both fp32 (B, H, R), in ONE pass: the fused
// backward's prep (flash_bwd_cols then takes both and launches no prep of its own)
std::tuple<at::Tensor, at::Tensor> flash_bwd_prep(const at::Tensor& dout, const at::Tensor& out, const at::Tensor& lse,
                                                  int64_t H) {
  Range rr_("xdot.flash_bwd_prep");
  TORCH_CHECK(dout.is_cuda() && dout.dim() == 3 && dout.is_contiguous() && out.sizes() == dout.sizes() &&
                  out.is_contiguous() && out.scalar_type() == dout.scalar_type() && out.device() == dout.device(),
              "xdot.flash_bwd_prep: dout/out must be matching contiguous (B, R, H*D) device tensors");
  TORCH_CHECK(H > 0 && dout.size(2) % H == 0, "xdot.flash_bwd_prep: H");
  TORCH_CHECK(lse.is_contiguous() && lse.scalar_type() == at::kFloat && lse.device() == dout.device() &&
                  lse.numel() == dout.size(0) * H * dout.size(1), "xdot.flash_bwd_prep: lse (B, H, R) fp32");
  xdot::fa::BwdArgs a{};
  a.dout = dout.data_ptr();
  a.B = (int)dout.size(0); a.R = (int)dout.size(1); a.H = (int)H;
  auto delta = at::empty({dout.size(0), H, dout.size(1)}, dout.options().dtype(at::kFloat));
  auto lse2 = at::empty_like(delta);
  a.lse = lse.data_ptr<float>();
  a.lse2 = lse2.data_ptr<float>();
  c10::DeviceGuard guard(dout.device());
  TORCH_CHECK(xdot_flash_bwd_delta_launch(&a, out.data_ptr(), delta.data_ptr<float>(), dt_code(dout.scalar_type()),
                                          (int)(dout.size(2) / H), cur_stream(dout)) == 0,
              "xdot.flash_bwd_prep: unsupported dtype/head dim");
  check_launch(hipGetLastError(), "flash_bwd_prep");
  return {delta, lse2};
}

// row-side grad (this rank's rows), column-split when the row count is small
at::Tensor flash_bwd_rows(const at::Tensor& dout, const at::Tensor& rows, const at::Tensor& kc, const at::Tensor& vc,
                          const at::Tensor& lse, const at::Tensor& delta, const c10::optional<at::Tensor>& bits,
                          const c10::optional<at::Tensor>& flags, int64_t H, double scale, int64_t nsplit,
                          bool prescaled, int64_t fp32_mode, const c10::optional<at::Tensor>& sbuf,
                          const c10::optional<at::Tensor>& dsbuf) {
  Range rr_("xdot.flash_bwd_rows");
  const FlashGeom g = flash_check(rows, kc, vc, H, bits, flags);
  float* sb = sbuf_ptr(sbuf, g, H, rows, fp32_mode, "xdot.flash_bwd_rows");
  float* dsb = sbuf_ptr(dsbuf, g, H, rows, fp32_mode, "xdot.flash_bwd_rows (dS buffer)");
  TORCH_CHECK(!dsb || sb || g.D <= 128, "xdot.flash_bwd_rows: a dS buffer without the score buffer needs D <= 128");
  TORCH_CHECK(delta.is_contiguous() && delta.scalar_type() == at::kFloat && delta.numel() == g.B * H * g.R,
              "xdot.flash_bwd_rows: delta");
  auto a = bwd_args(g, dout, rows, kc, vc, lse, bits, flags, H, scale);
  auto drows = at::empty_like(rows);
  int ns = nsplit > 0 ? pick_split(1, g.T, 1, nsplit) : rows_split(g.B, g.R, g.T, H);
  if (nsplit == 0 && rows.scalar_type() == at::kFloat) {
    const int f = xdot_flash_f32_row_splits(1, (int)fp32_mode, (int)g.D, sb != nullptr || dsb != nullptr,
                                            ((g.R + 127) / 128) * g.B * H, g.T);
    if (f > 0) ns = f;
  }
  if (nsplit == 0 && g.D > 128) {
    const int f = xdot_flash_wide_splits(1, dt_code(rows.scalar_type()), (int)g.D, sb != nullptr,
                                         ((g.R + 127) / 128) * g.B * H, (g.T + 31) / 32);
    if (f > 0) ns = f;
  }
  at::Tensor dpart;
  if (ns > 1) dpart = at::empty({ns, g.B, g.R, g.C}, rows.options().dtype(at::kFloat));
  a.delta = delta.data_ptr<float>(); a.drows = drows.data_ptr();
  a.nsplit = ns; a.dpart = ns > 1 ? dpart.data_ptr<float>() : nullptr;
  a.prescaled = prescaled ? 1 : 0;
  a.fp32_mode = (int)fp32_mode;
  a.sbuf = sb;
  a.dsbuf = dsb;
  c10::DeviceGuard guard(rows.device());
  TORCH_CHECK(xdot_flash_bwd_rows_launch(&a, dt_code(rows.scalar_type()), (int)g.D, cur_stream(rows)) == 0,
              "xdot.flash_bwd_rows: config");
  check_launch(hipGetLastError(), "flash_bwd_rows");
  return drows;
}

// ---- chunked launches (gather / reduce-scatter pipelining) ----------------------------
// column splits the row-block kernels would use for (R rows, T columns) — the caller sizes the
// partial buffers with it
int64_t flash_splits(int64_t B, int64_t R, int64_t T, int64_t H, bool rows_kernel) {
  if (rows_kernel) return rows_split(B, R, T, H);
  return pick_split(((R + 127) / 128) * B * H, T, 512, 0);
}

void check_part(const at::Tensor& t, int64_t slots_needed, int64_t per_slot, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kFloat && t.dim() >= 1 &&
                  t.size(0) >= slots_needed && t.numel() == t.size(0) * per_slot,
              "xdot: partial buffer ", what, " has the wrong shape/dtype");
}

// forward over this column chunk into partial slots [sp0, sp0 + nsplit) of opart / lpart
void flash_fwd_partial(const at::Tensor& rows, const at::Tensor& kc, const at::Tensor& vc,
                       const c10::optional<at::Tensor>& bits, const c10::optional<at::Tensor>& flags, int64_t H,
                       double scale, at::Tensor& opart, at::Tensor& lpart, int64_t sp0, int64_t nsplit,
                       bool prescaled, int64_t fp32_mode) {
  Range rr_("xdot.flash_fwd_partial");
  const FlashGeom g = flash_check(rows, kc, vc, H, bits, flags);
  TORCH_CHECK(sp0 >= 0 && nsplit >= 1, "xdot.flash_fwd_partial: slots");
  const int ns = pick_split(1, g.T, 1, nsplit);  // clamps nsplit to the column tiles
  check_part(opart, sp0 + ns, g.B * g.R * g.C, "opart");
  check_part(lpart, sp0 + ns, g.B * H * g.R, "lpart");
  xdot::fa::FwdArgs a{};
  a.rows = rows.data_ptr(); a.kc = kc.data_ptr(); a.vc = vc.data_ptr();
  const bool hb = bits.has_value() && bits->defined();
  a.mbits = hb ? reinterpret_cast<const uint64_t*>(bits->data_ptr()) : nullptr;
  a.mflags = hb ? flags->data_ptr<uint8_t>() : nullptr;
  a.B = (int)g.B; a.H = (int)H; a.R = (int)g.R; a.T = (int)g.T; a.scale = (float)scale;
  a.ldkv = g.ld;
  a.nsplit = ns; a.sp0 = (int)sp0; a.force_partial = 1;
  a.opart = opart.data_ptr<float>(); a.lpart = lpart.data_ptr<float>();
  a.prescaled = prescaled ? 1 : 0;
  a.fp32_mode = (int)fp32_mode;
  c10::DeviceGuard guard(rows.device());
  TORCH_CHECK(xdot_flash_fwd_launch(&a, dt_code(rows.scalar_type()), (int)g.D, cur_stream(rows)) == 0,
              "xdot.flash_fwd_partial: config");
  check_launch(hipGetLastError(), "flash_fwd_partial");
}

// merge all slots of opart / lpart -> (out in like's dtype, lse)
std::tuple<at::Tensor, at::Tensor> flash_fwd_combine(const at::Tensor& opart, const at::Tensor& lpart, int64_t H,
                                                     const at::Tensor& like) {
  Range rr_("xdot.flash_fwd_combine");
  TORCH_CHECK(like.dim() == 3 && like.is_cuda(), "xdot.flash_fwd_combine: like (B, R, C)");
  const int64_t B = like.size(0), R = like.size(1), C = like.size(2), S = opart.size(0);
  TORCH_CHECK(H > 0 && C % H == 0, "xdot.flash_fwd_combine: H");
  check_part(opart, S, B * R * C, "opart");
  check_part(lpart, S, B * H * R, "lpart");
  auto out = at::empty_like(like);
  auto lse = at::empty({B, H, R}, like.options().dtype(at::kFloat));
  xdot::fa::FwdArgs a{};
  a.out = out.data_ptr(); a.lse = lse.data_ptr<float>();
  a.B = (int)B; a.H = (int)H; a.R = (int)R; a.nsplit = (int)S;
  a.opart = opart.data_ptr<float>(); a.lpart = lpart.data_ptr<float>();
  c10::DeviceGuard guard(like.device());
  TORCH_CHECK(xdot_flash_fwd_combine_launch(&a, dt_code(like.scalar_type()), (int)(C / H), cur_stream(like)) == 0,
              "xdot.flash_fwd_combine: config");
  check_launch(hipGetLastError(), "flash_fwd_combine");
  return {out, lse};
}

// merge all slots of opart / lpart into slot 0 in fp32 (the running partial of the ring
// forward: two slots of memory per block instead of one per ring step).  O is merged in place
// (each element is read and written by one thread); the merged LSE goes to lrun (lpart slot 0
// is still read by the other threads of its row) and is copied back by the caller.
void flash_fwd_merge(at::Tensor& opart, const at::Tensor& lpart, at::Tensor& lrun, int64_t H) {
  Range rr_("xdot.flash_fwd_merge");
  TORCH_CHECK(opart.dim() == 4 && opart.is_cuda(), "xdot.flash_fwd_merge: opart (S, B, R, C)");
  const int64_t S = opart.size(0), B = opart.size(1), R = opart.size(2), C = opart.size(3);
  TORCH_CHECK(H > 0 && C % H == 0 && (C / H) % 32 == 0, "xdot.flash_fwd_merge: H");
  check_part(opart, S, B * R * C, "opart");
  check_part(lpart, S, B * H * R, "lpart");
  TORCH_CHECK(lrun.is_cuda() && lrun.is_contiguous() && lrun.scalar_type() == at::kFloat && lrun.numel() == B * H * R,
              "xdot.flash_fwd_merge: lrun (B, H, R) fp32");
  xdot::fa::FwdArgs a{};
  a.out32 = opart.data_ptr<float>(); a.lse = lrun.data_ptr<float>();
  a.B = (int)B; a.H = (int)H; a.R = (int)R; a.nsplit = (int)S;
  a.opart = opart.data_ptr<float>(); a.lpart = lpart.data_ptr<float>();
  c10::DeviceGuard guard(opart.device());
  // dtype only selects the (unused) 16-bit output path
  TORCH_CHECK(xdot_flash_fwd_combine_launch(&a, xdot::DT_BF16, (int)(C / H), cur_stream(opart)) == 0,
              "xdot.flash_fwd_merge: config");
  check_launch(hipGetLastError(), "flash_fwd_merge");
}

// out = Σ_s part[s] in fp32; out may be part[0] (running sums: each element is read and
// written by one thread)
void sum_partials_into(const at::Tensor& part, at::Tensor& out) {
  Range rr_("xdot.sum_partials_into");
  TORCH_CHECK(part.is_cuda() && part.is_contiguous() && part.scalar_type() == at::kFloat && part.dim() >= 2,
              "xdot.sum_partials_into: contiguous fp32 (S, ...) device tensor");
  const int64_t n = part.numel() / part.size(0);
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.scalar_type() == at::kFloat && out.numel() == n,
              "xdot.sum_partials_into: out must be a contiguous fp32 slot");
  TORCH_CHECK(n % 4 == 0 && aligned16(part.data_ptr()) && aligned16(out.data_ptr()),
              "xdot.sum_partials_into: numel % 4 and 16-byte alignment");
  c10::DeviceGuard guard(part.device());
  TORCH_CHECK(xdot_sum_partials_launch(part.data_ptr<float>(), out.data_ptr(), (int)part.size(0), n, xdot::DT_F32,
                                       cur_stream(part)) == 0, "xdot.sum_partials_into");
  check_launch(hipGetLastError(), "sum_partials_into");
}

// row-side grads of this column chunk into partial slots [sp0, sp0 + nsplit) of dpart
void flash_bwd_rows_partial(const at::Tensor& dout, const at::Tensor& rows, const at::Tensor& kc, const at::Tensor& vc,
                            const at::Tensor& lse, const at::Tensor& delta, const c10::optional<at::Tensor>& bits,
                            const c10::optional<at::Tensor>& flags, int64_t H, double scale, at::Tensor& dpart,
                            int64_t sp0, int64_t nsplit, bool prescaled, int64_t fp32_mode) {
  Range rr_("xdot.flash_bwd_rows_partial");
  const FlashGeom g = flash_check(rows, kc, vc, H, bits, flags);
  TORCH_CHECK(delta.is_contiguous() && delta.scalar_type() == at::kFloat && delta.numel() == g.B * H * g.R,
              "xdot.flash_bwd_rows_partial: delta");
  TORCH_CHECK(sp0 >= 0 && nsplit >= 1, "xdot.flash_bwd_rows_partial: slots");
  const int ns = pick_split(1, g.T, 1, nsplit);
  check_part(dpart, sp0 + ns, g.B * g.R * g.C, "dpart");
  auto a = bwd_args(g, dout, rows, kc, vc, lse, bits, flags, H, scale);
  a.delta = delta.data_ptr<float>();
  a.nsplit = ns; a.sp0 = (int)sp0; a.force_partial = 1; a.dpart = dpart.data_ptr<float>();
  a.prescaled = prescaled ? 1 : 0;
  a.fp32_mode = (int)fp32_mode;
  c10::DeviceGuard guard(rows.device());
  TORCH_CHECK(xdot_flash_bwd_rows_launch(&a, dt_code(rows.scalar_type()), (int)g.D, cur_stream(rows)) == 0,
              "xdot.flash_bwd_rows_partial: config");
  check_launch(hipGetLastError(), "flash_bwd_rows_partial");
}

// Σ of all dpart slots -> (B, R, C) in like's dtype
at::Tensor flash_bwd_rows_sum(const at::Tensor& dpart, int64_t H, const at::Tensor& like) {
  Range rr_("xdot.flash_bwd_rows_sum");
  const int64_t B = like.size(0), R = like.size(1), C = like.size(2), S = dpart.size(0);
  check_part(dpart, S, B * R * C, "dpart");
  auto out = at::empty_like(like);
  xdot::fa::BwdArgs a{};
  a.drows = out.data_ptr(); a.dpart = dpart.data_ptr<float>();
  a.B = (int)B; a.H = (int)H; a.R = (int)R; a.nsplit = (int)S;
  c10::DeviceGuard guard(like.device());
  TORCH_CHECK(xdot_flash_bwd_rows_sum_launch(&a, dt_code(like.scalar_type()), (int)(C / H), cur_stream(like)) == 0,
              "xdot.flash_bwd_rows_sum: config");
  check_launch(hipGetLastError(), "flash_bwd_rows_sum");
  return out;
}


// ---- native xGMI pull collectives (csrc/ipc.hip; driven by xdot/utils/ipc.py) ----
void ipc_ok(int rc, const char* what) { TORCH_CHECK(rc == 0, "xdot.", what, ": HIP error ", rc); }

std::vector<int64_t> ipc_info() {
  return {xdot_ipc_sig_bytes(), xdot_ipc_max_ranks(), xdot_ipc_max_wgs(), xdot_ipc_handle_bytes(),
          xdot_ipc_wall_clock_khz()};
}
int64_t ipc_alloc(int64_t nbytes, bool uncached) {
  TORCH_CHECK(nbytes > 0, "xdot.ipc_alloc: size");
  void* p = nullptr;
  ipc_ok(xdot_ipc_alloc(nbytes, uncached ? 1 : 0, &p), "ipc_alloc");
  return (int64_t)(uintptr_t)p;
}
void ipc_free(int64_t p) { ipc_ok(xdot_ipc_free((void*)(uintptr_t)p), "ipc_free"); }
at::Tensor ipc_get_handle(int64_t p) {
  auto h = at::empty({xdot_ipc_handle_bytes()}, at::TensorOptions().dtype(at::kByte));
  ipc_ok(xdot_ipc_get_handle((void*)(uintptr_t)p, h.data_ptr()), "ipc_get_handle");
  return h;
}
int64_t ipc_open(const at::Tensor& h) {
  TORCH_CHECK(!h.is_cuda() && h.scalar_type() == at::kByte && h.is_contiguous() && h.numel() == xdot_ipc_handle_bytes(),
              "xdot.ipc_open: a CPU uint8 handle tensor");
  void* p = nullptr;
  ipc_ok(xdot_ipc_open(h.data_ptr(), &p), "ipc_open");
  return (int64_t)(uintptr_t)p;
}
void ipc_close(int64_t p) { ipc_ok(xdot_ipc_close((void*)(uintptr_t)p), "ipc_close"); }
std::vector<int64_t> ipc_host_word() {
  void *host = nullptr, *dev = nullptr;
  ipc_ok(xdot_ipc_host_word(&host, &dev), "ipc_host_word");
  return {(int64_t)(uintptr_t)host, (int64_t)(uintptr_t)dev};
}
int64_t ipc_read_word(int64_t host) { return (int64_t)*reinterpret_cast<volatile uint32_t*>((uintptr_t)host); }
void ipc_write_word(int64_t host, int64_t v) { *reinterpret_cast<volatile uint32_t*>((uintptr_t)host) = (uint32_t)v; }

xdot::ipc::Args ipc_args(const at::Tensor& inp, at::Tensor& out, at::IntArrayRef stage, at::IntArrayRef sig,
                         int64_t status, int64_t rank, int64_t epoch, int64_t ticks, int64_t nwg, const char* what) {
  const int64_t n = (int64_t)stage.size();
  TORCH_CHECK(n >= 2 && n <= xdot::ipc::MAXR && (int64_t)sig.size() == n && rank >= 0 && rank < n, "xdot.", what,
              ": ranks");
  TORCH_CHECK(nwg >= 1 && nwg <= xdot::ipc::MAXG && epoch >= 1 && status != 0, "xdot.", what, ": config");
  TORCH_CHECK(inp.is_cuda() && out.is_cuda() && inp.is_contiguous() && out.is_contiguous() &&
              inp.device() == out.device() && inp.element_size() >= 2 &&
              (uintptr_t)inp.data_ptr() % 2 == 0 && (uintptr_t)out.data_ptr() % 2 == 0,
              "xdot.", what, ": contiguous 16/32-bit device tensors");
  xdot::ipc::Args a{};
  a.src = static_cast<const char*>(inp.data_ptr());
  a.out = static_cast<char*>(out.data_ptr());
  for (int64_t p = 0; p < n; ++p) {
    TORCH_CHECK(stage[p] != 0 && sig[p] != 0 && stage[p] % 16 == 0, "xdot.", what, ": peer pointers");
    a.stage[p] = reinterpret_cast<char*>((uintptr_t)stage[p]);
    a.sig[p] = reinterpret_cast<uint32_t*>((uintptr_t)sig[p]);
  }
  a.status = reinterpret_cast<uint32_t*>((uintptr_t)status);
  a.timeout_ticks = ticks;
  a.rank = (int)rank; a.n = (int)n; a.epoch = (int)epoch; a.nwg = (int)nwg;
  return a;
}

// out (N * inp bytes, rank-major) <- every rank's inp, pulled over xGMI from the peers' staging slots
void ipc_all_gather(const at::Tensor& inp, at::Tensor& out, at::IntArrayRef stage, at::IntArrayRef sig, int64_t status,
                    int64_t rank, int64_t epoch, int64_t ticks, int64_t nwg) {
  Range rr_("xdot.ipc_all_gather");
  auto a = ipc_args(inp, out, stage, sig, status, rank, epoch, ticks, nwg, "ipc_all_gather");
  const int64_t bytes = inp.numel() * inp.element_size();
  TORCH_CHECK(out.numel() * out.element_size() == bytes * a.n && bytes % 16 == 0, "xdot.ipc_all_gather: sizes");
  a.shard = bytes;
  c10::DeviceGuard guard(inp.device());
  TORCH_CHECK(xdot_ipc_all_gather_launch(&a, cur_stream(inp)) == 0, "xdot.ipc_all_gather: config");
  check_launch(hipGetLastError(), "ipc_all_gather");
}

// out <- Σ over ranks (rank order, fp32) of block `rank` of the rank-major inp
void ipc_reduce_scatter(const at::Tensor& inp, at::Tensor& out, at::IntArrayRef stage, at::IntArrayRef sig,
                        int64_t status, int64_t rank, int64_t epoch, int64_t ticks, int64_t nwg) {
  Range rr_("xdot.ipc_reduce_scatter");
  auto a = ipc_args(inp, out, stage, sig, status, rank, epoch, ticks, nwg, "ipc_reduce_scatter");
  TORCH_CHECK(inp.scalar_type() == out.scalar_type(), "xdot.ipc_reduce_scatter: dtype");
  const int64_t bytes = out.numel() * out.element_size();
  TORCH_CHECK(inp.numel() == out.numel() * a.n && bytes % 16 == 0, "xdot.ipc_reduce_scatter: sizes");
  a.shard = bytes;
  a.dt = dt_code(inp.scalar_type());
  c10::DeviceGuard guard(inp.device());
  TORCH_CHECK(xdot_ipc_reduce_scatter_launch(&a, cur_stream(inp)) == 0, "xdot.ipc_reduce_scatter: config");
  check_launch(hipGetLastError(), "ipc_reduce_scatter");
}

// ---- HIP graph node priorities: diagnostics (benchmarks/micro/graph_prio_probe.py) ----
// Stream capture records the fork/join topology but not the stream priorities, and on ROCm 7.2
// hipGraphKernelNodeSetAttribute(.., hipKernelNodeAttributePriority, ..) returns invalid
// argument, so a captured two-stream backward cannot get its priority back
// (profiles/r3_graph.md); these two ops let the probe re-check a newer runtime.
void graph_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) (void)hipGetLastError();  // do not leave the error for the next HIP call
  TORCH_CHECK(e == hipSuccess, "xdot.", what, ": ", hipGetErrorString(e));
}

bool is_kernel_node(hipGraphNode_t n) {
  hipGraphNodeType t;
  return hipGraphNodeGetType(n, &t) == hipSuccess && t == hipGraphNodeTypeKernel;
}

// priorities of every kernel node of a graph (diagnostics / tests)
std::vector<int64_t> graph_kernel_priorities(int64_t raw) {
  hipGraph_t g = reinterpret_cast<hipGraph_t>((uintptr_t)raw);
  size_t n = 0;
  graph_ok(hipGraphGetNodes(g, nullptr, &n), "graph_kernel_priorities");
  std::vector<hipGraphNode_t> nodes(n);
  graph_ok(hipGraphGetNodes(g, nodes.data(), &n), "graph_kernel_priorities");
  std::vector<int64_t> out;
  for (auto nd : nodes) {
    if (!is_kernel_node(nd)) continue;
    hipKernelNodeAttrValue v{};
    graph_ok(hipGraphKernelNodeGetAttribute(nd, hipKernelNodeAttributePriority, &v), "graph_kernel_priorities");
    out.push_back(v.priority);
  }
  return out;
}

// set the priority attribute of the i-th kernel node of a graph (diagnostics)
void graph_set_kernel_priority(int64_t raw, int64_t index, int64_t prio) {
  hipGraph_t g = reinterpret_cast<hipGraph_t>((uintptr_t)raw);
  size_t n = 0;
  graph_ok(hipGraphGetNodes(g, nullptr, &n), "graph_set_kernel_priority");
  std::vector<hipGraphNode_t> nodes(n);
  graph_ok(hipGraphGetNodes(g, nodes.data(), &n), "graph_set_kernel_priority");
  int64_t k = 0;
  for (auto nd : nodes) {
    if (!is_kernel_node(nd)) continue;
    if (k++ != index) continue;
    hipKernelNodeAttrValue v{};
    v.priority = (int)prio;
    graph_ok(hipGraphKernelNodeSetAttribute(nd, hipKernelNodeAttributePriority, &v), "graph_set_kernel_priority");
    return;
  }
  TORCH_CHECK(false, "xdot.graph_set_kernel_priority: no kernel node ", index);
}

}  // namespace

TORCH_LIBRARY(xdot, m) {
  m.def("gemm(Tensor A, Tensor B, Tensor(a!) C, int M, int N, int K, int nseg, int nb1, int nb2, "
        "int lda, int ldb, int ldc, int sA1, int sA2, int sB1, int sB2, int sC1, int sC2, "
        "int sAseg, int sBseg, bool a_mc, bool b_mc, float alpha, float beta=0.0, int path=0) -> ()");
  m.def("softmax_fwd(Tensor x, Tensor? mask, float scale, int mdiv, int mmul, int mmod) -> Tensor");
  m.def("softmax_bwd(Tensor y, Tensor dy, float scale) -> Tensor");
  m.def("mask_pack(Tensor mask) -> (Tensor, Tensor, Tensor)");
  m.def("flash_fwd(Tensor rows, Tensor kc, Tensor vc, Tensor? bits, Tensor? flags, int H, float scale, int nsplit=0, bool prescaled=False, int fp32_mode=0, Tensor(a!)? sbuf=None) -> (Tensor, Tensor)");
  m.def("flash_bwd_cols(Tensor dout, Tensor rows, Tensor kc, Tensor vc, Tensor out, Tensor lse, Tensor? bits, "
        "Tensor? flags, int H, float scale, Tensor? delta=None, bool fp32_out=True, bool prescaled=False, "
        "Tensor? lse2=None, int fp32_mode=0, Tensor(a!)? sbuf=None, Tensor(b!)? dsbuf=None, int passes=3, "
        "Tensor(c!)? dkv_out=None) -> (Tensor, Tensor)");
  m.def("flash_bwd_prep(Tensor dout, Tensor out, Tensor lse, int H) -> (Tensor, Tensor)");
  m.def("flash_bwd_delta(Tensor dout, Tensor out, int H) -> Tensor");
  m.def("sum_partials(Tensor part, ScalarType out_dtype) -> Tensor");
  m.def("flash_splits(int B, int R, int T, int H, bool rows_kernel) -> int");
  m.def("flash_fwd_partial(Tensor rows, Tensor kc, Tensor vc, Tensor? bits, Tensor? flags, int H, float scale, "
        "Tensor(a!) opart, Tensor(b!) lpart, int sp0, int nsplit, bool prescaled=False, int fp32_mode=0) -> ()");
  m.def("flash_fwd_combine(Tensor opart, Tensor lpart, int H, Tensor like) -> (Tensor, Tensor)");
  m.def("flash_bwd_rows_partial(Tensor dout, Tensor rows, Tensor kc, Tensor vc, Tensor lse, Tensor delta, Tensor? bits, "
        "Tensor? flags, int H, float scale, Tensor(a!) dpart, int sp0, int nsplit, bool prescaled=False, int fp32_mode=0) -> ()");
  m.def("flash_bwd_rows_sum(Tensor dpart, int H, Tensor like) -> Tensor");
  m.def("flash_fwd_merge(Tensor(a!) opart, Tensor lpart, Tensor(b!) lrun, int H) -> ()");
  m.def("sum_partials_into(Tensor part, Tensor(a!) out) -> ()");
  m.def("cast_multi(Tensor[] src, Tensor(a!)[] dst) -> ()");
  m.def("adamw_step(Tensor(a!)[] params, Tensor[] grads, Tensor(b!)[] exp_avg, Tensor(c!)[] exp_avg_sq, float lr, "
        "float beta1, float beta2, float eps, float weight_decay, int step, Tensor[] step_ts, Tensor? lr_t, "
        "Tensor(d!)[] grad_out) -> ()");
  m.def("flash_bwd_rows(Tensor dout, Tensor rows, Tensor kc, Tensor vc, Tensor lse, Tensor delta, Tensor? bits, "
        "Tensor? flags, int H, float scale, int nsplit=0, bool prescaled=False, int fp32_mode=0, Tensor? sbuf=None, "
        "Tensor? dsbuf=None) -> Tensor");
  m.def("flash_prescale(Tensor x, float scale) -> Tensor");
  m.def("mse_fwd(Tensor y, Tensor t) -> (Tensor, Tensor)");
  m.def("proj(Tensor x, Tensor w, Tensor? bias, bool nn, Tensor(a!)? out=None, int force=0, float alpha=1.0) -> Tensor");
  m.def("wgrad(Tensor dy, Tensor x, ScalarType out_dtype, int splits=0) -> Tensor");
  m.def("wgrad2(Tensor dy0, Tensor x0, Tensor dy1, Tensor x1, ScalarType out_dtype) -> Tensor[]");
  m.def("ipc_info() -> int[]");
  m.def("ipc_alloc(int nbytes, bool uncached) -> int");
  m.def("ipc_free(int ptr) -> ()");
  m.def("ipc_get_handle(int ptr) -> Tensor");
  m.def("ipc_open(Tensor handle) -> int");
  m.def("ipc_close(int ptr) -> ()");
  m.def("ipc_host_word() -> int[]");
  m.def("ipc_read_word(int host) -> int");
  m.def("ipc_write_word(int host, int v) -> ()");
  m.def("ipc_all_gather(Tensor inp, Tensor(a!) out, int[] stage, int[] sig, int status, int rank, int epoch, "
        "int ticks, int nwg) -> ()");
  m.def("ipc_reduce_scatter(Tensor inp, Tensor(a!) out, int[] stage, int[] sig, int status, int rank, int epoch, "
        "int ticks, int nwg) -> ()");
  m.def("build_id() -> str");
  m.def("graph_kernel_priorities(int graph) -> int[]");
  m.def("graph_set_kernel_priority(int graph, int index, int prio) -> ()");
}

TORCH_LIBRARY_IMPL(xdot, CompositeExplicitAutograd, m) {
  m.impl("build_id", &build_id);
  m.impl("graph_kernel_priorities", &graph_kernel_priorities);
  m.impl("graph_set_kernel_priority", &graph_set_kernel_priority);
  m.impl("flash_splits", &flash_splits);
  m.impl("ipc_info", &ipc_info);
  m.impl("ipc_alloc", &ipc_alloc);
  m.impl("ipc_free", &ipc_free);
  m.impl("ipc_get_handle", &ipc_get_handle);
  m.impl("ipc_open", &ipc_open);
  m.impl("ipc_close", &ipc_close);
  m.impl("ipc_host_word", &ipc_host_word);
  m.impl("ipc_read_word", &ipc_read_word);
  m.impl("ipc_write_word", &ipc_write_word);
}

TORCH_LIBRARY_IMPL(xdot, CUDA, m) {
  m.impl("gemm", &gemm);
  m.impl("softmax_fwd", &softmax_fwd);
  m.impl("softmax_bwd", &softmax_bwd);
  m.impl("mask_pack", &mask_pack);
  m.impl("flash_fwd", &flash_fwd);
  m.impl("flash_bwd_cols", &flash_bwd_cols);
  m.impl("flash_bwd_rows", &flash_bwd_rows);
  m.impl("flash_bwd_delta", &flash_bwd_delta);
  m.impl("flash_bwd_prep", &flash_bwd_prep);
  m.impl("sum_partials", &sum_partials);
  m.impl("flash_prescale", &flash_prescale);
  m.impl("mse_fwd", &mse_fwd);
  m.impl("proj", &proj);
  m.impl("wgrad", &wgrad);
  m.impl("wgrad2", &wgrad2);
  m.impl("flash_fwd_partial", &flash_fwd_partial);
  m.impl("flash_fwd_combine", &flash_fwd_combine);
  m.impl("flash_bwd_rows_partial", &flash_bwd_rows_partial);
  m.impl("flash_bwd_rows_sum", &flash_bwd_rows_sum);
  m.impl("flash_fwd_merge", &flash_fwd_merge);
  m.impl("sum_partials_into", &sum_partials_into);
  m.impl("adamw_step", &adamw_step);
  m.impl("cast_multi", &cast_multi);
  m.impl("ipc_all_gather", &ipc_all_gather);
  m.impl("ipc_reduce_scatter", &ipc_reduce_scatter);
}
