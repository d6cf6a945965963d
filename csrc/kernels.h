// xdot — host-visible argument structs and C-ABI launchers of the gfx950 kernels.
// Shared between the kernel translation units (*.hip) and the torch binding (bindings.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xdot {

enum DType : int { DT_F32 = 0, DT_BF16 = 1, DT_F16 = 2 };

struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  int M, N, K;     // K = length of one segment
  int nseg;        // number of K segments
  int nb2;         // inner batch extent (z2 = z % nb2, z1 = z / nb2)
  int tiles_m, tiles_n;
  int64_t lda, ldb, ldc;
  int64_t sA1, sA2, sB1, sB2, sC1, sC2;  // batch strides (elements)
  int64_t sAseg, sBseg;                  // segment strides (elements)
  float alpha;
};

namespace smx {
struct Args {
  const void* x;      // fwd: scores ; bwd: y (probabilities)
  const void* dy;     // bwd only
  void* out;          // fwd: y ; bwd: dx
  const uint8_t* mask;
  int64_t rows, T;
  int64_t mdiv, mmul, mmod;
  float scale;
};
}  // namespace smx

}  // namespace xdot

extern "C" {
int xdot_gemm_launch(const xdot::GemmArgs* a, int batches, int dt_in, int dt_out, int a_mc,
                     int b_mc, int vec, hipStream_t st);
int xdot_softmax_fwd_launch(const xdot::smx::Args* a, int dt, int vec, hipStream_t st);
int xdot_softmax_bwd_launch(const xdot::smx::Args* a, int dt, int vec, hipStream_t st);
}
