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
  float beta;      // C = alpha * A.B + beta * C (beta = 0: C is not read)
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

namespace fa {
struct FwdArgs {
  const void* rows;        // (B, R, H*D)
  const void* kc;          // gathered key side (B, T, ldkv), first H*D columns used
  const void* vc;          // gathered value side (B, T, ldkv)
  void* out;               // (B, R, H*D)
  float* lse;              // (B, H, R) natural-log LSE
  const uint64_t* mbits;   // (B, NKT, R) bit k = col kt*64+k masked, or null
  const uint8_t* mflags;   // (B, ceil(R/32), NKT) 0 none / 1 all / 2 partial, or null
  int B, H, R, T;
  int64_t ldkv;            // element stride between gathered rows (H*D, or 2*H*D when packed [q|v])
  float scale;             // softmax scale (not log2-scaled)
  int nsplit;              // column splits (>1: partials to opart/lpart, then combine)
  float* opart;            // (slots, B, R, H*D) fp32 normalised partial outputs
  float* lpart;            // (slots, B, H, R) partial LSE
  int sp0;                 // first partial slot of this launch (chunked launches)
  int force_partial;       // 1: write partials even with nsplit == 1 (no combine here)
  int prescaled;           // 1: rows hold K * scale * log2(e) (xdot_prescale_rows_launch)
  float* out32;            // combine only: non-null -> write the merged O in fp32 here (fully
                           // masked rows: 0 with lse -inf), a running partial for the ring
  int fp32_mode;           // fp32 inputs: 0 exact (flash_f32.hip), 1 split-bf16 (flash_x3.hip)
  // head-heavy grid (16-bit forward, xrbs > 0): XCD x = blockIdx % 8 owns row blocks
  // [x*xrbs, (x+1)*xrbs) (linear index bh*nrb + rb); the first xwhole run whole, the last xrem
  // are split into nsplit column pieces whose partials go to a compact buffer
  // opart/lpart[(piece * 8*xrem + tail) * 128 + row-in-block] (* D for opart)
  int xrbs, xwhole, xrem;
  // exact fp32 only: non-null -> the raw scores S of every computed 32x32 tile are stored here
  // ((B*H, ceil(R/32), ceil(T/32)) blocks of 1024 floats, flash_f32.hip "score buffer")
  float* sbuf;
};

struct BwdArgs {
  const void* rows;        // (B, R, H*D)   row side (k)
  const void* kc;          // gathered key side (q)
  const void* vc;          // gathered value side (v)
  const void* dout;        // (B, R, H*D)   upstream grad of out
  const float* lse;        // (B, H, R)
  const float* delta;      // (B, H, R) rowsum(dO * O)
  float* lse2;             // (B, H, R) lse * log2(e) for the column kernel (written by the prep kernel), or null
  void* drows;             // (B, R, H*D)   grad of row side (out dtype)
  void* dkc;               // (B, T, ldg) partial grads of the gathered key side (fp32 or the input dtype)
  void* dvc;               // (B, T, ldg) partial grads of the gathered value side
  int dkv16;               // 1: dkc/dvc are in the input dtype (bf16/fp16), 0: fp32
  const uint64_t* mbits;
  const uint8_t* mflags;
  int B, H, R, T;
  int64_t ldkv;            // element stride between gathered input rows
  int64_t ldg;             // element stride between rows of the dkc/dvc outputs
  float scale;
  int nsplit;              // column splits of the row-side kernel
  float* dpart;            // (slots, B, R, H*D) fp32 partial row-side grads (nsplit > 1)
  int sp0;                 // first partial slot of this launch (chunked launches)
  int force_partial;       // 1: write partials even with nsplit == 1 (summed separately)
  int prescaled;           // 1: rows hold K * scale * log2(e) (same buffer as the forward's)
  int fp32_mode;           // fp32 inputs: 0 exact (flash_f32.hip), 1 split-bf16 (flash_x3.hip)
  // fp32 (exact / split): the forward's score buffer (FwdArgs::sbuf).  The column kernel reads S
  // from it instead of recomputing it and writes dS; the row kernel then reads dS
  float* sbuf;
  // dS buffer (same block layout), or nullptr: dS overwrites S in place (the dV pass must then
  // run before the dQ pass).  With it the dV pass can run after the dQ pass, concurrently with the
  // row kernel (D <= 128 kernels)
  float* dsbuf;
  int sb_passes;           // column launch in score-buffer mode: bit 0 dV pass, bit 1 dQ pass (0: both)
  // row splits of the fp32 column kernels (0 / 1: none).  A (b, h) x 128-column workgroup sweeps
  // all R rows, so B*H*T/128 workgroups run in ceil(W / slots) rounds and a last round of a few
  // workgroups idles the GPU (T = R = 25000, H = 8: 1568 workgroups over 512 slots = 3.06 rounds
  // in 4).  With splits, workgroup (sp, b, h, cb) sweeps row tiles [sp NRT / s, (sp+1) NRT / s)
  // and writes fp32 partials (s, B*T, H*D) to cpq (dQ, or both grads of the recompute kernel's
  // main pass) / cpv (dV); xdot_flash_cols_sum_launch adds them up in order.
  int csq, csv;
  float* cpq;
  float* cpv;
  // head-heavy grid of the exact-fp32 fused column pass (xcb > 0): XCD x = blockIdx % 8 owns column
  // blocks [x*xcb, (x+1)*xcb) (linear index bh*ncb + cb); the first xwhole sweep all rows and write
  // the gradients directly, the last xrem run in csq row pieces whose partials are compact:
  // cpq/cpv[((piece * 8*xrem + tail) * 128 + column-in-block) * D]
  int xcb, xwhole, xrem;
};

}  // namespace fa

}  // namespace xdot

namespace xdot {
// multi-tensor AdamW (csrc/optim.hip): up to ADAM_MAX_T tensors per launch
constexpr int ADAM_MAX_T = 32;
constexpr int ADAM_BLOCK_ELEMS = 256 * 4;
struct AdamArgs {
  void* p[ADAM_MAX_T];
  const void* g[ADAM_MAX_T];
  float* m[ADAM_MAX_T];
  float* v[ADAM_MAX_T];
  int64_t n[ADAM_MAX_T];
  int blk0[ADAM_MAX_T + 1];  // first block of each tensor (prefix sum)
  int nt;
  float lr, beta1, beta2, eps, wd, bc1, bc2_sqrt;
  // graph-capturable optimizer (dev_state = 1): every tensor's step count lives on the device
  // (the optimizer's per-parameter state["step"], advanced by a device op before the update)
  // and so does the learning rate (refreshed from the param group before each replay); bc1 /
  // bc2_sqrt / lr are then read in the kernel
  int dev_state;
  const float* step_dev[ADAM_MAX_T];
  const float* lr_dev;
  // g32 = 1: the gradients are fp32 (GradSync's reduced fp32 sums of 16-bit parameters) and each
  // is also written, rounded to the parameter dtype, into gout (the parameter's .grad): the
  // write-back pass of GradSync.wait() folded into the update
  int g32;
  void* gout[ADAM_MAX_T];
};
// multi-tensor dtype conversion (csrc/optim.hip): dst[i] = (dst dtype) src[i] for up to CAST_MAX_T
// tensor pairs per launch (GradSync's fp32 reduce buffers <-> 16-bit gradients)
constexpr int CAST_MAX_T = 32;
constexpr int CAST_BLOCK_ELEMS = 256 * 8;
struct CastArgs {
  const void* src[CAST_MAX_T];
  void* dst[CAST_MAX_T];
  int64_t n[CAST_MAX_T];
  int sdt[CAST_MAX_T], ddt[CAST_MAX_T];
  int blk0[CAST_MAX_T + 1];  // first block of each pair (prefix sum)
  int nt;
};
// projection GEMM (csrc/gemm_proj.hip): C[M, N] = A[M, K] . op(B) (+ bias[N]); A k-contiguous,
// B = W[N, K] (NT, forward) or W[K, N] (NN, input gradient), 16-bit, C row-major
struct ProjArgs {
  const void* A;
  const void* B;
  const void* bias;  // nullptr: none
  void* C;
  int M, N, K;
  int64_t lda, ldb, ldc;
  float alpha;       // C = alpha * (A . op(B) + bias)
};
namespace ipc {
constexpr int MAXR = 8;     // ranks of one node
constexpr int MAXG = 256;   // workgroups (byte ranges) per collective
constexpr int SIG_WORDS = 2 * MAXR * MAXG;  // arrive[MAXR][MAXG], done[MAXR][MAXG]

// one xGMI pull collective (csrc/ipc.hip)
struct Args {
  const char* src;           // local input
  char* out;                 // local output
  char* stage[MAXR];         // staging slot of every rank (own: local pointer)
  uint32_t* sig[MAXR];       // signal page of every rank (own: local pointer)
  uint32_t* status;          // host-mapped error word
  int64_t shard;             // bytes per rank block (multiple of 16)
  int64_t timeout_ticks;     // wall-clock ticks per wait
  int rank, n, epoch, nwg, dt;
};
}  // namespace ipc
}  // namespace xdot

extern "C" {
int xdot_gemm_launch(const xdot::GemmArgs* a, int batches, int dt_in, int dt_out, int a_mc,
                     int b_mc, int vec, hipStream_t st);
// exact-fp32 GEMM (csrc/gemm_f32.hip): fp32 in / out, same arguments as xdot_gemm_launch
int xdot_gemm_f32_launch(const xdot::GemmArgs* a, int batches, int a_mc, int b_mc, int vec, hipStream_t st);
// 256x256 LDS-DMA 16-bit GEMM (csrc/gemm2.hip); splits > 1 needs ws: splits*batches*M*N fp32
int xdot_gemm2_launch(const xdot::GemmArgs* a, int batches, int dt_in, int dt_out, int a_mc, int b_mc,
                      int splits, float* ws, hipStream_t st);
// persistent 256x256 LDS-DMA exact-fp32 GEMM (csrc/gemm2_f32.hip); eligibility in the file;
// splits > 1 needs ws (splits*batches*M*N fp32) and runs the ordered sum itself
int xdot_gemm2_f32_launch(const xdot::GemmArgs* a, int batches, int a_mc, int b_mc, int splits, float* ws,
                          hipStream_t st);
// compute units of the current device (csrc/gemm2.hip)
int xdot_num_cus();
// C = alpha * (ordered sum of `splits` fp32 partials ws[s][z][M][N]) + beta * C  (csrc/gemm2.hip)
int xdot_gemm_reduce_launch(const xdot::GemmArgs* a, const float* ws, int splits, int batches, int dt_out,
                            hipStream_t st);
// 8-phase 16x16x32 16-bit GEMM (csrc/gemm3.hip): M, N >= 256, K % 8 == 0; -3 = not eligible
int xdot_gemm3_launch(const xdot::GemmArgs* a, int batches, int dt_in, int dt_out, int a_mc, int b_mc,
                      int splits, float* ws, hipStream_t st);
// projection GEMM; -3 = not eligible (16-bit, K % 64 == 0, N % 64 == 0 (NN: % 128), 16-byte
// aligned A / B with lda, ldb % 8 == 0, 8-byte aligned C with ldc % 4 == 0) or, unless force,
// large enough for the library to be faster
int xdot_gemm_proj_launch(const xdot::ProjArgs* a, int dt, int nn, int force, hipStream_t st);
// weight gradients dW_i = A_iᵀ B_i (csrc/gemm_wgrad.hip), np = 1 or 2 products in one launch: A (K, M),
// B (K, N) row-major 16-bit, S slabs of K -> fp32 partials part (S, M, N); -3 = not eligible
// (M, N % 128, lda / ldb % 8, 16-byte bases)
int xdot_gemm_wgrad_launch(int np, const void* const* A, const void* const* B, float* const* part, const int* M,
                           const int* N, const int* K, const int* S, const int64_t* lda, const int64_t* ldb, int dt,
                           hipStream_t st);
// fp32 operand -> compact bf16 parts [z1][z2][3][seg][R][C] (hi, or lo where lo_mask bit p is set)
int xdot_split3_launch(const float* src, void* dst, int64_t s1, int64_t s2, int64_t sseg, int64_t ld,
                       int nb1, int nb2, int nseg, int R, int C, int lo_mask, hipStream_t st);
int xdot_softmax_fwd_launch(const xdot::smx::Args* a, int dt, int vec, hipStream_t st);
int xdot_softmax_bwd_launch(const xdot::smx::Args* a, int dt, int vec, hipStream_t st);
// bool mask (B, R, T) -> row-major bits (B, R, NKT), column-major bits (B, ceil(R/64),
// ceil(T/128)*128) and tile flags (B, ceil(R/32), NKT4); one read of the mask
int xdot_mask_pack_launch(const uint8_t* mask, uint64_t* bits, uint64_t* bt, uint8_t* flags, int B, int R, int T,
                          hipStream_t st);
int xdot_flash_fwd_launch(const xdot::fa::FwdArgs* a, int dt, int D, hipStream_t st);
// δ = rowsum(dO ⊙ O) (reads a->dout, a->B/R/H)
int xdot_flash_bwd_delta_launch(const xdot::fa::BwdArgs* a, const void* out, float* delta, int dt, int D, hipStream_t st);
// gathered-side grads; a->delta must hold δ
int xdot_flash_bwd_cols_launch(const xdot::fa::BwdArgs* a, int dt, int D, hipStream_t st);
int xdot_flash_bwd_rows_launch(const xdot::fa::BwdArgs* a, int dt, int D, hipStream_t st);
// software-pipelined column kernel (csrc/flash_cols.hip): pre-scaled 16-bit, D <= 96; -1 = not taken
int xdot_flash_bwd_cols2_launch(const xdot::fa::BwdArgs* a, int dt, int D, hipStream_t st);
// out (n elements, dtype dto) = Σ_s part[s] (fp32 partials, n % 4 == 0)
int xdot_sum_partials_launch(const float* part, void* out, int S, int64_t n, int dto, hipStream_t st);
// both products of a paired weight-gradient launch in one pass (a: n_a elements, b: n_b)
int xdot_sum_partials2_launch(const float* pa, void* oa, int Sa, int64_t na, const float* pb, void* ob, int Sb,
                              int64_t nb, int dto, hipStream_t st);
// out = (16-bit) (x * (scale * log2 e)) elementwise, n % 8 == 0: the pre-scaled row side of the
// flash kernels (the factor is formed in fp32 exactly as the kernels form it)
int xdot_prescale_rows_launch(const void* x, void* out, int64_t n, float scale, int dt, hipStream_t st);
// rows per workgroup of the forward kernel (128)
int xdot_flash_fwd_rows_per_wg();
// one AdamW step over a->nt tensors of dtype dt (params/grads), fp32 moments
int xdot_adamw_launch(const xdot::AdamArgs* a, int dt, hipStream_t st);
// resident workgroups per CU of the exact-fp32 forward (head-heavy grid planning), 0: no kernel
int xdot_flash_f32_fwd_occ(int D, bool sbuf);
// XDOT_F32_HEAVY (default 1): the exact-fp32 forward may take the head-heavy grid
int xdot_flash_f32_heavy();
// a->nt conversions in one launch (DT_F32 / DT_BF16 / DT_F16 each side)
int xdot_cast_multi_launch(const xdot::CastArgs* a, hipStream_t st);
int xdot_mse_fwd_launch(const void* y, const void* t, void* dy, float* part, int nparts, void* loss, int64_t n, int dt,
                        hipStream_t st);
// merge a->nsplit partial slots (a->opart, a->lpart) into a->out / a->lse
int xdot_flash_fwd_combine_launch(const xdot::fa::FwdArgs* a, int dt, int D, hipStream_t st);
// sum a->nsplit slots of a->dpart into a->drows
int xdot_flash_bwd_rows_sum_launch(const xdot::fa::BwdArgs* a, int dt, int D, hipStream_t st);
// exact-fp32 flash family (csrc/flash_f32.hip); the launchers above route DT_F32 here
int xdot_flash_fwd_f32_launch(const xdot::fa::FwdArgs* a, int D, hipStream_t st);
int xdot_flash_combine_f32_launch(const xdot::fa::FwdArgs* a, int D, hipStream_t st);
int xdot_flash_bwd_prep_f32_launch(const xdot::fa::BwdArgs* a, const void* out, float* delta, int D, hipStream_t st);
int xdot_flash_bwd_rows_f32_launch(const xdot::fa::BwdArgs* a, int D, hipStream_t st);
int xdot_flash_bwd_cols_f32_launch(const xdot::fa::BwdArgs* a, int D, hipStream_t st);
// row splits the fp32 column launch would use (occupancy-aware round model): *sq for the dQ /
// recompute pass, *sv for the dV pass (score-buffer mode); both 1 for other families
int xdot_flash_cols_splits(const xdot::fa::BwdArgs* a, int dt, int D, int* sq, int* sv);
int xdot_flash_cols_splits_f32(const xdot::fa::BwdArgs* a, int D, int* sq, int* sv);
// head-heavy plan of the exact-fp32 fused column pass (sbuf, 4 passes, D <= 128): 1 and
// (whole, rem, split) per XCD when the round model prefers it over the uniform split sq, else 0
int xdot_flash_f32_cols_heavy(const xdot::fa::BwdArgs* a, int D, int sq, int* whole, int* rem, int* split);
int xdot_flash_cols_splits_x3(const xdot::fa::BwdArgs* a, int D, int* sq, int* sv);
// out[r * ldo + c] = Σ_s part[(s * rows + r) * C + c] for r < rows, c < C (C % 4 == 0): fp32
// partials, output in dtype `dt` (DT_F32 / DT_BF16 / DT_F16)
int xdot_flash_cols_sum_launch(const float* part, void* out, int S, int64_t rows, int C, int64_t ldo, int dt,
                               hipStream_t st);
int xdot_flash_cols_splits_cols2(const xdot::fa::BwdArgs* a, int dt, int D, int* sq);
// column splits of the fp32 row-block kernels (kernel 0: forward, 1: row-side backward) for W
// unsplit workgroups over T columns: occupancy of the instantiation x CUs, round model
// (XDOT_F32_SPLIT: unset / auto = model, "old" = the 16-bit model, n = forced); 0: not handled
int xdot_flash_f32_row_splits(int kernel, int fp32_mode, int D, bool sbuf, int64_t W, int64_t T);
int xdot_flash_f32_row_splits_exact(int kernel, int D, bool sbuf, int64_t W, int64_t T);
int xdot_flash_f32_row_splits_x3(int kernel, int D, bool sbuf, int64_t W, int64_t T);
// split counts of the wide (D > 128) kernels from their own occupancy: kernel 0 / 1 = column
// splits of the forward / row side (0: use the caller's model), 2 / 3 = row splits of the
// column side's dQ / dV pass (XDOT_WIDE_SPLIT: auto, 0 = off, n = forced)
int xdot_flash_wide_splits(int kernel, int dt, int D, bool sbuf, int64_t W, int64_t n);
int xdot_flash_rows_sum_f32_launch(const xdot::fa::BwdArgs* a, int D, hipStream_t st);
// wide head dims (csrc/flash_wide.hip): D = 160 / 192 / 256 / 384, 16-bit and exact fp32 (a wide
// fp32 launch always runs exact); -1 = not a wide (dtype, D), -2 = needs the score buffer (fp32 D > 256)
int xdot_flash_wide_fwd_launch(const xdot::fa::FwdArgs* a, int dt, int D, hipStream_t st);
int xdot_flash_wide_rows_launch(const xdot::fa::BwdArgs* a, int dt, int D, hipStream_t st);
int xdot_flash_wide_cols_launch(const xdot::fa::BwdArgs* a, int dt, int D, hipStream_t st);
// split-bf16 fp32 family (csrc/flash_x3.hip, fp32_mode = 1); prep / combine / sum are shared
int xdot_flash_fwd_x3_launch(const xdot::fa::FwdArgs* a, int D, hipStream_t st);
int xdot_flash_bwd_rows_x3_launch(const xdot::fa::BwdArgs* a, int D, hipStream_t st);
int xdot_flash_bwd_cols_x3_launch(const xdot::fa::BwdArgs* a, int D, hipStream_t st);
// native xGMI pull collectives (csrc/ipc.hip)
int xdot_ipc_sig_bytes();
int xdot_ipc_max_ranks();
int xdot_ipc_max_wgs();
int xdot_ipc_alloc(int64_t bytes, int uncached, void** p);
int xdot_ipc_free(void* p);
int xdot_ipc_handle_bytes();
int xdot_ipc_get_handle(void* p, void* out);
int xdot_ipc_open(const void* handle, void** p);
int xdot_ipc_close(void* p);
int xdot_ipc_host_word(void** host, void** dev);
int xdot_ipc_wall_clock_khz();
int xdot_ipc_all_gather_launch(const xdot::ipc::Args* a, hipStream_t st);
int xdot_ipc_reduce_scatter_launch(const xdot::ipc::Args* a, hipStream_t st);
}
