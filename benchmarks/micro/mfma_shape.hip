// Bare bf16 MFMA throughput by shape on random operands (MI355X_MICROARCH.md 'DVFS give-back'
// item 7): v_mfma_f32_32x32x16_bf16 vs v_mfma_f32_16x16x32_bf16, same FLOP per wave, operands
// in registers (re-randomised per launch), 2 waves per SIMD, every CU busy.  Prints TFLOP/s.
// `mfma_shape f32`: the exact-fp32 shapes instead (v_mfma_f32_32x32x2_f32 vs
// v_mfma_f32_16x16x4_f32, 64 FLOP/clk/SIMD both): the clock-limited fp32 matrix rate that
// prices the exact-fp32 flash kernels (profiles/r6_fp32.md §2).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

template <int SHAPE, int ITERS>
__global__ __launch_bounds__(512) void mfma_loop(const u32x4* in, float* out) {
  const int t = blockIdx.x * 512 + threadIdx.x;
  u32x4 a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { a[i] = in[(t * 8 + i) & 0xfffff]; b[i] = in[(t * 8 + 4 + i) & 0xfffff]; }
  float s = 0.f;
  if constexpr (SHAPE == 32) {
    f32x16 c[4] = {};
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        c[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[i]), __builtin_bit_cast(bf16x8, b[i]), c[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) for (int r = 0; r < 16; ++r) s += c[i][r];
  } else if constexpr (SHAPE == 2) {  // f32 32x32x2: 4096 FLOP; 8 per iter
    f32x16 c[4] = {};
    const f32x4 fa = __builtin_bit_cast(f32x4, a[0]), fb = __builtin_bit_cast(f32x4, b[0]);
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) c[i & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i & 3], fb[(i + 1) & 3], c[i & 3], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) for (int r = 0; r < 16; ++r) s += c[i][r];
  } else if constexpr (SHAPE == 4) {  // f32 16x16x4: 2048 FLOP; 16 per iter
    f32x4 c[8] = {};
    const f32x4 fa = __builtin_bit_cast(f32x4, a[0]), fb = __builtin_bit_cast(f32x4, b[0]);
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int i = 0; i < 16; ++i) c[i & 7] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i & 3], fb[(i + (i >> 2)) & 3], c[i & 7], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) for (int r = 0; r < 4; ++r) s += c[i][r];
  } else {
    f32x4 c[8] = {};
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        c[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[i & 3]), __builtin_bit_cast(bf16x8, b[(i + (i >> 2)) & 3]), c[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) for (int r = 0; r < 4; ++r) s += c[i][r];
  }
  out[t] = s;
}

int main(int argc, char** argv) {
  const int nblk = 256 * 2 * 4;  // 4 rounds of 2 x 512-thread workgroups per CU (2 waves / SIMD)
  const int n = 1 << 20;
  std::vector<unsigned> h(4 * n);
  srand(1);
  for (auto& x : h) x = (unsigned)rand() * 2654435761u;  // random bf16 pairs (incl. large exponents)
  const bool f32 = argc > 1 && !strcmp(argv[1], "f32");
  if (f32) {
    for (auto& x : h) x = 0x3f800000u | (x & 0x807fffffu);  // fp32 in +-[1, 2): random mantissas
  } else {
    for (auto& x : h) x &= 0xbfffbfffu;                   // keep every bf16 finite (exponent < 255)
  }
  u32x4* din;
  float* dout;
  hipMalloc(&din, 16ull * n);
  hipMalloc(&dout, 4ull * nblk * 512);
  hipMemcpy(din, h.data(), 16ull * n, hipMemcpyHostToDevice);
  constexpr int IT = 4000, ITF = 1000;  // f32: 8 x 64 cycles per iteration vs 4 x 32
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = argc > 3 ? atoi(argv[3]) : 3;
  for (int rep = 0; rep < reps; ++rep) {
    for (int shape : f32 ? std::vector<int>{2, 4} : std::vector<int>{32, 16}) {
      float ms = 0;
      const int nl = argc > 2 ? atoi(argv[2]) : 1;  // launches per timed window (long windows: DVFS steady state)
      for (int w = 0; w < 2; ++w) {  // warm-up window then the timed one
        hipEventRecord(e0);
        for (int l = 0; l < nl; ++l) {
        if (shape == 32) hipLaunchKernelGGL((mfma_loop<32, IT>), dim3(nblk), dim3(512), 0, 0, din, dout);
        else if (shape == 16) hipLaunchKernelGGL((mfma_loop<16, IT>), dim3(nblk), dim3(512), 0, 0, din, dout);
        else if (shape == 2) hipLaunchKernelGGL((mfma_loop<2, ITF * 4>), dim3(nblk), dim3(512), 0, 0, din, dout);
        else hipLaunchKernelGGL((mfma_loop<4, ITF * 4>), dim3(nblk), dim3(512), 0, 0, din, dout);
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
      }
      // 32x32x16: 32768 FLOP x 4 per iter; 16x16x32: 16384 x 8 per iter (same)
      // f32 32x32x2: 4096 FLOP x 8 per iter; 16x16x4: 2048 x 16 per iter (same)
      const double flop = shape >= 16 ? 2.0 * 32 * 32 * 16 * 4 * (double)IT * (nblk * 8.0)
                                      : 2.0 * 32 * 32 * 2 * 8 * (double)(ITF * 4) * (nblk * 8.0);
      const char* nm = shape == 32 ? "32x32x16_bf16" : shape == 16 ? "16x16x32_bf16" : shape == 2 ? "32x32x2_f32" : "16x16x4_f32";
      printf("{\"shape\": \"%s\", \"rep\": %d, \"launches\": %d, \"ms\": %.3f, \"TFLOPs\": %.1f}\n", nm, rep, nl, ms,
             flop * nl / ms / 1e9);
    }
  }
  return 0;
}
