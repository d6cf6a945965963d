// Measures the cross-workgroup reduction a fused (5-product) flash backward would need for the
// row-side gradient dK (see profiles/r2_fused_bwd_analysis.md): every workgroup that owns a block
// of Cspan gathered columns sweeps all R local rows and contributes a 64 x D fp32 tile of dK per
// 64-row tile.  Three ways to sum those contributions, timed on the real sizes:
//   atomic      global fp32 atomic adds straight into dK (vector atomics, return value unused)
//   atomic_pk   packed bf16 atomic adds (half the bytes, bf16 accumulation)
//   slab+sum    plain 16-byte stores into per-column-block slabs, then an ordered sum pass
// Workgroups start their row sweep at a staggered tile (as a real kernel would) or all at 0.
// Build: hipcc -O3 --offload-arch=gfx950 -o benchmarks/native/atomic_partials benchmarks/native/atomic_partials.hip
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

constexpr int D = 96, RT = 64, NT = 256, PER = RT * D / NT;  // 24 floats per thread per tile

__global__ __launch_bounds__(NT) void k_atomic(float* dk, int R, int ncb, int stagger) {
  const int cb = blockIdx.x % ncb, h = blockIdx.x / ncb;
  const int nrt = R / RT;
  float* base = dk + (size_t)h * R * D;
  for (int i = 0; i < nrt; ++i) {
    const int rt = stagger ? (i + cb * 7) % nrt : i;
    float* t = base + (size_t)rt * RT * D;
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int idx = e * NT + threadIdx.x;
      __hip_atomic_fetch_add(t + idx, 1.0f + 1e-3f * (float)(cb & 7), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ __launch_bounds__(NT) void k_atomic_pk(__hip_bfloat162* dk, int R, int ncb, int stagger) {
  const int cb = blockIdx.x % ncb, h = blockIdx.x / ncb;
  const int nrt = R / RT;
  __hip_bfloat162* base = dk + (size_t)h * R * D / 2;
  for (int i = 0; i < nrt; ++i) {
    const int rt = stagger ? (i + cb * 7) % nrt : i;
    __hip_bfloat162* t = base + (size_t)rt * RT * D / 2;
#pragma unroll
    for (int e = 0; e < PER / 2; ++e) {
      const int idx = e * NT + threadIdx.x;
      unsafeAtomicAdd(t + idx, __hip_bfloat162{__float2bfloat16(1.0f), __float2bfloat16(1.0f)});
    }
  }
}

__global__ __launch_bounds__(NT) void k_slab(float4* slab, int R, int ncb, int stagger) {
  const int cb = blockIdx.x % ncb, h = blockIdx.x / ncb;
  const int nrt = R / RT;
  float4* base = slab + ((size_t)h * ncb + cb) * R * D / 4;
  for (int i = 0; i < nrt; ++i) {
    const int rt = stagger ? (i + cb * 7) % nrt : i;
    float4* t = base + (size_t)rt * RT * D / 4;
#pragma unroll
    for (int e = 0; e < PER / 4; ++e) {
      const int idx = e * NT + threadIdx.x;
      const float v = 1.0f + 1e-3f * (float)(cb & 7);
      t[idx] = float4{v, v, v, v};
    }
  }
}

// dk[h, r, d] = sum over column blocks in order (deterministic)
__global__ __launch_bounds__(NT) void k_sum(const float4* slab, float4* dk, int R, int ncb, int H) {
  const size_t n4 = (size_t)R * D / 4;
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n4 * H) return;
  const size_t h = i / n4, o = i % n4;
  float4 acc = slab[(h * ncb) * n4 + o];
  for (int c = 1; c < ncb; ++c) {
    const float4 v = slab[(h * ncb + c) * n4 + o];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  dk[i] = acc;
}

template <class F> float timeit(F f, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int i = 0; i < iters; ++i) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? std::atoi(argv[1]) : 25000 / RT * RT;  // 24960: whole 64-row tiles
  const int T = argc > 2 ? std::atoi(argv[2]) : 25000;
  const int H = 8, iters = 5;
  float* dk; CK(hipMalloc(&dk, (size_t)H * R * D * 4));
  for (int cspan : {128, 256}) {
    const int ncb = (T + cspan - 1) / cspan;
    const double bytes = (double)ncb * H * R * D * 4;
    for (int st = 0; st < 2; ++st) {
      const float ta = timeit([&] { hipLaunchKernelGGL(k_atomic, dim3(ncb * H), dim3(NT), 0, 0, dk, R, ncb, st); }, iters);
      const float tp = timeit([&] { hipLaunchKernelGGL(k_atomic_pk, dim3(ncb * H), dim3(NT), 0, 0, (__hip_bfloat162*)dk, R, ncb, st); }, iters);
      std::printf("{\"R\": %d, \"T\": %d, \"cspan\": %d, \"stagger\": %d, \"partial_GB\": %.2f, \"atomic_f32_ms\": %.3f, \"atomic_f32_TBps\": %.2f, \"atomic_pk_bf16_ms\": %.3f, \"atomic_pk_bf16_TBps\": %.2f}\n",
                  R, T, cspan, st, bytes / 1e9, ta, bytes / ta / 1e9, tp, bytes / 2 / tp / 1e9);
      std::fflush(stdout);
    }
    float4* slab;
    CK(hipMalloc(&slab, (size_t)bytes));
    const float ts = timeit([&] { hipLaunchKernelGGL(k_slab, dim3(ncb * H), dim3(NT), 0, 0, slab, R, ncb, 1); }, iters);
    const size_t n4 = (size_t)H * R * D / 4;
    const float tsum = timeit([&] { hipLaunchKernelGGL(k_sum, dim3((unsigned)((n4 + NT - 1) / NT)), dim3(NT), 0, 0, slab, (float4*)dk, R, ncb, H); }, iters);
    std::printf("{\"R\": %d, \"T\": %d, \"cspan\": %d, \"partial_GB\": %.2f, \"slab_store_ms\": %.3f, \"slab_store_TBps\": %.2f, \"ordered_sum_ms\": %.3f, \"ordered_sum_TBps\": %.2f}\n",
                R, T, cspan, bytes / 1e9, ts, bytes / ts / 1e9, tsum, bytes / tsum / 1e9);
    std::fflush(stdout);
    CK(hipFree(slab));
  }
  CK(hipFree(dk));
  return 0;
}
