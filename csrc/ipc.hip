// xdot — native xGMI pull collectives over HIP IPC (SURVEY §5.8 stage 2).
//
// The reference moves every block through Horovod/NCCL collectives
// (distributed_dot_product/multiplication/functions.py:89-97 all-gather loop, :143-147 and
// :202-210 the N all-reduces of `all`/`tn`).  Stage 1 of this repo maps those onto RCCL
// (xdot/utils/comm.py TorchDistComm).  This file is stage 2: every rank exports a staging
// buffer and a signal page with hipIpcGetMemHandle, maps its peers' pages
// (hipIpcOpenMemHandle) once, and then
//   all-gather       each rank PULLS the N-1 peer shards straight out of the peers' staging
//                    buffers over the point-to-point xGMI links — all 7 links of an MI355X are
//                    read concurrently (workgroups start at different peers), not one ring hop
//                    per step;
//   reduce-scatter   each rank pulls ITS block from every peer and sums the N blocks in fp32,
//                    in rank order 0..N-1: deterministic, one rounding to the output dtype
//                    (RCCL rounds bf16 partials after every ring hop).
//
// One kernel per collective, one workgroup per byte range w (the same range partition on
// every rank and for every collective of a communicator), so synchronisation is per (peer, range) flag and needs no grid barrier:
//   1. wait until every peer has finished READING our staging slot from two collectives ago
//      (done[p][w] >= epoch - 2: the slots alternate);
//   2. copy range w of the input into our staging slot, write it back to memory
//      (system-scope release: the peers read HBM over xGMI, not our L2) and publish
//      arrive[r][w] = epoch into every peer's signal page (a remote 4-byte vector store);
//   3. for each peer: wait for its arrive[p][w] >= epoch (local spin on our own uncached
//      signal page), acquire at system scope (invalidates stale remote lines in this XCD's
//      L2), pull its range w, then publish done[r][w] = epoch into that peer's page.
// Every wait is bounded by a wall-clock budget: on expiry the kernel sets a host-mapped error
// word and drains (every wave reaches the end), and the host raises on its next call.
// All flag traffic uses vector memory instructions only.
#include "common.h"

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

namespace xdot {
namespace ipc {

__device__ inline uint32_t ld_flag(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline void st_flag(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// thread 0 spins until *p >= want (or the budget expires: error word set); returns true for
// every thread of the workgroup when the wait EXPIRED (the caller then poisons its output
// range with NaN instead of reading the peer's stale bytes)
__device__ inline bool wait_ge(const uint32_t* p, uint32_t want, const Args& a) {
  __shared__ int expired;
  if (threadIdx.x == 0) {
    int ex = 0;
    const uint64_t t0 = wall_clock64();
    while ((int32_t)(ld_flag(p) - want) < 0) {
      if ((int64_t)(wall_clock64() - t0) > a.timeout_ticks) {
        st_flag(a.status, 1u);
        ex = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    expired = ex;
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
  const bool ex = expired != 0;
  __syncthreads();  // `expired` is reused by the next wait
  return ex;
}

// dst[v] = all-ones (NaN in fp32 / bf16 / fp16) for 16-byte units v in [v0, v1)
__device__ inline void poison_units(char* dst, int64_t v0, int64_t v1) {
  u32x4_ua* d = reinterpret_cast<u32x4_ua*>(dst);
  for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) d[v] = u32x4{~0u, ~0u, ~0u, ~0u};
}

// publish: this workgroup's stores are in memory before the flag lands at the peer
__device__ inline void release_all() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
}

__device__ inline void range_of(const Args& a, int w, int64_t& v0, int64_t& v1) {
  const int64_t nv = a.shard / 16;
  const int64_t per = (nv + a.nwg - 1) / a.nwg;
  v0 = min(nv, (int64_t)w * per);
  v1 = min(nv, v0 + per);
}

// dst[v] = src[v] for 16-byte units v in [v0, v1); 4 units in flight per thread
__device__ inline void copy_units(char* dst, const char* src, int64_t v0, int64_t v1) {
  const u32x4_ua* s = reinterpret_cast<const u32x4_ua*>(src);
  u32x4_ua* d = reinterpret_cast<u32x4_ua*>(dst);
  const int64_t step = (int64_t)blockDim.x;
  int64_t v = v0 + threadIdx.x;
  for (; v + 3 * step < v1; v += 4 * step) {
    const u32x4 x0 = s[v], x1 = s[v + step], x2 = s[v + 2 * step], x3 = s[v + 3 * step];
    d[v] = x0; d[v + step] = x1; d[v + 2 * step] = x2; d[v + 3 * step] = x3;
  }
  for (; v < v1; v += step) d[v] = s[v];
}

// the peer workgroup w visits at step q (spreads the workgroups over all links)
__device__ inline int peer_at(const Args& a, int w, int q) { return (a.rank + 1 + (w + q) % (a.n - 1)) % a.n; }

__global__ __launch_bounds__(256) void all_gather_kernel(Args a) {
  const int w = blockIdx.x;
  uint32_t* arrive = a.sig[a.rank];
  uint32_t* done = a.sig[a.rank] + MAXR * MAXG;
  int64_t v0, v1;
  range_of(a, w, v0, v1);
  // 1. our slot is free once every peer finished reading it two collectives ago.  If that wait
  //    expires, a (merely slow) peer may still be reading the old epoch's bytes: overwriting the
  //    slot and raising our flag would hand it the new bytes as the old ones.  So this range is
  //    neither staged nor published (the peers' waits expire and poison theirs: loud on every
  //    rank) and our own output range is poisoned.
  bool busy = false;
  if (a.epoch > 2)
    for (int p = 0; p < a.n; ++p)
      if (p != a.rank) busy |= wait_ge(done + p * MAXG + w, (uint32_t)(a.epoch - 2), a);
  if (busy) {
    for (int p = 0; p < a.n; ++p) poison_units(a.out + p * a.shard, v0, v1);
    return;
  }
  // 2. stage range w (and our own output block), publish
  copy_units(a.stage[a.rank], a.src, v0, v1);
  if (a.src != a.out + a.rank * a.shard)  // in place (the producer wrote out[rank]): no own-block copy
    copy_units(a.out + a.rank * a.shard, a.src, v0, v1);
  release_all();
  if (threadIdx.x < a.n && threadIdx.x != a.rank)
    st_flag(a.sig[threadIdx.x] + a.rank * MAXG + w, (uint32_t)a.epoch);
  // 3. pull range w of every peer (NaN if the peer never arrived)
  for (int q = 0; q < a.n - 1; ++q) {
    const int p = peer_at(a, w, q);
    if (wait_ge(arrive + p * MAXG + w, (uint32_t)a.epoch, a)) {
      poison_units(a.out + p * a.shard, v0, v1);
      continue;
    }
    copy_units(a.out + p * a.shard, a.stage[p], v0, v1);
    release_all();  // the loads have returned (their data is stored) before the peer may refill
    if (threadIdx.x == 0) st_flag(a.sig[p] + MAXR * MAXG + a.rank * MAXG + w, (uint32_t)a.epoch);
  }
}

template <int DT>
__device__ inline void acc_unit(float (&acc)[8], const u32x4& x) {
  if constexpr (DT == DT_F32) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] += __uint_as_float(x[i]);
  } else {
    using T = typename dt_traits<DT>::T;
    union { u32x4 u; T e[8]; } c;
    c.u = x;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += (float)c.e[i];
  }
}

template <int DT>
__device__ inline u32x4 pack_unit(const float (&acc)[8]) {
  if constexpr (DT == DT_F32) {
    return u32x4{__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]), __float_as_uint(acc[3])};
  } else {
    using T = typename dt_traits<DT>::T;
    union { u32x4 u; T e[8]; } c;
#pragma unroll
    for (int i = 0; i < 8; ++i) c.e[i] = (T)acc[i];
    return c.u;
  }
}

// input: N blocks of `shard` bytes (rank-major); output: Σ_p block `rank` of rank p
template <int DT>
__global__ __launch_bounds__(256) void reduce_scatter_kernel(Args a) {
  const int w = blockIdx.x;
  uint32_t* arrive = a.sig[a.rank];
  uint32_t* done = a.sig[a.rank] + MAXR * MAXG;
  int64_t v0, v1;
  range_of(a, w, v0, v1);
  bool busy = false;  // slot still being read by a peer: no stage / publish (see all_gather_kernel)
  if (a.epoch > 2)
    for (int p = 0; p < a.n; ++p)
      if (p != a.rank) busy |= wait_ge(done + p * MAXG + w, (uint32_t)(a.epoch - 2), a);
  if (busy) {
    poison_units(a.out, v0, v1);
    return;
  }
  // stage range w of every block (peer p reads block p)
  for (int p = 0; p < a.n; ++p)
    if (p != a.rank) copy_units(a.stage[a.rank] + p * a.shard, a.src + p * a.shard, v0, v1);
  release_all();
  if (threadIdx.x < a.n && threadIdx.x != a.rank)
    st_flag(a.sig[threadIdx.x] + a.rank * MAXG + w, (uint32_t)a.epoch);
  bool lost = false;
  for (int q = 0; q < a.n - 1; ++q) lost |= wait_ge(arrive + peer_at(a, w, q) * MAXG + w, (uint32_t)a.epoch, a);
  // fixed summation order 0..N-1 on every rank (deterministic, fp32)
  const u32x4_ua* own = reinterpret_cast<const u32x4_ua*>(a.src + a.rank * a.shard);
  u32x4_ua* o = reinterpret_cast<u32x4_ua*>(a.out);
  if (lost) {  // a peer's partial is missing: the whole range is invalid
    poison_units(a.out, v0, v1);
    v1 = v0;
  }
  for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < a.n; ++p) {
      const u32x4 x = p == a.rank ? own[v] : reinterpret_cast<const u32x4*>(a.stage[p] + a.rank * a.shard)[v];
      acc_unit<DT>(acc, x);
    }
    o[v] = pack_unit<DT>(acc);
  }
  release_all();
  if (threadIdx.x < a.n && threadIdx.x != a.rank)
    st_flag(a.sig[threadIdx.x] + MAXR * MAXG + a.rank * MAXG + w, (uint32_t)a.epoch);
}

}  // namespace ipc
}  // namespace xdot

using xdot::ipc::Args;

extern "C" {

int xdot_ipc_sig_bytes() { return xdot::ipc::SIG_WORDS * 4; }
int xdot_ipc_max_ranks() { return xdot::ipc::MAXR; }
int xdot_ipc_max_wgs() { return xdot::ipc::MAXG; }

// device buffer for IPC export; uncached: flag pages (every access is system-coherent)
int xdot_ipc_alloc(int64_t bytes, int uncached, void** p) {
  hipError_t e = uncached ? hipExtMallocWithFlags(p, (size_t)bytes, hipDeviceMallocUncached) : hipMalloc(p, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*p, 0, (size_t)bytes);
}
int xdot_ipc_free(void* p) { return (int)hipFree(p); }
int xdot_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }
int xdot_ipc_get_handle(void* p, void* out) {
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e == hipSuccess) std::memcpy(out, &h, sizeof(h));
  return (int)e;
}
int xdot_ipc_open(const void* handle, void** p) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess);
}
int xdot_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }
// pinned host word mapped into the device (the kernels' error flag; read by the host without a sync)
int xdot_ipc_host_word(void** host, void** dev) {
  hipError_t e = hipHostMalloc(host, 64, hipHostMallocMapped);
  if (e != hipSuccess) return (int)e;
  std::memset(*host, 0, 64);
  return (int)hipHostGetDevicePointer(dev, *host, 0);
}
int xdot_ipc_wall_clock_khz() {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return -1;
  return khz;
}

int xdot_ipc_all_gather_launch(const Args* a, hipStream_t st) {
  if (a->n < 2 || a->n > xdot::ipc::MAXR || a->nwg < 1 || a->nwg > xdot::ipc::MAXG || a->shard % 16) return -1;
  hipLaunchKernelGGL(xdot::ipc::all_gather_kernel, dim3(a->nwg), dim3(256), 0, st, *a);
  return 0;
}

int xdot_ipc_reduce_scatter_launch(const Args* a, hipStream_t st) {
  using namespace xdot;
  if (a->n < 2 || a->n > ipc::MAXR || a->nwg < 1 || a->nwg > ipc::MAXG || a->shard % 16) return -1;
  switch (a->dt) {
    case DT_F32: hipLaunchKernelGGL(ipc::reduce_scatter_kernel<DT_F32>, dim3(a->nwg), dim3(256), 0, st, *a); return 0;
    case DT_BF16: hipLaunchKernelGGL(ipc::reduce_scatter_kernel<DT_BF16>, dim3(a->nwg), dim3(256), 0, st, *a); return 0;
    case DT_F16: hipLaunchKernelGGL(ipc::reduce_scatter_kernel<DT_F16>, dim3(a->nwg), dim3(256), 0, st, *a); return 0;
    default: return -1;
  }
}

}  // extern "C"
