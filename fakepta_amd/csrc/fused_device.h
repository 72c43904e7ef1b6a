// Device helpers shared by the persistent fused kernels (grid_fused.hip: k_grid_fused; grid_fused_w.hip:
// k_grid_fused_w): per-XCD item queues, the role barrier, the LDS-only wait, a lane-pair DPP exchange, and the
// FPTA_FUSED_PROF phase counters. Header-only.
#pragma once
#include <hip/hip_runtime.h>

#include "grid_device.h"

namespace fpta {
// -DFPTA_FUSED_PROF (make variant; tools/fused_prof.py): per-wave cycle counters of the kernel's phases
#ifdef FPTA_FUSED_PROF
struct Prof {
  unsigned long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t = 0;
  __device__ __forceinline__ void start() { t = clock64(); }
  __device__ __forceinline__ void lap(int i) {
    const unsigned long long n = clock64();
    v[i] += n - t;
    t = n;
  }
  __device__ __forceinline__ void count(int i) { ++v[i]; }
  __device__ __forceinline__ void flush(unsigned long long* out, int wave) {
    if (out && (threadIdx.x & 63) == 0)
      for (int i = 0; i < 8; ++i) out[((int64_t)blockIdx.x * 8 + wave) * 8 + i] = v[i];
  }
};
#else
struct Prof {
  __device__ __forceinline__ void start() {}
  __device__ __forceinline__ void lap(int) {}
  __device__ __forceinline__ void count(int) {}
  __device__ __forceinline__ void flush(unsigned long long*, int) {}
};
#endif

// a double from lane l ^ 1 (DPP quad_perm [1, 0, 3, 2] on both halves)
__device__ __forceinline__ double dpp_xor1(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ void fused_barrier() { asm volatile("s_barrier" ::: "memory"); }  // no vmcnt(0) fence
__device__ __forceinline__ void fused_wait_lgkm0() { __builtin_amdgcn_s_waitcnt(15 | (3 << 14) | (7 << 4)); }

// A workgroup's items come from its XCD's queue (workgroup b runs on XCD b % 8): the items of XCD x are a contiguous
// range (the items of one pulsar run side by side on one XCD, whose L2 then holds the pulsar's weights), handed out
// one at a time by a ticket counter, so a workgroup that starts late (a co-running kernel held its CU) takes fewer
// items instead of delaying the launch's end. Tickets are fetched two items ahead into an LDS ring of four; -1 = none.
struct FusedQueue {
  int first, end;
  uint32_t* ticket;
  __device__ __forceinline__ FusedQueue(int n_items, uint32_t* q) {
    const int per = (n_items + 7) >> 3;
    const int x = blockIdx.x & 7;
    first = x * per;
    end = min(n_items, first + per);
    ticket = q + x;
  }
  // one lane: the next item of this XCD or -1 (a vector atomic: the lane's own address)
  __device__ __forceinline__ int fetch() const {
    const int t = (int)__hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return first + t < end ? first + t : -1;
  }
};

}  // namespace fpta
