// Last-arrival reductions (the BatchNorm statistics finalisation, resnet_ops.hip
// bn_finalize, and the BatchNorm backward's strip sums): every block of a strip stores its
// partial write-through, drains, and takes a ticket; the block that takes the last ticket
// sums the partials in FIXED order (bitwise reproducible) and re-arms the ticket, so a
// captured graph replays them.  (Round 3 also ran the statistics finalisation inside the
// stats-producing conv launch; measured slower - profiles/r3_bn_fusion - and removed in
// round 5.)
#pragma once
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A strip of blocks reduces into per-block partials; the block that takes the strip's
// last ticket sums the partials in FIXED order and resets the ticket for the next launch.
// Cross-XCD visibility without fences: an agent-scope release fence writes back the
// XCD's whole L2 (measured: ~30 us per reduction at 400 blocks), so the partials are
// stored write-through (st_wt) and drained (vmcnt(0)) before the relaxed ticket
// increment, and the last block reads them with agent-scope atomic loads.
__device__ __forceinline__ bool last_arrival(int* ticket, int expected, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's st_wt partials are out
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == expected - 1;
    if (last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_flag = last;
  }
  __syncthreads();
  return *s_flag != 0;
}

}  // namespace ddp_amd
