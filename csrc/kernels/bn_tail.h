// BatchNorm statistics finalised inside the kernel that produces them (ResNet-18,
// BASELINE.json config 5): the stats-producing launches (conv_gemm_fwd, the halo forward,
// splitk_reduce) write their per-block [2][C] partial rows write-through and then run
// bn_stats_tail, a two-level last-arrival reduction:
//   level 1: the blocks of a column block (its channels) are grouped 32 rows at a time;
//            the last block of a group to arrive sums the group's rows in row order into
//            ws[group] (or, with one group, finalises directly);
//   level 2: the last group sums ws[0 .. groups) in group order and finalises: mean,
//            invstd, the running buffers with torch's semantics (momentum, unbiased
//            running variance) and num_batches_tracked.
// Fixed summation order (no float atomics: bitwise reproducible); the ticket words reset
// themselves, so a captured graph replays them.  This removes the separate bn_finalize
// launch per BatchNorm (20 per ResNet-18 step).
#pragma once
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

constexpr int BN_TAIL_GROUP = 32;  // stats rows per level-1 group

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

// Fixed-order sum of rows [r0, r1) of a [rows][2][C] slab for channels [c0, c0 + nc) of
// this block (256 threads): thread = (channel, row phase); phases sum rows r0 + ph,
// r0 + ph + NPH, ... and are combined in phase order.  Result for (which, c) in
// red[which][c - c0] (LDS, caller-provided, >= 2 * nc floats), valid after the barrier.
__device__ __forceinline__ void bn_tail_sum(const float* slab, long C, int r0, int r1, int c0, int nc,
                                            float* red, float* scratch /* [256][2] */) {
  const int tid = threadIdx.x;
  const int nph = nc >= 256 ? 1 : 256 / nc;  // nc in {64, 128, 256, 512}
  for (int cb = 0; cb < nc; cb += 256) {
    const int cl = cb + (nc >= 256 ? tid : tid % nc);
    const int ph = nc >= 256 ? 0 : tid / nc;
    float s = 0.f, q = 0.f;
    if (cl < nc) {
      // every load of a 16-row batch in flight before the in-order sum (these agent-scope
      // loads miss the XCD's L2: one memory round trip per batch, not per row)
      const float* p = slab + (long)c0 + cl;
      for (int rb = r0 + ph; rb < r1; rb += 16 * nph) {
        float a[16], b[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int r = rb + u * nph;
          a[u] = r < r1 ? ld_agent(p + (long)r * 2 * C) : 0.f;
          b[u] = r < r1 ? ld_agent(p + (long)r * 2 * C + C) : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          if (rb + u * nph < r1) { s += a[u]; q += b[u]; }
        }
      }
    }
    scratch[2 * tid] = s;
    scratch[2 * tid + 1] = q;
    __syncthreads();
    if (nph == 1) {
      if (cl < nc) { red[cl] = s; red[nc + cl] = q; }
    } else if (tid < nc) {
      float S = scratch[2 * tid], Q = scratch[2 * tid + 1];
      for (int k = 1; k < nph; ++k) {
        S += scratch[2 * (tid + k * nc)];
        Q += scratch[2 * (tid + k * nc) + 1];
      }
      red[tid] = S;
      red[nc + tid] = Q;
    }
    __syncthreads();
  }
}

// Called by every thread of a stats-producing block after its partial row `row`
// (channels [c0, c0 + nc) of column block `colblk`) was stored with st_wt.  `lds`: dead
// LDS of the caller (its staging tiles), >= 2 * nc + 512 floats.
__device__ __forceinline__ void bn_stats_tail(const BnFin& f, const float* stats, int row, int colblk, int c0,
                                           int nc, float* lds) {
  __shared__ int s_last;
  float* red = lds;
  float* scratch = lds + 2 * nc;
  const int ng = (f.rows + BN_TAIL_GROUP - 1) / BN_TAIL_GROUP;
  const int grp = row / BN_TAIL_GROUP;
  const int gr0 = grp * BN_TAIL_GROUP, gr1 = min(f.rows, gr0 + BN_TAIL_GROUP);
  int* tk = f.tickets + (long)colblk * (ng + 1);
  const long C = f.C;
  if (!last_arrival(tk + grp, gr1 - gr0, &s_last)) return;
  bn_tail_sum(stats, C, gr0, gr1, c0, nc, red, scratch);
  if (ng > 1) {
    for (int v = threadIdx.x; v < 2 * nc; v += 256) {
      const int which = v / nc, cl = v - which * nc;
      st_wt(f.ws + (long)grp * 2 * C + which * C + c0 + cl, red[v]);
    }
    if (!last_arrival(tk + ng, ng, &s_last)) return;
    bn_tail_sum(f.ws, C, 0, ng, c0, nc, red, scratch);
  }
  for (int cl = threadIdx.x; cl < nc; cl += 256) {
    const int c = c0 + cl;
    const float S = red[cl], Q = red[nc + cl];
    const float mean = S / f.count;
    const float var = fmaxf(Q / f.count - mean * mean, 0.f);
    f.save_mean[c] = mean;
    f.save_invstd[c] = rsqrtf(var + f.eps);
    if (f.running_mean) {
      const float unb = f.count > 1.f ? var * f.count / (f.count - 1.f) : var;
      f.running_mean[c] = (1.f - f.momentum) * f.running_mean[c] + f.momentum * mean;
      f.running_var[c] = (1.f - f.momentum) * f.running_var[c] + f.momentum * unb;
    }
  }
  if (f.nbt && colblk == 0 && threadIdx.x == 0) f.nbt[0] += 1;
}

}  // namespace ddp_amd
