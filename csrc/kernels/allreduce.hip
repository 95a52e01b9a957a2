// Direct (all-to-all) two-shot SUM all-reduce over xGMI for the DDP gradient buckets.
//
// Why not only RCCL: an 8x MI355X node is a full mesh of point-to-point xGMI links
// (7 per GPU).  A ring all-reduce moves 2(N-1)/N of the bucket over ONE link per step;
// the direct algorithm below moves each byte over its own link, all 7 links at once,
// in two hops, and runs as ONE kernel inside the step's hipGraph (no proxy thread, no
// protocol selection).  SimpleCNN's buckets are 2.0 MB and 75 KB (SURVEY.md §2.6
// I6/I7), i.e. latency-bound: two cross-GPU barriers + 2 x (bucket / N) per link.
//
//   B0  entry barrier: every rank's gradient bucket is final
//   RS  rank r pulls its slice r from all peers (system-scope loads over xGMI), sums in
//       FIXED rank order 0..N-1 (bitwise identical on every rank), writes the reduced
//       slice to its stage buffer (parity = call number & 1)
//   B1  every rank finished RS (so nobody reads any rank's gradient buffer any more)
//   AG  rank r pulls every peer's reduced slice from its stage buffer into its own
//       gradient buffer (local stores)
//
// Pull-only: no GPU ever writes another GPU's memory, so each GPU's own L2 stays
// coherent for its own buffers.  Everything a peer reads is produced with system-scope
// (write-through) stores and read with system-scope loads, and every storing wave
// drains its stores (s_waitcnt vmcnt(0)) before the block's flag store.  The stage
// buffer is double-buffered by call parity, which removes the exit barrier: call k+2
// reuses call k's stage only after every rank passed call k+1's B0.
//
// One-shot variant (XgmiArgs::oneshot, small buckets): every rank publishes its whole
// bucket to its stage buffer (parity-double-buffered), ONE barrier, then every rank pulls
// all N published buckets and sums them in fixed rank order - each rank computes the
// full result itself (bitwise identical everywhere), trading N x the bytes for one fewer
// cross-GPU barrier, which wins when the bucket is a few tens of KB (SimpleCNN's
// 75 KB conv bucket).  Stage reuse: call k+2 rewrites parity k's stage only after every
// rank passed call k+1's barrier, i.e. finished reading call k.
//
// Barriers are per block: block b of every rank handles the same element range of every
// slice, and only ever waits for block b of its peers.  Flags are monotonic per-block counters in
// uncached memory; every spin is bounded (XgmiArgs::timeout_ticks of the 100 MHz clock):
// on timeout the block sets the error word and stops waiting, so a broken peer makes
// the result wrong (detected by the host) instead of hanging the GPU.
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {



// bf16 shadows of one updated parameter (flat index j), same layouts as sgd_kernel
__device__ __forceinline__ void shadow_one(const ShadowSet& sh, long j, float v) {
#pragma unroll
  for (int r = 0; r < MAX_SHADOWS; ++r) {
    if (r >= sh.count) break;
    const long k = j - sh.r[r].off;
    if (k < 0 || k >= sh.r[r].n) continue;
    const bf16_t b = f2bf(v);
    if (sh.r[r].kind == SHADOW_BF16) {
      sh.r[r].dst[k] = b;
    } else if (sh.r[r].kind == SHADOW_BF16_FCFRAG) {
      sh.r[r].dst[fcfrag_index((int)k, sh.r[r].a, sh.r[r].b)] = b;
    } else if (sh.r[r].kind == SHADOW_BF16_PAD4) {  // [..][3] -> [..][4], 4th stays zero
      sh.r[r].dst[(k / 3) * 4 + k % 3] = b;
    } else if (sh.r[r].kind == SHADOW_F32_TAPT) {  // exact fp32 [tap][ci][co] copy
      const long per = (long)sh.r[r].b * sh.r[r].c;
      const long co = k / per;
      sh.r[r].dst32[(k - co * per) * sh.r[r].a + co] = v;
    } else {  // SHADOW_BF16_TAPT: OHWI [co][tap][ci] -> [tap][ci][co]
      const long per = (long)sh.r[r].b * sh.r[r].c;
      const long co = k / per;
      sh.r[r].dst[(k - co * per) * sh.r[r].a + co] = b;
    }
  }
}

// Signal all peers (lane p of wave 0 -> peer p) and wait until every peer's block b
// has signalled `target` to us.  Caller guarantees every wave drained its stores.
// On a timeout the FIRST stalled wait is recorded in the error word (xgmi_error_code:
// block, peer, barrier); the word stays non-zero (sticky) for every later call.
__device__ __forceinline__ void xgmi_barrier(const XgmiArgs& a, unsigned target, unsigned* s_fail, int phase) {
  __syncthreads();
  const int t = threadIdx.x;
  if (t < a.world && !*s_fail) {
    unsigned* dst = a.sig[t] + XGMI_FLAG_OFF + blockIdx.x * XGMI_MAX_RANKS + a.rank;
    __hip_atomic_store(dst, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* src = a.sig[a.rank] + XGMI_FLAG_OFF + blockIdx.x * XGMI_MAX_RANKS + t;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
        unsigned expected = 0u;
        __hip_atomic_compare_exchange_strong(a.sig[a.rank] + XGMI_ERR_OFF, &expected,
                                             xgmi_error_code((int)blockIdx.x, t, phase), __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        *s_fail = 1u;
        break;
      }
    }
  }
  __syncthreads();
}

// Element i of the slice per thread and rank, blocks striding over 256-element chunks
// (chunk c, c + gridDim.x, ...: the grid is capped at XGMI_GRID_CAP blocks so the
// all-reduce, which overlaps the conv backward on its own stream, keeps few waves
// resident while it waits in its barriers).  All N loads of a chunk - two chunks at a
// time - are in flight at once, so each phase is about one xGMI round trip per two chunks.
__device__ __forceinline__ float rank_sum(const XgmiArgs& a, float* const* src, long k, int N) {
  float v[XGMI_MAX_RANKS];
#pragma unroll
  for (int p = 0; p < XGMI_MAX_RANKS; ++p) v[p] = p < N ? ld_sys(src[p] + k) : 0.f;
  float sum = v[0];
#pragma unroll
  for (int p = 1; p < XGMI_MAX_RANKS; ++p)
    if (p < N) sum += v[p];
  return sum;
}

// the reduced gradient g of flat bucket element k -> my gradient buffer (+ fused SGD)
__device__ __forceinline__ void finish(const XgmiArgs& a, long k, float g) {
  a.data[a.rank][a.off + k] = g;
  if (a.sgd.update) {  // fused optimizer: same update on every rank
    const long j = a.off + k;
    float m = a.mbuf ? a.mbuf[j] : 0.f;
    const float pn = sgd_one(a.params[j], g, &m, a.sgd);
    a.params[j] = pn;
    if (a.mbuf) a.mbuf[j] = m;
    shadow_one(a.sh, j, pn);
  }
}

__global__ __launch_bounds__(XGMI_THREADS) void xgmi_allreduce_kernel(XgmiArgs a) {
  __shared__ unsigned s_epoch, s_fail;
  const int N = a.world, r = a.rank;
  unsigned* my = a.sig[r];
  // sticky failure: after any timeout every later call skips its barriers at once
  // (the host raises on the error word; a broken run must not cost timeouts per step)
  const bool failed_before = __hip_atomic_load(my + XGMI_ERR_OFF, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
  if (threadIdx.x == 0) {
    // per-block call counter (only this block of this rank touches it); every call of a
    // channel uses the same grid, so the counters of all blocks stay equal
    const unsigned e = my[XGMI_SEQ_OFF + blockIdx.x] + 1u;
    my[XGMI_SEQ_OFF + blockIdx.x] = e;
    s_epoch = e;
    s_fail = failed_before ? 1u : 0u;
  }
  __syncthreads();
  const unsigned e = s_epoch;
  const long G = (long)gridDim.x * XGMI_THREADS;     // elements per grid stride
  const long i0 = (long)blockIdx.x * XGMI_THREADS + threadIdx.x;

  if (a.oneshot) {
    // ---- publish my whole bucket, one barrier, sum every rank's copy in rank order
    const long par1 = (long)(e & 1u) * a.n;
    for (long i = i0; i < a.n; i += G) st_sys(a.stage[r] + par1 + i, a.data[r][a.off + i]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    xgmi_barrier(a, 2u * e, &s_fail, XGMI_PHASE_ONESHOT);
    if (!s_fail) {
      float* src[XGMI_MAX_RANKS];
#pragma unroll
      for (int p = 0; p < XGMI_MAX_RANKS; ++p) src[p] = p < N ? a.stage[p] + par1 : nullptr;
      long i = i0;
      for (; i + G < a.n; i += 2 * G) {
        const float s0 = rank_sum(a, src, i, N), s1 = rank_sum(a, src, i + G, N);
        finish(a, i, s0 * a.scale);
        finish(a, i + G, s1 * a.scale);
      }
      if (i < a.n) finish(a, i, rank_sum(a, src, i, N) * a.scale);
    }
    if (a.step_ctr && blockIdx.x == 0 && threadIdx.x == 0) a.step_ctr[0] += 1;
    return;
  }
  const long slice = a.slice;  // elements per rank slice (the last rank's may be shorter)
  const long par = (long)(e & 1u) * slice;
  if (a.publish) {
    // the peers' block b reads element i of every slice of my bucket for exactly this
    // block's i: make those elements system-visible (write-through) before arriving
    float* mine = a.data[r] + a.off;
    for (int p = 0; p < N; ++p) {
      const long lim = min(slice, a.n - (long)p * slice);
      for (long i = i0; i < lim; i += G) st_sys(mine + (long)p * slice + i, mine[(long)p * slice + i]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  xgmi_barrier(a, 2u * e, &s_fail, XGMI_PHASE_B0);  // B0
  if (!s_fail) {
    // ---- RS: elements of my slice, fixed-order sum over ranks 0..N-1
    float* src[XGMI_MAX_RANKS];
#pragma unroll
    for (int p = 0; p < XGMI_MAX_RANKS; ++p) src[p] = p < N ? a.data[p] + a.off + (long)r * slice : nullptr;
    const long lim = min(slice, a.n - (long)r * slice);  // my slice's real length
    long i = i0;
    for (; i + G < lim; i += 2 * G) {
      const float s0 = rank_sum(a, src, i, N), s1 = rank_sum(a, src, i + G, N);
      st_sys(a.stage[r] + par + i, s0);
      st_sys(a.stage[r] + par + i + G, s1);
    }
    if (i < lim) st_sys(a.stage[r] + par + i, rank_sum(a, src, i, N));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  xgmi_barrier(a, 2u * e + 1u, &s_fail, XGMI_PHASE_B1);  // B1
  if (!s_fail) {
    // ---- AG: element i of every rank's reduced slice into my gradient buffer
    for (long i = i0; i < slice; i += G) {
      float v[XGMI_MAX_RANKS];
#pragma unroll
      for (int p = 0; p < XGMI_MAX_RANKS; ++p)
        v[p] = (p < N && (long)p * slice + i < a.n) ? ld_sys(a.stage[p] + par + i) : 0.f;
#pragma unroll
      for (int p = 0; p < XGMI_MAX_RANKS; ++p) {
        const long k = (long)p * slice + i;
        if (p < N && k < a.n) finish(a, k, v[p] * a.scale);
      }
    }
  }
  if (a.step_ctr && blockIdx.x == 0 && threadIdx.x == 0) a.step_ctr[0] += 1;
}

int xgmi_blocks(long n, int world, bool oneshot) {
  const long slice = oneshot ? n : (n + world - 1) / world;
  long b = (slice + XGMI_THREADS - 1) / XGMI_THREADS;
  if (b > XGMI_GRID_CAP) b = XGMI_GRID_CAP;
  return (int)(b < 1 ? 1 : b);
}

void xgmi_allreduce(const XgmiArgs& a, int blocks, hipStream_t s) {
  hipLaunchKernelGGL(xgmi_allreduce_kernel, dim3(blocks), dim3(XGMI_THREADS), 0, s, a);
}

}  // namespace ddp_amd
