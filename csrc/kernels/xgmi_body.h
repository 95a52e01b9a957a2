// Device side of the direct xGMI all-reduce (see allreduce.hip for the algorithm): the
// body runs as the standalone bucket kernel (xgmi_allreduce_kernel) or as an in-launch role
// of the SimpleCNN conv backward (conv3x3.hip XAR), parameterised by its block index / count.
//
// Store policy of every buffer a PEER reads.  The barrier below has no
// release / acquire fence, so each peer-read byte must be stored write-through at system
// scope (sc0 sc1: the line goes to HBM, not only to the writer XCD's L2), drained by its
// wave (s_waitcnt vmcnt(0)) before the block's flag store, and read with system-scope loads
// (sc0 sc1: no L1 / L2 hit on a stale line).
//
//   buffer            written by (cache policy)                                   read by peers
//   ----------------  -----------------------------------------------------------  ---------------
//   data[r] bucket    engine producers with sys_store = 1: the fc role / fc_bwd dW    RS ld4_sys,
//     (gradients)     (st_sys), the fused slab reducer / grad_reduce dst (st_sys),    one-shot: not
//                     the fc bias (st_sys); module path: plain autograd stores, then   read (the
//                     the publish pass re-stores them st4_sys (a.publish)              stage is)
//   stage[r]          RS output / one-shot publish: st4_sys                         AG / one-shot
//                                                                                   sum: ld4_sys
//   sig[r]            flags: relaxed system-scope atomic stores into uncached        relaxed system
//                     memory (hipDeviceMallocUncached)                              atomic loads
//
// The AG's reduced values land in data[rank] with PLAIN stores: peers read that range again
// only in the next call's RS, after the next step's producers rewrote it write-through, and
// at least one kernel boundary (which writes back this XCD's dirty L2 lines) lies between.
// The one-shot publish reads the local bucket with system-scope loads (its producers may run
// in the same launch on another XCD: dist_mode 2).  tests/test_hygiene_cpu.py checks the ISA
// of the hot kernels for cache write-back / invalidate instructions; the start-up chain check
// (engine/fused_step.py verify_chain) compares the reduced gradient with an oracle summed
// outside this code.
#pragma once

#include "kernels/common.h"
#include "kernels/launchers.h"
#include "kernels/shadow.h"

namespace ddp_amd {

// loads in flight per thread in the reduce-scatter / all-gather loops (XgmiArgs items)
constexpr int XGMI_BATCH = 8;

// DDP_AMD_XGMI_FENCED=1 (a build switch): put a system-scope release fence before
// each barrier flag store and an acquire fence after the wait - the conservative protocol,
// for a node where the write-through + drain argument above is in doubt.  Off by default:
// on gfx950 each fence is a whole-L2 write-back / invalidate (profiles/r5_dist: ~4 us per
// multi-GPU step), and the hot kernels' ISA is checked to contain neither.
#ifndef DDP_AMD_XGMI_FENCED
#define DDP_AMD_XGMI_FENCED 0
#endif

// Signal all peers (lane p of wave 0 -> peer p) and wait until every peer's block b
// has signalled `target` to us.  Caller guarantees every wave drained its stores.
// On a timeout the FIRST stalled wait is recorded in the error word (xgmi_error_code:
// block, peer, barrier); the word stays non-zero (sticky) for every later call.
__device__ __forceinline__ void xgmi_barrier(const XgmiArgs& a, unsigned target, unsigned* s_fail, int phase, int blk) {
  __syncthreads();
  const int t = threadIdx.x;
  if (t < a.world && !*s_fail) {
    unsigned* dst = a.sig[t] + XGMI_FLAG_OFF + blk * XGMI_MAX_RANKS + a.rank;
    // No fences: everything a peer reads (gradient buckets, stage buffers) is written with
    // system-scope write-through stores that every wave drained (s_waitcnt vmcnt(0)) before
    // this flag store, and read with system-scope loads that bypass the caches - so a
    // release (write-back of the whole L2) and an acquire (invalidation of L1 / L2, after
    // which this block's own parameter loads missed) only cost time.  Producers with plain
    // stores go through the publish pass (a.publish), which re-stores write-through.
    if constexpr (DDP_AMD_XGMI_FENCED) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(dst, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* src = a.sig[a.rank] + XGMI_FLAG_OFF + blk * XGMI_MAX_RANKS + t;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
        unsigned expected = 0u;
        __hip_atomic_compare_exchange_strong(a.sig[a.rank] + XGMI_ERR_OFF, &expected,
                                             xgmi_error_code(blk, t, phase), __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        *s_fail = 1u;
        break;
      }
    }
    if constexpr (DDP_AMD_XGMI_FENCED) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
}

// Data movement is in 16-byte quads (4 floats): thread t of block b handles quad
// q = b * XGMI_THREADS + t, then q + G, q + 2G, ... (G = grid x XGMI_THREADS quads), two
// quads at a time, with all N ranks' loads of both in flight at once - 32 B x N per lane,
// so a small grid (XGMI_GRID_CAP blocks, leaving most CUs to the concurrent backward)
// still keeps megabytes in flight over the 7 links.  Peer memory is read with
// system-scope (sc0 sc1) buffer loads, stage buffers written with system-scope stores.
// Two-shot slices are whole quads (XgmiComm rounds the slice up to a multiple of 4), so
// every rank's slice starts on a quad; the bucket's last quad may be partial and takes
// the per-element path.
constexpr int SYS_CPOL = 1 | 16;  // sc0 | sc1: system scope
typedef __attribute__((ext_vector_type(4))) int ar_i32x4;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t sys_rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float4 ld4_sys(__amdgpu_buffer_rsrc_t r, long q) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(q * 16), 0, SYS_CPOL));
}
__device__ __forceinline__ void st4_sys(__amdgpu_buffer_rsrc_t r, long q, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ar_i32x4, v), r, (int)(q * 16), 0, SYS_CPOL);
}
__device__ __forceinline__ float4 add4(float4 x, float4 y) {
  return make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
}

// fixed rank-order (0..N-1) sum of quad q of every rank's source
__device__ __forceinline__ float4 rank_sum4(const __amdgpu_buffer_rsrc_t* src, long q, int N) {
  float4 v[XGMI_MAX_RANKS];
#pragma unroll
  for (int p = 0; p < XGMI_MAX_RANKS; ++p) v[p] = p < N ? ld4_sys(src[p], q) : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 sum = v[0];
#pragma unroll
  for (int p = 1; p < XGMI_MAX_RANKS; ++p)
    if (p < N) sum = add4(sum, v[p]);
  return sum;
}
// the same for the elements [4q, lim) of a partial last quad (element loads)
__device__ __forceinline__ float4 rank_sum_tail(float* const* src, long q, long lim, int N) {
  float e[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long k = 4 * q + j;
    float sum = 0.f;
    if (k < lim) {
      sum = ld_sys(src[0] + k);
#pragma unroll
      for (int p = 1; p < XGMI_MAX_RANKS; ++p)
        if (p < N) sum += ld_sys(src[p] + k);
    }
    e[j] = sum;
  }
  return make_float4(e[0], e[1], e[2], e[3]);
}

// the fused optimizer on flat bucket element k with reduced gradient g: same update on
// every rank, so parameters stay bitwise identical
// WT (the dist_mode 4 launch): parameters and shadows stored write-through - the next step's
// forward blocks of the same launch read them with sc1 loads (conv3x3.hip step_head_kernel)
template <bool WT = false>
__device__ __forceinline__ void sgd_elem(const XgmiArgs& a, long k, float g) {
  const long j = a.off + k;
  float m = a.mbuf ? a.mbuf[j] : 0.f;
  const float pn = sgd_one(a.params[j], g, &m, a.sgd);
  put_f<WT>(a.params + j, pn);
  if (a.mbuf) a.mbuf[j] = m;
  shadow_one<WT>(a.sh, j, pn);
}
// quad q (elements 4q.., below lim) of the reduced bucket times scale -> my gradient
// buffer and, with the fused optimizer (a.sgd.update), the parameters / momentum / shadows.
// Whole quads of a 4-aligned bucket are 16-byte accesses (sgd_quad / shadow_quad: the
// same writers as sgd_kernel); a partial last quad goes element by element.
__device__ __forceinline__ float4 scale4(const XgmiArgs& a, float4 v) {
  return make_float4(v.x * a.scale, v.y * a.scale, v.z * a.scale, v.w * a.scale);
}
template <bool WT = false>
__device__ __forceinline__ void finish_quad(const XgmiArgs& a, long q, float4 v, long lim) {
  if (4 * q + 3 < lim && (a.off & 3) == 0) {
    const long j = a.off + 4 * q;
    *reinterpret_cast<float4*>(a.data[a.rank] + j) = v;
    if (a.sgd.update) {
      const float4 pm = ld_quad(a.params, j);
      const float4 mm = a.sgd.momentum != 0.f ? ld_quad(a.mbuf, j) : make_float4(0.f, 0.f, 0.f, 0.f);
      sgd_quad_apply<WT>(a.params, a.mbuf, j, v, pm, mm, a.sgd, a.sh);
    }
    return;
  }
  float* d = a.data[a.rank] + a.off + 4 * q;
  const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (4 * q + j >= lim) continue;
    d[j] = e[j];
    if (a.sgd.update) sgd_elem<WT>(a, 4 * q + j, e[j]);
  }
}
template <bool WT = false>
__device__ __forceinline__ void finish4(const XgmiArgs& a, long q, float4 v, long lim) {
  finish_quad<WT>(a, q, scale4(a, v), lim);
}

// The all-reduce as block `blk` of `nblk` (the standalone kernel: blockIdx.x of gridDim.x;
// the in-launch role of the conv backward (conv3x3.hip XAR): its role-local block index).
// Every call of a channel must use the same nblk on every rank (the per-block sequence
// counters, barrier flags and quad mapping are per block index).  s_epoch / s_fail: two
// words of the block's LDS.  Returns with the block's stores drained.
// skid: the phase-stamp kernel id (scripts/stamps.py; the dist_mode 4 step head stamps apart)
template <bool WT = false>
__device__ __forceinline__ void xgmi_allreduce_body(const XgmiArgs& a, int blk, int nblk, unsigned* s_sh,
                                                    int skid = STAMP_K_XGMI) {
  unsigned& s_epoch = s_sh[0];
  unsigned& s_fail = s_sh[1];
  const int N = a.world, r = a.rank;
  unsigned* my = a.sig[r];
  // sticky failure: after any timeout every later call skips its barriers at once
  // (the host raises on the error word; a broken run must not cost timeouts per step)
  const bool failed_before = __hip_atomic_load(my + XGMI_ERR_OFF, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
  const long q0 = (long)blk * XGMI_THREADS + threadIdx.x;
  // one-shot: this thread's first quad of the local bucket, requested before the call
  // counter's round trip (only the stage store needs the counter's parity) - the two
  // latencies overlap instead of adding up on the conv bucket's path into the step head
  float4 first = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool first_ok = a.oneshot && q0 < a.n / 4;
  if (first_ok) {
    const float* mine = a.data[r] + a.off;
    first = make_float4(ld_sys(mine + 4 * q0), ld_sys(mine + 4 * q0 + 1), ld_sys(mine + 4 * q0 + 2),
                        ld_sys(mine + 4 * q0 + 3));
  }
  if (threadIdx.x == 0) {
    // per-block call counter (only this block of this rank touches it); every call of a
    // channel uses the same grid, so the counters of all blocks stay equal
    const unsigned e = my[XGMI_SEQ_OFF + blk] + 1u;
    my[XGMI_SEQ_OFF + blk] = e;
    s_epoch = e;
    s_fail = failed_before ? 1u : 0u;
  }
  __syncthreads();
  const unsigned e = s_epoch;
  const long G = (long)nblk * XGMI_THREADS;     // quads per grid stride

  if (a.oneshot) {
    // ---- publish my whole bucket, one barrier, sum every rank's copy in rank order
    const long n = a.n, nq = (n + 3) / 4, fq = n / 4;  // quads, full quads
    const long par1 = (long)(e & 1u) * ((nq * 4 + 3) & ~3L);
    const float* mine = a.data[r] + a.off;
    const __amdgpu_buffer_rsrc_t mystage = sys_rsrc(a.stage[r] + par1);
    // `mine` with system-scope loads: in the in-launch placement (dist_mode 2) the
    // gradient was written in this same launch by blocks on other XCDs, and this XCD's L2 may
    // still hold the previous step's lines - a plain load could read them
    for (long q = q0; q < nq; q += G) {
      float4 v;
      const float ps = a.prescale;
      if (q == q0 && first_ok) {
        v = make_float4(first.x * ps, first.y * ps, first.z * ps, first.w * ps);
      } else if (q < fq) {
        v = make_float4(ld_sys(mine + 4 * q) * ps, ld_sys(mine + 4 * q + 1) * ps, ld_sys(mine + 4 * q + 2) * ps,
                        ld_sys(mine + 4 * q + 3) * ps);
      } else {
        float t[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) t[j] = 4 * q + j < n ? ld_sys(mine + 4 * q + j) * ps : 0.f;
        v = make_float4(t[0], t[1], t[2], t[3]);
      }
      st4_sys(mystage, q, v);  // the stage holds whole quads (zero-padded tail)
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    DDP_STAMP(skid, 1);
    xgmi_barrier(a, 2u * e, &s_fail, XGMI_PHASE_ONESHOT, blk);
    DDP_STAMP(skid, 2);
    if (!s_fail) {
      __amdgpu_buffer_rsrc_t src[XGMI_MAX_RANKS];
#pragma unroll
      for (int p = 0; p < XGMI_MAX_RANKS; ++p) src[p] = sys_rsrc(p < N ? a.stage[p] + par1 : a.stage[r]);
      long q = q0;
      for (; q + G < nq; q += 2 * G) {
        const float4 s0 = rank_sum4(src, q, N), s1 = rank_sum4(src, q + G, N);
        finish4<WT>(a, q, s0, n);
        finish4<WT>(a, q + G, s1, n);
      }
      if (q < nq) finish4<WT>(a, q, rank_sum4(src, q, N), n);
    }
    if (a.step_ctr && blk == 0 && threadIdx.x == 0) a.step_ctr[0] += 1;
    return;
  }
  const long slice = a.slice;  // elements per rank slice, a multiple of 4 (the last rank's may be shorter)
  const long sq = slice / 4;
  const long par = (long)(e & 1u) * slice;
  if (a.publish) {
    // the peers' block b reads quad q of every slice of my bucket for exactly this
    // block's q: make those elements system-visible (write-through) before arriving.
    // Slice-relative quads, the same thread <-> quad map as RS / AG below: the AG's
    // reduced value must land after (program order) this re-store of the local value.
    float* mine = a.data[r] + a.off;
    const __amdgpu_buffer_rsrc_t rm = sys_rsrc(mine);
    const float ps = a.prescale;  // (x * 1.f == x: the plain re-store when not prescaling)
    for (int p = 0; p < N; ++p) {
      const long lim = min(slice, a.n - (long)p * slice);
      for (long q = q0; 4 * q < lim; q += G) {
        const long k = (long)p * slice + 4 * q;
        if (4 * q + 3 < lim) {
          st4_sys(rm, k / 4, make_float4(mine[k] * ps, mine[k + 1] * ps, mine[k + 2] * ps, mine[k + 3] * ps));
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (4 * q + j < lim) st_sys(mine + k + j, mine[k + j] * ps);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  DDP_STAMP(skid, 1);
  xgmi_barrier(a, 2u * e, &s_fail, XGMI_PHASE_B0, blk);  // B0
  DDP_STAMP(skid, 2);
  if (!s_fail) {
    // ---- RS: quads of my slice, fixed-order sum over ranks 0..N-1
    float* srcp[XGMI_MAX_RANKS];
    __amdgpu_buffer_rsrc_t src[XGMI_MAX_RANKS];
#pragma unroll
    for (int p = 0; p < XGMI_MAX_RANKS; ++p) {
      srcp[p] = (p < N ? a.data[p] : a.data[r]) + a.off + (long)r * slice;
      src[p] = sys_rsrc(srcp[p]);
    }
    const long lim = min(slice, a.n - (long)r * slice);  // my slice's real length (may be <= 0)
    const long fq = lim > 0 ? lim / 4 : 0, nq = lim > 0 ? (lim + 3) / 4 : 0;
    const __amdgpu_buffer_rsrc_t mystage = sys_rsrc(a.stage[r] + par);
    // the thread's full quads q0, q0 + G, ... below fq as (quad j, rank p) items in order,
    // XGMI_BATCH loads in flight per batch whatever N is (N = 1 would otherwise wait on one
    // load per quad); each quad's sum runs p = 0..N-1 exactly as rank_sum4 (same bits)
    const long J = fq > q0 ? (fq - q0 + G - 1) / G : 0;
    const long items = J * N;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (long i0 = 0; i0 < items; i0 += XGMI_BATCH) {
      float4 v[XGMI_BATCH];
      long jj = i0 / N;
      int pp = (int)(i0 - jj * N);
#pragma unroll
      for (int u = 0; u < XGMI_BATCH; ++u) {
        v[u] = i0 + u < items ? ld4_sys(sys_rsrc(a.data[pp] + a.off + (long)r * slice), q0 + jj * G)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
        if (++pp == N) { pp = 0; ++jj; }
      }
      jj = i0 / N;
      pp = (int)(i0 - jj * N);
#pragma unroll
      for (int u = 0; u < XGMI_BATCH; ++u) {
        if (i0 + u < items) {
          acc = pp == 0 ? v[u] : add4(acc, v[u]);
          if (pp == N - 1) st4_sys(mystage, q0 + jj * G, acc);
        }
        if (++pp == N) { pp = 0; ++jj; }
      }
    }
    // the partial last quad of the bucket (element loads)
    for (long q = q0 + J * G; q < nq; q += G) st4_sys(mystage, q, rank_sum_tail(srcp, q, lim, N));
    (void)src;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  DDP_STAMP(skid, 3);
  // ---- AG: quad q of every rank's reduced slice into my gradient buffer
  // the thread's quads q0, q0 + G, ... of every rank's reduced slice as (quad j, rank p)
  // items in order, XGMI_BATCH per batch: every load of a batch (reduced quads over xGMI,
  // and with the fused optimizer the local parameter / momentum quads) is issued before
  // the first store, whatever N is.  The first batch's parameter / momentum loads (local,
  // independent of the reduction) go out before B1, their latency under the barrier's.
  const bool vec = (a.off & 3) == 0;
  const bool mom = a.sgd.momentum != 0.f;
  const long Jg = sq > q0 ? (sq - q0 + G - 1) / G : 0;
  const long items_g = Jg * N;
  float4 pv[XGMI_BATCH], mv[XGMI_BATCH];
  auto load_pm = [&](long i0) {
    long jj = i0 / N;
    int pp = (int)(i0 - jj * N);
#pragma unroll
    for (int u = 0; u < XGMI_BATCH; ++u) {
      const long qq = (long)pp * sq + q0 + jj * G;
      const bool whole = i0 + u < items_g && vec && 4 * qq + 3 < a.n && a.sgd.update;
      pv[u] = whole ? ld_quad(a.params, a.off + 4 * qq) : make_float4(0.f, 0.f, 0.f, 0.f);
      mv[u] = whole && mom ? ld_quad(a.mbuf, a.off + 4 * qq) : make_float4(0.f, 0.f, 0.f, 0.f);
      if (++pp == N) { pp = 0; ++jj; }
    }
  };
  load_pm(0);
  xgmi_barrier(a, 2u * e + 1u, &s_fail, XGMI_PHASE_B1, blk);  // B1
  DDP_STAMP(skid, 4);
  if (!s_fail) {
    const long items = items_g;
    for (long i0 = 0; i0 < items; i0 += XGMI_BATCH) {
      float4 v[XGMI_BATCH];
      if (i0 > 0) load_pm(i0);
      long jj = i0 / N;
      int pp = (int)(i0 - jj * N);
#pragma unroll
      for (int u = 0; u < XGMI_BATCH; ++u) {
        const long q = q0 + jj * G, qq = (long)pp * sq + q;
        const bool ok = i0 + u < items && 4 * qq < a.n;
        v[u] = ok ? ld4_sys(sys_rsrc(a.stage[pp] + par), q) : make_float4(0.f, 0.f, 0.f, 0.f);
        if (++pp == N) { pp = 0; ++jj; }
      }
      // finish one item per trip (the finishing code once, not XGMI_BATCH times: unrolled it
      // made the kernel too large to unroll); the trip's registers are picked from the arrays
      // by a select chain on the (uniform) slot index - constant array indices only
      jj = i0 / N;
      pp = (int)(i0 - jj * N);
      // one wait for the whole batch: inside the rolled loop the compiler waits for every
      // outstanding memory operation (the previous items' stores included) before each item
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#pragma unroll 1
      for (int u = 0; u < XGMI_BATCH; ++u) {
        const long q = q0 + jj * G, qq = (long)pp * sq + q;
        if (++pp == N) { pp = 0; ++jj; }
        if (i0 + u >= items) break;
        if (4 * qq >= a.n) continue;
        float4 vv = v[0], pq = pv[0], mq = mv[0];
#pragma unroll
        for (int w = 1; w < XGMI_BATCH; ++w)
          if (u == w) { vv = v[w]; pq = pv[w]; mq = mv[w]; }
        const float4 d = scale4(a, vv);
        if (vec && 4 * qq + 3 < a.n) {
          const long j = a.off + 4 * qq;
          *reinterpret_cast<float4*>(a.data[r] + j) = d;
          if (a.sgd.update) sgd_quad_apply<WT>(a.params, a.mbuf, j, d, pq, mq, a.sgd, a.sh);
        } else {
          finish_quad<WT>(a, qq, d, a.n);
        }
      }
    }
  }
  if (a.step_ctr && blk == 0 && threadIdx.x == 0) a.step_ctr[0] += 1;
}

}  // namespace ddp_amd
