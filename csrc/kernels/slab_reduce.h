// Fixed-order split-K slab reduction (+ fused SGD) of one 64-output chunk, shared by the
// standalone grad_reduce kernel (optim.hip, NT = 64 * GR threads) and the reducer role
// of the fused conv backward (conv3x3.hip, 256 threads, in-launch hand-off).
//
// Output space: the SlabSet's segments back to back, each padded to a multiple of 64
// outputs, so chunk q (64 outputs) never straddles two segments.  Order of the float
// operations, independent of NT: row group g (rows g, g + GR, ...) is summed in batches of
// 8 rows (sequential adds), then the tail rows; the GR group sums are then added in order
// 0, 1, ..., GR-1 - bitwise reproducible and identical between the two launch shapes.
#pragma once
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

// segment k and element i of output lane c of chunk q; false past the last segment.
// The segment is found from the chunk base alone (q is block-uniform), so k stays a
// scalar and the segment fields are scalar loads (a per-lane k would turn every field
// access into a vector load, ordered behind the slab loads in flight).
__device__ __forceinline__ bool slab_locate(const SlabSet& ss, long q, int c, int& k, long& i) {
  long ib = q * 64;
  for (k = 0; k < ss.count; ++k) {
    const long padded = (ss.s[k].n + 63) / 64 * 64;
    if (ib < padded) break;
    ib -= padded;
  }
  i = ib + c;
  return k < ss.count && i < ss.s[k].n;
}

// Fused-SGD operands of the chunk's outputs for threads of wave 0 (prefetch them before
// waiting for the slabs: they do not depend on this step's gradients).
// (mine: this thread owns output threadIdx.x & 63 of chunk q - wave 0 in slab_reduce_chunk)
__device__ __forceinline__ void slab_sgd_prefetch(const SlabSet& ss, long q, float& p0, float& m0,
                                                  bool mine = true) {
  p0 = m0 = 0.f;
  if (!ss.sgd.update || !mine) return;
  int k;
  long i;
  if (slab_locate(ss, q, threadIdx.x & 63, k, i) && ss.s[k].p) {
    p0 = ss.s[k].p[i];
    m0 = ss.s[k].m ? ss.s[k].m[i] : 0.f;
  }
}

template <bool SC1>
__device__ __forceinline__ float slab_ld(const float* p) {
  if constexpr (SC1) return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}

// part: GR * 64 floats of LDS.  Every thread of the block calls it (contains barriers).
// SC1: the slab rows are read with agent-scope loads (written write-through inside the
// same launch).  p0 / m0: slab_sgd_prefetch's values for this chunk.
template <int GR, int NT, bool SC1>
__device__ __forceinline__ void slab_reduce_chunk(const SlabSet& ss, long q, float* part, float p0, float m0) {
  constexpr int NW = NT / 64, GPW = GR / NW;
  static_assert(GR % NW == 0, "row groups must split evenly over the waves");
  const int c = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int k;
  long i;
  const bool live = slab_locate(ss, q, c, k, i);
  if (live) {
    const SlabSeg& sg = ss.s[k];
    const float* src = sg.slab + sg.src_off + i;
    const long st = sg.row_stride;
    // every group's first batch of 8 rows in flight at once, then the rest in order
    float a[GPW][8];
    int r[GPW];
#pragma unroll
    for (int j = 0; j < GPW; ++j) {
      r[j] = wave + NW * j;
      if (r[j] + 7 * GR < sg.rows)
#pragma unroll
        for (int u = 0; u < 8; ++u) a[j][u] = slab_ld<SC1>(src + (long)(r[j] + GR * u) * st);
    }
#pragma unroll
    for (int j = 0; j < GPW; ++j) {
      float acc = 0.f;
      if (r[j] + 7 * GR < sg.rows) {
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += a[j][u];
        r[j] += 8 * GR;
      }
      for (; r[j] + 7 * GR < sg.rows; r[j] += 8 * GR) {
        float b[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) b[u] = slab_ld<SC1>(src + (long)(r[j] + GR * u) * st);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += b[u];
      }
      for (; r[j] < sg.rows; r[j] += GR) acc += slab_ld<SC1>(src + (long)r[j] * st);
      part[(wave + NW * j) * 64 + c] = acc;
    }
  } else {
#pragma unroll
    for (int j = 0; j < GPW; ++j) part[(wave + NW * j) * 64 + c] = 0.f;
  }
  __syncthreads();
  if (wave == 0 && live) {
    const SlabSeg& sg = ss.s[k];  // k is block-uniform
    float g = part[c];
#pragma unroll
    for (int qq = 1; qq < GR; ++qq) g += part[qq * 64 + c];
    g *= sg.scale;
    if (sg.accum) g += sg.dst[i];
    if (ss.sys_store) st_sys(sg.dst + i, g);
    else sg.dst[i] = g;
    if (ss.sgd.update && sg.p) {  // single-process step: the gradient is final -> fused SGD
      float m = m0;
      const float pn = sgd_one(p0, g, &m, ss.sgd);
      sg.p[i] = pn;
      if (sg.m) sg.m[i] = m;
      if (sg.sh) sg.sh[i] = f2bf(pn);
      if (sg.sh_t || sg.sh_t32) {  // OHWI [co][tap][ci] -> [tap][ci][co]
        const long per = (long)sg.t_taps * sg.t_ci;
        const long co = i / per;
        if (sg.sh_t) sg.sh_t[(i - co * per) * sg.t_co + co] = f2bf(pn);
        if (sg.sh_t32) sg.sh_t32[(i - co * per) * sg.t_co + co] = pn;
      }
    }
  }
  __syncthreads();  // part is reused by the next chunk
}

// ---- the fused conv backward's reducer (256 threads, GR = 16): 4 consecutive outputs
// per thread, one 16-byte sc1 buffer load per row, and J chunks' first 8 rows per group
// in flight together.  Thread (wave w, lane l): column quad cq = l & 15, row group
// g = 4 w + (l >> 4).  Every group is summed by ONE thread in increasing row order
// (sequential adds, exactly as grad_reduce: its batching of 8 rows does not change the
// sequence of additions) and the 16 group sums are combined in order 0..15: bit-identical
// to slab_reduce_chunk<16, *>.  Branch-free loads (a load issued on only some paths makes
// the compiler wait for outstanding loads where the paths join): rows past the segment's
// end are clamped and not added (select); a quad that would cross the segment's end n
// loads the last 4 elements [n-4, n) and shifts (segments need n >= 4, checked by the
// host); lanes past n read element 0 and are never finalised.
// All index work (segment lookups: dependent scalar loads of the SlabSet kernel argument)
// happens in slab_fused_plan, BEFORE the reducer waits for the slabs; after the wait only
// address arithmetic and the loads remain.
template <int J>
struct SlabFusedPlan {
  const float* base[J];  // segment slab + src_off (block-uniform)
  long stride[J];
  int rows[J];
  long ic[J];  // this thread's clamped quad start
  int sh[J];   // shift of the quad that crosses the segment end
  // the output this thread finalises (chunk threadIdx >> 6, element threadIdx & 63)
  bool own_live;
  long own_i;
  float* dst;
  float *p, *m, *sh32;
  bf16_t *shb, *sht;
  float scale;
  int accum, t_co, t_taps, t_ci;
  float p0, m0;
};

__device__ __forceinline__ float4 slab_ld4_sc1(const float* base, long e) {
  // dword-aligned 16-byte sc1 buffer load of elements [e, e + 4) of a segment (byte
  // offsets fit 31 bits: the engine's slabs are < 2 GB)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
  typedef __attribute__((ext_vector_type(4))) int i32x4_t;
  const i32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(e * 4), 0, 16 /* sc1 */);
  return __builtin_bit_cast(float4, v);
}
// v holds elements [i - s, i - s + 4); return elements i.. (components past 3 - s unused).
// Bit-mask selects: a ternary chain on the components is turned into a dynamically
// indexed vector, which the backend lowers through scratch memory.
__device__ __forceinline__ float4 shift4(const float4& v, int s) {
  const unsigned m0 = s == 0 ? ~0u : 0u, m1 = s == 1 ? ~0u : 0u, m2 = s == 2 ? ~0u : 0u, m3 = s == 3 ? ~0u : 0u;
  const unsigned x = __float_as_uint(v.x), y = __float_as_uint(v.y), z = __float_as_uint(v.z), w = __float_as_uint(v.w);
  float4 o;
  o.x = __uint_as_float((x & m0) | (y & m1) | (z & m2) | (w & m3));
  o.y = __uint_as_float((y & m0) | (z & m1) | (w & (m2 | m3)));
  o.z = __uint_as_float((z & m0) | (w & (m1 | m2 | m3)));
  o.w = v.w;
  return o;
}
__device__ __forceinline__ void add4_if(float4& a, const float4& b, bool ok) {
  a.x = ok ? a.x + b.x : a.x;
  a.y = ok ? a.y + b.y : a.y;
  a.z = ok ? a.z + b.z : a.z;
  a.w = ok ? a.w + b.w : a.w;
}

// chunks q0 + j * qs (< nq), j < J
template <int J>
__device__ __forceinline__ void slab_fused_plan(const SlabSet& ss, long q0, long qs, long nq, SlabFusedPlan<J>& pl) {
  const int lane = threadIdx.x & 63;
  const int cq = lane & 15;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const long q = q0 + j * qs;
    int k;
    long ib;
    const bool ok = q < nq && slab_locate(ss, q, 0, k, ib) && k < ss.count;  // ib: the chunk's first element
    const int ks = ok ? k : 0;  // chunks past the end read segment 0 row 0, unused
    const SlabSeg& sg = ss.s[ks];
    pl.base[j] = sg.slab + sg.src_off;
    pl.stride[j] = sg.row_stride;
    pl.rows[j] = ok ? sg.rows : 0;
    const long i = ok && ib + 4 * cq < sg.n ? ib + 4 * cq : 0;  // dead lanes: element 0
    const long last4 = sg.n - 4;
    pl.ic[j] = i < last4 ? i : last4;
    pl.sh[j] = (int)(i - pl.ic[j]);
  }
  // own output
  const int jt = threadIdx.x >> 6;
  const long q = q0 + (long)jt * qs;
  int k;
  long i;
  pl.own_live = jt < J && q < nq && slab_locate(ss, q, lane, k, i);
  pl.own_i = pl.own_live ? i : 0;
  const SlabSeg& sg = ss.s[pl.own_live ? k : 0];
  pl.dst = sg.dst;
  pl.p = sg.p;
  pl.m = sg.m;
  pl.shb = sg.sh;
  pl.sht = sg.sh_t;
  pl.sh32 = sg.sh_t32;
  pl.scale = sg.scale;
  pl.accum = sg.accum;
  pl.t_co = sg.t_co;
  pl.t_taps = sg.t_taps;
  pl.t_ci = sg.t_ci;
  pl.p0 = pl.m0 = 0.f;
  if (pl.own_live && ss.sgd.update && pl.p) {  // SGD operands (independent of the slabs)
    pl.p0 = pl.p[pl.own_i];
    pl.m0 = pl.m ? pl.m[pl.own_i] : 0.f;
  }
}

// group sums acc (this thread's quad of group g) -> LDS -> the finalising threads combine
// groups 0..15 in order, scale, store and apply the fused SGD
template <int J>
__device__ __forceinline__ void slab_fused_finish(const SlabSet& ss, const SlabFusedPlan<J>& pl, float* part,
                                                  const float4* acc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cq = lane & 15, g = 4 * wave + (lane >> 4);
#pragma unroll
  for (int j = 0; j < J; ++j) *reinterpret_cast<float4*>(part + (j * 16 + g) * 64 + 4 * cq) = acc[j];
  __syncthreads();
  DDP_STAMP(STAMP_K_GRAD_REDUCE, 4);  // group sums in LDS
  // combine + epilogue: thread t < 64 * J finalises output t & 63 of chunk t >> 6
  if (pl.own_live) {
    const int j = wave, c = lane;
    const long i = pl.own_i;
    float gsum = part[(j * 16) * 64 + c];
#pragma unroll
    for (int qq = 1; qq < 16; ++qq) gsum += part[(j * 16 + qq) * 64 + c];
    gsum *= pl.scale;
    if (pl.accum) gsum += pl.dst[i];
    if (ss.sys_store) st_sys(pl.dst + i, gsum);
    else pl.dst[i] = gsum;
    if (ss.sgd.update && pl.p) {
      float m = pl.m0;
      const float pn = sgd_one(pl.p0, gsum, &m, ss.sgd);
      pl.p[i] = pn;
      if (pl.m) pl.m[i] = m;
      if (pl.shb) pl.shb[i] = f2bf(pn);
      if (pl.sht || pl.sh32) {
        const long per = (long)pl.t_taps * pl.t_ci;
        const long co = i / per;
        if (pl.sht) pl.sht[(i - co * per) * pl.t_co + co] = f2bf(pn);
        if (pl.sh32) pl.sh32[(i - co * per) * pl.t_co + co] = pn;
      }
    }
  }
  __syncthreads();
}

// part: J * 16 * 64 floats of LDS.  Every thread of the block calls it.
template <int J>
__device__ __forceinline__ void slab_fused_run(const SlabSet& ss, const SlabFusedPlan<J>& pl, float* part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = 4 * wave + (lane >> 4);
  float4 a[J][8];
  // every chunk's first 8 rows per group in ONE straight-line block
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int rl = pl.rows[j] > 0 ? pl.rows[j] - 1 : 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) a[j][u] = slab_ld4_sc1(pl.base[j], pl.ic[j] + (long)min(g + 16 * u, rl) * pl.stride[j]);
  }
  __builtin_amdgcn_sched_barrier(0);
  DDP_STAMP(STAMP_K_GRAD_REDUCE, 3);  // loads issued
  float4 acc[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 8; ++u) add4_if(acc[j], shift4(a[j][u], pl.sh[j]), g + 16 * u < pl.rows[j]);
  }
  // deeper slabs (e.g. the w1 slab, one row per dgrad block): the remaining rows, in order
#pragma clang loop unroll(full)
  for (int j = 0; j < J; ++j) {
    if (pl.rows[j] > 8 * 16) {  // block-uniform
      float4 t = acc[j];
      for (int r0 = 8 * 16; r0 < pl.rows[j]; r0 += 8 * 16) {
        float4 b[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          b[u] = slab_ld4_sc1(pl.base[j], pl.ic[j] + (long)min(g + r0 + 16 * u, pl.rows[j] - 1) * pl.stride[j]);
#pragma unroll
        for (int u = 0; u < 8; ++u) add4_if(t, shift4(b[u], pl.sh[j]), g + r0 + 16 * u < pl.rows[j]);
      }
      acc[j] = t;
    }
  }
  slab_fused_finish<J>(ss, pl, part, acc);
}

// Deep slab sets (128 < rows <= 256: the exact-fp32 step's 224 weight-gradient rows, bf16 at
// B = 64: 256): all 16 rows of every group of the J chunks in flight at once.  The 8-row
// variant above made one serial load round per further 128 rows and chunk - 1 + J rounds
// after the arrival wait.  Same summation order (rows g, g + 16, ... sequentially).  Rows
// past 256 (the fp32 w1 slab: one row per dgrad block) continue in serial 8-row rounds.
template <int J>
__device__ __forceinline__ void slab_fused_run16(const SlabSet& ss, const SlabFusedPlan<J>& pl, float* part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = 4 * wave + (lane >> 4);
  float4 a[J][16];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int rl = pl.rows[j] > 0 ? pl.rows[j] - 1 : 0;
#pragma unroll
    for (int u = 0; u < 16; ++u) a[j][u] = slab_ld4_sc1(pl.base[j], pl.ic[j] + (long)min(g + 16 * u, rl) * pl.stride[j]);
  }
  __builtin_amdgcn_sched_barrier(0);
  DDP_STAMP(STAMP_K_GRAD_REDUCE, 3);  // loads issued
  float4 acc[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 16; ++u) add4_if(acc[j], shift4(a[j][u], pl.sh[j]), g + 16 * u < pl.rows[j]);
  }
#pragma clang loop unroll(full)
  for (int j = 0; j < J; ++j) {
    if (pl.rows[j] > 16 * 16) {  // block-uniform
      float4 t = acc[j];
      for (int r0 = 16 * 16; r0 < pl.rows[j]; r0 += 8 * 16) {
        float4 b[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          b[u] = slab_ld4_sc1(pl.base[j], pl.ic[j] + (long)min(g + r0 + 16 * u, pl.rows[j] - 1) * pl.stride[j]);
#pragma unroll
        for (int u = 0; u < 8; ++u) add4_if(t, shift4(b[u], pl.sh[j]), g + r0 + 16 * u < pl.rows[j]);
      }
      acc[j] = t;
    }
  }
  slab_fused_finish<J>(ss, pl, part, acc);
}

// number of 64-output chunks of a SlabSet
__host__ __device__ inline long slab_chunks(const SlabSet& ss) {
  long b = 0;
  for (int k = 0; k < ss.count; ++k) b += (ss.s[k].n + 63) / 64;
  return b;
}

}  // namespace ddp_amd
