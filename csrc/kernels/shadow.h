// Reduced-precision / re-laid-out parameter shadows written by the optimizer passes.
//
// The fp32 master parameters live in the flat buffer; the MFMA kernels read copies in
// their own operand layout (bf16 plain, the conv2 weight's [tap][ci][co] transpose, the
// fc weight's MFMA-fragment order, ...: ShadowRegion kinds in launchers.h).  Every pass
// that updates a parameter refreshes its shadows in the same pass: sgd_kernel (optim.hip)
// and the fused SGD of the xGMI all-reduce (allreduce.hip) share these writers, so both
// produce the same bytes.
//
// shadow_quad: flat elements [i, i + 4) with new values v.  A quad wholly inside a
// region whose offset is 4-aligned goes out as ONE vector store where the layout keeps
// the 4 elements contiguous (plain bf16: 8 B; fc fragment order: c % 4 is the fastest
// index, so 8 B bf16 / 16 B fp32); transposed layouts and straddling quads fall back to
// element stores.
#pragma once

#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

// WT: write-through stores (agent scope, sc1) - a consumer in the SAME launch on another XCD
// reads the shadow with sc1 loads (the dist_mode 4 launch: the all-reduce's fused SGD, then
// the next step's forward blocks; conv3x3.hip step_head_kernel)
template <bool WT = false>
__device__ __forceinline__ void put_bf(bf16_t* p, bf16_t v) {
  if constexpr (WT) st_wt(p, v); else *p = v;
}
template <bool WT = false>
__device__ __forceinline__ void put_f(float* p, float v) {
  if constexpr (WT) st_wt(p, v); else *p = v;
}
template <bool WT = false>
__device__ __forceinline__ void put_u2(uint2* p, uint2 v) {
  if constexpr (WT) st_wt(p, v); else *p = v;
}
template <bool WT = false>
__device__ __forceinline__ void put_f4(float* p, float4 v) {  // 16-byte aligned p
  if constexpr (WT) st_wt(reinterpret_cast<float4*>(p), v);  // (two 8-byte sc1 stores)
  else *reinterpret_cast<float4*>(p) = v;
}

template <bool WT = false>
__device__ __forceinline__ void shadow_put(const ShadowRegion& s, long j, float v) {
  if (j < 0 || j >= s.n) return;
  if (s.kind == SHADOW_BF16) {
    put_bf<WT>(s.dst + j, f2bf(v));
  } else if (s.kind == SHADOW_BF16_FCFRAG) {
    put_bf<WT>(s.dst + fcfrag_index((int)j, s.a, s.b), f2bf(v));
  } else if (s.kind == SHADOW_F32_FCFRAG) {
    put_f<WT>(s.dst32 + fcfrag_index((int)j, s.a, s.b), v);
  } else if (s.kind == SHADOW_BF16_PAD4) {  // [..][3] -> [..][4], the 4th stays zero
    put_bf<WT>(s.dst + (j / 3) * 4 + j % 3, f2bf(v));
  } else if (s.kind == SHADOW_F32_TAPT) {  // exact fp32 [tap][ci][co] copy
    const long per = (long)s.b * s.c;
    const long co = j / per;
    put_f<WT>(s.dst32 + (j - co * per) * s.a + co, v);
  } else {  // SHADOW_BF16_TAPT: OHWI [co][tap][ci] -> [tap][ci][co]
    const long per = (long)s.b * s.c;
    const long co = j / per;
    put_bf<WT>(s.dst + (j - co * per) * s.a + co, f2bf(v));
  }
}

// every region containing flat element i (constant trip count: a loop to sh.count
// indexing the by-value ShadowSet dynamically put it in scratch)
template <bool WT = false>
__device__ __forceinline__ void shadow_one(const ShadowSet& sh, long i, float v) {
#pragma unroll
  for (int r = 0; r < MAX_SHADOWS; ++r) {
    if (r >= sh.count) break;
    shadow_put<WT>(sh.r[r], i - sh.r[r].off, v);
  }
}

template <bool WT = false>
__device__ __forceinline__ void shadow_quad(const ShadowSet& sh, long i, float4 v) {
#pragma unroll
  for (int r = 0; r < MAX_SHADOWS; ++r) {
    if (r >= sh.count) break;
    const ShadowRegion& s = sh.r[r];
    const long j = i - s.off;
    if (j + 3 < 0 || j >= s.n) continue;
    const bool whole = j >= 0 && j + 3 < s.n && ((s.off & 3) == 0);
    if (s.kind == SHADOW_BF16 && whole) {
      put_u2<WT>(reinterpret_cast<uint2*>(s.dst + j), pack4(v.x, v.y, v.z, v.w));
    } else if (s.kind == SHADOW_BF16_FCFRAG && whole) {
      // C % 4 == 0: the quad is 4 consecutive channels of one (o, hw) -> 8 contiguous bytes
      put_u2<WT>(reinterpret_cast<uint2*>(s.dst + fcfrag_index((int)j, s.a, s.b)), pack4(v.x, v.y, v.z, v.w));
    } else if (s.kind == SHADOW_F32_FCFRAG && whole) {
      put_f4<WT>(s.dst32 + fcfrag_index((int)j, s.a, s.b), v);
    } else {
      // four explicit calls, not a loop over a local array (a dynamic index puts it in scratch)
      shadow_put<WT>(s, j, v.x);
      shadow_put<WT>(s, j + 1, v.y);
      shadow_put<WT>(s, j + 2, v.z);
      shadow_put<WT>(s, j + 3, v.w);
    }
  }
}

// SGD (torch semantics, sgd_one) on flat quad [i, i + 4) with gradient d, from the
// already loaded parameter quad v and momentum quad m (zero without momentum); stores the
// parameters / momentum (16-byte accesses: i % 4 == 0, 16-byte-aligned buffers) and
// refreshes the shadows.  Split from the loads so a caller with several quads in flight
// can issue every load before the first dependent store.
template <bool WT = false>
__device__ __forceinline__ void sgd_quad_apply(float* __restrict__ p, float* __restrict__ mbuf, long i,
                                               float4 d, float4 v, float4 m, const SgdArgs& a,
                                               const ShadowSet& sh) {
  v.x = sgd_one(v.x, d.x, &m.x, a);
  v.y = sgd_one(v.y, d.y, &m.y, a);
  v.z = sgd_one(v.z, d.z, &m.z, a);
  v.w = sgd_one(v.w, d.w, &m.w, a);
  put_f4<WT>(p + i, v);
  if (a.momentum != 0.f) *reinterpret_cast<float4*>(mbuf + i) = m;  // (read only by later launches)
  // (from a local copy: the regions read through a reference into the xGMI kernel's
  // by-value argument struct made the compiler copy the whole struct to scratch)
  const ShadowSet shl = sh;
  shadow_quad<WT>(shl, i, v);
}
__device__ __forceinline__ float4 ld_quad(const float* __restrict__ p, long i) {
  return *reinterpret_cast<const float4*>(p + i);
}

}  // namespace ddp_amd
