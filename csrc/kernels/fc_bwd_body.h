// fc backward body (SimpleCNN's Linear(50176, 10) over the NHWC-flattened ReLU2 output,
// reference model.py:16,19), shared by the standalone fc_bwd kernel (linear.hip) and the
// fc role of the fused fc + conv backward launch (conv3x3.hip, fuse level 2).
//
// One pass over the activation computing
//   dX[b][k] = (MASK ? X>0 : 1) * sum_o dL[b][o] W[o][k]      (bf16 / fp32, write-through)
//   dW[o][k] = scale * sum_b dL[b][o] X[b][k]                    (fp32)
// i.e. fc dgrad + fc wgrad + ReLU2 mask fused.
//
// Geometry: a block of WPB waves owns COLS = 64 * CPL consecutive columns k (CPL per
// lane, one 2*CPL- or 4*CPL-byte load per row).  The batch rows are split over VW
// "virtual" waves (virtual wave v: rows v, v + VW, ...; physical wave w runs the virtual
// waves w, w + WPB, ...) and the dW partials are summed in virtual-wave order
// v = 0, 1, ..., VW-1 through LDS, WPB slots per round - so every (WPB, CPL) with the
// same VW gives bit-identical dW, and dX never depends on the geometry at all.  The W
// columns and the first rows of X are requested BEFORE the prologue (cross-entropy
// backward or dL copy) so they land while it runs.  Every branch on the row count or the
// class count is wave-uniform, row addresses are clamped instead of guarded, so a wave
// keeps all its loads in flight.  NOT = compile-time class capacity (NOT == 10 fixes NO).
//
// ready != nullptr (fused level 2): after its dX stores every wave drains them
// (vmcnt(0)), the block syncs and lane 0 stores ready[bx] = 1 with an agent-scope
// (sc1) store; the conv roles poll it with sc1 loads and read dX with sc1 loads
// (MI355X_MICROARCH.md, hand-off table row 1: sc1 stores, drained, one flag per block).
#pragma once
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

constexpr int FCB_RB = 8;  // rows in flight per virtual wave

template <int CPL>
struct ColF {
  float v[CPL];
};
// CPL consecutive columns of one row as floats
template <int CPL>
__device__ __forceinline__ ColF<CPL> ldc(const bf16_t* p) {
  ColF<CPL> r;
  if constexpr (CPL == 2) {
    const unsigned u = *reinterpret_cast<const unsigned*>(p);
    r.v[0] = __builtin_bit_cast(float, u << 16);
    r.v[1] = __builtin_bit_cast(float, u & 0xffff0000u);
  } else {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    r.v[0] = __builtin_bit_cast(float, u.x << 16);
    r.v[1] = __builtin_bit_cast(float, u.x & 0xffff0000u);
    r.v[2] = __builtin_bit_cast(float, u.y << 16);
    r.v[3] = __builtin_bit_cast(float, u.y & 0xffff0000u);
  }
  return r;
}
template <int CPL>
__device__ __forceinline__ ColF<CPL> ldc(const float* p) {
  ColF<CPL> r;
  if constexpr (CPL == 2) {
    const float2 a = *reinterpret_cast<const float2*>(p);
    r.v[0] = a.x; r.v[1] = a.y;
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p);
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  }
  return r;
}
template <int CPL>
__device__ __forceinline__ void stc_wt(bf16_t* p, const float* v) {
  const unsigned a = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
  if constexpr (CPL == 2) {
    st_wt(reinterpret_cast<unsigned*>(p), a);
  } else {
    const unsigned b = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
    st_wt(reinterpret_cast<uint2*>(p), make_uint2(a, b));
  }
}
template <int CPL>
__device__ __forceinline__ void stc_wt(float* p, const float* v) {
  if constexpr (CPL == 2) st_wt(reinterpret_cast<float2*>(p), make_float2(v[0], v[1]));
  else st_wt(reinterpret_cast<float4*>(p), make_float4(v[0], v[1], v[2], v[3]));
}

template <int WPB, int NOT, int CPL>
__host__ __device__ constexpr int fcb_red_floats() { return WPB * NOT * 64 * CPL; }

// LDS floats of the body: [B][NO] dL, [B] loss, (XENT: [B][NO] logits, [B] labels),
// then the dW reduction slots [WPB][NOT][COLS], which the cross-entropy prologue's copy
// of the partial logits (npart floats) aliases.
__host__ __device__ inline long fcb_lds_floats(int B, int NO, bool xent, long npart, int red) {
  const long head = ((long)(xent ? 2 * B * NO + B : B * NO) + B + 3) & ~3L;
  return head + (red > npart ? red : npart);
}

// The fc bias gradient (fixed batch order), the fused SGD of the bias and the batch-mean
// loss from the block's LDS dL / per-row losses - wave 0 of block 0, or of the last block to
// arrive (FcBwdExtras::last_ctr).
template <bool XENT>
__device__ __forceinline__ void fc_bwd_bias_loss(const FcBwdExtras& ex, const float* s_dl, const float* s_loss,
                                                 int B, int NO, bool last) {
  const int lane = threadIdx.x & 63;
  if (ex.dbias && lane < NO) {
    float acc = 0.f;
#pragma unroll 16
    for (int b = 0; b < B; ++b) acc += s_dl[b * NO + lane];  // (unrolled: the reads go out together)
    const float g = acc * ex.dbias_scale;
    if (ex.sys_store) st_sys(ex.dbias + lane, g);
    else ex.dbias[lane] = g;
    if (last && ex.p_b && ex.sgd.update) {
      // == the 1-row in-place slab the fused slab reduction used to apply it from (0 + g)
      float m = ex.m_b ? ex.m_b[lane] : 0.f;
      const float pn = sgd_one(ex.p_b[lane], 0.f + g, &m, ex.sgd);
      ex.p_b[lane] = pn;
      if (ex.m_b) ex.m_b[lane] = m;
    }
  }
  if ((XENT || ex.loss_rows) && ex.loss_out) {
    // (every caller runs this with a whole wave) one load per lane, then the same
    // sequential b = 0, 1, ... sum through v_readlane: the loop of dependent-address-free
    // but serially waited loads on one lane took ~12 us at B = 64 (profiles/r4_b64/final_sweep)
    const float* lr = XENT ? s_loss : ex.loss_rows;
    const int at = ex.step_ctr ? *ex.step_ctr : 0;
    float acc = 0.f;
    for (int b0 = 0; b0 < B; b0 += 64) {
      const float v = b0 + lane < B ? lr[b0 + lane] : 0.f;
      const int nb = B - b0 < 64 ? B - b0 : 64;
      for (int k = 0; k < nb; ++k)
        acc += __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), k));
    }
    if (lane == 63) {
      ex.loss_out[at] = acc / (float)B;
      if (last && ex.step_inc) *ex.step_inc = at + 1;  // ex.step_inc == ex.step_ctr (read just above)
    }
  }
  if (ex.zero_i32 && (last || !ex.last_ctr))  // (block 0 when there is no last-block count)
    for (int i = lane; i < ex.n_zero; i += 64) ex.zero_i32[(long)i * ex.zero_stride] = 0;
}

// Wave-independent fc weight gradient (+ fused SGD) of 128 consecutive columns [col0,
// col0 + 128): lane l owns columns col0 + 2l, +1 and sums their dW over the whole batch
// itself, in fc_bwd_body's virtual-wave order for VW = 8 (virtual wave v: rows v, v + 8,
// ..., an fma chain from 0; partials combined v = 0, 1, ..., 7) - bit-identical to the
// block-wide body, with no LDS reduction and no block barrier per chunk.  dL comes from
// LDS, rows padded to FCDW_LD floats (s_dl [B][FCDW_LD], filled by the caller; read as
// broadcast 16-byte loads).  B <= MAXB.  Every global load of the chunk (the SGD operands,
// then all B rows) is issued up front; a scheduling barrier per virtual wave keeps only
// that wave's dL values live.  The level-3 conv backward's fc role runs it on the launch's
// otherwise idle resident slots (conv3x3.hip FCR).
// X is the bf16 activation (4-byte loads: the lane's column pair) or, for the exact-fp32
// step, the fp32 one (8-byte loads); the fp32 step's fc operand copy is the fp32 FCFRAG
// shadow (ex.sh_frag32).
constexpr int FCDW_LD = 12;
template <int MAXB, typename T>
__device__ __forceinline__ void fc_dw_wave_chunk(const float* s_dl, const T* __restrict__ X,
                                                 float* __restrict__ dW, float scale, int B, long K,
                                                 const FcBwdExtras& ex, long col0) {
  constexpr bool F32 = sizeof(T) == 4;
  constexpr int NO = 10, VW = 8, RPV = (MAXB + VW - 1) / VW;
  const int lane = threadIdx.x & 63;
  const long col = col0 + 2 * lane;
  const bool active = col < K;  // host guarantees K % 2 == 0
  const long cc = active ? col : 0;
  // buffer loads: one scalar base per tensor, the row / class offset in the scalar offset
  // field, the lane's column offset in ONE VGPR shared by every load (no per-load 64-bit
  // addresses; the fc tensors are < 2 GiB)
  typedef __attribute__((ext_vector_type(2))) int i32x2_t;
  const int vo4 = (int)cc * 4, vo2 = (int)cc * 2;
  float2 pp[NO], mm[NO];
  if (ex.sgd.update) {
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(ex.p_w, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rm =
        __builtin_amdgcn_make_buffer_rsrc(ex.m_w ? ex.m_w : ex.p_w, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      pp[o] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rp, vo4, (int)(o * K * 4), 0));
      mm[o] = ex.m_w ? __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rm, vo4, (int)(o * K * 4), 0))
                     : make_float2(0.f, 0.f);
    }
  }
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(X), (short)0, 0x7fffffff,
                                                                      0x00020000);
  unsigned xw[F32 ? 1 : MAXB];
  float2 xf[F32 ? MAXB : 1];
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    if constexpr (F32)
      xf[b] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, vo4, (int)((long)min(b, B - 1) * K * 4), 0));
    else
      xw[b] = (unsigned)__builtin_amdgcn_raw_buffer_load_b32(rx, vo2, (int)((long)min(b, B - 1) * K * 2), 0);
  }
  float acc[NO][2];
#pragma unroll
  for (int v = 0; v < VW; ++v) {
    __builtin_amdgcn_sched_barrier(0);
    float p[NO][2];
#pragma unroll
    for (int o = 0; o < NO; ++o) p[o][0] = p[o][1] = 0.f;
#pragma unroll
    for (int u = 0; u < RPV; ++u) {
      const int b = v + VW * u;
      if (b < MAXB && b < B) {  // wave-uniform
        const float x0 = F32 ? xf[F32 ? b : 0].x : __builtin_bit_cast(float, xw[F32 ? 0 : b] << 16);
        const float x1 = F32 ? xf[F32 ? b : 0].y : __builtin_bit_cast(float, xw[F32 ? 0 : b] & 0xffff0000u);
        const float4 d0 = *reinterpret_cast<const float4*>(s_dl + b * FCDW_LD);
        const float4 d1 = *reinterpret_cast<const float4*>(s_dl + b * FCDW_LD + 4);
        const float2 d2 = *reinterpret_cast<const float2*>(s_dl + b * FCDW_LD + 8);
        const float d[NO] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w, d2.x, d2.y};
#pragma unroll
        for (int o = 0; o < NO; ++o) {
          p[o][0] = fmaf(d[o], x0, p[o][0]);
          p[o][1] = fmaf(d[o], x1, p[o][1]);
        }
      }
    }
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      acc[o][0] = v == 0 ? p[o][0] : acc[o][0] + p[o][0];
      acc[o][1] = v == 0 ? p[o][1] : acc[o][1] + p[o][1];
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  if (!active) return;
  const long frag0 = (ex.sh_frag || ex.sh_frag32) ? fcfrag_index((int)col, ex.frag_HW, ex.frag_C) : 0;
#pragma unroll
  for (int o = 0; o < NO; ++o) {
    const float g0 = acc[o][0] * scale, g1 = acc[o][1] * scale;
    const long idx = (long)o * K + col;
    if (dW) {
      if (ex.sys_store) {
        st_sys(dW + idx, g0);
        st_sys(dW + idx + 1, g1);
      } else {
        *reinterpret_cast<float2*>(dW + idx) = make_float2(g0, g1);
      }
    }
    if (ex.sgd.update) {
      float m0 = mm[o].x, m1 = mm[o].y;
      const float p0 = sgd_one(pp[o].x, g0, &m0, ex.sgd), p1 = sgd_one(pp[o].y, g1, &m1, ex.sgd);
      st_wt(reinterpret_cast<float2*>(ex.p_w + idx), make_float2(p0, p1));
      if (ex.m_w) *reinterpret_cast<float2*>(ex.m_w + idx) = make_float2(m0, m1);
      const unsigned pb = (unsigned)f2bf(p0) | ((unsigned)f2bf(p1) << 16);
      if (ex.sh_plain) st_wt(reinterpret_cast<unsigned*>(ex.sh_plain + idx), pb);
      // FCFRAG keeps channel pairs (c, c + 1), c even, adjacent: one 4-byte store; the class
      // is its outermost dimension, so class o's index is class 0's + o * K
      if (ex.sh_frag) st_wt(reinterpret_cast<unsigned*>(ex.sh_frag + frag0 + (long)o * K), pb);
      if (ex.sh_frag32) st_wt(reinterpret_cast<float2*>(ex.sh_frag32 + frag0 + (long)o * K), make_float2(p0, p1));
    }
  }
}

template <typename T, bool MASK, bool XENT, int NOT, int WPB, int VW, int CPL, bool DXO = true>
__device__ __forceinline__ void fc_bwd_body(const float* __restrict__ dL, const T* __restrict__ X,
                                            const T* __restrict__ Wf, T* __restrict__ dX,
                                            float* __restrict__ dW, float scale, int B, long K, int NO_rt,
                                            const FcBwdExtras& ex, float* smem, int bx, int* ready) {
  static_assert(VW % WPB == 0, "virtual waves must be a multiple of the physical waves");
  constexpr int COLS = 64 * CPL, NT = WPB * 64, KV = VW / WPB;
  DDP_STAMP(STAMP_K_FC_BWD, 0);
  const int NO = NOT == 10 ? 10 : NO_rt;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* s_dl = smem;             // [B][NO]
  float* s_loss = s_dl + B * NO;  // [B]
  float* s_lg = s_loss + B;       // [B][NO] cross-entropy scratch (XENT)
  int* s_lab = reinterpret_cast<int*>(s_lg + B * NO);  // [B] labels (XENT)
  float* s_red = smem + (((XENT ? 2 * B * NO + B : B * NO) + B + 3) & ~3);  // [WPB][NOT][COLS]

  const long col = (long)bx * COLS + CPL * lane;
  const bool active = col < K;  // host guarantees K % CPL == 0
  const long cc = active ? col : 0;
  // ---- this block's column loads first (independent of the prologue)
  ColF<CPL> wr[DXO ? NOT : 1];
  if constexpr (DXO) {
#pragma unroll
    for (int o = 0; o < NOT; ++o) {
      if (o < NO) wr[o] = ldc<CPL>(Wf + (long)o * K + cc);
      else
#pragma unroll
        for (int j = 0; j < CPL; ++j) wr[o].v[j] = 0.f;
    }
  }
  // rows of virtual wave v = wave + WPB * kv (uniform)
  int nr[KV];
#pragma unroll
  for (int kv = 0; kv < KV; ++kv) {
    const int v = wave + WPB * kv;
    nr[kv] = B > v ? (B - v + VW - 1) / VW : 0;
  }
  ColF<CPL> xr[KV][FCB_RB];
#pragma unroll
  for (int kv = 0; kv < KV; ++kv)
#pragma unroll
    for (int u = 0; u < FCB_RB; ++u) {
      const int b = min(wave + WPB * kv + VW * u, B - 1);
      xr[kv][u] = ldc<CPL>(X + (long)b * K + cc);
    }
  // fused-SGD operands of this thread's dW outputs (final loop below): requested now so
  // the optimizer tail has no dependent global round trip
  constexpr int PRE = (NOT * COLS + NT - 1) / NT;
  float pre_p[PRE], pre_m[PRE];
  if (ex.sgd.update) {
#pragma unroll
    for (int j = 0; j < PRE; ++j) {
      const int i = threadIdx.x + j * NT;
      const int o = i / COLS, c = i - (i / COLS) * COLS;
      const long k = (long)bx * COLS + c;
      const bool ok = i < NO * COLS && k < K;
      const long idx = ok ? (long)o * K + k : 0;
      pre_p[j] = ex.p_w[idx];
      pre_m[j] = ex.m_w ? ex.m_w[idx] : 0.f;
    }
  }
  // ---- then the cross-entropy's (labels, partial logits: coalesced, to LDS).  Issued
  // first instead, they made the rows phase wait for the later column loads (measured
  // 10.6 vs 9.4 us per kernel): the prologue is not what the kernel waits on.
  XentPre xp;
  const int npart = XENT ? ((B * ex.HW + ex.CH - 1) / ex.CH) * 2 * NO : 0;
  if (XENT) xent_prefetch(ex.part, npart, ex.fc_bias, NO, B, ex.labels32, ex.bi, xp);
  DDP_STAMP(STAMP_K_XENT, 0);  // loads of W / X issued
  // ---- prologue: dL of the whole batch into LDS
  if (XENT) {
    // the partials' LDS copy aliases s_red (first written after the next barrier)
    xent_finish(xp, ex.part, npart, ex.HW, ex.CH, ex.fc_bias, NO, B, ex.labels32, ex.bi, ex.gscale, s_dl,
                s_loss, s_lg, s_lab, s_red);
  } else {
    for (int i = threadIdx.x; i < B * NO; i += NT) s_dl[i] = dL[i];
  }
  __syncthreads();
  DDP_STAMP(STAMP_K_FC_BWD, 1);
  // fc bias gradient (sum over the batch, fixed order) and the batch-mean loss
  if (bx == 0 && !ex.last_ctr && wave == 0) fc_bwd_bias_loss<XENT>(ex, s_dl, s_loss, B, NO, false);
  float dw[KV][NOT][CPL];
#pragma unroll
  for (int kv = 0; kv < KV; ++kv)
#pragma unroll
    for (int o = 0; o < NOT; ++o)
#pragma unroll
      for (int j = 0; j < CPL; ++j) dw[kv][o][j] = 0.f;
#pragma unroll
  for (int kv = 0; kv < KV; ++kv) {
    const int v = wave + WPB * kv;
    for (int u0 = 0; u0 < nr[kv]; u0 += FCB_RB) {
      if (u0 > 0) {
#pragma unroll
        for (int u = 0; u < FCB_RB; ++u) {
          const int b = min(v + VW * (u0 + u), B - 1);
          xr[kv][u] = ldc<CPL>(X + (long)b * K + cc);
        }
      }
#pragma unroll
      for (int u = 0; u < FCB_RB; ++u) {
        if (u0 + u < nr[kv]) {  // wave-uniform
          const int b = v + VW * (u0 + u);
          const float* dl = s_dl + b * NO;
          float dz[CPL];
#pragma unroll
          for (int j = 0; j < CPL; ++j) dz[j] = 0.f;
#pragma unroll
          for (int o = 0; o < NOT; ++o)
            if (o < NO) {
              const float d = dl[o];
#pragma unroll
              for (int j = 0; j < CPL; ++j) {
                if constexpr (DXO) dz[j] = fmaf(d, wr[o].v[j], dz[j]);
                dw[kv][o][j] = fmaf(d, xr[kv][u].v[j], dw[kv][o][j]);
              }
            }
          if constexpr (DXO) {
            if (MASK) {
#pragma unroll
              for (int j = 0; j < CPL; ++j) dz[j] = xr[kv][u].v[j] > 0.f ? dz[j] : 0.f;
            }
            if (active) stc_wt<CPL>(dX + (long)b * K + col, dz);  // dZ2: write-through
          }
        }
      }
    }
  }
  DDP_STAMP(STAMP_K_FC_BWD, 2);
  if (ready) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's dZ2 stores are out
  // ---- fixed-order reduction of the virtual waves' dW partials, WPB slots per round
  float acc[PRE];
#pragma unroll
  for (int kv = 0; kv < KV; ++kv) {
    if (kv > 0) __syncthreads();  // the previous round's slots were read
#pragma unroll
    for (int o = 0; o < NOT; ++o)
      if (o < NO) {
        float* dst = s_red + (wave * NOT + o) * COLS + CPL * lane;
        if constexpr (CPL == 2) *reinterpret_cast<float2*>(dst) = make_float2(dw[kv][o][0], dw[kv][o][1]);
        else *reinterpret_cast<float4*>(dst) = make_float4(dw[kv][o][0], dw[kv][o][1], dw[kv][o][2], dw[kv][o][3]);
      }
    __syncthreads();
    if (kv == 0 && ready && threadIdx.x == 0)  // every wave drained its dZ2 stores before the barrier
      __hip_atomic_store(ready + bx, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int jj = 0; jj < PRE; ++jj) {
      const int i = threadIdx.x + jj * NT;
      if (i < NO * COLS) {
        const int o = i / COLS, c = i - (i / COLS) * COLS;
        float a = kv == 0 ? s_red[o * COLS + c] : acc[jj] + s_red[o * COLS + c];
#pragma unroll
        for (int w = 1; w < WPB; ++w) a += s_red[(w * NOT + o) * COLS + c];
        acc[jj] = a;
      }
    }
  }
  DDP_STAMP(STAMP_K_FC_BWD, 3);
#pragma unroll
  for (int jj = 0; jj < PRE; ++jj) {
    const int i = threadIdx.x + jj * NT;
    if (i >= NO * COLS) break;
    const int o = i / COLS, c = i - (i / COLS) * COLS;
    const long k = (long)bx * COLS + c;
    if (k < K) {
      const float g = acc[jj] * scale;
      const long idx = (long)o * K + k;
      if (dW) {  // null: fused optimizer consumes it in registers
        if (ex.sys_store) st_sys(dW + idx, g);
        else dW[idx] = g;
      }
      if (ex.sgd.update) {  // single-process step: dW is final -> fused SGD + shadows
        float m = pre_m[jj];
        const float pn = sgd_one(pre_p[jj], g, &m, ex.sgd);
        st_wt(ex.p_w + idx, pn);  // write-through: no dirty L2 at the kernel boundary
        if (ex.m_w) ex.m_w[idx] = m;
        const bf16_t pb = f2bf(pn);
        if (ex.sh_plain) st_wt(ex.sh_plain + idx, pb);
        if (ex.sh_frag) st_wt(ex.sh_frag + fcfrag_index((int)idx, ex.frag_HW, ex.frag_C), pb);
        if (ex.sh_frag32) st_wt(ex.sh_frag32 + fcfrag_index((int)idx, ex.frag_HW, ex.frag_C), pn);
      }
    }
  }
  if (ex.last_ctr && wave == 0) {
    // arrival after the block's whole body: every read of the fc bias (prologue) is done.
    // Only wave 0 of the last block goes on; its LDS dL / losses are the block's own.
    int old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(ex.last_ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old == (ex.last_n > 0 ? ex.last_n : (int)gridDim.x) - 1) fc_bwd_bias_loss<XENT>(ex, s_dl, s_loss, B, NO, true);
  }
  DDP_STAMP(STAMP_K_FC_BWD, 4);
}

}  // namespace ddp_amd
