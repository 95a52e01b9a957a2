// Shared device helpers for the gfx950 (CDNA4) kernels of ddp_amd.
//
// Conventions used by every kernel in this directory:
//  * activations are NHWC bf16 (channels contiguous = the GEMM K dimension of an
//    implicit-GEMM convolution), stored as raw 16-bit words (bf16_t);
//  * master parameters are fp32; kernels that feed MFMA read bf16 "shadow"
//    copies that the fused SGD kernel rewrites after every update;
//  * MFMA tile = v_mfma_f32_16x16x32_bf16.  Lane maps (cdna_hip_programming.md §3):
//      A[row = l&15][k = 8*(l>>4) + j],  B[k = 8*(l>>4) + j][col = l&15],  j = 0..7
//      D[row = 4*(l>>4) + r][col = l&15], r = 0..3
//    The convolution kernels put output CHANNELS on the MFMA rows and PIXELS on
//    the columns, so each lane ends with 4 consecutive channels of one pixel
//    (one 8-byte NHWC store per 16x16 tile).
//  * wave = 64 lanes; all reductions are fixed-order (bitwise reproducible).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels/types.h"

namespace ddp_amd {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int WAVE = 64;

__device__ __forceinline__ float bf2f(bf16_t b) {
  return __builtin_bit_cast(float, ((unsigned)b) << 16);
}
__device__ __forceinline__ bf16_t f2bf(float f) {  // RNE, NaN-preserving (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}
__device__ __forceinline__ float bf16_round(float f) { return bf2f(f2bf(f)); }

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  return z;
}
__device__ __forceinline__ bf16x8 ld8(const bf16_t* p) {  // 16-byte global load
  return *reinterpret_cast<const bf16x8*>(p);
}
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 8 contiguous bytes = 4 bf16 packed from 4 floats
__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
  uint2 r;
  r.x = (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
  r.y = (unsigned)f2bf(c) | ((unsigned)f2bf(d) << 16);
  return r;
}
__device__ __forceinline__ void unpack4(uint2 v, float* o) {
  o[0] = __builtin_bit_cast(float, v.x << 16);
  o[1] = __builtin_bit_cast(float, v.x & 0xffff0000u);
  o[2] = __builtin_bit_cast(float, v.y << 16);
  o[3] = __builtin_bit_cast(float, v.y & 0xffff0000u);
}

// Element-wise ReLU mask of an 8-wide bf16 fragment by a second fragment (y > 0).
__device__ __forceinline__ bf16x8 mask8(bf16x8 g, bf16x8 y) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    // torch threshold_backward keeps grad unless (y <= 0): sign bit clear and not +0
    const unsigned short u = (unsigned short)y[j];
    const bool pos = (u & 0x8000u) == 0 && u != 0;
    r[j] = pos ? g[j] : (short)0;
  }
  return r;
}

// SimpleCNN conv1 (Cin = 1, 3x3): relu(b1[c] + sum_k w1[c*9+k] * v[k]) with exactly the
// FMA order of conv1_fwd_kernel, so kernels that recompute a1 instead of reading it
// from memory reproduce the stored bf16 values bit for bit.
__device__ __forceinline__ float conv1_eval(const float* w1, const float* b1, const float* v, int c) {
  float acc = b1[c];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc = fmaf(w1[c * 9 + k], v[k], acc);
  return fmaxf(acc, 0.f);
}

// ---- cross-lane reductions on DPP (VALU modifiers, no LDS round trips) --------------
// dpp<CTRL>(v): v of the lane selected by the DPP control (quad_perm 0x00-0xFF,
// row_half_mirror 0x141, row_mirror 0x140), all rows / banks enabled.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}
// Sum / max over each 16-lane row (lanes sharing lane >> 4); every lane of the row
// gets the result.  Pairs, quads, halves, row: a fixed association order, identical
// on every lane (each step combines two equal-shaped partial sums commutatively).
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  v = fmaxf(v, dpp<0x141>(v));
  v = fmaxf(v, dpp<0x140>(v));
  return v;
}
__device__ __forceinline__ float lane_bcast(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}
// fixed-order sum over all 64 lanes (every lane gets the total): rows, then
// ((r0 + r1) + (r2 + r3)) from lane reads
__device__ __forceinline__ float wave_sum(float v) {
  v = row16_sum(v);
  return (lane_bcast(v, 0) + lane_bcast(v, 16)) + (lane_bcast(v, 32) + lane_bcast(v, 48));
}
// sum over the 16 lanes that share (lane >> 4)
__device__ __forceinline__ float sum16(float v) { return row16_sum(v); }
__device__ __forceinline__ float wave_max(float v) {
  v = row16_max(v);
  return fmaxf(fmaxf(lane_bcast(v, 0), lane_bcast(v, 16)), fmaxf(lane_bcast(v, 32), lane_bcast(v, 48)));
}

// Whole-batch softmax cross-entropy on one workgroup, fixed summation order.
// part: split-K partial logits [B][G][NO] (G partials per logit), NO <= 16.
// One 16-lane row per batch row, lane o = class o: the lane sums its G partials
// (all loads of a 64-chunk in flight, clamped addresses, masked afterwards), then
// max / sum-exp / the label's logit are 16-lane DPP reductions.  Writes
// dl[b*NO + o] = (softmax - onehot) * gscale and loss[b] = logsumexp - x[label].
// Used by xent_rows (own kernel) and by the XENT prologue of fc_bwd, so both
// produce bit-identical values.  blockDim.x must be a multiple of 64.
__device__ __forceinline__ void xent_batch_block(const float* __restrict__ part, int G,
                                                 const float* __restrict__ bias, int NO, int B,
                                                 const int* __restrict__ labels32, const BatchIdx& bi,
                                                 float gscale, float* dl, float* loss) {
  const int o = threadIdx.x & 15;
  const bool own = o < NO;
  const int base = bi.base();
  for (int b = threadIdx.x >> 4; b < B; b += blockDim.x >> 4) {
    const int label = labels32[bi.row(b, base)];
    const float* src = part + (long)b * G * NO + (own ? o : 0);
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    for (int g0 = 0; g0 < G; g0 += 64) {
      float v[64];
#pragma unroll
      for (int u = 0; u < 64; ++u) v[u] = src[(long)min(g0 + u, G - 1) * NO];
#pragma unroll
      for (int u = 0; u < 64; ++u) a[u & 3] += (g0 + u < G) ? v[u] : 0.f;
    }
    const float x = own ? bias[o] + ((a[0] + a[1]) + (a[2] + a[3])) : -INFINITY;
    const float mx = row16_max(x);
    const float e = own ? __expf(x - mx) : 0.f;
    const float se = row16_sum(e);
    const float xl = row16_sum(own && o == label ? x : 0.f);
    if (own) dl[b * NO + o] = (e / se - (o == label ? 1.f : 0.f)) * gscale;
    if (o == 0) loss[b] = mx + __logf(se) - xl;
  }
}

}  // namespace ddp_amd
