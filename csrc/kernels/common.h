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

// fixed-order butterfly sum over all 64 lanes (every lane gets the total)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
// sum over the 16 lanes that share (lane >> 4)
__device__ __forceinline__ float sum16(float v) {
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
  return v;
}

// Softmax cross-entropy of one row on one wave from split-K fc partials laid out
// [NO][G] (part_row = part + b*NO*G): 4 lanes per class, fixed summation order.
// Writes dl_row[c] = (softmax - onehot) * gscale (lanes with j == 0) and returns
// the row loss (valid on every lane).  Shared by xent_rows and the XENT prologue of
// fc_bwd so both produce bit-identical values.
__device__ __forceinline__ float xent_row_wave(const float* __restrict__ part_row, int G,
                                               const float* __restrict__ bias, int NO, int label,
                                               float gscale, float* dl_row) {
  const int lane = threadIdx.x & 63;
  const int c = lane >> 2, j = lane & 3;
  const bool own = c < NO;
  float s = 0.f;
  if (own) {
    const float* src = part_row + (long)c * G;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int g = j;
    for (; g + 12 < G; g += 16) {  // 4 independent loads in flight
      a0 += src[g]; a1 += src[g + 4]; a2 += src[g + 8]; a3 += src[g + 12];
    }
    for (; g < G; g += 4) a0 += src[g];
    s = ((a0 + a1) + a2) + a3;
  }
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  const float x = own ? s + bias[c] : -INFINITY;
  const float mx = wave_max(x);
  const float e = (own && j == 0) ? __expf(x - mx) : 0.f;
  const float se = wave_sum(e);
  const float xl = wave_sum((own && j == 0 && c == label) ? x : 0.f);
  if (own && j == 0) dl_row[c] = (e / se - (c == label ? 1.f : 0.f)) * gscale;
  return mx + __logf(se) - xl;
}

}  // namespace ddp_amd
