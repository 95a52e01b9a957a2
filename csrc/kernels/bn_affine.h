// A BatchNorm + ReLU applied by the consumer of a conv output while it loads the raw
// output (launchers.h BnAffine): bf16(relu(x * sc + sh)) with sc = invstd * gamma,
// sh = beta - mean * sc - ONE definition shared by bn_apply, the BN backward's recomputed
// ReLU mask and every consumer-side application (maxpool, halo conv forward / weight
// gradient), so all of them see bitwise the value bn_apply would have stored.
#pragma once
#include "kernels/common.h"

namespace ddp_amd {

// The raw BatchNorm parameters of 8 channels (loaded early, e.g. beside a staging load)
struct BnRaw8 {
  float4 is[2], g[2], mu[2], be[2];
};
__device__ __forceinline__ BnRaw8 bn_raw8(const float* invstd, const float* gamma, const float* mean,
                                          const float* beta, int c0) {
  BnRaw8 r;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    r.is[h] = *reinterpret_cast<const float4*>(invstd + c0 + 4 * h);
    r.g[h] = *reinterpret_cast<const float4*>(gamma + c0 + 4 * h);
    r.mu[h] = *reinterpret_cast<const float4*>(mean + c0 + 4 * h);
    r.be[h] = *reinterpret_cast<const float4*>(beta + c0 + 4 * h);
  }
  return r;
}
// sc = invstd * gamma, sh = beta - mean * sc (explicit fma: no contraction differences)
__device__ __forceinline__ void bn_affine8_of(const BnRaw8& r, float* sc, float* sh) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float isv[4] = {r.is[h].x, r.is[h].y, r.is[h].z, r.is[h].w};
    const float gv[4] = {r.g[h].x, r.g[h].y, r.g[h].z, r.g[h].w};
    const float mv[4] = {r.mu[h].x, r.mu[h].y, r.mu[h].z, r.mu[h].w};
    const float bv[4] = {r.be[h].x, r.be[h].y, r.be[h].z, r.be[h].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sc[4 * h + j] = isv[j] * gv[j];
      sh[4 * h + j] = fmaf(-mv[j], sc[4 * h + j], bv[j]);
    }
  }
}
// sc / sh of channels c0 .. c0 + 7
__device__ __forceinline__ void bn_affine8(const float* invstd, const float* gamma, const float* mean,
                                           const float* beta, int c0, float* sc, float* sh) {
  bn_affine8_of(bn_raw8(invstd, gamma, mean, beta, c0), sc, sh);
}

// 8 raw bf16 values -> bf16(relu(x * sc + sh))
__device__ __forceinline__ bf16x8 bn_relu8(bf16x8 v, const float* sc, const float* sh) {
  const uint4 u = __builtin_bit_cast(uint4, v);
  float x[8];
  unpack4(make_uint2(u.x, u.y), x);
  unpack4(make_uint2(u.z, u.w), x + 4);
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = fmaxf(fmaf(x[j], sc[j], sh[j]), 0.f);
  const uint2 lo = pack4(x[0], x[1], x[2], x[3]), hi = pack4(x[4], x[5], x[6], x[7]);
  return __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
}

}  // namespace ddp_amd
