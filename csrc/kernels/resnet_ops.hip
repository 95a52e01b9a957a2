// Non-convolution ResNet-18 kernels on NHWC bf16 activations (BASELINE.json config 5;
// SURVEY.md §2.4 north-star list: BatchNorm2d train-mode fwd/bwd with running stats,
// MaxPool 3x3/s2, global average pool, residual add, fc head).
//
// BatchNorm statistics come from the producing convolution's epilogue (per-block
// per-channel sum / sum-of-squares slabs, conv_gemm.hip); bn_finalize reduces them
// in fixed order and updates the running buffers with torch's semantics (momentum
// 0.1, unbiased running variance, num_batches_tracked).  bn_apply fuses normalise +
// affine + residual add + ReLU.  The backward is two kernels: strip-parallel sums of
// dy and dy*xhat (with the ReLU mask from the saved output) finished by the strip's
// last block, which also writes dgamma / dbeta straight into the parameter
// gradients; then the per-element input gradient.  All float reductions are
// fixed-order (the only atomics are integer tickets).
#include <type_traits>
#include <stdexcept>
#include <string>

#include "kernels/bn_affine.h"
#include "kernels/bn_tail.h"
#include "kernels/common.h"
#include "kernels/launchers.h"

#define RN_CHECK(expr)                                                                   \
  do {                                                                                   \
    const hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e_)); \
  } while (0)

namespace ddp_amd {

// ---------------------------------------------------------------- last-arrival reductions
// (ld_agent / last_arrival: kernels/bn_tail.h)

// ---------------------------------------------------------------- BatchNorm
// stats slab [rows][2][C] -> mean / invstd (+ running stats with torch's semantics:
// momentum, unbiased running variance; + num_batches_tracked).  Latency-bound (a few KB
// per layer), so the kernel is built around memory round trips: grid (ceil(C/64), G),
// block (strip, y) owns rows [y*RPB, (y+1)*RPB) (RPB = 64 up to 4096 rows); its 4 row
// phases x 64 channels issue ALL their loads (16 rows each) before summing in row order,
// phases combined in order -> ws[y].  G == 1 finalises straight away (no ticket, one
// round trip); otherwise the strip's last block (ticket) sums ws[0..G) the same way
// (G <= 64: one batch) and finalises.
constexpr int BNF_RPB = 64;
constexpr int BNF_MAXG = 64;

// rows [r0, r1) (<= 64 of them) of a [rows][2][C] slab, channel c: phase grp sums rows
// r0 + grp, r0 + grp + 4, ... (all 16 loads in flight), in order
template <bool AGENT>
__device__ __forceinline__ void bnf_rows(const float* slab, long C2, int C, int c, int r0, int r1, int grp,
                                         float& s, float& q) {
  s = q = 0.f;
  for (int rb = r0; rb < r1; rb += 64) {  // one batch unless a block owns > 64 rows
    float a[16], b[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int r = rb + grp + 4 * u;
      const bool ok = r < r1;
      const float* p = slab + (long)(ok ? r : r0) * C2 + c;
      a[u] = ok ? (AGENT ? ld_agent(p) : *p) : 0.f;
      b[u] = ok ? (AGENT ? ld_agent(p + C) : p[C]) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (rb + grp + 4 * u < r1) { s += a[u]; q += b[u]; }
    }
  }
}

__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ slab, int rows,
                                                          int C, float count, float eps, float momentum,
                                                          float* __restrict__ running_mean,
                                                          float* __restrict__ running_var,
                                                          float* __restrict__ save_mean,
                                                          float* __restrict__ save_invstd,
                                                          long long* __restrict__ nbt,
                                                          float* __restrict__ ws, int* __restrict__ tickets,
                                                          int rpb) {
  __shared__ float ps[4][64], pq[4][64];
  __shared__ int s_last;
  const int l = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + l;
  const int G = gridDim.y, y = blockIdx.y;
  const long C2 = 2L * C;
  float s = 0.f, q = 0.f;
  if (c < C) bnf_rows<false>(slab, C2, C, c, y * rpb, min(rows, (y + 1) * rpb), grp, s, q);
  ps[grp][l] = s;
  pq[grp][l] = q;
  __syncthreads();
  if (G > 1) {
    if (grp == 0 && c < C) {
      st_wt(ws + (long)y * C2 + c, ((ps[0][l] + ps[1][l]) + ps[2][l]) + ps[3][l]);
      st_wt(ws + (long)y * C2 + C + c, ((pq[0][l] + pq[1][l]) + pq[2][l]) + pq[3][l]);
    }
    if (!last_arrival(&tickets[blockIdx.x], G, &s_last)) return;
    s = q = 0.f;
    if (c < C) bnf_rows<true>(ws, C2, C, c, 0, G, grp, s, q);
    __syncthreads();
    ps[grp][l] = s;
    pq[grp][l] = q;
    __syncthreads();
  }
  if (grp == 0 && c < C) {
    const float S = ((ps[0][l] + ps[1][l]) + ps[2][l]) + ps[3][l];
    const float Q = ((pq[0][l] + pq[1][l]) + pq[2][l]) + pq[3][l];
    const float mean = S / count;
    const float var = fmaxf(Q / count - mean * mean, 0.f);
    save_mean[c] = mean;
    save_invstd[c] = rsqrtf(var + eps);
    if (running_mean) {
      const float unb = count > 1.f ? var * count / (count - 1.f) : var;
      running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
    }
  }
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
}

__device__ __forceinline__ void ld8f(const float* p, float* o) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
__device__ __forceinline__ void unpack8(bf16x8 v, float* o) {
  const uint4 u = __builtin_bit_cast(uint4, v);
  unpack4(make_uint2(u.x, u.y), o);
  unpack4(make_uint2(u.z, u.w), o + 4);
}
// Upstream gradient of a tensor with two consumers (ResNet block input: the conv branch and
// the residual branch): d = bf16(d1 + d2), the exact value autograd's separate bf16 add
// kernel would have produced - fused into the loads of the kernel that consumes the sum.
__device__ __forceinline__ void unpack8_sum(bf16x8 a, const bf16_t* b2, long off, float* o) {
  unpack8(a, o);
  if (b2) {
    float t[8];
    unpack8(ld8(b2 + off), t);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = bf16_round(o[j] + t[j]);
  }
}
// ReLU mask source of the BatchNorm backward: MSK 0 none, 1 the saved output (out > 0),
// 2 recomputed from the BN input y: bf16(y * sc + sh) > 0 - bitwise the stored output's
// sign (same affine, same rounding), for BatchNorms without a residual add; saves the
// read of the output tensor in both backward passes.
template <int MSK>
__device__ __forceinline__ void bn_mask8(bf16x8 go, const float* xv, const float* msc, const float* msh,
                                         float* d) {
  if constexpr (MSK == 1) {
    float ov[8];
    unpack8(go, ov);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (!(ov[j] > 0.f)) d[j] = 0.f;
  } else if constexpr (MSK == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (!(bf16_round(fmaf(xv[j], msc[j], msh[j])) > 0.f)) d[j] = 0.f;
  }
}

__device__ __forceinline__ uint4 pack8(const float* v) {
  const uint2 lo = pack4(v[0], v[1], v[2], v[3]), hi = pack4(v[4], v[5], v[6], v[7]);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

// (bn_affine8: kernels/bn_affine.h - shared with the consumer-side applications)

// y = act(x * sc + sh [+ res]), sc = invstd * gamma, sh = beta - mean * sc; 8 channels per
// thread.  The grid stride is a multiple of C/8 (which divides 256), so a thread's
// channel group - and its 16 per-channel constants - never change.
template <bool RES, bool RELU>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t* __restrict__ x, long n8, int C,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta,
                                                       const bf16_t* __restrict__ res,
                                                       bf16_t* __restrict__ y) {
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  const int c0 = (int)(t0 % (C / 8)) * 8;
  float sc[8], sh[8];
  bn_affine8(invstd, gamma, mean, beta, c0, sc, sh);
  for (long i = t0; i < n8; i += stride) {
    float v[8], r[8];
    unpack8(ld8(x + i * 8), v);
    if (RES) unpack8(ld8(res + i * 8), r);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = fmaf(v[j], sc[j], sh[j]);
      if (RES) v[j] += r[j];
      if (RELU) v[j] = fmaxf(v[j], 0.f);
    }
    *reinterpret_cast<uint4*>(y + i * 8) = pack8(v);
  }
}

// Backward pass 1: sums of dy and dy * xhat per channel, dy = the gradient w.r.t. the BN
// output masked by the ReLU (out > 0) when RELU.  grid (C/64, R): block = 8 channel
// groups (64 channels) x 32 pixel lanes over `rpb` pixels -> ws[y]; the strip's last
// block sums ws[0..R) in fixed order into sums[2C] = [sum dy | sum dy*xhat] and the
// affine gradients (dbeta = sum dy, dgamma = sum dy*xhat; `accum` adds to them).
//
// (A one-launch variant - every block applying pass 2 to its own pixels after an in-launch
// wait for the strip's sums - measured slower at every ResNet-18 layer and was removed in
// round 5: profiles/r3_bn_fusion.)
template <int MSK>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const bf16_t* __restrict__ dout,
                                                            const bf16_t* __restrict__ dout2,
                                                            const bf16_t* __restrict__ out,
                                                            const bf16_t* __restrict__ x, int P, int C,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, int rpb,
                                                            float* __restrict__ ws, int* __restrict__ tickets,
                                                            float* __restrict__ sums,
                                                            float* __restrict__ dgamma,
                                                            float* __restrict__ dbeta, int accum,
                                                            const float* __restrict__ mgamma,
                                                            const float* __restrict__ mbeta) {
  __shared__ float sred[32][2][64];
  __shared__ float sfin[8][128];
  __shared__ int s_last;
  const int tg = threadIdx.x & 7, tp = threadIdx.x >> 3;
  const int cb = blockIdx.x * 64;
  const int c0 = cb + tg * 8;
  float mu[8], is[8], s[8], q[8];
  ld8f(mean + c0, mu);
  ld8f(invstd + c0, is);
  float msc[8], msh[8];  // MSK 2: the forward's affine (bn_affine8)
  if constexpr (MSK == 2) bn_affine8(invstd, mgamma, mean, mbeta, c0, msc, msh);
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  const int p0 = blockIdx.y * rpb, p1 = min(P, p0 + rpb);
  auto acc8 = [&](bf16x8 gd, long off, bf16x8 gx, bf16x8 go) {
    float d[8], xv[8];
    unpack8_sum(gd, dout2, off, d);
    unpack8(gx, xv);
    bn_mask8<MSK>(go, xv, msc, msh, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] += d[j];
      q[j] = fmaf(d[j], (xv[j] - mu[j]) * is[j], q[j]);
    }
  };
  int p = p0 + tp;
  // groups of four pixels (a block streams ~150 KB at layer1; with two in flight the pass
  // was latency-bound at ~2.2 TB/s), software-pipelined: group k + 1's loads (dout2's
  // too) are issued before group k is summed, so a block waits out about one memory round
  // trip instead of one per group (256 blocks = one 4-wave block per CU: nothing else
  // hides it).  Then two, then one pixel - the per-thread summation order is pixel order.
  bf16x8 gd[2][4], gx[2][4], gr[2][4], g2[2][4];
  auto load_g = [&](int pp, auto SET) {
    constexpr int st = decltype(SET)::value;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long o = (long)(pp + 32 * u) * C + c0;
      gd[st][u] = ld8(dout + o);
      gx[st][u] = ld8(x + o);
      gr[st][u] = MSK == 1 ? ld8(out + o) : zero8();
      g2[st][u] = dout2 ? ld8(dout2 + o) : zero8();
    }
  };
  auto sum_g = [&](auto SET) {
    constexpr int st = decltype(SET)::value;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float d[8], xv[8];
      unpack8(gd[st][u], d);
      if (dout2) {  // unpack8_sum's add, on the prefetched second gradient
        float t[8];
        unpack8(g2[st][u], t);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = bf16_round(d[j] + t[j]);
      }
      unpack8(gx[st][u], xv);
      bn_mask8<MSK>(gr[st][u], xv, msc, msh, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += d[j];
        q[j] = fmaf(d[j], (xv[j] - mu[j]) * is[j], q[j]);
      }
    }
  };
  const int n4 = p1 - p - 96 > 0 ? (p1 - p - 96 + 127) / 128 : 0;  // groups with p + 96 < p1
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  if (n4 > 0) load_g(p, S0{});
  for (int k = 0; k < n4; k += 2) {
    if (k + 1 < n4) load_g(p + 128 * (k + 1), S1{});
    sum_g(S0{});
    if (k + 1 < n4) {
      if (k + 2 < n4) load_g(p + 128 * (k + 2), S0{});
      sum_g(S1{});
    }
  }
  p += 128 * n4;
  for (; p + 32 < p1; p += 64) {  // two pixels' loads in flight
    const long o0 = (long)p * C + c0, o1 = o0 + 32L * C;
    const bf16x8 d0 = ld8(dout + o0), x0 = ld8(x + o0), d1 = ld8(dout + o1), x1 = ld8(x + o1);
    const bf16x8 r0 = MSK == 1 ? ld8(out + o0) : zero8(), r1 = MSK == 1 ? ld8(out + o1) : zero8();
    acc8(d0, o0, x0, r0);
    acc8(d1, o1, x1, r1);
  }
  for (; p < p1; p += 32) {
    const long o0 = (long)p * C + c0;
    acc8(ld8(dout + o0), o0, ld8(x + o0), MSK == 1 ? ld8(out + o0) : zero8());
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sred[tp][0][tg * 8 + j] = s[j];
    sred[tp][1][tg * 8 + j] = q[j];
  }
  __syncthreads();
  const int R = gridDim.y;
  const int v = threadIdx.x & 127, which = v >> 6, cc = v & 63;
  if (threadIdx.x < 128) {
    float a = 0.f;
    for (int t = 0; t < 32; ++t) a += sred[t][which][cc];
    st_wt(ws + ((long)blockIdx.y * 2 + which) * C + cb + cc, a);
  }
  if (!last_arrival(&tickets[blockIdx.x], R, &s_last)) return;
  // Fixed-order sum of the R partial rows: thread = 4 of the strip's 128 values (float4)
  // x one of 8 row phases, up to 8 rows in flight.  Plain loads are coherent here: the
  // rows were stored write-through and no block of this kernel read them before.
  {
    const int vq = threadIdx.x & 31, ph = threadIdx.x >> 5;
    const int wh = vq >> 4, c4 = (vq & 15) * 4;
    const float* src = ws + (long)wh * C + cb + c4;
    float4 a4 = make_float4(0.f, 0.f, 0.f, 0.f);
    int yy = ph;
    for (; yy + 56 < R; yy += 64) {
      float4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = *reinterpret_cast<const float4*>(src + (long)(yy + 8 * u) * 2 * C);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a4.x += t[u].x; a4.y += t[u].y; a4.z += t[u].z; a4.w += t[u].w;
      }
    }
    for (; yy < R; yy += 8) {
      const float4 t = *reinterpret_cast<const float4*>(src + (long)yy * 2 * C);
      a4.x += t.x; a4.y += t.y; a4.z += t.z; a4.w += t.w;
    }
    float* sp = &sfin[ph][wh * 64 + c4];
    sp[0] = a4.x; sp[1] = a4.y; sp[2] = a4.z; sp[3] = a4.w;
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    float tot = sfin[0][v];
#pragma unroll
    for (int k = 1; k < 8; ++k) tot += sfin[k][v];
    const int c = cb + cc;
    sums[which * C + c] = tot;
    float* dst = which ? dgamma : dbeta;
    if (dst) dst[c] = accum ? dst[c] + tot : tot;
  }
}

// Backward pass 2: dx = gamma*invstd/count * (count*dy - sum_dy - xhat*sum_dyxh); also
// writes the residual-branch gradient (= dy masked) when dres != null.  Same
// fixed-channel-group grid stride as bn_apply.
template <int MSK>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16_t* __restrict__ dout,
                                                           const bf16_t* __restrict__ dout2,
                                                           const bf16_t* __restrict__ out,
                                                           const bf16_t* __restrict__ x, long n8,
                                                           int C, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ sums,
                                                           float count, bf16_t* __restrict__ dx,
                                                           bf16_t* __restrict__ dres,
                                                           const float* __restrict__ mbeta) {
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  const int c0 = (int)(t0 % (C / 8)) * 8;
  float mu[8], is[8], k[8], sd[8], sq[8];
  ld8f(mean + c0, mu);
  ld8f(invstd + c0, is);
  ld8f(gamma + c0, k);
  ld8f(sums + c0, sd);
  ld8f(sums + C + c0, sq);
  float msc[8], msh[8];
  if constexpr (MSK == 2) bn_affine8(invstd, gamma, mean, mbeta, c0, msc, msh);
#pragma unroll
  for (int j = 0; j < 8; ++j) k[j] = k[j] * is[j] / count;
  for (long i = t0; i < n8; i += stride) {
    float d[8], xv[8], o[8];
    unpack8_sum(ld8(dout + i * 8), dout2, i * 8, d);
    unpack8(ld8(x + i * 8), xv);
    bn_mask8<MSK>(MSK == 1 ? ld8(out + i * 8) : zero8(), xv, msc, msh, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xh = (xv[j] - mu[j]) * is[j];
      o[j] = k[j] * (count * d[j] - sd[j] - xh * sq[j]);
    }
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(o);
    if (dres) *reinterpret_cast<uint4*>(dres + i * 8) = pack8(d);
  }
}

// ---------------------------------------------------------------- pooling
// 3x3 / stride 2 / pad 1 max pool, 8 channels per thread (16-B loads); argmax (window
// index 0..8, first max in row-major window order = torch's tie rule) saved as uint8.
// AFF: x is the stem conv's raw output and the window reads the BatchNorm + ReLU of it
// (bn_apply's exact value, bn_affine8): the stem's bn_apply pass (51 MB read + write at
// batch 32) disappears; the BN backward recomputes its mask from x (MSK 2).
template <bool AFF>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16_t* __restrict__ x, int N, int H,
                                                          int W, int C, int OH, int OW,
                                                          bf16_t* __restrict__ y,
                                                          unsigned char* __restrict__ amax, BnAffine bn) {
  const int cg = C / 8;
  const int total = N * OH * OW * cg;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int g8 = (i % cg) * 8;
  float sc[8], sh[8];
  if constexpr (AFF) bn_affine8(bn.invstd, bn.gamma, bn.mean, bn.beta, g8, sc, sh);
  const int p = i / cg;
  const int n = p / (OH * OW);
  const int r = p - n * OH * OW;
  const int oh = r / OW, ow = r - oh * OW;
  float best[8];
  unsigned bi[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0u; }
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int ih = oh * 2 - 1 + k / 3, iw = ow * 2 - 1 + k % 3;
    if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
      float v[8];
      unpack8(ld8(x + (((long)n * H + ih) * W + iw) * C + g8), v);
      if constexpr (AFF) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = bf16_round(fmaxf(fmaf(v[j], sc[j], sh[j]), 0.f));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (v[j] > best[j] || (v[j] != v[j] && best[j] == best[j])) { best[j] = v[j]; bi[j] = k; }
    }
  }
  const long o = (long)p * C + g8;
  *reinterpret_cast<uint4*>(y + o) = pack8(best);
  *reinterpret_cast<uint2*>(amax + o) =
      make_uint2(bi[0] | bi[1] << 8 | bi[2] << 16 | bi[3] << 24, bi[4] | bi[5] << 8 | bi[6] << 16 | bi[7] << 24);
}

// Gather form of the backward (deterministic).  One thread per 2x2 input quad (rows 2a,
// 2a+1 x cols 2b, 2b+1) and 8 channels: with stride 2 the quad's pixels are covered only
// by the windows (a|a+1, b|b+1), so the thread loads those four dy / argmax vectors once
// (a per-pixel gather loads 9 per quad) and sums each pixel's matches in the window order
// kh, kw = 0..2 (bitwise equal to the per-pixel form).
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16_t* __restrict__ dy,
                                                          const bf16_t* __restrict__ dy2,
                                                          const unsigned char* __restrict__ amax,
                                                          int N, int H, int W, int C, int OH, int OW,
                                                          bf16_t* __restrict__ dx) {
  const int cg = C / 8;
  const int QH = (H + 1) / 2, QW = (W + 1) / 2;
  const int total = N * QH * QW * cg;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int g8 = (i % cg) * 8;
  const int q = i / cg;
  const int n = q / (QH * QW);
  const int r = q - n * QH * QW;
  const int qa = r / QW, qb = r - qa * QW;
  float d[2][2][8];
  uint2 am[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int oh = qa + u, ow = qb + v;
      if (oh < OH && ow < OW) {
        const long o = (((long)n * OH + oh) * OW + ow) * C + g8;
        am[u][v] = *reinterpret_cast<const uint2*>(amax + o);
        unpack8_sum(ld8(dy + o), dy2, o, d[u][v]);
      } else {
        am[u][v] = make_uint2(0xffffffffu, 0xffffffffu);  // matches no tap
#pragma unroll
        for (int j = 0; j < 8; ++j) d[u][v][j] = 0.f;
      }
    }
#pragma unroll
  for (int dr = 0; dr < 2; ++dr) {
    const int ih = 2 * qa + dr;
    if (ih >= H) continue;
#pragma unroll
    for (int dc = 0; dc < 2; ++dc) {
      const int iw = 2 * qb + dc;
      if (iw >= W) continue;
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
      // even row: window row qa at kh = 1; odd row: qa + 1 at kh = 0, then qa at kh = 2
#pragma unroll
      for (int ru = 0; ru < (dr ? 2 : 1); ++ru) {
        const int u = dr ? 1 - ru : 0, kh = dr ? 2 * ru : 1;
#pragma unroll
        for (int cv = 0; cv < (dc ? 2 : 1); ++cv) {
          const int v = dc ? 1 - cv : 0, kw = dc ? 2 * cv : 1;
          const unsigned kk = kh * 3 + kw;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const unsigned bsel = ((j < 4 ? am[u][v].x : am[u][v].y) >> (8 * (j & 3))) & 0xffu;
            if (bsel == kk) acc[j] += d[u][v][j];
          }
        }
      }
      *reinterpret_cast<uint4*>(dx + (((long)n * H + ih) * W + iw) * C + g8) = pack8(acc);
    }
  }
}

// global average pool: [N][HW][C] bf16 -> [N][C] fp32.  Block = (n, 64 channels): 8 channel
// groups (16-B loads) x 32 pixel lanes, lanes summed in fixed order through LDS.
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const bf16_t* __restrict__ x, int N, int HW,
                                                          int C, float* __restrict__ y) {
  __shared__ float s_p[32][65];
  const int n = blockIdx.x, c0 = blockIdx.y * 64;
  const int cgp = threadIdx.x & 7, pl = threadIdx.x >> 3;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int p = pl; p < HW; p += 32) {
    float v[8];
    unpack8(ld8(x + ((long)n * HW + p) * C + c0 + cgp * 8), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) s_p[pl][cgp * 8 + j] = acc[j];
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = 0.f;
    for (int l = 0; l < 32; ++l) t += s_p[l][threadIdx.x];
    y[(long)n * C + c0 + threadIdx.x] = t / (float)HW;
  }
}

__global__ void avgpool_bwd_kernel(const float* __restrict__ dy, int N, int HW, int C,
                                   bf16_t* __restrict__ dx) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)N * HW * C) return;
  const int c = (int)(i % C);
  const int n = (int)(i / ((long)HW * C));
  dx[i] = f2bf(dy[(long)n * C + c] / (float)HW);
}

// ---------------------------------------------------------------- classifier loss
// Mean softmax cross-entropy over [B][C] fp32 logits (C <= 1024) for wide heads: one wave
// per row (4 rows per block, B/4 blocks) instead of one block looping over the rows.
// Per-row losses go out write-through; the last block sums them in row order.
constexpr int XR_M = 16;
__global__ __launch_bounds__(256) void xent_wave_rows_kernel(const float* __restrict__ logits, int C,
                                                             int B, const long long* __restrict__ labels,
                                                             float* __restrict__ dlogits,
                                                             float* __restrict__ loss_out,
                                                             float* __restrict__ ws, int* __restrict__ ticket,
                                                             float gscale) {
  __shared__ int s_last;
  const int lane = threadIdx.x & 63, b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b < B) {
    const int label = (int)labels[b];
    float x[XR_M];
    float mx = -INFINITY;
#pragma unroll
    for (int m = 0; m < XR_M; ++m) {
      const int c = lane + 64 * m;
      x[m] = c < C ? logits[(long)b * C + c] : -INFINITY;
      mx = fmaxf(mx, x[m]);
    }
    mx = wave_max(mx);
    float se = 0.f, xl = 0.f;
#pragma unroll
    for (int m = 0; m < XR_M; ++m) {
      const int c = lane + 64 * m;
      if (c == label) xl = x[m];
      x[m] = c < C ? __expf(x[m] - mx) : 0.f;
      se += x[m];
    }
    se = wave_sum(se);
    xl = wave_sum(xl);  // logit[label]
    const float inv = 1.f / se;
#pragma unroll
    for (int m = 0; m < XR_M; ++m) {
      const int c = lane + 64 * m;
      if (c < C) dlogits[(long)b * C + c] = (x[m] * inv - (c == label ? 1.f : 0.f)) * gscale;
    }
    if (lane == 0) st_wt(ws + b, mx + __logf(se) - xl);
  }
  if (!last_arrival(ticket, gridDim.x, &s_last)) return;
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int r = 0; r < B; ++r) t += ld_agent(ws + r);
    loss_out[0] = t / (float)B;
  }
}

// ---------------------------------------------------------------- input pipeline
// Device-resident uint8 RGB images [N][HW][3] + batch indices -> the stem's input:
// NHWC bf16 [B][HW][4] = u8 / 255 with the 4th channel zero (one pixel per thread,
// 3-byte read, 8-byte write).
__global__ __launch_bounds__(256) void image_gather_nhwc4_kernel(const unsigned char* __restrict__ imgs,
                                                                 const long long* __restrict__ idx,
                                                                 int B, int HW, long N,
                                                                 bf16_t* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * HW) return;
  const int b = (int)(i / HW);
  const int p = (int)(i - (long)b * HW);
  long n = idx[b];
  n = n < 0 ? 0 : (n >= N ? N - 1 : n);  // host validates; never read out of bounds
  const unsigned char* src = imgs + (n * HW + p) * 3;
  const float k = 1.f / 255.f;
  *reinterpret_cast<uint2*>(out + i * 4) = pack4(src[0] * k, src[1] * k, src[2] * k, 0.f);
}

// ---------------------------------------------------------------- small fp32 GEMM
// C[m][n] = alpha * sum_k A(m,k) B(k,n) + (bias ? bias[n] : 0), A(m,k) = A[m*sam + k*sak],
// B(k,n) = B[k*sbk + n*sbn]; A/B element type float or bf16 (template).  16x16 LDS
// tiles; used for the 512 -> 1000 classifier head fwd/bwd.
template <typename TA, typename TB>
__global__ __launch_bounds__(256) void sgemm_kernel(int M, int N, int K, const TA* __restrict__ A,
                                                    long sam, long sak, const TB* __restrict__ B,
                                                    long sbk, long sbn, float* __restrict__ Cm,
                                                    long ldc, const float* __restrict__ bias,
                                                    float alpha, int accum) {
  __shared__ float sA[16][17], sB[16][17];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m = blockIdx.y * 16 + ty, n = blockIdx.x * 16 + tx;
  float acc = 0.f;
  auto ld = [](const auto* p, long i) -> float {
    if constexpr (sizeof(*p) == 2) return bf2f(reinterpret_cast<const bf16_t*>(p)[i]);
    else return reinterpret_cast<const float*>(p)[i];
  };
  for (int k0 = 0; k0 < K; k0 += 16) {
    const int ka = k0 + tx, kb = k0 + ty;
    sA[ty][tx] = (m < M && ka < K) ? ld(A, (long)m * sam + (long)ka * sak) : 0.f;
    sB[ty][tx] = (kb < K && n < N) ? ld(B, (long)kb * sbk + (long)n * sbn) : 0.f;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) acc = fmaf(sA[ty][k], sB[k][tx], acc);
    __syncthreads();
  }
  if (m < M && n < N) {
    float v = alpha * acc + (bias ? bias[n] : 0.f);
    if (accum) v += Cm[(long)m * ldc + n];  // direct gradient accumulation (C += A.B)
    Cm[(long)m * ldc + n] = v;
  }
}

// Small-M fp32 GEMM (M <= 32: the classifier head's batch rows) on v_mfma_f32_16x16x4_f32:
// block = 16 waves over one 32 x 16 output tile, the K range split across the waves (each
// wave: two 16x16 accumulators), partial tiles summed through LDS in fixed wave order
// (deterministic).  Exact fp32 products; long K (512 / 1000) spreads over 16 waves
// instead of one 16x16 VALU tile walking all of it.
constexpr int SMM_WAVES = 16;
template <typename TA, typename TB>
__global__ __launch_bounds__(64 * SMM_WAVES) void gemm_small_m_kernel(
    int M, int N, int K, const TA* __restrict__ A, long sam, long sak, const TB* __restrict__ B, long sbk,
    long sbn, float* __restrict__ Cm, long ldc, const float* __restrict__ bias, float alpha, int accum) {
  __shared__ float red[SMM_WAVES][32][17];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16;
  auto ld = [](const auto* p, long i) -> float {
    if constexpr (sizeof(*p) == 2) return bf2f(reinterpret_cast<const bf16_t*>(p)[i]);
    else return reinterpret_cast<const float*>(p)[i];
  };
  const int kq = ((K + SMM_WAVES - 1) / SMM_WAVES + 3) & ~3;  // this wave's K range (multiple of 4)
  const int kb = wave * kq, ke = min(K, kb + kq);
  const int r = lane & 15, kl = lane >> 4;
  const int n = n0 + r;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = kb; k0 < ke; k0 += 32) {
    float a0[8], a1[8], bv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {  // 8 MFMA steps' operands in flight
      const int k = k0 + 4 * u + kl;
      const bool kok = k < ke;
      a0[u] = (kok && r < M) ? ld(A, (long)r * sam + (long)k * sak) : 0.f;
      a1[u] = (kok && r + 16 < M) ? ld(A, (long)(r + 16) * sam + (long)k * sak) : 0.f;
      bv[u] = (kok && n < N) ? ld(B, (long)k * sbk + (long)n * sbn) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[u], bv[u], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[u], bv[u], acc1, 0, 0, 0);
    }
  }
  // D[row = 4(l>>4) + j][col = l & 15]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[wave][4 * kl + j][r] = acc0[j];
    red[wave][16 + 4 * kl + j][r] = acc1[j];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 32 * 16; t += 64 * SMM_WAVES) {
    const int m = t >> 4, c = t & 15, nn = n0 + c;
    if (m >= M || nn >= N) continue;
    float v = red[0][m][c];
#pragma unroll
    for (int w = 1; w < SMM_WAVES; ++w) v += red[w][m][c];
    v = alpha * v + (bias ? bias[nn] : 0.f);
    if (accum) v += Cm[(long)m * ldc + nn];
    Cm[(long)m * ldc + nn] = v;
  }
}

// OHWI [Co][T][Ci] (fp32 master) -> bf16 [Ci][T][Co] (conv_gemm dgrad operand)
__global__ void transpose_w_kernel(const float* __restrict__ w, int Co, int T, int Ci,
                                   bf16_t* __restrict__ wt) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Co * T * Ci) return;
  const int ci = (int)(i % Ci);
  const int t = (int)((i / Ci) % T);
  const int co = (int)(i / ((long)Ci * T));
  wt[((long)ci * T + t) * Co + co] = f2bf(w[i]);
}

// ---------------------------------------------------------------- launchers
static unsigned grid_for(long n, int per_thread = 1) {
  const long t = (n + per_thread - 1) / per_thread;
  const long b = (t + 255) / 256;
  return (unsigned)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

// Ticket words for last_arrival: one zeroed pool per device, handed out round-robin
// (every kernel resets the tickets it used, so a slot is clean when it comes round).
int* bn_ticket_slots(int n) {
  constexpr int kSlots = 1 << 16;
  static int* pool[64] = {};
  static int next[64] = {};
  int dev = 0;
  RN_CHECK(hipGetDevice(&dev));
  dev &= 63;
  if (!pool[dev]) {
    RN_CHECK(hipMalloc(reinterpret_cast<void**>(&pool[dev]), sizeof(int) * kSlots));
    RN_CHECK(hipMemset(pool[dev], 0, sizeof(int) * kSlots));
    RN_CHECK(hipDeviceSynchronize());
  }
  if (next[dev] + n > kSlots) next[dev] = 0;
  int* p = pool[dev] + next[dev];
  next[dev] += n;
  return p;
}

// blocks per strip: one per BNF_RPB rows (more only past BNF_MAXG * BNF_RPB rows)
static int bnf_rpb(int rows) {
  int r = BNF_RPB;
  while ((rows + r - 1) / r > BNF_MAXG) r *= 2;
  return r;
}
int bn_finalize_groups(int rows) { return (rows + bnf_rpb(rows) - 1) / bnf_rpb(rows); }

void bn_finalize(const float* slab, int rows, int C, float count, float eps, float momentum,
                 float* running_mean, float* running_var, float* save_mean, float* save_invstd,
                 long long* nbt, float* ws, hipStream_t s) {
  const int strips = (C + 63) / 64, G = bn_finalize_groups(rows), rpb = bnf_rpb(rows);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(strips, G), dim3(256), 0, s, slab, rows, C, count, eps,
                     momentum, running_mean, running_var, save_mean, save_invstd, nbt, ws,
                     G > 1 ? bn_ticket_slots(strips) : nullptr, rpb);
}

void bn_apply(const bf16_t* x, long P, int C, const float* mean, const float* invstd,
              const float* gamma, const float* beta, const bf16_t* res, bool relu, bf16_t* y,
              hipStream_t s) {
  const unsigned g = grid_for(P * C, 8);
#define BA(R, L) hipLaunchKernelGGL((bn_apply_kernel<R, L>), dim3(g), dim3(256), 0, s, x, P * C / 8, C, mean, invstd, gamma, beta, res, y)
  if (res) { if (relu) BA(true, true); else BA(true, false); }
  else { if (relu) BA(false, true); else BA(false, false); }
#undef BA
}

// Rows of the reduce grid: about 392 pixels per block.  The last-arrival tail (write-through
// partials, R same-address ticket increments, the last block's R-row sum) grows with R,
// so small layers want few fat blocks: scripts/bn_sweep.py at batch 32 measured
// 13.1 -> 8.5 us (7x7x512), 14.9 -> 10.8 us (14x14x256), 19.8 -> 15.4 us (28x28x128)
// against a fixed 512-block grid.  Settable for the sweep; ws is sized by bn_bwd_rows at
// the same setting.
static int g_bn_bwd_px = 392;
void bn_bwd_set_px_per_block(int px) { g_bn_bwd_px = px < 32 ? 32 : px; }

int bn_bwd_rows(long P, int C, int* rpb) {
  // (a floor of ~256 blocks for the deep layers' few pixels measured 0.9 % slower: more
  // partial rows for the last block to sum, profiles/r4_resnet/bn_bwd)
  (void)C;
  long R = P / g_bn_bwd_px;
  if (R > 256) R = 256;
  if (R < 1) R = 1;
  const long r = (P + R - 1) / R;
  if (rpb) *rpb = (int)r;
  return (int)((P + r - 1) / r);
}

void bn_bwd(const bf16_t* dout, const bf16_t* out, const bf16_t* x, long P, int C, const float* mean,
            const float* invstd, const float* gamma, float count, float* ws, float* sums,
            float* dgamma, float* dbeta, bool accum, bf16_t* dx, bf16_t* dres, hipStream_t s,
            const bf16_t* dout2, const float* mask_beta) {
  int rpb = 0;
  const int R = bn_bwd_rows(P, C, &rpb);
  const dim3 grid(C / 64, R);
  int* tk = bn_ticket_slots(C / 64);
  // ReLU mask: the saved output, or (no output given, mask_beta given) recomputed from x
  const int msk = out ? 1 : (mask_beta ? 2 : 0);
#define BNR(M) hipLaunchKernelGGL((bn_bwd_reduce_kernel<M>), grid, dim3(256), 0, s, dout, dout2, out, x, (int)P, C, mean, invstd, rpb, ws, tk, sums, dgamma, dbeta, (int)accum, gamma, mask_beta)
  if (msk == 1) BNR(1); else if (msk == 2) BNR(2); else BNR(0);
#undef BNR
  const unsigned g = grid_for(P * C, 8);
#define BNA(M) hipLaunchKernelGGL(bn_bwd_apply_kernel<M>, dim3(g), dim3(256), 0, s, dout, dout2, out, x, P * C / 8, C, mean, invstd, gamma, sums, count, dx, dres, mask_beta)
  if (msk == 1) BNA(1); else if (msk == 2) BNA(2); else BNA(0);
#undef BNA
}

void maxpool_fwd(const bf16_t* x, int N, int H, int W, int C, int OH, int OW, bf16_t* y,
                 unsigned char* amax, hipStream_t s, const BnAffine* bn) {
  const long total = (long)N * OH * OW * (C / 8);
  const dim3 grid((unsigned)((total + 255) / 256));
  if (bn && bn->mean)
    hipLaunchKernelGGL(maxpool_fwd_kernel<true>, grid, dim3(256), 0, s, x, N, H, W, C, OH, OW, y, amax, *bn);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<false>, grid, dim3(256), 0, s, x, N, H, W, C, OH, OW, y, amax, BnAffine{});
}

void maxpool_bwd(const bf16_t* dy, const unsigned char* amax, int N, int H, int W, int C, int OH,
                 int OW, bf16_t* dx, hipStream_t s, const bf16_t* dy2) {
  const long total = (long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, dy,
                     dy2, amax, N, H, W, C, OH, OW, dx);
}

void image_gather_nhwc4(const unsigned char* imgs, const long long* idx, int B, int HW, long N,
                        bf16_t* out, hipStream_t s) {
  const long total = (long)B * HW;
  hipLaunchKernelGGL(image_gather_nhwc4_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                     imgs, idx, B, HW, N, out);
}

void avgpool_fwd(const bf16_t* x, int N, int HW, int C, float* y, hipStream_t s) {
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(N, C / 64), dim3(256), 0, s, x, N, HW, C, y);
}

bool xent_wave_rows(const float* logits, int C, int B, const long long* labels, float* dlogits,
                    float* loss_out, float gscale, hipStream_t s) {
  constexpr int kMaxB = 8192;
  if (C > 64 * XR_M || B > kMaxB || B < 1) return false;
  static float* wsp[64] = {};
  int dev = 0;
  RN_CHECK(hipGetDevice(&dev));
  dev &= 63;
  if (!wsp[dev]) RN_CHECK(hipMalloc(reinterpret_cast<void**>(&wsp[dev]), sizeof(float) * kMaxB));
  hipLaunchKernelGGL(xent_wave_rows_kernel, dim3((B + 3) / 4), dim3(256), 0, s, logits, C, B, labels,
                     dlogits, loss_out, wsp[dev], bn_ticket_slots(1), gscale);
  return true;
}

void avgpool_bwd(const float* dy, int N, int HW, int C, bf16_t* dx, hipStream_t s) {
  const long total = (long)N * HW * C;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, dy, N,
                     HW, C, dx);
}

void sgemm(int M, int N, int K, const void* A, bool a_bf16, long sam, long sak, const void* B,
           bool b_bf16, long sbk, long sbn, float* C, long ldc, const float* bias, float alpha,
           hipStream_t s, bool accum) {
  if (M <= 32 && K >= 64) {  // long-K, few rows: the MFMA small-M kernel
    const dim3 g2((N + 15) / 16);
#define SM(TA, TB) hipLaunchKernelGGL((gemm_small_m_kernel<TA, TB>), g2, dim3(64 * SMM_WAVES), 0, s, M, N, K, (const TA*)A, sam, sak, (const TB*)B, sbk, sbn, C, ldc, bias, alpha, (int)accum)
    if (a_bf16) { if (b_bf16) SM(bf16_t, bf16_t); else SM(bf16_t, float); }
    else { if (b_bf16) SM(float, bf16_t); else SM(float, float); }
#undef SM
    return;
  }
  const dim3 grid((N + 15) / 16, (M + 15) / 16);
#define SG(TA, TB) hipLaunchKernelGGL((sgemm_kernel<TA, TB>), grid, dim3(256), 0, s, M, N, K, (const TA*)A, sam, sak, (const TB*)B, sbk, sbn, C, ldc, bias, alpha, (int)accum)
  if (a_bf16) { if (b_bf16) SG(bf16_t, bf16_t); else SG(bf16_t, float); }
  else { if (b_bf16) SG(float, bf16_t); else SG(float, float); }
#undef SG
}

void transpose_w(const float* w, int Co, int T, int Ci, bf16_t* wt, hipStream_t s) {
  const long n = (long)Co * T * Ci;
  hipLaunchKernelGGL(transpose_w_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, Co, T,
                     Ci, wt);
}

}  // namespace ddp_amd
