// Non-convolution ResNet-18 kernels on NHWC bf16 activations (BASELINE.json config 5;
// SURVEY.md §2.4 north-star list: BatchNorm2d train-mode fwd/bwd with running stats,
// MaxPool 3x3/s2, global average pool, residual add, fc head).
//
// BatchNorm statistics come from the producing convolution's epilogue (per-block
// per-channel sum / sum-of-squares slabs, conv_gemm.hip); bn_finalize reduces them
// in fixed order and updates the running buffers with torch's semantics (momentum
// 0.1, unbiased running variance).  bn_apply fuses normalise + affine + residual
// add + ReLU.  The backward is two passes: per-block partial sums of dy and
// dy*xhat (with the ReLU mask from the saved output), then the per-element
// input gradient.  All reductions are fixed-order (no atomics).
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

// ---------------------------------------------------------------- BatchNorm
// stats slab [nblk][2][C] -> mean/invstd (+ running stats).  Block = 64 channels x 4 groups.
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ slab, int nblk,
                                                          int C, float count, float eps, float momentum,
                                                          float* __restrict__ running_mean,
                                                          float* __restrict__ running_var,
                                                          float* __restrict__ save_mean,
                                                          float* __restrict__ save_invstd) {
  __shared__ float ps[4][64], pq[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), grp = threadIdx.x >> 6;
  float s = 0.f, q = 0.f;
  if (c < C)
    for (int b = grp; b < nblk; b += 4) {
      s += slab[(long)b * 2 * C + c];
      q += slab[(long)b * 2 * C + C + c];
    }
  ps[grp][threadIdx.x & 63] = s;
  pq[grp][threadIdx.x & 63] = q;
  __syncthreads();
  if (grp == 0 && c < C) {
    const int l = threadIdx.x;
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
}

// y = act((x - mean) * invstd * gamma + beta [+ res]); 8 channels per thread.
template <bool RES, bool RELU>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t* __restrict__ x, long P, int C,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta,
                                                       const bf16_t* __restrict__ res,
                                                       bf16_t* __restrict__ y) {
  const long n8 = P * C / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    const int c0 = (int)((i * 8) % C);
    const bf16x8 xv = ld8(x + i * 8);
    bf16x8 rv = zero8();
    if (RES) rv = ld8(res + i * 8);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      float v = (bf2f((bf16_t)xv[j]) - mean[c]) * invstd[c] * gamma[c] + beta[c];
      if (RES) v += bf2f((bf16_t)rv[j]);
      if (RELU) v = fmaxf(v, 0.f);
      o[j] = v;
    }
    uint4 pk;
    const uint2 lo = pack4(o[0], o[1], o[2], o[3]), hi = pack4(o[4], o[5], o[6], o[7]);
    pk.x = lo.x; pk.y = lo.y; pk.z = hi.x; pk.w = hi.y;
    *reinterpret_cast<uint4*>(y + i * 8) = pk;
  }
}

// Backward pass 1: per-block partials of sum(dy) and sum(dy * xhat), where dy is the
// gradient w.r.t. the BN output masked by the ReLU (out > 0) when RELU.  Block = 256
// threads = (256 / (C/8)) pixel lanes x (C/8) channel groups over `rows` pixels.
template <bool RELU>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const bf16_t* __restrict__ dout,
                                                            const bf16_t* __restrict__ out,
                                                            const bf16_t* __restrict__ x, long P,
                                                            int C, const float* __restrict__ mean,
                                                            const float* __restrict__ invstd,
                                                            float* __restrict__ slab, int rows) {
  extern __shared__ __attribute__((aligned(16))) float sred[];  // [pl][2][C]
  const int cg = C / 8;
  const int pl = 256 / cg;  // pixel lanes
  const int tg = threadIdx.x % cg, tp = threadIdx.x / cg;
  float s[8], q[8], mu[8], is[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s[j] = q[j] = 0.f;
    mu[j] = mean[tg * 8 + j];
    is[j] = invstd[tg * 8 + j];
  }
  const long p0 = (long)blockIdx.x * rows;
  const long p1 = min(P, p0 + rows);
  if (tp < pl)
    for (long p = p0 + tp; p < p1; p += pl) {
      const long off = p * C + tg * 8;
      const bf16x8 g = ld8(dout + off), xv = ld8(x + off);
      bf16x8 ov = zero8();
      if (RELU) ov = ld8(out + off);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float d = bf2f((bf16_t)g[j]);
        if (RELU && !(bf2f((bf16_t)ov[j]) > 0.f)) d = 0.f;
        const float xh = (bf2f((bf16_t)xv[j]) - mu[j]) * is[j];
        s[j] += d;
        q[j] = fmaf(d, xh, q[j]);
      }
    }
  if (tp < pl) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sred[(tp * 2) * C + tg * 8 + j] = s[j];
      sred[(tp * 2 + 1) * C + tg * 8 + j] = q[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float S = 0.f, Q = 0.f;
    for (int t = 0; t < pl; ++t) {
      S += sred[(t * 2) * C + c];
      Q += sred[(t * 2 + 1) * C + c];
    }
    slab[(long)blockIdx.x * 2 * C + c] = S;
    slab[(long)blockIdx.x * 2 * C + C + c] = Q;
  }
}

// Backward pass 2: dx = gamma*invstd/count * (count*dy - sum_dy - xhat*sum_dyxh); also
// writes the residual-branch gradient (= dy masked) when dres != null.
template <bool RELU>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16_t* __restrict__ dout,
                                                           const bf16_t* __restrict__ out,
                                                           const bf16_t* __restrict__ x, long P,
                                                           int C, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ sums,
                                                           float count, bf16_t* __restrict__ dx,
                                                           bf16_t* __restrict__ dres) {
  const long n8 = P * C / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    const int c0 = (int)((i * 8) % C);
    const bf16x8 g = ld8(dout + i * 8), xv = ld8(x + i * 8);
    bf16x8 ov = zero8();
    if (RELU) ov = ld8(out + i * 8);
    float o[8], dm[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      float d = bf2f((bf16_t)g[j]);
      if (RELU && !(bf2f((bf16_t)ov[j]) > 0.f)) d = 0.f;
      dm[j] = d;
      const float xh = (bf2f((bf16_t)xv[j]) - mean[c]) * invstd[c];
      const float k = gamma[c] * invstd[c] / count;
      o[j] = k * (count * d - sums[c] - xh * sums[C + c]);
    }
    uint4 pk;
    uint2 lo = pack4(o[0], o[1], o[2], o[3]), hi = pack4(o[4], o[5], o[6], o[7]);
    pk.x = lo.x; pk.y = lo.y; pk.z = hi.x; pk.w = hi.y;
    *reinterpret_cast<uint4*>(dx + i * 8) = pk;
    if (dres) {
      lo = pack4(dm[0], dm[1], dm[2], dm[3]);
      hi = pack4(dm[4], dm[5], dm[6], dm[7]);
      pk.x = lo.x; pk.y = lo.y; pk.z = hi.x; pk.w = hi.y;
      *reinterpret_cast<uint4*>(dres + i * 8) = pk;
    }
  }
}

// ---------------------------------------------------------------- pooling
// 3x3 / stride 2 / pad 1 max pool; argmax (window index 0..8, first max in row-major
// window order = torch's tie rule) saved as uint8 for the backward.
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16_t* __restrict__ x, int N, int H,
                                                          int W, int C, int OH, int OW,
                                                          bf16_t* __restrict__ y,
                                                          unsigned char* __restrict__ amax) {
  const long total = (long)N * OH * OW * C;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  const long p = i / C;
  const int n = (int)(p / ((long)OH * OW));
  const int r = (int)(p - (long)n * OH * OW);
  const int oh = r / OW, ow = r - (r / OW) * OW;
  float best = -INFINITY;
  int bi = 0;
  for (int k = 0; k < 9; ++k) {
    const int ih = oh * 2 - 1 + k / 3, iw = ow * 2 - 1 + k % 3;
    if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
      const float v = bf2f(x[(((long)n * H + ih) * W + iw) * C + c]);
      if (v > best || (v != v && best == best)) { best = v; bi = k; }  // NaN propagates like torch
    }
  }
  y[i] = f2bf(best);
  amax[i] = (unsigned char)bi;
}

// Gather form of the backward (deterministic): each input element sums dy over the
// (at most 4) windows that selected it.
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16_t* __restrict__ dy,
                                                          const unsigned char* __restrict__ amax,
                                                          int N, int H, int W, int C, int OH, int OW,
                                                          bf16_t* __restrict__ dx) {
  const long total = (long)N * H * W * C;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  const long p = i / C;
  const int n = (int)(p / ((long)H * W));
  const int r = (int)(p - (long)n * H * W);
  const int ih = r / W, iw = r - (r / W) * W;
  float acc = 0.f;
  for (int kh = 0; kh < 3; ++kh) {
    const int th = ih + 1 - kh;
    if (th < 0 || (th & 1)) continue;
    const int oh = th >> 1;
    if (oh >= OH) continue;
    for (int kw = 0; kw < 3; ++kw) {
      const int tw = iw + 1 - kw;
      if (tw < 0 || (tw & 1)) continue;
      const int ow = tw >> 1;
      if (ow >= OW) continue;
      const long o = (((long)n * OH + oh) * OW + ow) * C + c;
      if (amax[o] == kh * 3 + kw) acc += bf2f(dy[o]);
    }
  }
  dx[i] = f2bf(acc);
}

// global average pool: [N][HW][C] bf16 -> [N][C] fp32 (thread per (n, c), fixed order)
__global__ void avgpool_fwd_kernel(const bf16_t* __restrict__ x, int N, int HW, int C,
                                   float* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i - (i / C) * C;
  float s = 0.f;
  for (int p = 0; p < HW; ++p) s += bf2f(x[((long)n * HW + p) * C + c]);
  y[i] = s / (float)HW;
}

__global__ void avgpool_bwd_kernel(const float* __restrict__ dy, int N, int HW, int C,
                                   bf16_t* __restrict__ dx) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)N * HW * C) return;
  const int c = (int)(i % C);
  const int n = (int)(i / ((long)HW * C));
  dx[i] = f2bf(dy[(long)n * C + c] / (float)HW);
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
                                                    float alpha) {
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
  if (m < M && n < N) Cm[(long)m * ldc + n] = alpha * acc + (bias ? bias[n] : 0.f);
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

void bn_finalize(const float* slab, int nblk, int C, float count, float eps, float momentum,
                 float* running_mean, float* running_var, float* save_mean, float* save_invstd,
                 hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, s, slab, nblk, C, count,
                     eps, momentum, running_mean, running_var, save_mean, save_invstd);
}

void bn_apply(const bf16_t* x, long P, int C, const float* mean, const float* invstd,
              const float* gamma, const float* beta, const bf16_t* res, bool relu, bf16_t* y,
              hipStream_t s) {
  const unsigned g = grid_for(P * C, 8);
#define BA(R, L) hipLaunchKernelGGL((bn_apply_kernel<R, L>), dim3(g), dim3(256), 0, s, x, P, C, mean, invstd, gamma, beta, res, y)
  if (res) { if (relu) BA(true, true); else BA(true, false); }
  else { if (relu) BA(false, true); else BA(false, false); }
#undef BA
}

int bn_bwd_blocks(long P, int rows) { return (int)((P + rows - 1) / rows); }

void bn_bwd_reduce(const bf16_t* dout, const bf16_t* out, const bf16_t* x, long P, int C,
                   const float* mean, const float* invstd, float* slab, int rows, hipStream_t s) {
  const int pl = 256 / (C / 8);
  const size_t lds = sizeof(float) * pl * 2 * C;
  const dim3 grid(bn_bwd_blocks(P, rows));
  if (out)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<true>, grid, dim3(256), lds, s, dout, out, x, P, C, mean, invstd, slab, rows);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<false>, grid, dim3(256), lds, s, dout, out, x, P, C, mean, invstd, slab, rows);
}

void bn_bwd_apply(const bf16_t* dout, const bf16_t* out, const bf16_t* x, long P, int C,
                  const float* mean, const float* invstd, const float* gamma, const float* sums,
                  float count, bf16_t* dx, bf16_t* dres, hipStream_t s) {
  const unsigned g = grid_for(P * C, 8);
  if (out)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(g), dim3(256), 0, s, dout, out, x, P, C, mean, invstd, gamma, sums, count, dx, dres);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<false>, dim3(g), dim3(256), 0, s, dout, out, x, P, C, mean, invstd, gamma, sums, count, dx, dres);
}

void maxpool_fwd(const bf16_t* x, int N, int H, int W, int C, int OH, int OW, bf16_t* y,
                 unsigned char* amax, hipStream_t s) {
  const long total = (long)N * OH * OW * C;
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, x, N,
                     H, W, C, OH, OW, y, amax);
}

void maxpool_bwd(const bf16_t* dy, const unsigned char* amax, int N, int H, int W, int C, int OH,
                 int OW, bf16_t* dx, hipStream_t s) {
  const long total = (long)N * H * W * C;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, dy,
                     amax, N, H, W, C, OH, OW, dx);
}

void avgpool_fwd(const bf16_t* x, int N, int HW, int C, float* y, hipStream_t s) {
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((N * C + 255) / 256), dim3(256), 0, s, x, N, HW, C, y);
}

void avgpool_bwd(const float* dy, int N, int HW, int C, bf16_t* dx, hipStream_t s) {
  const long total = (long)N * HW * C;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, dy, N,
                     HW, C, dx);
}

void sgemm(int M, int N, int K, const void* A, bool a_bf16, long sam, long sak, const void* B,
           bool b_bf16, long sbk, long sbn, float* C, long ldc, const float* bias, float alpha,
           hipStream_t s) {
  const dim3 grid((N + 15) / 16, (M + 15) / 16);
#define SG(TA, TB) hipLaunchKernelGGL((sgemm_kernel<TA, TB>), grid, dim3(256), 0, s, M, N, K, (const TA*)A, sam, sak, (const TB*)B, sbk, sbn, C, ldc, bias, alpha)
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
