// Skinny Linear layer over an NHWC-flattened bf16 activation (SimpleCNN's fc,
// reference model.py:16,19: nn.Linear(50176, 10)).
//
// The weight is kept in the activation's memory order, [out][H*W][C] (bf16
// shadow of the fp32 master), so both passes stream it contiguously.  The
// checkpoint still stores the reference's NCHW-flatten [out][C*H*W] order: the
// permutation happens only at save/load (ddp_amd/models/layers.py).
//
//  fc_partial : per-16-pixel-tile partial logits (fixed-order split-K); the fused
//               engine gets these from the conv2 epilogue instead.
//  fc_reduce  : logits[b][o] = bias[o] + sum_g part[b][g][o] (fixed order).
//  fc_bwd     : one pass over the activation computing
//                 dX[b][k] = (MASK ? X>0 : 1) * sum_o dL[b][o] W[o][k]      (bf16)
//                 dW[o][k] = scale * sum_b dL[b][o] X[b][k]                    (fp32)
//               i.e. fc dgrad + fc wgrad + ReLU2 mask fused;
//               dW is written straight into the gradient bucket, prescaled.
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

constexpr int FC_MAXO = 16;

__global__ __launch_bounds__(256) void fc_partial_kernel(const bf16_t* __restrict__ X,
                                                         const bf16_t* __restrict__ Wf,
                                                         float* __restrict__ part, int B, int HW,
                                                         int C, int NO) {
  const int lane = threadIdx.x & 63;
  const long tile = (long)blockIdx.x * 4 + (threadIdx.x >> 6);  // 16-pixel tile over B*HW
  const int G = HW / 16;
  if (tile >= (long)B * G) return;
  const int n = (int)(tile / G), g = (int)(tile - (long)n * G);
  const long xoff = ((long)n * HW + g * 16) * C;
  const long woff = (long)g * 16 * C;
  const int te = 16 * C;
  float s[FC_MAXO];
#pragma unroll
  for (int o = 0; o < FC_MAXO; ++o) s[o] = 0.f;
  for (int e = lane * 8; e < te; e += 512) {
    const bf16x8 xv = ld8(X + xoff + e);
#pragma unroll
    for (int o = 0; o < FC_MAXO; ++o) {
      if (o < NO) {
        const bf16x8 wv = ld8(Wf + (long)o * HW * C + woff + e);
        float a = s[o];
#pragma unroll
        for (int j = 0; j < 8; ++j) a = fmaf(bf2f((bf16_t)xv[j]), bf2f((bf16_t)wv[j]), a);
        s[o] = a;
      }
    }
  }
#pragma unroll
  for (int o = 0; o < FC_MAXO; ++o)
    if (o < NO) {
      const float t = wave_sum(s[o]);
      if (lane == 0) part[tile * NO + o] = t;
    }
}

__global__ void fc_reduce_kernel(const float* __restrict__ part, const float* __restrict__ bias,
                                 float* __restrict__ out, int B, int G, int NO) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * NO) return;
  const int b = i / NO, o = i - (i / NO) * NO;
  float s = 0.f;
  for (int g = 0; g < G; ++g) s += part[((long)b * G + g) * NO + o];
  out[i] = s + (bias ? bias[o] : 0.f);
}

template <bool MASK, bool XENT>
__global__ __launch_bounds__(256) void fc_bwd_kernel(const float* __restrict__ dL,
                                                     const bf16_t* __restrict__ X,
                                                     const bf16_t* __restrict__ Wf,
                                                     bf16_t* __restrict__ dX, float* __restrict__ dW,
                                                     float scale, int B, long K, int NO,
                                                     FcBwdExtras ex) {
  extern __shared__ __attribute__((aligned(16))) float s_dl[];  // [B][NO] (+ [B] row losses)
  if (XENT) {
    // every block recomputes the (tiny) cross-entropy backward: B rows, one wave per row
    const int base = ex.bi.base();
    for (int b = threadIdx.x >> 6; b < B; b += 4) {
      const int label = ex.labels32[ex.bi.row(b, base)];
      const float l = xent_row_wave(ex.part + (long)b * NO * ex.G, ex.G, ex.fc_bias, NO, label,
                                    ex.gscale, s_dl + b * NO);
      if ((threadIdx.x & 63) == 0) s_dl[B * NO + b] = l;
    }
  } else {
    for (int i = threadIdx.x; i < B * NO; i += 256) s_dl[i] = dL[i];
  }
  __syncthreads();
  if (blockIdx.x == 0) {
    // fc bias gradient (sum over the batch, fixed order) and the batch-mean loss
    if (ex.dbias && threadIdx.x < NO) {
      float acc = 0.f;
      for (int b = 0; b < B; ++b) acc += s_dl[b * NO + threadIdx.x];
      ex.dbias[threadIdx.x] = acc * ex.dbias_scale;
    }
    if ((XENT || ex.loss_rows) && ex.loss_out && threadIdx.x == 64) {
      const float* lr = XENT ? s_dl + B * NO : ex.loss_rows;
      float acc = 0.f;
      for (int b = 0; b < B; ++b) acc += lr[b];
      ex.loss_out[ex.step_ctr ? *ex.step_ctr : 0] = acc / (float)B;
    }
  }
  const long k = (long)blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  float w[FC_MAXO], dw[FC_MAXO];
#pragma unroll
  for (int o = 0; o < FC_MAXO; ++o) {
    w[o] = (o < NO) ? bf2f(Wf[(long)o * K + k]) : 0.f;
    dw[o] = 0.f;
  }
  // 32 rows per chunk: all activation loads of the chunk are issued before any math
  for (int b0 = 0; b0 < B; b0 += 32) {
    const int nb = min(32, B - b0);
    float xa[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) xa[u] = (u < nb) ? bf2f(X[(long)(b0 + u) * K + k]) : 0.f;
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      if (u < nb) {
        const float* dl = s_dl + (b0 + u) * NO;
        float dz = 0.f;
#pragma unroll
        for (int o = 0; o < FC_MAXO; ++o)
          if (o < NO) {
            dz = fmaf(dl[o], w[o], dz);
            dw[o] = fmaf(dl[o], xa[u], dw[o]);
          }
        if (MASK && !(xa[u] > 0.f)) dz = 0.f;
        dX[(long)(b0 + u) * K + k] = f2bf(dz);
      }
    }
  }
#pragma unroll
  for (int o = 0; o < FC_MAXO; ++o)
    if (o < NO) dW[(long)o * K + k] = dw[o] * scale;
}

void fc_partial(const bf16_t* X, const bf16_t* Wf, float* part, int B, int HW, int C, int NO,
                hipStream_t s) {
  const long tiles = (long)B * (HW / 16);
  hipLaunchKernelGGL(fc_partial_kernel, dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, s, X, Wf,
                     part, B, HW, C, NO);
}

void fc_reduce(const float* part, const float* bias, float* out, int B, int G, int NO,
               hipStream_t s) {
  hipLaunchKernelGGL(fc_reduce_kernel, dim3((B * NO + 255) / 256), dim3(256), 0, s, part, bias, out,
                     B, G, NO);
}

void fc_bwd(const float* dL, const bf16_t* X, const bf16_t* Wf, bf16_t* dX, float* dW, float scale,
            int B, long K, int NO, bool mask, hipStream_t s, const FcBwdExtras& ex) {
  const dim3 grid((unsigned)((K + 255) / 256));
  const bool xe = ex.part != nullptr;
  const size_t lds = sizeof(float) * B * (NO + (xe ? 1 : 0));
#define LB(M, XE) hipLaunchKernelGGL((fc_bwd_kernel<M, XE>), grid, dim3(256), lds, s, dL, X, Wf, dX, dW, scale, B, K, NO, ex)
  if (xe) { if (mask) LB(true, true); else LB(false, true); }
  else { if (mask) LB(true, false); else LB(false, false); }
#undef LB
}

}  // namespace ddp_amd
