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

// fc backward: a block owns 256 consecutive columns k (4 per lane, 8-byte loads)
// and its 4 waves split the batch rows (wave w: rows w, w+4, ...), so every wave has
// its rows' loads in flight at once; the per-wave dW partials are summed in fixed
// wave order through LDS.  NOT = compile-time class capacity (guards o < NO).
template <bool MASK, bool XENT, int NOT>
__global__ __launch_bounds__(256) void fc_bwd_kernel(const float* __restrict__ dL,
                                                     const bf16_t* __restrict__ X,
                                                     const bf16_t* __restrict__ Wf,
                                                     bf16_t* __restrict__ dX, float* __restrict__ dW,
                                                     float scale, int B, long K, int NO,
                                                     FcBwdExtras ex) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* s_dl = smem;                 // [B][NO]
  float* s_loss = smem + B * NO;      // [B]        (XENT)
  float* s_red = smem + (XENT ? B * (NO + 1) : B * NO);  // [3][NO][256] wave partials
  s_red = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(s_red) + 15) & ~(uintptr_t)15);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (XENT) {
    // every block recomputes the (tiny) cross-entropy backward of the whole batch
    xent_batch_block(ex.part, ex.G, ex.fc_bias, NO, B, ex.labels32, ex.bi, ex.gscale, s_dl, s_loss);
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
      const float* lr = XENT ? s_loss : ex.loss_rows;
      float acc = 0.f;
      for (int b = 0; b < B; ++b) acc += lr[b];
      ex.loss_out[ex.step_ctr ? *ex.step_ctr : 0] = acc / (float)B;
    }
  }
  const long k0 = (long)blockIdx.x * 256 + lane * 4;
  const bool active = k0 < K;  // host guarantees K % 4 == 0
  float w[NOT][4], dw[NOT][4];
#pragma unroll
  for (int o = 0; o < NOT; ++o) {
    float t[4] = {0.f, 0.f, 0.f, 0.f};
    if (active && o < NO) unpack4(*reinterpret_cast<const uint2*>(Wf + (long)o * K + k0), t);
#pragma unroll
    for (int c = 0; c < 4; ++c) { w[o][c] = t[c]; dw[o][c] = 0.f; }
  }
  constexpr int RB = 8;  // rows in flight per wave
  for (int b0 = wave; b0 < B; b0 += 4 * RB) {
    uint2 xr[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int b = b0 + 4 * u;
      xr[u] = (active && b < B) ? *reinterpret_cast<const uint2*>(X + (long)b * K + k0) : make_uint2(0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int b = b0 + 4 * u;
      if (b < B) {
        float xa[4];
        unpack4(xr[u], xa);
        const float* dl = s_dl + b * NO;
        float dz[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int o = 0; o < NOT; ++o)
          if (o < NO) {
            const float d = dl[o];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              dz[c] = fmaf(d, w[o][c], dz[c]);
              dw[o][c] = fmaf(d, xa[c], dw[o][c]);
            }
          }
        if (MASK) {
#pragma unroll
          for (int c = 0; c < 4; ++c) dz[c] = xa[c] > 0.f ? dz[c] : 0.f;
        }
        if (active) *reinterpret_cast<uint2*>(dX + (long)b * K + k0) = pack4(dz[0], dz[1], dz[2], dz[3]);
      }
    }
  }
  // fixed-order reduction of the 4 waves' dW partials
  if (wave > 0) {
#pragma unroll
    for (int o = 0; o < NOT; ++o)
      if (o < NO)
        *reinterpret_cast<float4*>(s_red + ((wave - 1) * NO + o) * 256 + lane * 4) =
            make_float4(dw[o][0], dw[o][1], dw[o][2], dw[o][3]);
  }
  __syncthreads();
  if (wave == 0 && active) {
#pragma unroll
    for (int o = 0; o < NOT; ++o)
      if (o < NO) {
        float4 r = make_float4(dw[o][0], dw[o][1], dw[o][2], dw[o][3]);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const float4 t = *reinterpret_cast<const float4*>(s_red + (q * NO + o) * 256 + lane * 4);
          r.x += t.x; r.y += t.y; r.z += t.z; r.w += t.w;
        }
        r.x *= scale; r.y *= scale; r.z *= scale; r.w *= scale;
        *reinterpret_cast<float4*>(dW + (long)o * K + k0) = r;
      }
  }
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

size_t fc_bwd_lds(int B, int NO, bool xent) {
  return sizeof(float) * ((size_t)B * (xent ? NO + 1 : NO) + 4 + (size_t)3 * NO * 256);
}

void fc_bwd(const float* dL, const bf16_t* X, const bf16_t* Wf, bf16_t* dX, float* dW, float scale,
            int B, long K, int NO, bool mask, hipStream_t s, const FcBwdExtras& ex) {
  const dim3 grid((unsigned)((K + 255) / 256));
  const bool xe = ex.part != nullptr;
  const size_t lds = fc_bwd_lds(B, NO, xe);
#define LB(M, XE, N) hipLaunchKernelGGL((fc_bwd_kernel<M, XE, N>), grid, dim3(256), lds, s, dL, X, Wf, dX, dW, scale, B, K, NO, ex)
  if (NO == 10) {
    if (xe) { if (mask) LB(true, true, 10); else LB(false, true, 10); }
    else { if (mask) LB(true, false, 10); else LB(false, false, 10); }
  } else {
    if (xe) { if (mask) LB(true, true, FC_MAXO); else LB(false, true, FC_MAXO); }
    else { if (mask) LB(true, false, FC_MAXO); else LB(false, false, FC_MAXO); }
  }
#undef LB
}

}  // namespace ddp_amd
