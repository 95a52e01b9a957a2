// Fused softmax cross-entropy forward + backward (reference train_ddp.py:40,198:
// nn.CrossEntropyLoss(), mean reduction).
//
// One workgroup of 4 waves; wave w owns rows b = w, w+4, ...; lane l owns
// classes c = l, l+64, ...  Per row: logits = bias + sum_g partials (fixed
// order: the split-K partial logits of the fc layer), max / sum-exp by wave
// butterflies, loss_b = logsumexp - logit[label],
// dlogits = (softmax - onehot) * gscale (gscale = 1/B for the mean).
// Also produces the fc bias gradient sum_b dlogits (prescaled for DDP) and the
// mean loss as a device scalar that the host reads only when it logs
// (every 100 batches, reference train_ddp.py:201-202).
// Labels come either from an int64 tensor or from the device-resident dataset
// labels through the epoch index list (BatchIdx).
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

constexpr int XE_MAXM = 16;  // up to 1024 classes

__global__ __launch_bounds__(1024) void xent_kernel(const float* __restrict__ part, int G,
                                                   const float* __restrict__ bias, int C, int B,
                                                   const long long* __restrict__ labels64,
                                                   const int* __restrict__ labels32, BatchIdx bi,
                                                   float* __restrict__ logits_out,
                                                   float* __restrict__ dlogits,
                                                   float* __restrict__ loss_out,
                                                   float* __restrict__ dbias, float gscale,
                                                   float dbias_scale) {
  __shared__ float s_loss[16];
  __shared__ float s_db[4][XE_MAXM * 64];  // dbias: 4 waves only (see xent())
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int M = (C + 63) / 64;
  float db[XE_MAXM];
#pragma unroll
  for (int m = 0; m < XE_MAXM; ++m) db[m] = 0.f;
  float lsum = 0.f;
  const int base = labels32 ? bi.base() : 0;
  for (int b = wave; b < B; b += nw) {
    const int label = labels64 ? (int)labels64[b] : labels32[bi.row(b, base)];
    float x[XE_MAXM];
    float mx = -INFINITY;
#pragma unroll
    for (int m = 0; m < XE_MAXM; ++m) {
      const int c = lane + 64 * m;
      x[m] = -INFINITY;
      if (m < M && c < C) {
        float s = 0.f;
        for (int g = 0; g < G; ++g) s += part[((long)b * G + g) * C + c];
        x[m] = s + (bias ? bias[c] : 0.f);
        if (logits_out) logits_out[(long)b * C + c] = x[m];
        mx = fmaxf(mx, x[m]);
      }
    }
    mx = wave_max(mx);
    float se = 0.f, xl = 0.f;
#pragma unroll
    for (int m = 0; m < XE_MAXM; ++m) {
      const int c = lane + 64 * m;
      if (m < M && c < C) {
        se += __expf(x[m] - mx);
        if (c == label) xl = x[m];
      }
    }
    se = wave_sum(se);
    xl = wave_sum(xl);
    const float lse = mx + __logf(se);
    lsum += lse - xl;
    const float inv = 1.f / se;
#pragma unroll
    for (int m = 0; m < XE_MAXM; ++m) {
      const int c = lane + 64 * m;
      if (m < M && c < C) {
        const float d = (__expf(x[m] - mx) * inv - (c == label ? 1.f : 0.f)) * gscale;
        dlogits[(long)b * C + c] = d;
        db[m] += d;
      }
    }
  }
  if (lane == 0) s_loss[wave] = lsum;
  if (dbias) {
#pragma unroll
    for (int m = 0; m < XE_MAXM; ++m)
      if (m < M) s_db[wave][lane + 64 * m] = db[m];
  }
  __syncthreads();
  // graph-replayed steps log their loss into a per-epoch history indexed by the step counter
  if (threadIdx.x == 0 && loss_out) {
    float t = s_loss[0];
    for (int w = 1; w < nw; ++w) t += s_loss[w];
    loss_out[bi.step_ctr ? *bi.step_ctr : 0] = t / (float)B;
  }
  if (dbias)
    for (int c = threadIdx.x; c < C; c += 256)
      dbias[c] = (((s_db[0][c] + s_db[1][c]) + s_db[2][c]) + s_db[3][c]) * dbias_scale;
}

// Engine variant (fusion level 0): one workgroup over the per-block partial logits
// [blk][2][NO] written by the fused conv2 epilogue, see xent_batch_block (common.h).
// Writes per-row loss and dlogits; the batch mean loss and the fc bias gradient are
// finished by fc_bwd's first block (it holds dlogits).
__global__ __launch_bounds__(1024) void xent_rows_kernel(const float* __restrict__ part, int HW, int CH,
                                                        const float* __restrict__ bias, int NO,
                                                        int B, const int* __restrict__ labels32,
                                                        BatchIdx bi, float* __restrict__ dlogits,
                                                        float* __restrict__ loss_rows,
                                                        float gscale) {
  extern __shared__ float s_lg[];  // [B][NO] logits, then [B] labels
  xent_batch_block(part, HW, CH, bias, NO, B, labels32, bi, gscale, dlogits, loss_rows, s_lg,
                   reinterpret_cast<int*>(s_lg + B * NO));
}

void xent_rows(const float* part, int HW, int CH, const float* bias, int NO, int B,
               const int* labels32, BatchIdx bi, float* dlogits, float* loss_rows, float gscale,
               hipStream_t s) {
  const int threads = B * NO <= 256 ? 256 : (B * NO <= 512 ? 512 : 1024);
  hipLaunchKernelGGL(xent_rows_kernel, dim3(1), dim3(threads), sizeof(float) * B * (NO + 1), s, part, HW, CH,
                     bias, NO, B, labels32, bi, dlogits, loss_rows, gscale);
}

void xent(const float* part, int G, const float* bias, int C, int B, const long long* labels64,
          const int* labels32, BatchIdx bi, float* logits_out, float* dlogits, float* loss_out,
          float* dbias, float gscale, float dbias_scale, hipStream_t s) {
  // one wave per row when there is no bias gradient to fold (it is reduced over 4 waves)
  if (G == 1 && !bias && !dbias && !logits_out && labels64 && !bi.step_ctr && C > 64 &&
      xent_wave_rows(part, C, B, labels64, dlogits, loss_out, gscale, s))
    return;
  const int waves = dbias ? 4 : (B < 16 ? (B < 4 ? 4 : B) : 16);
  hipLaunchKernelGGL(xent_kernel, dim3(1), dim3(64 * waves), 0, s, part, G, bias, C, B, labels64, labels32,
                     bi, logits_out, dlogits, loss_out, dbias, gscale, dbias_scale);
}

DDP_STAMPS_SETTER(stamps_set_xent)

}  // namespace ddp_amd
