// Skinny Linear layer over an NHWC-flattened bf16 or fp32 activation (SimpleCNN's fc,
// reference model.py:16,19: nn.Linear(50176, 10)).  The fp32 instantiations (--dtype fp32)
// read the fp32 master weight itself - no shadow copy.
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
#include <stdexcept>

#include "kernels/common.h"
#include "kernels/fc_bwd_body.h"
#include "kernels/launchers.h"

namespace ddp_amd {

constexpr int FC_MAXO = 16;

__device__ __forceinline__ void ld8f(const bf16_t* p, float* o) {
  const bf16x8 v = ld8(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = bf2f((bf16_t)v[j]);
}
__device__ __forceinline__ void ld8f(const float* p, float* o) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

template <typename T>
__global__ __launch_bounds__(256) void fc_partial_kernel(const T* __restrict__ X,
                                                         const T* __restrict__ Wf,
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
    float xv[8];
    ld8f(X + xoff + e, xv);
#pragma unroll
    for (int o = 0; o < FC_MAXO; ++o) {
      if (o < NO) {
        float wv[8];
        ld8f(Wf + (long)o * HW * C + woff + e, wv);
        float a = s[o];
#pragma unroll
        for (int j = 0; j < 8; ++j) a = fmaf(xv[j], wv[j], a);
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

// fc backward (body: fc_bwd_body.h): 8 waves of 2 columns per lane, one virtual wave per
// physical wave (the fused level-2 launch runs the same body at 4 waves x 2 virtual waves
// and gets bit-identical results).
constexpr int FCB_WPB = 8, FCB_CPL = 2, FCB_COLS = 64 * FCB_CPL;

template <typename T, bool MASK, bool XENT, int NOT, int WPB, bool DXO = true>
__global__ __launch_bounds__(WPB * 64) void fc_bwd_kernel(const float* __restrict__ dL,
                                                          const T* __restrict__ X,
                                                          const T* __restrict__ Wf,
                                                          T* __restrict__ dX,
                                                          float* __restrict__ dW, float scale,
                                                          int B, long K, int NO_rt,
                                                          FcBwdExtras ex) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  fc_bwd_body<T, MASK, XENT, NOT, WPB, WPB, FCB_CPL, DXO>(dL, X, Wf, dX, dW, scale, B, K, NO_rt, ex, smem,
                                                          blockIdx.x, nullptr);
}

void fc_partial(const bf16_t* X, const bf16_t* Wf, float* part, int B, int HW, int C, int NO,
                hipStream_t s) {
  const long tiles = (long)B * (HW / 16);
  hipLaunchKernelGGL(fc_partial_kernel<bf16_t>, dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, s, X, Wf,
                     part, B, HW, C, NO);
}
void fc_partial(const float* X, const float* Wf, float* part, int B, int HW, int C, int NO,
                hipStream_t s) {
  const long tiles = (long)B * (HW / 16);
  hipLaunchKernelGGL(fc_partial_kernel<float>, dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, s, X, Wf,
                     part, B, HW, C, NO);
}

void fc_reduce(const float* part, const float* bias, float* out, int B, int G, int NO,
               hipStream_t s) {
  hipLaunchKernelGGL(fc_reduce_kernel, dim3((B * NO + 255) / 256), dim3(256), 0, s, part, bias, out,
                     B, G, NO);
}

// npart: floats of the cross-entropy prologue's partial-logit copy (aliases s_red)
size_t fc_bwd_lds(int B, int NO, bool xent, long npart) {
  const int red = NO == 10 ? fcb_red_floats<FCB_WPB, 10, FCB_CPL>() : fcb_red_floats<FCB_WPB, FC_MAXO, FCB_CPL>();
  return sizeof(float) * (size_t)fcb_lds_floats(B, NO, xent, npart, red);
}

template <typename T>
static void fc_bwd_launch(const float* dL, const T* X, const T* Wf, T* dX, float* dW, float scale,
                          int B, long K, int NO, bool mask, hipStream_t s, const FcBwdExtras& ex) {
  const dim3 grid((unsigned)((K + FCB_COLS - 1) / FCB_COLS));
  const bool xe = ex.part != nullptr;
  if (xe && ((long)B * ex.HW >= (1L << 31) || ex.CH <= 0 || ex.HW / ex.CH + 2 > XENT_MAX_BLK))
    throw std::runtime_error("fc_bwd: cross-entropy prologue geometry out of range");
  const long npart = xe ? (((long)B * ex.HW + ex.CH - 1) / ex.CH) * 2 * NO : 0;
  const size_t lds = fc_bwd_lds(B, NO, xe, npart);
  if (lds > 65536) {
#define OPT(M, XE, N) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fc_bwd_kernel<T, M, XE, N, FCB_WPB>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)
    OPT(true, true, 10); OPT(false, true, 10); OPT(true, true, FC_MAXO); OPT(false, true, FC_MAXO);
#undef OPT
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fc_bwd_kernel<T, false, true, 10, FCB_WPB, false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fc_bwd_kernel<T, false, false, 10, FCB_WPB, false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  }
  if (ex.last_ctr && (NO != 10 || dX))
    throw std::runtime_error("fc_bwd: the last-block epilogue is the level-3 variant (10 classes, no dX)");
#define LB(M, XE, N) hipLaunchKernelGGL((fc_bwd_kernel<T, M, XE, N, FCB_WPB>), grid, dim3(FCB_WPB * 64), lds, s, dL, X, Wf, dX, dW, scale, B, K, NO, ex)
  if (!dX) {  // level 3: no data gradient (the conv forward produced dZ2); dL from the prologue or given
    if (NO != 10 || (!xe && !dL)) throw std::runtime_error("fc_bwd: dX == nullptr needs 10 classes and dL (or its prologue)");
    if (xe)
      hipLaunchKernelGGL((fc_bwd_kernel<T, false, true, 10, FCB_WPB, false>), grid, dim3(FCB_WPB * 64), lds, s, dL, X,
                         Wf, dX, dW, scale, B, K, NO, ex);
    else
      hipLaunchKernelGGL((fc_bwd_kernel<T, false, false, 10, FCB_WPB, false>), grid, dim3(FCB_WPB * 64), lds, s, dL,
                         X, Wf, dX, dW, scale, B, K, NO, ex);
  } else if (NO == 10) {
    if (xe) { if (mask) LB(true, true, 10); else LB(false, true, 10); }
    else { if (mask) LB(true, false, 10); else LB(false, false, 10); }
  } else {
    if (xe) { if (mask) LB(true, true, FC_MAXO); else LB(false, true, FC_MAXO); }
    else { if (mask) LB(true, false, FC_MAXO); else LB(false, false, FC_MAXO); }
  }
#undef LB
}

void fc_bwd(const float* dL, const bf16_t* X, const bf16_t* Wf, bf16_t* dX, float* dW, float scale,
            int B, long K, int NO, bool mask, hipStream_t s, const FcBwdExtras& ex) {
  fc_bwd_launch<bf16_t>(dL, X, Wf, dX, dW, scale, B, K, NO, mask, s, ex);
}
void fc_bwd(const float* dL, const float* X, const float* Wf, float* dX, float* dW, float scale,
            int B, long K, int NO, bool mask, hipStream_t s, const FcBwdExtras& ex) {
  fc_bwd_launch<float>(dL, X, Wf, dX, dW, scale, B, K, NO, mask, s, ex);
}

DDP_STAMPS_SETTER(stamps_set_linear)

}  // namespace ddp_amd
