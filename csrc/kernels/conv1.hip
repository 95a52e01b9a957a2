// First convolution of SimpleCNN: Conv2d(1 -> Cout, 3x3, padding=1) + bias + ReLU.
//
// Reference op: model.py:9-10 (nn.Conv2d(1,32,3,padding=1) -> nn.ReLU()).
// With a single input channel the GEMM K dimension is only 9, far too thin for
// MFMA, so this is a VALU direct convolution.  Its input is read straight out of
// the device-resident uint8 MNIST tensor through the epoch index list (the
// DistributedSampler gather, reference data.py:16-25) with ToTensor's /255 fused
// into the load, so no batch tensor is ever materialised.  Output: NHWC bf16.
//
// conv1_wgrad_kernel is the standalone weight/bias gradient used by the autograd
// (module) path; the fused training engine computes the same sums inside the
// conv2 data-gradient epilogue instead (conv3x3.hip).
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

template <typename T, bool U8>
__global__ __launch_bounds__(256) void conv1_fwd_kernel(const void* __restrict__ x, BatchIdx bi,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ bias,
                                                        T* __restrict__ y, int B, int H, int W,
                                                        int Cout) {
  extern __shared__ __attribute__((aligned(16))) float s_w[];  // [Cout][9] then [Cout]
  const int t = threadIdx.x;
  for (int i = t; i < Cout * 10; i += 256) s_w[i] = (i < Cout * 9) ? w[i] : bias[i - Cout * 9];
  __syncthreads();
  const int CG = Cout >> 3;  // channel groups of 8 per pixel
  const int ppb = 256 / CG;  // pixels per block
  const int cg = t % CG;
  const int HW = H * W;
  const long P = (long)blockIdx.x * ppb + t / CG;
  if (P >= (long)B * HW) return;
  const int n = (int)(P / HW);
  const int rem = (int)(P - (long)n * HW);
  const int h = rem / W, wc = rem - (rem / W) * W;
  float v[9];
  if (U8) {
    const int base = bi.base();
    const unsigned char* img = (const unsigned char*)x + (long)bi.row(n, base) * HW;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int hh = h + kh - 1, ww = wc + kw - 1;
        const bool ok = (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
        v[kh * 3 + kw] = ok ? (float)img[hh * W + ww] / 255.0f : 0.f;
      }
  } else {
    const float* img = (const float*)x + (long)n * HW;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int hh = h + kh - 1, ww = wc + kw - 1;
        const bool ok = (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
        v[kh * 3 + kw] = ok ? img[hh * W + ww] : 0.f;
      }
  }
  float o[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) o[c] = conv1_eval(s_w, s_w + Cout * 9, v, cg * 8 + c);
  if constexpr (sizeof(T) == 4) {  // exact fp32 activations (--dtype fp32)
    float* d = reinterpret_cast<float*>(y + P * Cout + cg * 8);
    *reinterpret_cast<float4*>(d) = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4*>(d + 4) = make_float4(o[4], o[5], o[6], o[7]);
  } else {
    uint4 pk;
    uint2 lo = pack4(o[0], o[1], o[2], o[3]), hi = pack4(o[4], o[5], o[6], o[7]);
    pk.x = lo.x; pk.y = lo.y; pk.z = hi.x; pk.w = hi.y;
    *reinterpret_cast<uint4*>(y + P * Cout + cg * 8) = pk;
  }
}

__device__ __forceinline__ float to_f(bf16_t v) { return bf2f(v); }
__device__ __forceinline__ float to_f(float v) { return v; }

// Partial weight/bias gradient of conv1 over a chunk of CHUNK pixels per block:
//   slab[blk][co*9 + tap] = sum_P dZ[P][co] * x[P shifted by tap],  slab[blk][Cout*9 + co] = sum_P dZ[P][co]
// dZ = dY * (Y > 0) when MASK (Y = conv1's ReLU output).  Reduced in fixed order by grad_reduce.
template <typename T, bool U8, bool MASK>
__global__ __launch_bounds__(320) void conv1_wgrad_kernel(const void* __restrict__ x, BatchIdx bi,
                                                          const T* __restrict__ dy,
                                                          const T* __restrict__ yact,
                                                          float* __restrict__ slab, int B, int H,
                                                          int W, int Cout, int chunk) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* s_x = smem;                  // [chunk][9]
  float* s_dz = smem + chunk * 9;     // [chunk][Cout]
  const int t = threadIdx.x;
  const int HW = H * W;
  const long P0 = (long)blockIdx.x * chunk;
  const long Ptot = (long)B * HW;
  const int base = U8 ? bi.base() : 0;
  for (int i = t; i < chunk * 9; i += blockDim.x) {
    const int p = i / 9, k = i - (i / 9) * 9;
    const long P = P0 + p;
    float v = 0.f;
    if (P < Ptot) {
      const int n = (int)(P / HW), rem = (int)(P - (long)n * HW);
      const int hh = rem / W + k / 3 - 1, ww = rem % W + k % 3 - 1;
      if ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W) {
        if (U8) v = (float)((const unsigned char*)x)[(long)bi.row(n, base) * HW + hh * W + ww] / 255.0f;
        else v = ((const float*)x)[(long)n * HW + hh * W + ww];
      }
    }
    s_x[i] = v;
  }
  for (int i = t; i < chunk * Cout; i += blockDim.x) {
    const long P = P0 + i / Cout;
    float g = 0.f;
    if (P < Ptot) {
      const long off = P0 * Cout + i;
      g = to_f(dy[off]);
      if (MASK && !(to_f(yact[off]) > 0.f)) g = 0.f;
    }
    s_dz[i] = g;
  }
  __syncthreads();
  const int nout = Cout * 10;
  for (int o = t; o < nout; o += blockDim.x) {
    float acc = 0.f;
    if (o < Cout * 9) {
      const int co = o / 9, k = o - (o / 9) * 9;
      for (int p = 0; p < chunk; ++p) acc = fmaf(s_dz[p * Cout + co], s_x[p * 9 + k], acc);
    } else {
      const int co = o - Cout * 9;
      for (int p = 0; p < chunk; ++p) acc += s_dz[p * Cout + co];
    }
    slab[(long)blockIdx.x * nout + o] = acc;
  }
}

template <typename T>
static void conv1_fwd_launch(const void* x, bool x_is_u8, BatchIdx bi, const float* w, const float* b,
                             T* y, int B, int H, int W, int Cout, hipStream_t s) {
  const int ppb = 256 / (Cout / 8);
  const long P = (long)B * H * W;
  const dim3 grid((unsigned)((P + ppb - 1) / ppb));
  const size_t lds = sizeof(float) * Cout * 10;
  if (x_is_u8)
    hipLaunchKernelGGL((conv1_fwd_kernel<T, true>), grid, dim3(256), lds, s, x, bi, w, b, y, B, H, W, Cout);
  else
    hipLaunchKernelGGL((conv1_fwd_kernel<T, false>), grid, dim3(256), lds, s, x, bi, w, b, y, B, H, W, Cout);
}
void conv1_fwd(const void* x, bool x_is_u8, BatchIdx bi, const float* w, const float* b, bf16_t* y,
               int B, int H, int W, int Cout, hipStream_t s) {
  conv1_fwd_launch<bf16_t>(x, x_is_u8, bi, w, b, y, B, H, W, Cout, s);
}
void conv1_fwd(const void* x, bool x_is_u8, BatchIdx bi, const float* w, const float* b, float* y,
               int B, int H, int W, int Cout, hipStream_t s) {
  conv1_fwd_launch<float>(x, x_is_u8, bi, w, b, y, B, H, W, Cout, s);
}

int conv1_wgrad_blocks(int B, int H, int W, int chunk) {
  const long P = (long)B * H * W;
  return (int)((P + chunk - 1) / chunk);
}

template <typename T>
static void conv1_wgrad_launch(const void* x, bool x_is_u8, BatchIdx bi, const T* dy, const T* yact,
                               float* slab, int B, int H, int W, int Cout, int chunk, hipStream_t s) {
  const dim3 grid(conv1_wgrad_blocks(B, H, W, chunk));
  const size_t lds = sizeof(float) * chunk * (9 + Cout);
  const bool mask = yact != nullptr;
#define L1W(U, M) hipLaunchKernelGGL((conv1_wgrad_kernel<T, U, M>), grid, dim3(320), lds, s, x, bi, dy, yact, slab, B, H, W, Cout, chunk)
  if (x_is_u8) { if (mask) L1W(true, true); else L1W(true, false); }
  else { if (mask) L1W(false, true); else L1W(false, false); }
#undef L1W
}
void conv1_wgrad(const void* x, bool x_is_u8, BatchIdx bi, const bf16_t* dy, const bf16_t* yact,
                 float* slab, int B, int H, int W, int Cout, int chunk, hipStream_t s) {
  conv1_wgrad_launch<bf16_t>(x, x_is_u8, bi, dy, yact, slab, B, H, W, Cout, chunk, s);
}
void conv1_wgrad(const void* x, bool x_is_u8, BatchIdx bi, const float* dy, const float* yact,
                 float* slab, int B, int H, int W, int Cout, int chunk, hipStream_t s) {
  conv1_wgrad_launch<float>(x, x_is_u8, bi, dy, yact, slab, B, H, W, Cout, chunk, s);
}

DDP_STAMPS_SETTER(stamps_set_conv1)

}  // namespace ddp_amd
