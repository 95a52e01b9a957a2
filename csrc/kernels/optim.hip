// Flat-buffer optimizer + gradient-slab reduction kernels.
//
// sgd_kernel: one multi-tensor SGD step over the whole flat fp32 parameter
// buffer (reference train_ddp.py:41,200: optim.SGD(lr=0.01); torch semantics of
// torch/optim/sgd.py _single_tensor_sgd incl. weight decay, momentum,
// dampening, nesterov, maximize).  In the same pass it refreshes the bf16
// shadows that the MFMA kernels read (plain copy, or the [tap][ci][co]
// transpose used by the conv data-gradient), and bumps the device step counter
// that the graph-captured step uses to find its batch.
//
// grad_reduce_kernel: fixed-order sum of split-K weight-gradient slabs into
// gradient-bucket views, prescaled by 1/world_size (DDP averaging).
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ mbuf, long n, SgdArgs a,
                                                  ShadowSet sh, int* __restrict__ step_ctr) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float v = p[i];
    if (a.update) {
      float d = g[i];
      if (a.maximize) d = -d;
      if (a.weight_decay != 0.f) d = fmaf(a.weight_decay, v, d);
      if (a.momentum != 0.f) {
        float buf;
        if (a.first_step) buf = d;
        else buf = fmaf(1.f - a.dampening, d, a.momentum * mbuf[i]);
        mbuf[i] = buf;
        d = a.nesterov ? fmaf(a.momentum, buf, d) : buf;
      }
      v = fmaf(-a.lr, d, v);
      p[i] = v;
    }
#pragma unroll
    for (int r = 0; r < MAX_SHADOWS; ++r) {
      if (r < sh.count) {
        const long j = i - sh.r[r].off;
        if (j >= 0 && j < sh.r[r].n) {
          if (sh.r[r].kind == SHADOW_BF16) {
            sh.r[r].dst[j] = f2bf(v);
          } else {  // SHADOW_BF16_TAPT: OHWI [co][tap][ci] -> [tap][ci][co]
            const int Co = sh.r[r].a, T = sh.r[r].b, Ci = sh.r[r].c;
            const long co = j / ((long)T * Ci);
            const long rr = j - co * T * Ci;
            sh.r[r].dst[rr * Co + co] = f2bf(v);
          }
        }
      }
    }
  }
  if (step_ctr && blockIdx.x == 0 && threadIdx.x == 0) step_ctr[0] += 1;
}

// Block = 64 consecutive outputs x 4 row groups: thread (c, g) sums rows g, g+4, ...
// (8 loads in flight), then the 4 group sums are added in fixed order via LDS.
__global__ __launch_bounds__(256) void grad_reduce_kernel(SlabSet ss) {
  __shared__ float part[4][64];
  const int c = threadIdx.x & 63, grp = threadIdx.x >> 6;
  // segments are laid out back to back, each padded to a multiple of 64 outputs, so
  // a block (64 outputs) never straddles two segments
  long i = (long)blockIdx.x * 64 + c;
  int k = 0;
  for (; k < ss.count; ++k) {
    const long padded = (ss.s[k].n + 63) / 64 * 64;
    if (i < padded) break;
    i -= padded;
  }
  const bool live = k < ss.count && i < ss.s[k].n;
  float acc = 0.f;
  if (live) {
    const SlabSeg& sg = ss.s[k];
    const float* src = sg.slab + sg.src_off + i;
    float a[8];
    int r = grp;
    for (; r + 28 < sg.rows; r += 32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = src[(long)(r + 4 * u) * sg.row_stride];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += a[u];
    }
    for (; r < sg.rows; r += 4) acc += src[(long)r * sg.row_stride];
  }
  part[grp][c] = acc;
  __syncthreads();
  if (grp == 0 && live) {
    const SlabSeg& sg = ss.s[k];  // k is block-uniform
    sg.dst[i] = (((part[0][c] + part[1][c]) + part[2][c]) + part[3][c]) * sg.scale;
  }
}

__global__ void scale_copy_kernel(float* __restrict__ dst, const float* __restrict__ src, long n,
                                  float scale) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = src[i] * scale;
}

void sgd_step(float* p, const float* g, float* mbuf, long n, const SgdArgs& a, const ShadowSet& sh,
              int* step_ctr, hipStream_t s) {
  const long blocks = (n + 255) / 256;
  const unsigned grid = (unsigned)(blocks < 2048 ? (blocks > 0 ? blocks : 1) : 2048);
  hipLaunchKernelGGL(sgd_kernel, dim3(grid), dim3(256), 0, s, p, g, mbuf, n, a, sh, step_ctr);
}

void grad_reduce(const SlabSet& ss, hipStream_t s) {
  long blocks = 0;
  for (int k = 0; k < ss.count; ++k) blocks += (ss.s[k].n + 63) / 64;
  if (blocks == 0) return;
  hipLaunchKernelGGL(grad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ss);
}

void scale_copy(float* dst, const float* src, long n, float scale, hipStream_t s) {
  const long blocks = (n + 255) / 256;
  const unsigned grid = (unsigned)(blocks < 1024 ? (blocks > 0 ? blocks : 1) : 1024);
  hipLaunchKernelGGL(scale_copy_kernel, dim3(grid), dim3(256), 0, s, dst, src, n, scale);
}

}  // namespace ddp_amd
