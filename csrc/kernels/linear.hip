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
#include "kernels/common.h"
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

// fc backward: a block of WPB waves owns FCB_COLS = 128 consecutive columns k (2 per
// lane, one 4-byte load per row) and its waves split the batch rows (wave w: rows
// w, w + WPB, ...).  The W columns and the first RB rows of X are requested BEFORE the
// prologue (cross-entropy backward / dL copy) so they land while it runs.  Every
// branch on the row count or the class count is wave-uniform (scalar), row addresses
// are clamped instead of guarded, so a wave keeps all its loads in flight.  dW: the
// waves' partials are summed in fixed wave order through LDS and written as coalesced
// rows.  NOT = compile-time class capacity (NOT == 10 fixes NO = 10).
constexpr int FCB_COLS = 128;
constexpr int FCB_RB = 8;  // rows in flight per wave

// 2 consecutive columns of one row as floats (bf16: one 4-byte load, fp32: one 8-byte load)
__device__ __forceinline__ float2 ld2f(const bf16_t* p) {
  const unsigned u = *reinterpret_cast<const unsigned*>(p);
  return make_float2(__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u));
}
__device__ __forceinline__ float2 ld2f(const float* p) { return *reinterpret_cast<const float2*>(p); }
__device__ __forceinline__ void st2_wt(bf16_t* p, float a, float b) {
  st_wt(reinterpret_cast<unsigned*>(p), (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16));
}
__device__ __forceinline__ void st2_wt(float* p, float a, float b) {
  st_wt(reinterpret_cast<float2*>(p), make_float2(a, b));
}

template <typename T, bool MASK, bool XENT, int NOT, int WPB>
__global__ __launch_bounds__(WPB * 64) void fc_bwd_kernel(const float* __restrict__ dL,
                                                          const T* __restrict__ X,
                                                          const T* __restrict__ Wf,
                                                          T* __restrict__ dX,
                                                          float* __restrict__ dW, float scale,
                                                          int B, long K, int NO_rt,
                                                          FcBwdExtras ex) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  DDP_STAMP(STAMP_K_FC_BWD, 0);
  const int NO = NOT == 10 ? 10 : NO_rt;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* s_dl = smem;            // [B][NO]
  float* s_loss = s_dl + B * NO;  // [B]
  float* s_lg = s_loss + B;       // [B][NO] cross-entropy scratch (XENT)
  int* s_lab = reinterpret_cast<int*>(s_lg + B * NO);  // [B] labels (XENT)
  float* s_red = smem + (((XENT ? 2 * B * NO + B : B * NO) + B + 3) & ~3);  // [WPB][NOT][COLS]

  const long col = (long)blockIdx.x * FCB_COLS + 2 * lane;
  const bool active = col < K;  // host guarantees K % 2 == 0
  const long cc = active ? col : 0;
  // ---- this block's loads first (independent of the prologue)
  float2 wr[NOT];
#pragma unroll
  for (int o = 0; o < NOT; ++o) wr[o] = (o < NO) ? ld2f(Wf + (long)o * K + cc) : make_float2(0.f, 0.f);
  const int nr = B > wave ? (B - wave + WPB - 1) / WPB : 0;  // rows of this wave (uniform)
  float2 xr[FCB_RB];
#pragma unroll
  for (int u = 0; u < FCB_RB; ++u) {
    const int b = min(wave + WPB * u, B - 1);
    xr[u] = ld2f(X + (long)b * K + cc);
  }
  // fused-SGD operands of this thread's dW outputs (final loop below): requested now so
  // the optimizer tail has no dependent global round trip
  constexpr int PRE = (NOT * FCB_COLS + WPB * 64 - 1) / (WPB * 64);
  float pre_p[PRE], pre_m[PRE];
  if (ex.sgd.update) {
#pragma unroll
    for (int j = 0; j < PRE; ++j) {
      const int i = threadIdx.x + j * WPB * 64;
      const int o = i / FCB_COLS, c = i - (i / FCB_COLS) * FCB_COLS;
      const long k = (long)blockIdx.x * FCB_COLS + c;
      const bool ok = i < NO * FCB_COLS && k < K;
      const long idx = ok ? (long)o * K + k : 0;
      pre_p[j] = ex.p_w[idx];
      pre_m[j] = ex.m_w ? ex.m_w[idx] : 0.f;
    }
  }
  DDP_STAMP(STAMP_K_XENT, 0);  // loads of W / X issued
  // ---- prologue: dL of the whole batch into LDS
  if (XENT) {
    xent_batch_block(ex.part, ex.HW, ex.CH, ex.fc_bias, NO, B, ex.labels32, ex.bi, ex.gscale, s_dl,
                     s_loss, s_lg, s_lab);
  } else {
    for (int i = threadIdx.x; i < B * NO; i += WPB * 64) s_dl[i] = dL[i];
  }
  __syncthreads();
  DDP_STAMP(STAMP_K_FC_BWD, 1);
  if (blockIdx.x == 0) {
    // fc bias gradient (sum over the batch, fixed order) and the batch-mean loss
    if (ex.dbias && threadIdx.x < NO) {
      float acc = 0.f;
      for (int b = 0; b < B; ++b) acc += s_dl[b * NO + threadIdx.x];
      if (ex.sys_store) st_sys(ex.dbias + threadIdx.x, acc * ex.dbias_scale);
      else ex.dbias[threadIdx.x] = acc * ex.dbias_scale;
    }
    if ((XENT || ex.loss_rows) && ex.loss_out && threadIdx.x == 64) {
      const float* lr = XENT ? s_loss : ex.loss_rows;
      float acc = 0.f;
      for (int b = 0; b < B; ++b) acc += lr[b];
      ex.loss_out[ex.step_ctr ? *ex.step_ctr : 0] = acc / (float)B;
    }
  }
  float w0[NOT], w1[NOT], dw0[NOT], dw1[NOT];
#pragma unroll
  for (int o = 0; o < NOT; ++o) {
    w0[o] = wr[o].x;
    w1[o] = wr[o].y;
    dw0[o] = 0.f;
    dw1[o] = 0.f;
  }
  for (int u0 = 0; u0 < nr; u0 += FCB_RB) {
    if (u0 > 0) {
#pragma unroll
      for (int u = 0; u < FCB_RB; ++u) {
        const int b = min(wave + WPB * (u0 + u), B - 1);
        xr[u] = ld2f(X + (long)b * K + cc);
      }
    }
#pragma unroll
    for (int u = 0; u < FCB_RB; ++u) {
      if (u0 + u < nr) {  // wave-uniform
        const int b = wave + WPB * (u0 + u);
        const float x0 = xr[u].x;
        const float x1 = xr[u].y;
        const float* dl = s_dl + b * NO;
        float dz0 = 0.f, dz1 = 0.f;
#pragma unroll
        for (int o = 0; o < NOT; ++o)
          if (o < NO) {
            const float d = dl[o];
            dz0 = fmaf(d, w0[o], dz0);
            dz1 = fmaf(d, w1[o], dz1);
            dw0[o] = fmaf(d, x0, dw0[o]);
            dw1[o] = fmaf(d, x1, dw1[o]);
          }
        if (MASK) {
          dz0 = x0 > 0.f ? dz0 : 0.f;
          dz1 = x1 > 0.f ? dz1 : 0.f;
        }
        if (active) st2_wt(dX + (long)b * K + col, dz0, dz1);  // dZ2: write-through
      }
    }
  }
  DDP_STAMP(STAMP_K_FC_BWD, 2);
  // ---- fixed-order reduction of the waves' dW partials
#pragma unroll
  for (int o = 0; o < NOT; ++o)
    if (o < NO)
      *reinterpret_cast<float2*>(s_red + (wave * NOT + o) * FCB_COLS + 2 * lane) = make_float2(dw0[o], dw1[o]);
  __syncthreads();
  DDP_STAMP(STAMP_K_FC_BWD, 3);
#pragma unroll
  for (int jj = 0; jj < PRE; ++jj) {
    const int i = threadIdx.x + jj * WPB * 64;
    if (i >= NO * FCB_COLS) break;
    const int o = i / FCB_COLS, c = i - (i / FCB_COLS) * FCB_COLS;
    const long k = (long)blockIdx.x * FCB_COLS + c;
    if (k < K) {
      float acc = s_red[o * FCB_COLS + c];
#pragma unroll
      for (int w = 1; w < WPB; ++w) acc += s_red[(w * NOT + o) * FCB_COLS + c];
      const float g = acc * scale;
      const long idx = (long)o * K + k;
      if (dW) {  // null: fused optimizer consumes it in registers
        if (ex.sys_store) st_sys(dW + idx, g);
        else dW[idx] = g;
      }
      if (ex.sgd.update) {  // single-process step: dW is final -> fused SGD + shadows
        float m = pre_m[jj];
        const float pn = sgd_one(pre_p[jj], g, &m, ex.sgd);
        st_wt(ex.p_w + idx, pn);  // write-through: no dirty L2 at the kernel boundary
        if (ex.m_w) ex.m_w[idx] = m;
        const bf16_t pb = f2bf(pn);
        if (ex.sh_plain) st_wt(ex.sh_plain + idx, pb);
        if (ex.sh_frag) st_wt(ex.sh_frag + fcfrag_index((int)idx, ex.frag_HW, ex.frag_C), pb);
      }
    }
  }
  DDP_STAMP(STAMP_K_FC_BWD, 4);
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

constexpr int FCB_WPB = 8;  // waves per fc_bwd block

size_t fc_bwd_lds(int B, int NO, bool xent) {
  const int NOT = NO == 10 ? 10 : FC_MAXO;
  const size_t head = (((size_t)(xent ? 2 * B * NO + B : B * NO) + B + 3) & ~(size_t)3);
  return sizeof(float) * (head + (size_t)FCB_WPB * NOT * FCB_COLS);
}

template <typename T>
static void fc_bwd_launch(const float* dL, const T* X, const T* Wf, T* dX, float* dW, float scale,
                          int B, long K, int NO, bool mask, hipStream_t s, const FcBwdExtras& ex) {
  const dim3 grid((unsigned)((K + FCB_COLS - 1) / FCB_COLS));
  const bool xe = ex.part != nullptr;
  const size_t lds = fc_bwd_lds(B, NO, xe);
#define LB(M, XE, N) hipLaunchKernelGGL((fc_bwd_kernel<T, M, XE, N, FCB_WPB>), grid, dim3(FCB_WPB * 64), lds, s, dL, X, Wf, dX, dW, scale, B, K, NO, ex)
  if (NO == 10) {
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
