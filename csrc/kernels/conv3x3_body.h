// Device code of the 3x3 MFMA convolution kernels (data gradient, weight gradient, the fused
// conv backward; the forward kernel is in conv3x3_fwd.h) and the host helpers the launchers of
// conv3x3.hip and conv3x3_bwd.hip share.  Split out of conv3x3.hip so that its two launcher
// TUs compile in parallel (the fused backward's many instantiations dominated the build).
#pragma once
#include <algorithm>
#include <stdexcept>

#include <cstdio>
#include <cstdlib>

#include "kernels/common.h"
#include "kernels/fc_bwd_body.h"
#include "kernels/launchers.h"
#include "kernels/slab_reduce.h"
#include "kernels/xgmi_body.h"

namespace ddp_amd {

// Cooperative global -> LDS copy of 16-byte chunks from up to two index spaces
// (n1 chunks of src1/dst1, then n2 of src2/dst2): every thread issues up to INF
// loads before its first LDS write, so a block's whole staging is ONE memory round
// trip when (n1 + n2) <= 256 * INF.  src(i) returns chunk i (zero-filled where out of
// range).
template <int INF, int NT = 256, typename S1, typename D1, typename S2, typename D2>
__device__ __forceinline__ void stage2(int n1, S1 src1, D1 dst1, int n2, S2 src2, D2 dst2) {
  const int n = n1 + n2;
  for (int base = threadIdx.x; base < n; base += NT * INF) {
    bf16x8 v[INF];
#pragma unroll
    for (int u = 0; u < INF; ++u) {
      const int i = base + u * NT;
      v[u] = (i < n1) ? src1(i) : ((i < n) ? src2(i - n1) : zero8());
    }
#pragma unroll
    for (int u = 0; u < INF; ++u) {
      const int i = base + u * NT;
      if (i < n1) dst1(i, v[u]);
      else if (i < n) dst2(i - n1, v[u]);
    }
  }
}
template <typename SrcFn, typename DstFn>
__device__ __forceinline__ void stage16(int n, SrcFn src, DstFn dst) {
  stage2<8>(n, src, dst, 0, src, dst);
}

constexpr unsigned long long DZ_WAIT_TICKS = 2000000;  // 20 ms of the 100 MHz clock (in-launch waits)

// Fused slab reduction of the conv backward (conv3x3_bwd_kernel<..., FRED>)
struct BwdReduce {
  SlabSet ss{};
  long nchunks = 0;
  int first_reducer = 0;  // blocks [first_reducer, nconv) reduce after the arrival count
  int nconv = 0;          // conv-role blocks (the arrivals the reducers wait for); fc-role blocks follow
  int* done = nullptr;  // 8 arrival counters, 32 ints apart (zeroed by the step's forward)
  int* err = nullptr;   // set to 2 when the wait times out
  // role order of the conv blocks: 0 = all dgrad blocks, then all wgrad blocks; 1 =
  // interleaved (d, w, d, w, ..., then the longer role's rest) so every CU holds a mix
  // of both roles instead of a dgrad phase followed by a wgrad phase (the reducers are the
  // last nr blocks whatever their role).  Set by the launcher (also without FRED).
  int interleave = 0;
  // 1: the slab set's largest segment has 128 < rows <= 256 (exact fp32, bf16 at B = 64):
  // the reducers take 2 chunks per pass with all 16 rows per group in flight
  // (slab_fused_run16); 0: 3 chunks per pass, 8 rows per group (slab_fused_run)
  int deep = 0;
};

// Geometry specialisation: kernels take <GH, GW, GCI, GCO>; non-zero values replace
// the runtime H, W, Cin, Cout so all index arithmetic (divisions by W, H*W, channel
// counts) folds to constants.  The launchers pick <28, 28, 32, 64> - SimpleCNN's
// conv2 - when the shape matches and the generic <0, 0, 0, 0> otherwise.
#define DDP_GEOM_OVERRIDE()                                    \
  if (GH) {                                                    \
    H = GH; W = GW; Cin = GCI; Cout = GCO;                     \
  }

// LDS geometry shared by fwd / dgrad: a block covers CH = 64*PXT consecutive output
// pixels of the flattened [B*H*W] space and stages the LINEAR pixel range
// [P0 - W - 1, P0 + CH + W + 1): every 3x3 neighbour of the block's pixels is in it
// (neighbours in another image row/image are zeroed by the (h,w) bounds test).
// Weight and activation rows are padded by 16 elements: a row stride of 8 mod 16 dwords
// is the one at which ds_read_b128's four 16-lane groups (rows l & 15, k offset
// 4 * (l >> 4) dwords) cover all 64 banks exactly once - conflict-free fragment reads
// (the previous 8-element pad gave 2-way conflicts).

// LDS bytes of the forward's staging area (weights, input rows, conv1 recompute
// scratch), rounded to 16; the fused-fc epilogue's per-tile partials follow it.
__host__ __device__ inline size_t fwd_stage_lds(int W, int Cin, int pxt, bool a1x, int es = 2) {
  const size_t XR = 64 * pxt + 2 * W + 2;  // a block covers CH = 64 * pxt pixels
  const int pad = es == 2 ? 16 : 8;        // Prec<T>::PAD
  const size_t b = (size_t)es * ((size_t)64 * (9 * Cin + pad) + XR * (Cin + pad)) +
                   (a1x ? sizeof(float) * ((XR + 2 * W + 2) + Cin * 10) : 0);
  return (b + 15) & ~(size_t)15;
}
constexpr int FC_MAX_NOF = 16;
// [16-pixel tile][channel group][class] floats (CH / 16 = 4 * pxt tiles per block)
__host__ __device__ inline size_t fc_epi_lds(int pxt, int nof) { return sizeof(float) * 4 * pxt * 4 * nof; }

// ---------------------------------------------------------------- data gradient
// A1X (with FUSE_W1, uint8 x0): the ReLU-input mask is recomputed from conv1 instead of
// being read from a stored a1 tensor (mask = bf16(relu(conv1(x))) > 0, bit-exact).
// WG (exact fp32, SimpleCNN geometry): the block computes ONE 16-channel half `by` of the
// input channels (two blocks per pixel chunk) and reads its weight fragments straight from
// the [tap][ci][co] fp32 copy in global memory (16-byte loads, one tap ahead of the MFMAs,
// L1/L2-resident: 73 KB) instead of staging 73 KB of fp32 weights in LDS - the block then
// needs ~60 KB of LDS, so two fit a CU (the fp32 conv backward ran at one block per CU,
// its dgrad and wgrad blocks serialised by residency: profiles/r3_fp32).  Each output's
// MFMA chain (tap-major, 32-wide K steps over the output channels) is unchanged, and the
// conv1 weight-gradient partials of a channel are summed over the same pixels in the same
// order, so dZ1 and the w1 slab row are bit-identical to the one-block-per-chunk kernel
// (each half writes its own 16 channels of the row).
template <typename T, int PXT, bool MASK_DY, bool MASK_X, bool FUSE_W1, bool A1X, int GH, int GW, int GCI,
          int GCO, int WGS = 0>
__device__ __forceinline__ void dgrad_body(
    const T* __restrict__ dY, const T* __restrict__ Yact, const T* __restrict__ WT,
    const T* __restrict__ Xact, T* __restrict__ dX, int B, int H, int W, int Cin, int Cout,
    const void* __restrict__ x0, int x0_u8, BatchIdx bi, float* __restrict__ w1slab, C1Src c1, char* smem, int bx, int by) {
  using P = Prec<T>;
  constexpr bool F32 = sizeof(T) == 4;
  // WGS: 0 = weights staged in LDS; 1 = from global, one 16-channel half `by` per block;
  // 2 = from global, both halves (all 32 input channels) per block
  constexpr bool WG = WGS > 0, HALF = WGS == 1;
  static_assert(!WG || (F32 && GCI == 32 && GCO == 64 && FUSE_W1), "weights-from-global dgrad: fp32 SimpleCNN conv2");
  constexpr int CE = P::CE;
  constexpr int NCT = HALF ? 1 : 2;  // 16-wide input-channel tiles per wave
  DDP_STAMP(STAMP_K_DGRAD, 0);
  DDP_GEOM_OVERRIDE();
  constexpr int CH = 64 * PXT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int HW = H * W;
  const long Ptot = (long)B * HW;
  const int ci_blk = HALF ? by * 16 : by * 32;
  const int KW = 9 * Cout, WS = KW + P::PAD, DS = Cout + P::PAD;  // row strides = 8 mod 16 dwords (conflict-free)
  const int XR = CH + 2 * W + 2;
  T* sWT = reinterpret_cast<T*>(smem);                   // [32 ci][9*Cout] (not WG)
  T* sDY = sWT + (WG ? 0 : 32 * WS);                     // [XR][Cout]
  float* sx0 = reinterpret_cast<float*>(sDY + XR * DS);  // [XR] conv1 input (FUSE_W1)
  float* s_w1 = sx0 + XR;                                // [4][320] (FUSE_W1)
  unsigned char* s_m1 = reinterpret_cast<unsigned char*>(s_w1 + 4 * 320);  // [CH][4] a1>0 bits (A1X)
  const long P0 = (long)bx * CH;
  const long Pbase = P0 - W - 1;
  // conv1 channel group of this wave's mask work: WG - the half's two groups, waves
  // (w, w + 2) splitting the pixels; otherwise group = wave
  const int mg = HALF ? 2 * by + (wave & 1) : wave;

  // conv1 input values for the fused w1 gradient: loads issued before the staging
  // round so the dependent index -> image chain overlaps it
  auto x0_at = [&](int r) {
    const long P = Pbase + r;
    float v = 0.f;
    if (P >= 0 && P < Ptot) {
      const int n = (int)(P / HW), rm = (int)(P - (long)n * HW);
      if (x0_u8) v = (float)((const unsigned char*)x0)[(long)bi.row(n, bi.base()) * HW + rm] / 255.0f;
      else v = ((const float*)x0)[P];
    }
    return v;
  };
  const float x0_pre = (FUSE_W1 && (int)threadIdx.x < XR) ? x0_at(threadIdx.x) : 0.f;
  Conv1Group cg;
  if (A1X) cg = conv1_group_load(c1.w, c1.b, mg);  // lands during the staging round
  // WG: tap 0's weight fragments, requested now so they land during the staging round
  const T* wg = WT + (long)(ci_blk + (lane & 15)) * Cout + P::kofs(lane);
  const long tstr = (long)Cin * Cout;
  typename P::Frag an[WG ? 2 : 1][WG ? NCT : 1];
  if constexpr (WG) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int t = 0; t < NCT; ++t) an[k][t] = P::frag(wg + 16 * t * Cout + 32 * k);
  }
  const int wc = KW / CE, cpc = Cout / CE;
  stage2<F32 ? 32 : 16>(WG ? 0 : 32 * wc,
          [&](int i) {
            const int r = i / wc, rest = (i - r * wc) * CE;  // rest = tap*Cout + co
            const int tap = rest / Cout, co = rest - tap * Cout;
            return ld16(WT + ((long)tap * Cin + ci_blk + r) * Cout + co);
          },
          [&](int i, bf16x8 v) { const int r = i / wc, c = (i - r * wc) * CE; st16(sWT + r * WS + c, v); },
          XR * cpc,
          [&](int i) {
            const int r = i / cpc, c = (i - r * cpc) * CE;
            const long Pq = Pbase + r;
            bf16x8 v = zero8();
            if (Pq >= 0 && Pq < Ptot) {
              v = ld16(dY + Pq * Cout + c);
              if (MASK_DY) v = mask16<T>(v, ld16(Yact + Pq * Cout + c));
            }
            return v;
          },
          [&](int i, bf16x8 v) { const int r = i / cpc, c = (i - r * cpc) * CE; st16(sDY + r * DS + c, v); });
  DDP_STAMP(STAMP_K_CONV1, 0);  // stage2 done (weights + dY in LDS, own waves)
  if (FUSE_W1) {
    if ((int)threadIdx.x < XR) sx0[threadIdx.x] = x0_pre;
    for (int r = threadIdx.x + 256; r < XR; r += 256) sx0[r] = x0_at(r);
  }
  DDP_STAMP(STAMP_K_CONV1, 1);  // x0 staged
  if (A1X) {
    // ReLU-input mask of the block's own pixels: bit j of s_m1[lp*4 + g] = (a1[lp][8g+j] > 0),
    // a1 recomputed from conv1 exactly as stored (bf16-rounded), channel group wave-uniform
    __syncthreads();
    const int g = mg;
    for (int lp = lane + (HALF ? 64 * (wave >> 1) : 0); lp < CH; lp += HALF ? 128 : 64) {
      const long P = P0 + lp;
      unsigned m = 0;
      if (P < Ptot) {
        const int rm = (int)(P % HW);
        const int hh = rm / W, ww = rm - (rm / W) * W;
        float v[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const int dh = k / 3 - 1, dw = k % 3 - 1;
          const bool ok = (unsigned)(hh + dh) < (unsigned)H && (unsigned)(ww + dw) < (unsigned)W;
          v[k] = ok ? sx0[lp + W + 1 + dh * W + dw] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a1v = conv1_eval_g(cg, v, j);  // the value the forward stored
          m |= ((F32 ? a1v : bf2f(f2bf(a1v))) > 0.f ? 1u : 0u) << j;
        }
      }
      s_m1[lp * 4 + g] = (unsigned char)m;
    }
    DDP_STAMP(STAMP_K_CONV1, 2);  // mask computed
  }
  const int kofs = P::kofs(lane);
  const int col = lane & 15;
  int h[PXT], w[PXT], rowc[PXT];
  bool valid[PXT];
  long Pp[PXT];
  float xa[PXT][2][4] = {};  // ReLU-input values of this lane's 2 x 4 outputs (MASK_X && !A1X)
#pragma unroll
  for (int pt = 0; pt < PXT; ++pt) {
    const int lp = (wave * PXT + pt) * 16 + col;
    Pp[pt] = P0 + lp;
    valid[pt] = Pp[pt] < Ptot;
    const long Pc = valid[pt] ? Pp[pt] : 0;
    const int n = (int)(Pc / HW);
    const int rm = (int)(Pc - (long)n * HW);
    h[pt] = rm / W;
    w[pt] = rm - h[pt] * W;
    rowc[pt] = lp + W + 1;
    if (MASK_X && !A1X) {  // prefetch the ReLU-input mask (lands during the MFMAs)
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
        const T* xp = Xact + Pc * Cin + ci_blk + 16 * t + 4 * (lane >> 4);
        if constexpr (F32) {
          const float4 x4 = *reinterpret_cast<const float4*>(xp);
          xa[pt][t][0] = x4.x; xa[pt][t][1] = x4.y; xa[pt][t][2] = x4.z; xa[pt][t][3] = x4.w;
        } else {
          unpack4(*reinterpret_cast<const uint2*>(xp), xa[pt][t]);
        }
      }
    }
  }
  lds_barrier();  // (the mask prefetch above stays in flight through the MFMA loop)
  DDP_STAMP(STAMP_K_DGRAD, 1);

  f32x4 acc[PXT][NCT];
#pragma unroll
  for (int pt = 0; pt < PXT; ++pt)
#pragma unroll
    for (int t = 0; t < NCT; ++t) acc[pt][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // one 32-wide K step (output channels co0 .. co0 + 31) of tap `tap` against A fragments a[]
  auto kstep = [&](int tap, int co0, const typename P::Frag* a) {
    const int dh = 1 - tap / 3, dw = 1 - tap % 3;  // dY pixel = (h + 1 - kh, w + 1 - kw)
    typename P::Frag b[PXT];
#pragma unroll
    for (int pt = 0; pt < PXT; ++pt) {
      const int hh = h[pt] + dh, ww = w[pt] + dw;
      const bool ok = valid[pt] && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
      const typename P::Frag v = P::frag(sDY + (rowc[pt] + dh * W + dw) * DS + co0 + kofs);
      b[pt] = fsel(ok, v, P::zero());  // unconditional read + select (see the forward)
    }
#pragma unroll
    for (int pt = 0; pt < PXT; ++pt)
#pragma unroll
      for (int t = 0; t < NCT; ++t) acc[pt][t] = P::mma(a[t], b[pt], acc[pt][t]);
  };
  if constexpr (WG) {
    // A fragments from the global [tap][ci][co] copy: lane (row ci + col, K offset kofs)
    // reads 2 x 16 bytes per 32-wide K step and channel tile; tap 0's were requested before
    // the staging round, every next tap's before this one's MFMAs (Cout == 64: two K steps
    // per tap)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      typename P::Frag ac[2][NCT];
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int t = 0; t < NCT; ++t) ac[k][t] = an[k][t];
      if (tap + 1 < 9) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int t = 0; t < NCT; ++t) an[k][t] = P::frag(wg + (tap + 1) * tstr + 16 * t * Cout + 32 * k);
      }
      kstep(tap, 0, ac[0]);
      kstep(tap, 32, ac[1]);
    }
  } else {
    const T* wrow = sWT + col * WS + kofs;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      for (int co0 = 0; co0 < Cout; co0 += 32) {
        const typename P::Frag a[2] = {P::frag(wrow + tap * Cout + co0), P::frag(wrow + 16 * WS + tap * Cout + co0)};
        kstep(tap, co0, a);
      }
    }
  }

  DDP_STAMP(STAMP_K_DGRAD, 2);
  float w1a[FUSE_W1 ? NCT : 1][4][10];
  if (FUSE_W1) {
#pragma unroll
    for (int t = 0; t < NCT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 10; ++k) w1a[t][j][k] = 0.f;
  }
#pragma unroll
  for (int pt = 0; pt < PXT; ++pt) {
    float xv[9];
    if (FUSE_W1) {
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int dh = k / 3 - 1, dw = k % 3 - 1;
        const int hh = h[pt] + dh, ww = w[pt] + dw;
        const bool ok = valid[pt] && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
        xv[k] = ok ? sx0[rowc[pt] + dh * W + dw] : 0.f;
      }
    }
#pragma unroll
    for (int t = 0; t < NCT; ++t) {
      const int ci = ci_blk + 16 * t + 4 * (lane >> 4);
      float v[4] = {acc[pt][t][0], acc[pt][t][1], acc[pt][t][2], acc[pt][t][3]};
      if (MASK_X && A1X) {
        const int lp = (wave * PXT + pt) * 16 + col;
        const unsigned m = s_m1[lp * 4 + (ci >> 3)] >> (ci & 7);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = ((m >> j) & 1u) ? v[j] : 0.f;
      } else if (MASK_X) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = xa[pt][t][j] > 0.f ? v[j] : 0.f;
      }
      float q[4] = {v[0], v[1], v[2], v[3]};  // the values stored (fp32: exact)
      if constexpr (F32) {
        if (dX && valid[pt]) *reinterpret_cast<float4*>(dX + Pp[pt] * Cin + ci) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        const uint2 pk = pack4(v[0], v[1], v[2], v[3]);
        if (dX && valid[pt]) *reinterpret_cast<uint2*>(dX + Pp[pt] * Cin + ci) = pk;  // dX null: only the fused w1 grad needs it
        unpack4(pk, q);
      }
      if (FUSE_W1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = valid[pt] ? q[j] : 0.f;
#pragma unroll
          for (int k = 0; k < 9; ++k) w1a[t][j][k] = fmaf(d, xv[k], w1a[t][j][k]);
          w1a[t][j][9] += d;
        }
      }
    }
  }
  DDP_STAMP(STAMP_K_DGRAD, 3);
  if (FUSE_W1) {
    // reduce over the 16 pixel lanes that share a channel group, then over waves (fixed order)
#pragma unroll
    for (int t = 0; t < NCT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 10; ++k) w1a[t][j][k] = sum16(w1a[t][j][k]);
    if (col == 0) {
#pragma unroll
      for (int t = 0; t < NCT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ci = ci_blk + 16 * t + 4 * (lane >> 4) + j;  // conv1 output channel (Cin == 32)
#pragma unroll
          for (int k = 0; k < 9; ++k) s_w1[wave * 320 + ci * 9 + k] = w1a[t][j][k];
          s_w1[wave * 320 + 288 + ci] = w1a[t][j][9];
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 320; i += 256) {
      // WG: only this half's 16 channels (the other half-block writes the rest of the row)
      if (HALF && ((i < 288 ? i / 9 : i - 288) >> 4) != by) continue;
      st_wt(w1slab + (long)bx * 320 + i, ((s_w1[i] + s_w1[320 + i]) + s_w1[640 + i]) + s_w1[960 + i]);
    }
  }
  DDP_STAMP(STAMP_K_DGRAD, 4);
}

template <typename T, int PXT, bool MASK_DY, bool MASK_X, bool FUSE_W1, bool A1X, int GH, int GW, int GCI,
          int GCO>
__global__ __launch_bounds__(256) void conv3x3_dgrad_kernel(
    const T* __restrict__ dY, const T* __restrict__ Yact, const T* __restrict__ WT,
    const T* __restrict__ Xact, T* __restrict__ dX, int B, int H, int W, int Cin, int Cout,
    const void* __restrict__ x0, int x0_u8, BatchIdx bi, float* __restrict__ w1slab, C1Src c1) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  dgrad_body<T, PXT, MASK_DY, MASK_X, FUSE_W1, A1X, GH, GW, GCI, GCO>(
      dY, Yact, WT, Xact, dX, B, H, W, Cin, Cout, x0, x0_u8, bi, w1slab, c1, smem, blockIdx.x, blockIdx.y);
}

// ---------------------------------------------------------------- weight gradient
// Block = (image n, chunk of R output rows).  LDS images (row strides C+16 elements,
// i.e. an odd multiple of 8 dwords, so 8 consecutive rows of ds_read_b64_tr_b16 hit
// 64 distinct banks):
//   sdY[slot][Cout]          slot = r*Wp + c, c < Wp = roundup(W,8); zero for c >= W
//   sX [(R+2)*(Wp+2)][Cin]   image rows r0-1..r0+R, cols -1..Wp; zero outside the image
// K index of a K-step (32 slots) for lane group g, element j:
//   slot = 4g + j (j<4),  16 + 4g + (j-4) (j>=4)   (same map for both operands)
// so the two 16-lane groups of a half-wave read 8 consecutive rows (conflict-free).
// A1X: the X tile (a1 rows r0-1 .. r0+R) is recomputed from the uint8 images (rows
// r0-2 .. r0+R+1) instead of being read from a stored a1 tensor.
// fp32 (exact) variant: the K dimension (pixel slots) is strided in NHWC for both operands,
// so each lane reads single floats - MFMA j takes slot s0 + 4j + (lane >> 4) - with row
// strides of 16 mod 32 dwords (Cout + 16, Cin + 16), conflict-free for ds_read_b32's two
// 32-lane groups (lanes l and l + 16 read adjacent slots).
// STAGE: the slab row goes through LDS (needs slab-row bytes of LDS, see conv3x3_bwd_lds)
// and leaves as 16-byte write-through stores - from the MFMA layout each lane holds one
// float per 64-byte run of the row, and 4-byte write-through stores took ~2.4 us per block.
// CS == 2 (bf16, STAGE, SimpleCNN geometry Cin 32 / Cout 64): the input channels are
// split over TWO blocks per (image, row chunk) - half h stages / recomputes only channels
// 16h .. 16h+15 of X (half the conv1 recompute) and each wave runs one 16x16 (co, ci)
// tile (half the MFMAs), so the wgrad role's critical path roughly halves.  Each output's
// MFMA chain over the K slots is unchanged: the slab row is bit-identical to CS == 1's,
// half 0 writes the ci < 16 columns and the bias, half 1 the rest.  The two halves of a
// row chunk are 8 blocks apart (same XCD: blocks go round-robin over the 8 XCDs), so the
// second one's dY tile reads hit the same L2.
// CS == 2 also for exact fp32 (slab rows stored directly): the half's 16 X channels are
// staged compactly (row stride 16 floats - the lanes of a ds_read_b32 then read 64
// consecutive dwords), so the block needs ~56 KB of LDS instead of ~82 KB and two blocks
// fit a CU next to the dgrad role (dgrad_body WG).
template <typename T, bool MASK_DY, bool A1X, int GH, int GW, int GCI, int GCO, bool STAGE = false, int CS = 1>
__device__ __forceinline__ void wgrad_body(
    const T* __restrict__ dY, const T* __restrict__ Yact, const T* __restrict__ X,
    float* __restrict__ slab, int B, int H, int W, int Cin, int Cout, int R, C1Src c1, char* smem, int bx, int by) {
  constexpr bool F32 = sizeof(T) == 4;
  constexpr int CE = Prec<T>::CE;
  static_assert(CS == 1 || (CS == 2 && (STAGE || F32) && !(STAGE && F32) && GCI == 32 && GCO == 64),
                "the channel-split wgrad role: bf16 with a staged slab row, or fp32 with direct stores");
  constexpr bool XC = F32 && CS == 2;  // compact X tile: only the half's 16 channels
  DDP_STAMP(STAMP_K_WGRAD, 0);
  DDP_GEOM_OVERRIDE();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nRC = (H + R - 1) / R;
  int rb = bx, half = 0;  // slab row (image, row chunk) and channel half of this block
  if constexpr (CS == 2) {
    if (((B * nRC) & 7) == 0) {
      half = (bx >> 3) & 1;
      rb = ((bx >> 4) << 3) | (bx & 7);
    } else {
      half = bx & 1;
      rb = bx >> 1;
    }
  }
  const int n = rb / nRC;
  const int r0 = (rb - n * nRC) * R;
  const int Wp = (W + 7) & ~7;
  const int DS = Cout + 16, XS = XC ? 16 : Cin + 16;  // LDS row strides (elements)
  const int nslot = ((R * Wp + 31) / 32) * 32;
  T* sdY = reinterpret_cast<T*>(smem);
  T* sX = sdY + (long)nslot * DS;
  const int XW = Wp + 2;

  // conv1 channel group of this wave (CS == 2: waves 2k, 2k+1 share the half's groups)
  const int c1g = CS == 2 ? 2 * half + (wave & 1) : wave;
  Conv1Group cg;
  if (A1X) cg = conv1_group_load(c1.w, c1.b, c1g);  // lands during the staging round
  // ---- stage dY rows (masked) and X rows with halo: one round of loads
  const int cxn = CS == 2 ? Cin / 2 : Cin, cx0 = half * cxn;  // staged X channels
  const int cpy_dy = Cout / CE, cpy_x = cxn / CE;
  auto dy_src = [&](int i) {
    const int slot = i / cpy_dy, ch = (i - slot * cpy_dy) * CE;
    const int r = slot / Wp, c = slot - (slot / Wp) * Wp;
    const int hh = r0 + r;
    bf16x8 v = zero8();
    if (r < R && hh < H && c < W) {
      const long off = (((long)n * H + hh) * W + c) * Cout + ch;
      v = ld16(dY + off);
      if (MASK_DY) v = mask16<T>(v, ld16(Yact + off));
    }
    return v;
  };
  auto dy_dst = [&](int i, bf16x8 v) {
    const int slot = i / cpy_dy, ch = (i - slot * cpy_dy) * CE;
    st16(sdY + (long)slot * DS + ch, v);
  };
  // A1X: uint8 x rows r0-2 .. r0+R+1, cols -2 .. Wp+1 -> LDS floats, then a1 (conv1 recompute)
  const int XW2 = Wp + 4, XR2 = R + 4, NXX = XR2 * XW2;
  float* sxx = reinterpret_cast<float*>(sX + (long)(R + 2) * XW * XS);
  const long img = A1X ? (long)c1.bi.row(n, c1.bi.base()) * H * W : 0;
  auto x_inside = [&](int i, int& off) {
    const int rr = i / XW2, cc = i - (i / XW2) * XW2;
    const int hh = r0 - 2 + rr, ww = cc - 2;
    off = hh * W + ww;
    return (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
  };
  auto recompute = [&]() {
    conv1_recompute_tile<T>(
        (R + 2) * XW, cg, c1g, CS == 2 ? 64 * (wave >> 1) : 0, CS == 2 ? 128 : 64,
        [&](int pos) {
          const int rr = pos / XW, cc = pos - (pos / XW) * XW;
          return (unsigned)(r0 - 1 + rr) < (unsigned)H && (unsigned)(cc - 1) < (unsigned)W;
        },
        [&](int pos, int k) {
          const int rr = pos / XW, cc = pos - (pos / XW) * XW;
          return sxx[(rr + k / 3) * XW2 + cc + k % 3];
        },
        [&](int pos, int g) { return sX + (long)pos * XS + 8 * (XC ? g - 2 * half : g); });
  };
  const int ndy = nslot * cpy_dy;
  stage2<F32 ? 32 : 16>(ndy, dy_src, dy_dst,
          A1X ? 0 : (R + 2) * XW * cpy_x,
          [&](int i) {
            const int pos = i / cpy_x, ch = cx0 + (i - pos * cpy_x) * CE;
            const int rr = pos / XW, cc = pos - (pos / XW) * XW;
            const int hh = r0 - 1 + rr, ww = cc - 1;
            return ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
                       ? ld16(X + (((long)n * H + hh) * W + ww) * Cin + ch) : zero8();
          },
          [&](int i, bf16x8 v) {
            const int pos = i / cpy_x, ch = cx0 + (i - pos * cpy_x) * CE;
            st16(sX + (long)pos * XS + (XC ? ch - cx0 : ch), v);
          });
  if (A1X) {
    for (int i = threadIdx.x; i < NXX; i += 256) {
      int off = 0;
      sxx[i] = x_inside(i, off) ? (float)c1.x[img + off] / 255.0f : 0.f;
    }
    __syncthreads();
    DDP_STAMP(STAMP_K_WGRAD, 1);
    recompute();
  }
  __syncthreads();
  DDP_STAMP(STAMP_K_WGRAD, 2);

  // ---- wave assignment: (pair of 16-wide co tiles) x (16-wide ci tile); CS == 2: one
  // 16-wide co tile per wave x the block's ci half
  constexpr int NCT = CS == 2 ? 1 : 2;  // 16-wide co tiles per wave
  const int nct = Cin / 16;
  const int asg = by * 4 + wave;
  const int coT = CS == 2 ? 16 * wave : (asg / nct) * 32;
  const int ciT = CS == 2 ? 16 * half : (asg - (asg / nct) * nct) * 16;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;

  f32x4 acc[NCT][9], accb[NCT];
#pragma unroll
  for (int c = 0; c < NCT; ++c) {
    accb[c] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 9; ++k) acc[c][k] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  if constexpr (F32) {
    const int ciL = XC ? 0 : ciT;  // the tile's column in the staged X rows
    const bool bias = CS == 1 || ciT == 0;  // CS == 2: only half 0 computes the bias (block-uniform)
#pragma unroll 1
    for (int s0 = 0; s0 < nslot; s0 += 32) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int sl = s0 + 4 * j + g;  // this lane's K slot of MFMA j
        float a[NCT];
#pragma unroll
        for (int c = 0; c < NCT; ++c) a[c] = sdY[(long)sl * DS + coT + 16 * c + i16];
        // padding slots (r >= R) carry dY == 0; clamp their row into initialised LDS
        const int rs0 = sl / Wp, cs = sl - rs0 * Wp, rs = min(rs0, R - 1);
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int kh = tap / 3, kw = tap % 3;
          const float bx_ = sX[(long)((rs + kh) * XW + cs + kw) * XS + ciL + i16];
#pragma unroll
          for (int c = 0; c < NCT; ++c) acc[c][tap] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c], bx_, acc[c][tap], 0, 0, 0);
        }
        if (bias) {
#pragma unroll
          for (int c = 0; c < NCT; ++c) accb[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c], 1.f, accb[c], 0, 0, 0);
        }
      }
    }
  } else {
    bf16x8 ones;
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (short)0x3F80;

    // 32-bit LDS element offsets (64-bit generic-pointer math per read cost a
    // v_mad_u64_u32 each); a tap adds the constant (kh * XW + kw) * XS, which folds into
    // the ds_read offset field under the geometry specialisation
    const int ldsX = nslot * DS;  // sX = sdY + nslot * DS
    lds_char* lsm = (lds_char*)smem;
    for (int s0 = 0; s0 < nslot; s0 += 32) {
      const int sA = s0 + 4 * g + q, sB = s0 + 16 + 4 * g + q;  // this lane's tr-read rows
      bf16x8 a[NCT];
#pragma unroll
      for (int c = 0; c < NCT; ++c) {
        const int oA = sA * DS + coT + 16 * c + 4 * p, oB = sB * DS + coT + 16 * c + 4 * p;
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(lds_ptr4(lsm, oA));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(lds_ptr4(lsm, oB));
        a[c] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      // X position of slot s for tap (kh,kw): sX row (r+kh), col (c+kw).  Padding slots
      // (r >= R) carry dY == 0; clamp their row so the read stays inside initialised LDS.
      const int rA0 = sA / Wp, cA = sA - rA0 * Wp, rB0 = sB / Wp, cB = sB - rB0 * Wp;
      const int rA = min(rA0, R - 1), rB = min(rB0, R - 1);
      const int xA = ldsX + (rA * XW + cA) * XS + ciT + 4 * p, xB = ldsX + (rB * XW + cB) * XS + ciT + 4 * p;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int kh = tap / 3, kw = tap % 3;
        const int to = (kh * XW + kw) * XS;
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(lds_ptr4(lsm, xA + to));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(lds_ptr4(lsm, xB + to));
        const bf16x8 b = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int c = 0; c < NCT; ++c) acc[c][tap] = mfma16(a[c], b, acc[c][tap]);
      }
      if (CS == 1 || ciT == 0) {  // CS == 2: only half 0 stores the bias (block-uniform)
#pragma unroll
        for (int c = 0; c < NCT; ++c) accb[c] = mfma16(a[c], ones, accb[c]);
      }
    }
  }

  DDP_STAMP(STAMP_K_WGRAD, 3);
  // ---- slab row: [Cout][3][3][Cin] (OHWI, the weight's native layout) then [Cout] bias
  const long row = (long)Cout * 9 * Cin + Cout;
  float* out = slab + (long)rb * row;
  if constexpr (STAGE) {
    __syncthreads();  // every wave is done with the staged tiles
    float* srow = reinterpret_cast<float*>(smem);
    // LDS position of row element e (output channel co): e + 16 * (co / 4), bias block
    // + 16 * Cout / 4.  The 4 output rows of an MFMA lane group sit 4 * 9 * Cin floats
    // apart (a multiple of the 64 banks); the skew spreads them over 4 bank quarters, and
    // keeps runs of 4 elements contiguous and 16-byte aligned for the read-back.
    const int wrow = 9 * Cin;
#pragma unroll
    for (int c = 0; c < NCT; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = coT + 16 * c + 4 * g + r;
        const int sk = 16 * (co >> 2);
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) srow[co * wrow + tap * Cin + ciT + i16 + sk] = acc[c][tap][r];
        if (ciT == 0 && i16 == 0) srow[Cout * wrow + 4 * Cout + co] = accb[c][r];
      }
    __syncthreads();
    // row % 4 == 0 and the slab rows are 16-byte aligned (checked by the launcher)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)(row * 4), 0x00020000);
    typedef __attribute__((ext_vector_type(4))) int i32x4_t;
    if constexpr (CS == 2) {
      // this half's 4-float runs: (co, tap) row ct, columns 16 * half + 4 * cq; half 0 also
      // the bias quads
      const int nq = Cout * 9 * 4;
      const int nst = nq + (half == 0 ? Cout / 4 : 0);
      for (int i = threadIdx.x; i < nst; i += 256) {
        const int e = i < nq ? (i >> 2) * Cin + 16 * half + 4 * (i & 3) : Cout * wrow + 4 * (i - nq);
        const int pos = e < Cout * wrow ? e + 16 * ((e / wrow) >> 2) : e + 4 * Cout;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, *reinterpret_cast<const float4*>(srow + pos)),
                                               rs, e * 4, 0, 16 /* sc1: write-through */);
      }
    } else {
      for (int i = threadIdx.x; i < row / 4; i += 256) {
        const int e = 4 * i;
        const int pos = e < Cout * wrow ? e + 16 * ((e / wrow) >> 2) : e + 4 * Cout;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, *reinterpret_cast<const float4*>(srow + pos)),
                                               rs, i * 16, 0, 16 /* sc1: write-through */);
      }
    }
  } else {
#pragma unroll
    for (int c = 0; c < NCT; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = coT + 16 * c + 4 * g + r;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) st_wt(out + ((long)co * 9 + tap) * Cin + ciT + i16, acc[c][tap][r]);
        if (ciT == 0 && i16 == 0) st_wt(out + (long)Cout * 9 * Cin + co, accb[c][r]);
      }
  }
  DDP_STAMP(STAMP_K_WGRAD, 4);
}

template <typename T, bool MASK_DY, bool A1X, int GH, int GW, int GCI, int GCO>
__global__ __launch_bounds__(256) void conv3x3_wgrad_kernel(
    const T* __restrict__ dY, const T* __restrict__ Yact, const T* __restrict__ X,
    float* __restrict__ slab, int B, int H, int W, int Cin, int Cout, int R, C1Src c1) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  wgrad_body<T, MASK_DY, A1X, GH, GW, GCI, GCO>(dY, Yact, X, slab, B, H, W, Cin, Cout, R, c1, smem,
                                              blockIdx.x, blockIdx.y);
}

// ---------------------------------------------------------------- fused conv backward
// SimpleCNN's whole conv backward in ONE launch (fusion level 1): blocks [0, nd) run the
// data gradient (+ fused conv1 weight gradient, recomputed ReLU mask), blocks [nd, nd+nw)
// the weight gradient.  Both only read dZ2 and the compact batch, so they are
// independent; one launch saves a dependent kernel boundary and lets the wgrad blocks
// fill the CUs the dgrad grid leaves idle (2 blocks per CU: <= 256 VGPR+AGPR per lane).
// Block-uniform role branch.
// DA1X / WA1X: the dgrad / wgrad role recomputes a1 = relu(conv1(x)) from the compact
// uint8 batch; otherwise it reads the a1 the forward stored (Xact).  Measured: the dgrad
// role only needs a1's ReLU mask of its own pixels and gets ~2 us faster reading it; the
// wgrad role needs full a1 tiles with halo and is as fast recomputing as loading.
// bf16: 2 blocks per CU (<= 256 VGPR+AGPR per lane); fp32 tiles take ~135 KiB of LDS, so
// one block per CU and the full register file
// FRED (fused reduction): the last blocks of the grid also do grad_reduce's work
// (slab_reduce.h).  Every block, once its slab rows are stored write-through and
// drained, adds 1 to one of 8 per-XCD-sharded counters (red.done[32 * (blockIdx % 8)],
// zeroed by the step's forward); the blocks from red.first_reducer on then wait until all
// blocks have arrived and reduce the 64-output chunks w, w + nr, ... (sc1 loads, grad_
// reduce's fixed order: bit-identical) with the fused SGD / shadows.  Deadlock-free: the
// blocks below first_reducer never wait, a waiting block has already arrived, and the
// host keeps the reducers within half the resident capacity (they are dispatched last,
// each into a slot it can hold while the rest are dispatched).
// CS: wgrad role channel split (see wgrad_body); the grid then has CS wgrad blocks per
// slab row.
// FCR (fuse level 3, single process): the fc weight gradient + fused SGD (fc_bwd_body
// without dX, dL given by the level-3 forward) as a third role: blocks [nconv, grid) after
// the conv roles.  They never wait and are not counted by the fused reduction, so the
// dispatch-order argument above is unchanged (every block a reducer waits for has a lower
// index than the reducer); the fc role's own last block (FcBwdExtras::last_ctr) finishes the
// fc bias, the loss and the step counter (launchers.h BwdFc).
constexpr int BFC_MAXB = 64;  // batch capacity of the fc role (the README's B = 64 example runs level 3)

// dL of the batch into LDS ([B][FCDW_LD] padded rows); the fc role's block 0 (first0) also
// finishes the fc bias, the loss and the step counter (nothing else in the launch reads them)
__device__ __forceinline__ float* fc_role_prologue(const BwdFc& fcr, int B, char* smem, bool first0) {
  float* s_dl = reinterpret_cast<float*>(smem);  // [B][FCDW_LD] (padded rows)
  for (int i = threadIdx.x; i < B * 10; i += 256) s_dl[(i / 10) * FCDW_LD + i % 10] = fcr.dl[i];
  __syncthreads();
  if (first0 && threadIdx.x < 64) {  // fc_bwd_bias_loss reads dense [B][10] rows
    float* s_dd = s_dl + B * FCDW_LD;
    for (int i = threadIdx.x; i < B * 10; i += 64) s_dd[i] = s_dl[(i / 10) * FCDW_LD + i % 10];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (same wave: the copy is in LDS)
    fc_bwd_bias_loss<false>(fcr.ex, s_dd, nullptr, B, 10, true);
  }
  return s_dl;
}
// one 128-column chunk of the fc weight gradient + SGD on this wave
template <typename T>
__device__ __forceinline__ void fc_role_chunk(const BwdFc& fcr, const float* s_dl, int B, long q) {
  const T* a2 = static_cast<const T*>(fcr.a2);
  // (B <= 32, the reference batch: 32 row loads per lane instead of 48 clamped ones)
  if (B <= 32) fc_dw_wave_chunk<32>(s_dl, a2, fcr.dW, fcr.scale, B, fcr.K, fcr.ex, q * 128);
  else fc_dw_wave_chunk<BFC_MAXB>(s_dl, a2, fcr.dW, fcr.scale, B, fcr.K, fcr.ex, q * 128);
}

// Spin until *cnt >= want (wave 0 polls with sleeps between polls, so the waiting block
// takes few issue slots from the conv waves sharing its CU); false on a timeout, after
// setting *err = code.  No acquire fence: everything the in-launch all-reduce reads after
// the wait was stored write-through by its producers and is read with system-scope loads
// (an agent-scope acquire is `buffer_inv sc1`, invalidating the XCD's L2 under the conv
// roles sharing it).
template <int SLEEP = 2>
__device__ __forceinline__ bool wait_count(const int* cnt, int want, int* err, int code) {
  __shared__ int s_ok;
  if (threadIdx.x < 64) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool ok = true;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > DZ_WAIT_TICKS) {
        if (threadIdx.x == 0 && err) __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(SLEEP);
    }
    if (threadIdx.x == 0) s_ok = ok ? 1 : 0;
  }
  __syncthreads();
  return s_ok != 0;
}

// this block's global stores are out (each wave drained - they are write-through: the
// producers of a multi-GPU step store their gradients system-scope), then one relaxed
// count.  (An agent-scope release here is `buffer_wbl2 sc1`: a write-back of the XCD's
// whole L2 per block.)
__device__ __forceinline__ void count_done(int* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T, int PXT, bool DA1X, bool WA1X, int GH, int GW, int GCI, int GCO, bool FRED, int CS = 1,
          bool FCR = false, int DG = 1, bool XAR = false>
__global__ __launch_bounds__(256, (sizeof(T) == 2 || CS == 2) ? 2 : 1) void conv3x3_bwd_kernel(
    const T* __restrict__ dY, const T* __restrict__ WT, T* __restrict__ dX,
    float* __restrict__ w1slab, float* __restrict__ slab, int B, int H, int W, int Cin, int Cout,
    int R, int nd, C1Src c1, const T* __restrict__ Xact, BwdReduce red, BwdFc fcr, BwdXar xar) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // conv-role index: the in-launch all-reduce blocks (XAR, the grid's head) and the fc-role
  // blocks [fc0, fc0 + nfc) are cut out of the grid order
  int cb = (int)blockIdx.x;
  if constexpr (XAR) {
    static_assert(FCR && FRED, "the in-launch all-reduce waits for the fc role and the fused reduction");
    // multi-GPU level-3 step (BwdXar): the bucket all-reduces run here, each as soon as its
    // gradients are final - the fc bucket while the conv roles still run (SURVEY.md §2.6 I6:
    // DDP's bucket 0 overlapping the rest of the backward), the conv bucket right behind the
    // last fused reducer.  Each role block waits only for this launch's producers and for the
    // same role block of its peers.  Deadlock freedom: the launcher takes this variant only
    // when the WHOLE grid (role + fc + conv + reducer blocks) fits the GPU's resident slots of
    // this instantiation (bwd_launch, hipOccupancy), so no block waits for an undispatched
    // one; a larger grid relies on in-order workgroup dispatch (these blocks come first) and
    // is opt-in, DDP_AMD_L3_INORDER=1, as for the level-3 forward.
    const int nx = xar.nblk0 + xar.nblk1;
    if (cb < nx) {
      unsigned* s_sh = reinterpret_cast<unsigned*>(smem);
      DDP_STAMP(STAMP_K_XGMI, 0);
      // the bucket's arguments into this block's LDS while it waits: read from global memory
      // inside the body, every field was re-loaded after each store (they may alias), ~1 us a
      // time; from LDS (another address space) the compiler keeps them
      const int k = cb < xar.nblk0 ? 0 : 1;
      XgmiArgs* s_xa = reinterpret_cast<XgmiArgs*>(smem + 64);
      {
        const int* src = reinterpret_cast<const int*>(xar.args + k);
        int* dst = reinterpret_cast<int*>(s_xa);
        for (int i = threadIdx.x; i < (int)(sizeof(XgmiArgs) / 4); i += 256) dst[i] = src[i];
      }
      if (k == 0) {
        const bool ok = wait_count(xar.fc_done, xar.fc_expect, xar.err, XAR_ERR);  // (its barrier orders the copy)
        DDP_STAMP(STAMP_K_XGMI, 5);
        if (ok) xgmi_allreduce_body(*s_xa, cb, xar.nblk0, s_sh);
      } else {
        const bool ok = wait_count(xar.fc_done, xar.fc_expect, xar.err, XAR_ERR) &&
                        wait_count(xar.red_done, xar.red_expect, xar.err, XAR_ERR);
        DDP_STAMP(STAMP_K_XGMI, 5);
        if (ok) xgmi_allreduce_body(*s_xa, cb - xar.nblk0, xar.nblk1, s_sh);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      DDP_STAMP(STAMP_K_XGMI, 7);
      if (threadIdx.x == 0) {
        // the step's last work item advances the batch window (the fc role read it before
        // counting itself into fc_done, which every role block waited for)
        // (relaxed: nothing is published through it - an agent-scope acq_rel is an L2
        // write-back + invalidate of the XCD per block)
        const int old = __hip_atomic_fetch_add(xar.xar_done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == nx - 1 && xar.step_ctr) xar.step_ctr[0] += 1;
      }
      return;
    }
    cb -= nx;
  }
  if constexpr (FCR) {
    const int f = cb - fcr.fc0;
    if (f >= 0 && f < fcr.nfc) {
      // fc role (persistent): dL of the batch into LDS once, block 0 finishes the fc bias,
      // the loss and the step counter (nothing else in this launch reads them), then every
      // wave takes 128-column chunks f * 4 + wave, + 4 * nfc, ... (fc_dw_wave_chunk)
      DDP_STAMP(STAMP_K_FC_BWD, 0);
      // raised issue priority: the fc role's late-dispatched blocks are one of the launch's
      // two tails (+0.9 %, profiles/r3_cnn/prio)
      __builtin_amdgcn_s_setprio(2);
      const float* s_dl = fc_role_prologue(fcr, B, smem, f == 0);
      DDP_STAMP(STAMP_K_FC_BWD, 1);
      // one 128-column chunk per wave, straight-line (a chunk loop let the compiler hoist
      // every row offset / guard of the unrolled body out of it: 300 spilled registers)
      const int nch = (int)((fcr.K + 127) / 128);
      const int q = f * 4 + (threadIdx.x >> 6);
      if (q < nch) fc_role_chunk<T>(fcr, s_dl, B, q);
      DDP_STAMP(STAMP_K_FC_BWD, 4);
      if constexpr (XAR) count_done(xar.fc_done);  // the fc bucket's gradient rows are out
      return;
    }
    if (f >= 0) cb -= fcr.nfc;
  }
  // exact fp32 with the channel split: the dgrad role reads its weights from global
  // (dgrad_body WGS); DG == 2 also splits it over input-channel halves, two blocks per pixel
  // chunk, paired 8 apart (same XCD, as the wgrad halves) - nd counts both halves
  constexpr bool WG = sizeof(T) == 4 && CS == 2;
  constexpr int WGS = WG ? (DG == 2 ? 1 : 2) : 0;
  const int nw = (red.nconv > 0 ? red.nconv : (int)gridDim.x) - nd;  // (nconv is always set by the launcher)
  int rd = cb;  // role-local index: dgrad block rd (rd < nd) or wgrad block rd - nd
  if (red.interleave) {
    const int m = nd < nw ? nd : nw;
    if (cb < 2 * m) rd = (cb & 1) ? nd + (cb >> 1) : (cb >> 1);
    else rd = nd > nw ? cb - m : nd + (cb - m);
  }
  if (rd < nd) {
    const int db = rd;
    int px = db, hf = 0;
    if constexpr (WGS == 1) {
      if (((nd >> 1) & 7) == 0) {
        hf = (db >> 3) & 1;
        px = ((db >> 4) << 3) | (db & 7);
      } else {
        hf = db & 1;
        px = db >> 1;
      }
    }
    dgrad_body<T, PXT, false, true, true, DA1X, GH, GW, GCI, GCO, WGS>(
        dY, nullptr, WT, DA1X ? nullptr : Xact, dX, B, H, W, Cin, Cout, c1.x, 1, c1.bi, w1slab, c1, smem, px, hf);
  } else {
    wgrad_body<T, false, WA1X, GH, GW, GCI, GCO, !WG, CS>(dY, nullptr, WA1X ? nullptr : Xact, slab, B, H,
                                                         W, Cin, Cout, R, c1, smem, rd - nd, 0);
  }
  if constexpr (FRED) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slab stores are out
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add(red.done + 32 * (blockIdx.x & 7), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cb < red.first_reducer) return;
    // reducer w of nr: the LAST nr conv blocks of the grid (dispatched after every block they
    // wait for; the host keeps nr within a quarter of the resident capacity)
    const int nblk = red.nconv > 0 ? red.nconv : (int)gridDim.x;
    const int w = cb - red.first_reducer, nw = nblk - red.first_reducer;
    // (a lambda capturing only scalars: capturing the kernel argument put the SlabSet in scratch)
    int* const done = red.done;
    int* const errw = red.err;
    auto wait_all = [done, errw, nblk]() {
      if (threadIdx.x < 64) {  // wave 0 polls the 8 shards (sc1 loads), sleeping between polls
        const int lane = threadIdx.x;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (true) {
          const int v = lane < 8 ? __hip_atomic_load(done + 32 * lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
          int tot = 0;
#pragma unroll
          for (int l = 0; l < 8; ++l) tot += __builtin_amdgcn_readlane(v, l);
          if (tot >= nblk) break;
          if (__builtin_amdgcn_s_memrealtime() - t0 > DZ_WAIT_TICKS) {
            if (lane == 0 && errw) __hip_atomic_store(errw, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      __syncthreads();
    };
    float* part = reinterpret_cast<float*>(smem);
    if (red.deep) {
      constexpr int J = 2;  // chunks per reducer pass (thread t < 64 * J finalises one output of chunk t >> 6)
      SlabFusedPlan<J> pl;
      slab_fused_plan<J>(red.ss, w, nw, red.nchunks, pl);  // index work + SGD operands before the wait
      DDP_STAMP(STAMP_K_GRAD_REDUCE, 0);
      wait_all();
      DDP_STAMP(STAMP_K_GRAD_REDUCE, 1);
      slab_fused_run16<J>(red.ss, pl, part);
      for (long q0 = w + (long)J * nw; q0 < red.nchunks; q0 += (long)J * nw) {  // few wgrad blocks: more passes
        slab_fused_plan<J>(red.ss, q0, nw, red.nchunks, pl);
        slab_fused_run16<J>(red.ss, pl, part);
      }
    } else {
      constexpr int J = 3;
      SlabFusedPlan<J> pl;
      slab_fused_plan<J>(red.ss, w, nw, red.nchunks, pl);
      DDP_STAMP(STAMP_K_GRAD_REDUCE, 0);
      wait_all();
      DDP_STAMP(STAMP_K_GRAD_REDUCE, 1);
      slab_fused_run<J>(red.ss, pl, part);
      for (long q0 = w + (long)J * nw; q0 < red.nchunks; q0 += (long)J * nw) {
        slab_fused_plan<J>(red.ss, q0, nw, red.nchunks, pl);
        slab_fused_run<J>(red.ss, pl, part);
      }
    }
    if (w == 0 && threadIdx.x == 0 && red.ss.step_ctr) red.ss.step_ctr[0] += 1;
    DDP_STAMP(STAMP_K_GRAD_REDUCE, 2);
    if constexpr (XAR) count_done(xar.red_done);  // this reducer's conv gradients are out
  }
}

// ---------------------------------------------------------------- launchers
// es = element size (2: bf16, 4: exact fp32)
static inline bool simplecnn_geom(int H, int W, int Cin, int Cout) {
  return H == 28 && W == 28 && Cin == 32 && Cout == 64;
}

// Kernels whose dynamic LDS exceeds the 64 KiB default must opt in once per
// instantiation (fp32 tiles use up to ~135 KiB of the CU's 160 KiB).
template <typename K>
static void lds_optin(K kernel, size_t bytes) {
  if (bytes > 65536) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// DDP_AMD_L3_INORDER=1: launches whose spinning blocks would not all be resident at once may
// rely on in-order workgroup dispatch (the hardware does not promise it) - the level-3
// forward beyond one wave of blocks, and the in-launch all-reduce (dist_mode 2)
static bool inorder_optin() {
  const char* e = getenv("DDP_AMD_L3_INORDER");  // (read per call: launch-plan time only)
  return e && e[0] == '1';
}

}  // namespace ddp_amd
