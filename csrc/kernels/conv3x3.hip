// 3x3 / stride 1 / padding 1 convolution on NHWC bf16 activations with MFMA
// (v_mfma_f32_16x16x32_bf16): forward, data gradient and weight gradient.
//
// Reference op: model.py:11-12 (nn.Conv2d(32,64,3,padding=1) -> nn.ReLU()), i.e.
// the layer that carries 95% of SimpleCNN's FLOPs.
//
// Implicit GEMM, output channels on the MFMA rows and pixels on the columns:
//   fwd   D[co][px] += W[co][tap][ci]   . X[px+tap][ci]        K = 9*Cin
//   dgrad D[ci][px] += WT[tap][ci][co]  . dY[px-tap][co]       K = 9*Cout
//   wgrad D[co][ci] += dY[px][co]       . X[px+tap][ci]        K = pixels (per tap)
// A K-step of 32 is one tap x 32 contiguous channels, so every A/B fragment is a
// single 16-byte load of 8 contiguous bf16.  Each lane finishes with 4
// consecutive channels of one pixel -> one 8-byte NHWC store per 16x16 tile.
//
// Fusions (templates):
//  * fwd:   bias + ReLU epilogue; FUSE_FC additionally dots the bf16 output tile
//           with the following Linear layer's weight (SimpleCNN's fc, stored
//           [out][H*W][C]) and writes per-16-pixel partial logits, so the fc
//           forward never re-reads the activation (SURVEY.md §2.4 K5 note).
//  * dgrad: ReLU mask of the upstream gradient (MASK_DY, module path) and of the
//           layer input (MASK_X: d(relu1)); FUSE_W1 accumulates conv1's weight
//           and bias gradient from the just-computed dZ1 (Cin=1 conv, K11).
//  * wgrad: split-K over image-row chunks, one fp32 slab row per block, bias
//           gradient from an extra MFMA against a ones fragment; fixed-order
//           reduction in grad_reduce (bitwise reproducible, no float atomics).
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

// ---------------------------------------------------------------- forward
template <int PXT, bool RELU, bool FUSE_FC>
__global__ __launch_bounds__(256) void conv3x3_fwd_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt, const float* __restrict__ bias,
    bf16_t* __restrict__ Y, int B, int H, int W, int Cin, int Cout,
    const bf16_t* __restrict__ wfc, float* __restrict__ fc_part, int NO) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int HW = H * W;
  const long Ptot = (long)B * HW;
  const int co0 = blockIdx.y * 64;
  const long pb = ((long)blockIdx.x * 4 + wave) * 16 * PXT;
  const int kofs = 8 * (lane >> 4);
  const int col = lane & 15;

  int n[PXT], h[PXT], w[PXT];
  bool valid[PXT];
#pragma unroll
  for (int pt = 0; pt < PXT; ++pt) {
    const long P = pb + pt * 16 + col;
    valid[pt] = P < Ptot;
    const long Pc = valid[pt] ? P : 0;
    n[pt] = (int)(Pc / HW);
    const int rem = (int)(Pc - (long)n[pt] * HW);
    h[pt] = rem / W;
    w[pt] = rem - h[pt] * W;
  }
  f32x4 acc[PXT][4];
#pragma unroll
  for (int pt = 0; pt < PXT; ++pt)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[pt][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const bf16_t* wrow = Wt + (long)(co0 + col) * 9 * Cin + kofs;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int dh = tap / 3 - 1, dw = tap % 3 - 1;
    for (int ci0 = 0; ci0 < Cin; ci0 += 32) {
      bf16x8 a[4], b[PXT];
#pragma unroll
      for (int t = 0; t < 4; ++t) a[t] = ld8(wrow + (long)16 * t * 9 * Cin + tap * Cin + ci0);
#pragma unroll
      for (int pt = 0; pt < PXT; ++pt) {
        const int hh = h[pt] + dh, ww = w[pt] + dw;
        const bool ok = valid[pt] && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
        b[pt] = ok ? ld8(X + (((long)n[pt] * H + hh) * W + ww) * Cin + ci0 + kofs) : zero8();
      }
#pragma unroll
      for (int pt = 0; pt < PXT; ++pt)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[pt][t] = mfma16(a[t], b[pt], acc[pt][t]);
    }
  }

  // epilogue: bias + ReLU + bf16 store (+ fc partial logits)
#pragma unroll
  for (int pt = 0; pt < PXT; ++pt) {
    const long P = pb + pt * 16 + col;
    float fcs[FUSE_FC ? 16 : 1];
    if (FUSE_FC) {
#pragma unroll
      for (int o = 0; o < 16; ++o) fcs[o] = 0.f;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int co = co0 + 16 * t + 4 * (lane >> 4);
      const float4 bv = *reinterpret_cast<const float4*>(bias + co);
      float v0 = acc[pt][t][0] + bv.x, v1 = acc[pt][t][1] + bv.y;
      float v2 = acc[pt][t][2] + bv.z, v3 = acc[pt][t][3] + bv.w;
      if (RELU) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f); }
      const uint2 pk = pack4(v0, v1, v2, v3);
      if (valid[pt]) *reinterpret_cast<uint2*>(Y + P * Cout + co) = pk;
      if (FUSE_FC) {
        float q[4];
        unpack4(pk, q);  // the bf16 values actually stored (what backward re-reads)
        const int rem = h[pt] * W + w[pt];
#pragma unroll
        for (int o = 0; o < 16; ++o) {
          if (o < NO) {
            float wv[4];
            unpack4(*reinterpret_cast<const uint2*>(wfc + ((long)o * HW + rem) * Cout + co), wv);
            float s = fcs[o];
            s = fmaf(q[0], wv[0], s); s = fmaf(q[1], wv[1], s);
            s = fmaf(q[2], wv[2], s); s = fmaf(q[3], wv[3], s);
            fcs[o] = valid[pt] ? s : 0.f;
          }
        }
      }
    }
    if (FUSE_FC) {
      // whole 16-pixel tile lies in one image (HW % 16 == 0, checked on host)
      const long g = (pb + pt * 16) / 16;
      const bool tile_ok = (pb + pt * 16) < Ptot;
#pragma unroll
      for (int o = 0; o < 16; ++o) {
        if (o < NO) {
          const float s = wave_sum(fcs[o]);
          if (lane == 0 && tile_ok) fc_part[g * NO + o] = s;
        }
      }
    }
  }
}

// ---------------------------------------------------------------- data gradient
template <int PXT, bool MASK_DY, bool MASK_X, bool FUSE_W1>
__global__ __launch_bounds__(256) void conv3x3_dgrad_kernel(
    const bf16_t* __restrict__ dY, const bf16_t* __restrict__ Yact, const bf16_t* __restrict__ WT,
    const bf16_t* __restrict__ Xact, bf16_t* __restrict__ dX, int B, int H, int W, int Cin, int Cout,
    const void* __restrict__ x0, int x0_u8, BatchIdx bi, float* __restrict__ w1slab) {
  __shared__ float s_w1[FUSE_W1 ? 4 * 320 : 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int HW = H * W;
  const long Ptot = (long)B * HW;
  const int ci_blk = blockIdx.y * 32;
  const long pb = ((long)blockIdx.x * 4 + wave) * 16 * PXT;
  const int kofs = 8 * (lane >> 4);
  const int col = lane & 15;

  int n[PXT], h[PXT], w[PXT];
  bool valid[PXT];
#pragma unroll
  for (int pt = 0; pt < PXT; ++pt) {
    const long P = pb + pt * 16 + col;
    valid[pt] = P < Ptot;
    const long Pc = valid[pt] ? P : 0;
    n[pt] = (int)(Pc / HW);
    const int rem = (int)(Pc - (long)n[pt] * HW);
    h[pt] = rem / W;
    w[pt] = rem - h[pt] * W;
  }
  f32x4 acc[PXT][2];
#pragma unroll
  for (int pt = 0; pt < PXT; ++pt) acc[pt][0] = acc[pt][1] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int dh = 1 - tap / 3, dw = 1 - tap % 3;  // dY pixel = (h + 1 - kh, w + 1 - kw)
    const bf16_t* wtap = WT + ((long)tap * Cin + ci_blk + col) * Cout + kofs;
    for (int co0 = 0; co0 < Cout; co0 += 32) {
      const bf16x8 a0 = ld8(wtap + co0);
      const bf16x8 a1 = ld8(wtap + (long)16 * Cout + co0);
      bf16x8 b[PXT];
#pragma unroll
      for (int pt = 0; pt < PXT; ++pt) {
        const int hh = h[pt] + dh, ww = w[pt] + dw;
        const bool ok = valid[pt] && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
        const long off = (((long)n[pt] * H + hh) * W + ww) * Cout + co0 + kofs;
        b[pt] = ok ? ld8(dY + off) : zero8();
        if (MASK_DY) b[pt] = ok ? mask8(b[pt], ld8(Yact + off)) : b[pt];
      }
#pragma unroll
      for (int pt = 0; pt < PXT; ++pt) {
        acc[pt][0] = mfma16(a0, b[pt], acc[pt][0]);
        acc[pt][1] = mfma16(a1, b[pt], acc[pt][1]);
      }
    }
  }

  float w1a[FUSE_W1 ? 2 : 1][4][10];
  if (FUSE_W1) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 10; ++k) w1a[t][j][k] = 0.f;
  }
  const int base = (FUSE_W1 && x0_u8) ? bi.base() : 0;
#pragma unroll
  for (int pt = 0; pt < PXT; ++pt) {
    const long P = pb + pt * 16 + col;
    float xv[9];
    if (FUSE_W1) {
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int hh = h[pt] + k / 3 - 1, ww = w[pt] + k % 3 - 1;
        const bool ok = valid[pt] && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
        float v = 0.f;
        if (ok) {
          if (x0_u8) v = (float)((const unsigned char*)x0)[(long)bi.row(n[pt], base) * HW + hh * W + ww] / 255.0f;
          else v = ((const float*)x0)[(long)n[pt] * HW + hh * W + ww];
        }
        xv[k] = v;
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int ci = ci_blk + 16 * t + 4 * (lane >> 4);
      float v[4] = {acc[pt][t][0], acc[pt][t][1], acc[pt][t][2], acc[pt][t][3]};
      if (MASK_X && valid[pt]) {
        float xa[4];
        unpack4(*reinterpret_cast<const uint2*>(Xact + P * Cin + ci), xa);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = xa[j] > 0.f ? v[j] : 0.f;
      }
      const uint2 pk = pack4(v[0], v[1], v[2], v[3]);
      if (valid[pt]) *reinterpret_cast<uint2*>(dX + P * Cin + ci) = pk;
      if (FUSE_W1) {
        float q[4];
        unpack4(pk, q);
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
  if (FUSE_W1) {
    // reduce over the 16 pixel lanes that share a channel group, then over waves (fixed order)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 10; ++k) w1a[t][j][k] = sum16(w1a[t][j][k]);
    if (col == 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ci = 16 * t + 4 * (lane >> 4) + j;  // conv1 output channel (Cin == 32)
#pragma unroll
          for (int k = 0; k < 9; ++k) s_w1[wave * 320 + ci * 9 + k] = w1a[t][j][k];
          s_w1[wave * 320 + 288 + ci] = w1a[t][j][9];
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 320; i += 256)
      w1slab[(long)blockIdx.x * 320 + i] = ((s_w1[i] + s_w1[320 + i]) + s_w1[640 + i]) + s_w1[960 + i];
  }
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
template <bool MASK_DY>
__global__ __launch_bounds__(256) void conv3x3_wgrad_kernel(
    const bf16_t* __restrict__ dY, const bf16_t* __restrict__ Yact, const bf16_t* __restrict__ X,
    float* __restrict__ slab, int B, int H, int W, int Cin, int Cout, int R) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nRC = (H + R - 1) / R;
  const int n = blockIdx.x / nRC;
  const int r0 = (blockIdx.x - n * nRC) * R;
  const int Wp = (W + 7) & ~7;
  const int DS = Cout + 16, XS = Cin + 16;  // LDS row strides (elements)
  const int nslot = ((R * Wp + 31) / 32) * 32;
  bf16_t* sdY = reinterpret_cast<bf16_t*>(smem);
  bf16_t* sX = sdY + (long)nslot * DS;
  const int XW = Wp + 2;

  // ---- stage dY rows (masked) and X rows with halo, 16 B per thread-iteration
  const int cpy_dy = Cout / 8, cpy_x = Cin / 8;
  for (int i = threadIdx.x; i < nslot * cpy_dy; i += 256) {
    const int slot = i / cpy_dy, ch = (i - slot * cpy_dy) * 8;
    const int r = slot / Wp, c = slot - (slot / Wp) * Wp;
    const int hh = r0 + r;
    bf16x8 v = zero8();
    if (r < R && hh < H && c < W) {
      const long off = (((long)n * H + hh) * W + c) * Cout + ch;
      v = ld8(dY + off);
      if (MASK_DY) v = mask8(v, ld8(Yact + off));
    }
    *reinterpret_cast<bf16x8*>(sdY + (long)slot * DS + ch) = v;
  }
  for (int i = threadIdx.x; i < (R + 2) * XW * cpy_x; i += 256) {
    const int pos = i / cpy_x, ch = (i - pos * cpy_x) * 8;
    const int rr = pos / XW, cc = pos - (pos / XW) * XW;
    const int hh = r0 - 1 + rr, ww = cc - 1;
    bf16x8 v = zero8();
    if ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
      v = ld8(X + (((long)n * H + hh) * W + ww) * Cin + ch);
    *reinterpret_cast<bf16x8*>(sX + (long)pos * XS + ch) = v;
  }
  __syncthreads();

  // ---- wave assignment: (pair of 16-wide co tiles) x (16-wide ci tile)
  const int nct = Cin / 16;
  const int asg = blockIdx.y * 4 + wave;
  const int coT = (asg / nct) * 32;
  const int ciT = (asg - (asg / nct) * nct) * 16;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;

  f32x4 acc[2][9], accb[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    accb[c] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 9; ++k) acc[c][k] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (short)0x3F80;

  for (int s0 = 0; s0 < nslot; s0 += 32) {
    const int sA = s0 + 4 * g + q, sB = s0 + 16 + 4 * g + q;  // this lane's tr-read rows
    bf16x8 a[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const bf16_t* pA = sdY + (long)sA * DS + coT + 16 * c + 4 * p;
      const bf16_t* pB = sdY + (long)sB * DS + coT + 16 * c + 4 * p;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)pA);
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)pB);
      a[c] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
    // X position of slot s for tap (kh,kw): sX row (r+kh), col (c+kw).  Padding slots
    // (r >= R) carry dY == 0; clamp their row so the read stays inside initialised LDS.
    const int rA0 = sA / Wp, cA = sA - rA0 * Wp, rB0 = sB / Wp, cB = sB - rB0 * Wp;
    const int rA = min(rA0, R - 1), rB = min(rB0, R - 1);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap % 3;
      const bf16_t* pA = sX + (long)((rA + kh) * XW + cA + kw) * XS + ciT + 4 * p;
      const bf16_t* pB = sX + (long)((rB + kh) * XW + cB + kw) * XS + ciT + 4 * p;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)pA);
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)pB);
      const bf16x8 b = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      acc[0][tap] = mfma16(a[0], b, acc[0][tap]);
      acc[1][tap] = mfma16(a[1], b, acc[1][tap]);
    }
    accb[0] = mfma16(a[0], ones, accb[0]);
    accb[1] = mfma16(a[1], ones, accb[1]);
  }

  // ---- slab row: [Cout][3][3][Cin] (OHWI, the weight's native layout) then [Cout] bias
  float* out = slab + (long)blockIdx.x * ((long)Cout * 9 * Cin + Cout);
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = coT + 16 * c + 4 * g + r;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) out[((long)co * 9 + tap) * Cin + ciT + i16] = acc[c][tap][r];
      if (ciT == 0 && i16 == 0) out[(long)Cout * 9 * Cin + co] = accb[c][r];
    }
}

// ---------------------------------------------------------------- launchers
void conv3x3_fwd(const bf16_t* X, const bf16_t* Wt, const float* bias, bf16_t* Y, int B, int H,
                 int W, int Cin, int Cout, bool relu, const bf16_t* wfc, float* fc_part, int NO,
                 int pxt, hipStream_t s) {
  const long P = (long)B * H * W;
  const int per_blk = 4 * 16 * pxt;
  const dim3 grid((unsigned)((P + per_blk - 1) / per_blk), Cout / 64);
  const bool fc = wfc != nullptr;
#define LF(PX, RL, FC) hipLaunchKernelGGL((conv3x3_fwd_kernel<PX, RL, FC>), grid, dim3(256), 0, s, X, Wt, bias, Y, B, H, W, Cin, Cout, wfc, fc_part, NO)
  if (pxt == 2) {
    if (fc) LF(2, true, true); else if (relu) LF(2, true, false); else LF(2, false, false);
  } else {
    if (fc) LF(1, true, true); else if (relu) LF(1, true, false); else LF(1, false, false);
  }
#undef LF
}

void conv3x3_dgrad(const bf16_t* dY, const bf16_t* Yact, const bf16_t* WT, const bf16_t* Xact,
                   bf16_t* dX, int B, int H, int W, int Cin, int Cout, const void* x0, bool x0_u8,
                   BatchIdx bi, float* w1slab, int pxt, hipStream_t s) {
  const long P = (long)B * H * W;
  const int per_blk = 4 * 16 * pxt;
  const dim3 grid((unsigned)((P + per_blk - 1) / per_blk), Cin / 32);
  const bool mdy = Yact != nullptr, mx = Xact != nullptr, w1 = w1slab != nullptr;
#define LD(PX, A, Bm, C) hipLaunchKernelGGL((conv3x3_dgrad_kernel<PX, A, Bm, C>), grid, dim3(256), 0, s, dY, Yact, WT, Xact, dX, B, H, W, Cin, Cout, x0, (int)x0_u8, bi, w1slab)
  if (pxt == 2) {
    if (w1) LD(2, false, true, true);
    else if (mdy && mx) LD(2, true, true, false);
    else if (mdy) LD(2, true, false, false);
    else if (mx) LD(2, false, true, false);
    else LD(2, false, false, false);
  } else {
    if (w1) LD(1, false, true, true);
    else if (mdy && mx) LD(1, true, true, false);
    else if (mdy) LD(1, true, false, false);
    else if (mx) LD(1, false, true, false);
    else LD(1, false, false, false);
  }
#undef LD
}

int conv3x3_dgrad_blocks(int B, int H, int W, int pxt) {
  const long P = (long)B * H * W;
  const int per_blk = 4 * 16 * pxt;
  return (int)((P + per_blk - 1) / per_blk);
}

int conv3x3_wgrad_blocks(int B, int H, int R) { return B * ((H + R - 1) / R); }

size_t conv3x3_wgrad_lds(int W, int Cin, int Cout, int R) {
  const int Wp = (W + 7) & ~7;
  const int nslot = ((R * Wp + 31) / 32) * 32;
  return sizeof(bf16_t) * ((size_t)nslot * (Cout + 16) + (size_t)(R + 2) * (Wp + 2) * (Cin + 16));
}

void conv3x3_wgrad(const bf16_t* dY, const bf16_t* Yact, const bf16_t* X, float* slab, int B,
                   int H, int W, int Cin, int Cout, int R, hipStream_t s) {
  const dim3 grid(conv3x3_wgrad_blocks(B, H, R), (Cout / 32) * (Cin / 16) / 4);
  const size_t lds = conv3x3_wgrad_lds(W, Cin, Cout, R);
  if (Yact)
    hipLaunchKernelGGL(conv3x3_wgrad_kernel<true>, grid, dim3(256), lds, s, dY, Yact, X, slab, B, H, W, Cin, Cout, R);
  else
    hipLaunchKernelGGL(conv3x3_wgrad_kernel<false>, grid, dim3(256), lds, s, dY, Yact, X, slab, B, H, W, Cin, Cout, R);
}

}  // namespace ddp_amd
