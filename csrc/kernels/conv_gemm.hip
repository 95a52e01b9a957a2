// General NHWC convolution as an LDS-tiled MFMA implicit GEMM (ResNet-18 layers:
// 3x3 s1/s2, 1x1 s2 downsample; SURVEY.md §2.4 "north-star" kernels).
//
// Forward, output channels on the MFMA rows, output pixels on the columns:
//   D[co][p] = sum_{tap, ci} W[co][tap][ci] * X[n][oh*s - pad + kh][ow*s - pad + kw][ci]
// K-step = one tap x 32 input channels (Cin % 32 == 0).  Block tile = BCO output
// channels x 128 output pixels, 4 waves arranged 2 (co) x 2 (px); each wave owns
// (BCO/2) x 64 = (BCO/32) x 4 tiles of 16x16.  Per K-step the block stages the
// weight tile [BCO][32] and the gathered input tile [128][32] into LDS (double
// buffered: the next K-step's global loads are issued before this step's MFMAs),
// rows padded to 40 elements (80 B) so the 16 rows of a fragment read hit distinct
// bank groups.
//
// Epilogue: bf16 NHWC store (+ optional bias / ReLU) and, when requested, per-block
// partial per-channel sum and sum-of-squares of the stored values (the training
// BatchNorm that follows needs exactly these; fixed-order reduction in bn_stats).
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

constexpr int CG_BP = 128;  // output pixels per block
constexpr int CG_KS = 32;   // K-step (channels of one tap)
constexpr int CG_RS = 40;   // LDS row stride (elements)

// STEM: Cin == 4 (3 real channels + 1 zero pad); a K-step covers 8 taps x 4 channels,
// k = tap*4 + c, so the weight row [KH*KW*4] is still contiguous per K-step.
template <int BCO, bool RELU, bool STATS, bool STEM>
__global__ __launch_bounds__(256) void conv_gemm_fwd_kernel(ConvGeom g, const bf16_t* __restrict__ X,
                                                            const bf16_t* __restrict__ Wt,
                                                            const float* __restrict__ bias,
                                                            bf16_t* __restrict__ Y,
                                                            float* __restrict__ stats) {
  __shared__ __attribute__((aligned(16))) bf16_t sA[2][BCO * CG_RS];
  __shared__ __attribute__((aligned(16))) bf16_t sB[2][CG_BP * CG_RS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wco = wave >> 1, wpx = wave & 1;
  constexpr int TCO = BCO / 32;  // 16-row tiles per wave (co)
  const long OHW = (long)g.OH * g.OW;
  const long Ptot = (long)g.N * OHW;
  const long p0 = (long)blockIdx.x * CG_BP;
  const int co0 = blockIdx.y * BCO;
  const int KWC = g.KH * g.KW * g.Cin;
  const int T = g.KH * g.KW;
  const int nk = STEM ? (T + 7) / 8 : T * (g.Cin / CG_KS);

  // this thread's staging slots: B: 2 chunks (pixel r = tid>>1 .. , 16 B each), A: BCO*4/256 chunks
  const int bp = tid >> 1, bh = (tid & 1) * 16;  // pixel row, element offset (two 16-B chunks)
  const long P = p0 + bp;
  const bool pv = P < Ptot;
  int n_ = 0, oh = 0, ow = 0;
  if (pv) {
    n_ = (int)(P / OHW);
    const int r = (int)(P - (long)n_ * OHW);
    oh = r / g.OW;
    ow = r - oh * g.OW;
  }
  auto load_k = [&](int ks, bf16x8* ra, bf16x8* rb) {
    if (STEM) {
      // this thread's 16 elements = taps ks*8 + bh/4 .. +3, 4 channels each (8 B per tap)
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        uint2 two[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int tap = ks * 8 + bh / 4 + h2 * 2 + u;
          const int kh = tap / g.KW, kw = tap - kh * g.KW;
          const int ih = oh * g.stride - g.pad + kh, iw = ow * g.stride - g.pad + kw;
          const bool ok = pv && tap < T && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
          two[u] = ok ? *reinterpret_cast<const uint2*>(X + (((long)n_ * g.H + ih) * g.W + iw) * 4)
                      : make_uint2(0u, 0u);
        }
        uint4 q4 = make_uint4(two[0].x, two[0].y, two[1].x, two[1].y);
        rb[h2] = __builtin_bit_cast(bf16x8, q4);
      }
#pragma unroll
      for (int u = 0; u < BCO * 4 / 256; ++u) {
        const int c = tid + u * 256;
        const int row = c >> 2, off = (c & 3) * 8;
        const int k = ks * CG_KS + off;
        ra[u] = (k < KWC) ? ld8(Wt + (long)(co0 + row) * KWC + k) : zero8();
      }
      return;
    }
    const int tap = ks / (g.Cin / CG_KS);
    const int ci0 = (ks - tap * (g.Cin / CG_KS)) * CG_KS;
    const int kh = tap / g.KW, kw = tap - kh * g.KW;
    // B: gathered input pixel (zero outside the image)
    const int ih = oh * g.stride - g.pad + kh, iw = ow * g.stride - g.pad + kw;
    const bool ok = pv && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
    const bf16_t* src = X + (((long)n_ * g.H + ih) * g.W + iw) * g.Cin + ci0 + bh;
    rb[0] = ok ? ld8(src) : zero8();
    rb[1] = ok ? ld8(src + 8) : zero8();
    // A: weight rows
#pragma unroll
    for (int u = 0; u < BCO * 4 / 256; ++u) {
      const int c = tid + u * 256;
      const int row = c >> 2, off = (c & 3) * 8;
      ra[u] = ld8(Wt + (long)(co0 + row) * KWC + tap * g.Cin + ci0 + off);
    }
  };
  auto store_k = [&](int buf, const bf16x8* ra, const bf16x8* rb) {
    *reinterpret_cast<bf16x8*>(&sB[buf][bp * CG_RS + bh]) = rb[0];
    *reinterpret_cast<bf16x8*>(&sB[buf][bp * CG_RS + bh + 8]) = rb[1];
#pragma unroll
    for (int u = 0; u < BCO * 4 / 256; ++u) {
      const int c = tid + u * 256;
      *reinterpret_cast<bf16x8*>(&sA[buf][(c >> 2) * CG_RS + (c & 3) * 8]) = ra[u];
    }
  };

  f32x4 acc[TCO][4];
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 ra[BCO * 4 / 256 > 0 ? BCO * 4 / 256 : 1], rb[2];
  load_k(0, ra, rb);
  store_k(0, ra, rb);
  __syncthreads();
  const int kofs = 8 * (lane >> 4), col = lane & 15;
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    const bool more = ks + 1 < nk;
    if (more) load_k(ks + 1, ra, rb);  // in flight during this step's MFMAs
    bf16x8 a[TCO], b[4];
#pragma unroll
    for (int i = 0; i < TCO; ++i)
      a[i] = *reinterpret_cast<const bf16x8*>(&sA[cur][(wco * (BCO / 2) + 16 * i + col) * CG_RS + kofs]);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      b[j] = *reinterpret_cast<const bf16x8*>(&sB[cur][(wpx * 64 + 16 * j + col) * CG_RS + kofs]);
#pragma unroll
    for (int i = 0; i < TCO; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
    if (more) store_k(cur ^ 1, ra, rb);
    __syncthreads();
  }

  // ---- epilogue
  float csum[TCO][4], csq[TCO][4];
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) csum[i][r] = csq[i][r] = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long Pj = p0 + wpx * 64 + 16 * j + col;
    const bool ok = Pj < Ptot;
#pragma unroll
    for (int i = 0; i < TCO; ++i) {
      const int co = co0 + wco * (BCO / 2) + 16 * i + 4 * (lane >> 4);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[i][j][r] + (bias ? bias[co + r] : 0.f);
        if (RELU) v[r] = fmaxf(v[r], 0.f);
      }
      const uint2 pk = pack4(v[0], v[1], v[2], v[3]);
      if (ok) *reinterpret_cast<uint2*>(Y + Pj * g.Cout + co) = pk;
      if (STATS) {
        float q[4];
        unpack4(pk, q);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = ok ? q[r] : 0.f;
          csum[i][r] += x;
          csq[i][r] = fmaf(x, x, csq[i][r]);
        }
      }
    }
  }
  if (STATS) {
    // per-block partials: reduce the 16 pixel lanes, then the two pixel-waves via LDS
    __shared__ float s_st[2][2][BCO];
#pragma unroll
    for (int i = 0; i < TCO; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = sum16(csum[i][r]), b = sum16(csq[i][r]);
        if (col == 0) {
          const int cl = wco * (BCO / 2) + 16 * i + 4 * (lane >> 4) + r;
          s_st[wpx][0][cl] = a;
          s_st[wpx][1][cl] = b;
        }
      }
    __syncthreads();
    // stats slab: [blocks_x][2][Cout]
    for (int c = tid; c < BCO; c += 256) {
      float* dst = stats + (long)blockIdx.x * 2 * g.Cout;
      dst[co0 + c] = s_st[0][0][c] + s_st[1][0][c];
      dst[g.Cout + co0 + c] = s_st[0][1][c] + s_st[1][1][c];
    }
  }
}

// ---------------------------------------------------------------- data gradient
// D[ci][p_in] = sum_{tap, co} WT[ci][tap][co] * dY[n][(ih + pad - kh)/s][(iw + pad - kw)/s][co]
// (taps whose offset is not divisible by the stride, or fall outside dY, contribute 0).
// WT is the [Cin][KH*KW][Cout] transpose of the OHWI weight.  Optional ReLU mask by
// the layer input's activation (MASK_X) in the epilogue.  Block = BCI input channels x
// 128 input pixels; K-step = one tap x 32 output channels.
template <int BCI, bool MASK_X>
__global__ __launch_bounds__(256) void conv_gemm_dgrad_kernel(ConvGeom g, const bf16_t* __restrict__ dY,
                                                              const bf16_t* __restrict__ WT,
                                                              const bf16_t* __restrict__ Xact,
                                                              bf16_t* __restrict__ dX) {
  __shared__ __attribute__((aligned(16))) bf16_t sA[2][BCI * CG_RS];
  __shared__ __attribute__((aligned(16))) bf16_t sB[2][CG_BP * CG_RS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wci = wave >> 1, wpx = wave & 1;
  constexpr int TCI = BCI / 32;
  const long HW = (long)g.H * g.W;
  const long Ptot = (long)g.N * HW;
  const long p0 = (long)blockIdx.x * CG_BP;
  const int ci0b = blockIdx.y * BCI;
  const int T = g.KH * g.KW;
  const int nk = T * (g.Cout / CG_KS);
  const int bp = tid >> 1, bh = (tid & 1) * 16;
  const long P = p0 + bp;
  const bool pv = P < Ptot;
  int n_ = 0, ih = 0, iw = 0;
  if (pv) {
    n_ = (int)(P / HW);
    const int r = (int)(P - (long)n_ * HW);
    ih = r / g.W;
    iw = r - ih * g.W;
  }
  auto load_k = [&](int ks, bf16x8* ra, bf16x8* rb) {
    const int tap = ks / (g.Cout / CG_KS);
    const int co0 = (ks - tap * (g.Cout / CG_KS)) * CG_KS;
    const int kh = tap / g.KW, kw = tap - kh * g.KW;
    const int th = ih + g.pad - kh, tw = iw + g.pad - kw;
    const int oh = th / g.stride, ow = tw / g.stride;
    const bool ok = pv && th >= 0 && tw >= 0 && th - oh * g.stride == 0 && tw - ow * g.stride == 0 &&
                    oh < g.OH && ow < g.OW;
    const bf16_t* src = dY + (((long)n_ * g.OH + oh) * g.OW + ow) * g.Cout + co0 + bh;
    rb[0] = ok ? ld8(src) : zero8();
    rb[1] = ok ? ld8(src + 8) : zero8();
#pragma unroll
    for (int u = 0; u < BCI * 4 / 256; ++u) {
      const int c = tid + u * 256;
      const int row = c >> 2, off = (c & 3) * 8;
      ra[u] = ld8(WT + ((long)(ci0b + row) * T + tap) * g.Cout + co0 + off);
    }
  };
  auto store_k = [&](int buf, const bf16x8* ra, const bf16x8* rb) {
    *reinterpret_cast<bf16x8*>(&sB[buf][bp * CG_RS + bh]) = rb[0];
    *reinterpret_cast<bf16x8*>(&sB[buf][bp * CG_RS + bh + 8]) = rb[1];
#pragma unroll
    for (int u = 0; u < BCI * 4 / 256; ++u) {
      const int c = tid + u * 256;
      *reinterpret_cast<bf16x8*>(&sA[buf][(c >> 2) * CG_RS + (c & 3) * 8]) = ra[u];
    }
  };
  f32x4 acc[TCI][4];
#pragma unroll
  for (int i = 0; i < TCI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 ra[BCI * 4 / 256 > 0 ? BCI * 4 / 256 : 1], rb[2];
  load_k(0, ra, rb);
  store_k(0, ra, rb);
  __syncthreads();
  const int kofs = 8 * (lane >> 4), col = lane & 15;
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    const bool more = ks + 1 < nk;
    if (more) load_k(ks + 1, ra, rb);
    bf16x8 a[TCI], b[4];
#pragma unroll
    for (int i = 0; i < TCI; ++i)
      a[i] = *reinterpret_cast<const bf16x8*>(&sA[cur][(wci * (BCI / 2) + 16 * i + col) * CG_RS + kofs]);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      b[j] = *reinterpret_cast<const bf16x8*>(&sB[cur][(wpx * 64 + 16 * j + col) * CG_RS + kofs]);
#pragma unroll
    for (int i = 0; i < TCI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
    if (more) store_k(cur ^ 1, ra, rb);
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long Pj = p0 + wpx * 64 + 16 * j + col;
    if (Pj >= Ptot) continue;
#pragma unroll
    for (int i = 0; i < TCI; ++i) {
      const int ci = ci0b + wci * (BCI / 2) + 16 * i + 4 * (lane >> 4);
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (MASK_X) {
        float xm[4];
        unpack4(*reinterpret_cast<const uint2*>(Xact + Pj * g.Cin + ci), xm);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = xm[r] > 0.f ? v[r] : 0.f;
      }
      *reinterpret_cast<uint2*>(dX + Pj * g.Cin + ci) = pack4(v[0], v[1], v[2], v[3]);
    }
  }
}

// ---------------------------------------------------------------- weight gradient
// D[co][(tap, ci)] = sum_p dY[p][co] * X[p @ tap][ci]; K = output pixels, split over
// blocks (grid.z = pixel chunks) into an fp32 slab [chunks][Cout][KH*KW][Cin] that
// grad_reduce sums in fixed order.  Block tile: 64 co x (one tap, 64 ci); per K-step
// 32 pixels of dY [32][64] and the gathered X [32][64] go to LDS (row stride 80
// elements = 40 dwords, an odd multiple of 8, so 8 consecutive rows of
// ds_read_b64_tr_b16 are conflict-free), and the K-along-lane MFMA fragments are read
// with the hardware transpose.  K index map: slot = 4g + j (j < 4), 16 + 4g + (j-4).
constexpr int WG_RS = 80;
// STEM (Cin == 4): the block's 64 columns are 16 taps x 4 channels (tap group
// blockIdx.y), so the slab row layout [Cout][T][4] is unchanged.
template <bool STEM>
__global__ __launch_bounds__(256) void conv_gemm_wgrad_kernel(ConvGeom g, const bf16_t* __restrict__ dY,
                                                              const bf16_t* __restrict__ X,
                                                              float* __restrict__ slab, int px_per_chunk) {
  __shared__ __attribute__((aligned(16))) bf16_t sD[2][32 * WG_RS];
  __shared__ __attribute__((aligned(16))) bf16_t sX[2][32 * WG_RS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int co0 = blockIdx.x * 64;
  const int T = g.KH * g.KW;
  const int tap = STEM ? 0 : blockIdx.y / (g.Cin / 64);
  const int ci0 = STEM ? 0 : (blockIdx.y - tap * (g.Cin / 64)) * 64;
  const int kh = tap / g.KW, kw = tap - kh * g.KW;
  const int tg0 = STEM ? blockIdx.y * 16 : 0;  // first tap of this block (STEM)
  const long OHW = (long)g.OH * g.OW;
  const long Ptot = (long)g.N * OHW;
  const long pbeg = (long)blockIdx.z * px_per_chunk;
  const long pend = min(Ptot, pbeg + px_per_chunk);
  // staging: 32 pixels x 64 ch for both tiles = 256 chunks of 16 B each -> one per thread each
  const int sp = tid >> 3, sc = (tid & 7) * 8;
  auto load = [&](long pk, bf16x8& vd, bf16x8& vx) {
    const long P = pk + sp;
    vd = zero8();
    vx = zero8();
    if (P < pend) {
      const int n_ = (int)(P / OHW);
      const int r = (int)(P - (long)n_ * OHW);
      const int oh = r / g.OW, ow = r - (r / g.OW) * g.OW;
      vd = ld8(dY + P * g.Cout + co0 + sc);
      if (STEM) {
        uint2 two[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int t = tg0 + sc / 4 + u;
          const int th = t / g.KW, tw = t - th * g.KW;
          const int ih = oh * g.stride - g.pad + th, iw = ow * g.stride - g.pad + tw;
          two[u] = (t < T && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
                       ? *reinterpret_cast<const uint2*>(X + (((long)n_ * g.H + ih) * g.W + iw) * 4)
                       : make_uint2(0u, 0u);
        }
        vx = __builtin_bit_cast(bf16x8, make_uint4(two[0].x, two[0].y, two[1].x, two[1].y));
      } else {
        const int ih = oh * g.stride - g.pad + kh, iw = ow * g.stride - g.pad + kw;
        if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
          vx = ld8(X + (((long)n_ * g.H + ih) * g.W + iw) * g.Cin + ci0 + sc);
      }
    }
  };
  // wave w: co tiles (2 of 4) x ci tiles (2 of 4)
  const int wco = (wave >> 1) * 32, wci = (wave & 1) * 32;
  const int gq = lane >> 4, i16 = lane & 15, q = i16 >> 2, pq = i16 & 3;
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 vd, vx;
  load(pbeg, vd, vx);
  *reinterpret_cast<bf16x8*>(&sD[0][sp * WG_RS + sc]) = vd;
  *reinterpret_cast<bf16x8*>(&sX[0][sp * WG_RS + sc]) = vx;
  __syncthreads();
  int cur = 0;
  for (long pk = pbeg; pk < pend; pk += 32) {
    const bool more = pk + 32 < pend;
    if (more) load(pk + 32, vd, vx);
    const int sA = 4 * gq + q, sB = 16 + 4 * gq + q;
    bf16x8 fa[2], fb[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)&sD[cur][sA * WG_RS + wco + 16 * a + 4 * pq]);
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)&sD[cur][sB * WG_RS + wco + 16 * a + 4 * pq]);
      fa[a] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)&sX[cur][sA * WG_RS + wci + 16 * b + 4 * pq]);
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)&sX[cur][sB * WG_RS + wci + 16 * b + 4 * pq]);
      fb[b] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[a][b] = mfma16(fa[a], fb[b], acc[a][b]);
    if (more) {
      *reinterpret_cast<bf16x8*>(&sD[cur ^ 1][sp * WG_RS + sc]) = vd;
      *reinterpret_cast<bf16x8*>(&sX[cur ^ 1][sp * WG_RS + sc]) = vx;
    }
    __syncthreads();
    cur ^= 1;
  }
  float* out = slab + (long)blockIdx.z * g.Cout * T * g.Cin;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wco + 16 * a + 4 * gq + r;
        if (STEM) {
          const int j = wci + 16 * b + i16;  // column = tap offset * 4 + channel
          const int t = tg0 + j / 4;
          if (t < T) out[((long)co * T + t) * 4 + (j & 3)] = acc[a][b][r];
        } else {
          const int ci = ci0 + wci + 16 * b + i16;
          out[((long)co * T + tap) * g.Cin + ci] = acc[a][b][r];
        }
      }
}

int conv_gemm_fwd_blocks(const ConvGeom& g) {
  const long P = (long)g.N * g.OH * g.OW;
  return (int)((P + CG_BP - 1) / CG_BP);
}

void conv_gemm_fwd(const ConvGeom& g, const bf16_t* X, const bf16_t* Wt, const float* bias,
                   bf16_t* Y, bool relu, float* stats, hipStream_t s) {
  const int bco = (g.Cout % 128 == 0) ? 128 : 64;
  const dim3 grid(conv_gemm_fwd_blocks(g), g.Cout / bco);
  if (g.Cin == 4) {  // stem: 8 taps x 4 channels per K-step
    if (bco != 64) return;  // host enforces Cout == 64 for the stem
    if (stats) hipLaunchKernelGGL((conv_gemm_fwd_kernel<64, false, true, true>), grid, dim3(256), 0, s, g, X, Wt, bias, Y, stats);
    else if (relu) hipLaunchKernelGGL((conv_gemm_fwd_kernel<64, true, false, true>), grid, dim3(256), 0, s, g, X, Wt, bias, Y, stats);
    else hipLaunchKernelGGL((conv_gemm_fwd_kernel<64, false, false, true>), grid, dim3(256), 0, s, g, X, Wt, bias, Y, stats);
    return;
  }
#define CGF(BC, RL, ST) hipLaunchKernelGGL((conv_gemm_fwd_kernel<BC, RL, ST, false>), grid, dim3(256), 0, s, g, X, Wt, bias, Y, stats)
  if (bco == 128) {
    if (stats) { if (relu) CGF(128, true, true); else CGF(128, false, true); }
    else { if (relu) CGF(128, true, false); else CGF(128, false, false); }
  } else {
    if (stats) { if (relu) CGF(64, true, true); else CGF(64, false, true); }
    else { if (relu) CGF(64, true, false); else CGF(64, false, false); }
  }
#undef CGF
}


void conv_gemm_dgrad(const ConvGeom& g, const bf16_t* dY, const bf16_t* WT, const bf16_t* Xact,
                     bf16_t* dX, hipStream_t s) {
  const long P = (long)g.N * g.H * g.W;
  const int bci = (g.Cin % 128 == 0) ? 128 : 64;
  const dim3 grid((unsigned)((P + CG_BP - 1) / CG_BP), g.Cin / bci);
#define CGD(BC, MX) hipLaunchKernelGGL((conv_gemm_dgrad_kernel<BC, MX>), grid, dim3(256), 0, s, g, dY, WT, Xact, dX)
  if (bci == 128) { if (Xact) CGD(128, true); else CGD(128, false); }
  else { if (Xact) CGD(64, true); else CGD(64, false); }
#undef CGD
}

int conv_gemm_wgrad_chunks(const ConvGeom& g, int px_per_chunk) {
  const long P = (long)g.N * g.OH * g.OW;
  return (int)((P + px_per_chunk - 1) / px_per_chunk);
}

void conv_gemm_wgrad(const ConvGeom& g, const bf16_t* dY, const bf16_t* X, float* slab,
                     int px_per_chunk, hipStream_t s) {
  if (g.Cin == 4) {
    const dim3 grid(g.Cout / 64, (g.KH * g.KW + 15) / 16, conv_gemm_wgrad_chunks(g, px_per_chunk));
    hipLaunchKernelGGL(conv_gemm_wgrad_kernel<true>, grid, dim3(256), 0, s, g, dY, X, slab, px_per_chunk);
    return;
  }
  const dim3 grid(g.Cout / 64, g.KH * g.KW * (g.Cin / 64), conv_gemm_wgrad_chunks(g, px_per_chunk));
  hipLaunchKernelGGL(conv_gemm_wgrad_kernel<false>, grid, dim3(256), 0, s, g, dY, X, slab, px_per_chunk);
}

}  // namespace ddp_amd
