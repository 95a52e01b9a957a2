// General NHWC convolution as an LDS-tiled MFMA implicit GEMM (ResNet-18 layers:
// 7x7/s2 stem, 3x3 s1/s2, 1x1 s2 downsample; SURVEY.md §2.4 "north-star" kernels).
//
// Forward, output channels on the MFMA rows, output pixels on the columns:
//   D[co][p] = sum_{tap, ci} W[co][tap][ci] * X[n][oh*s - pad + kh][ow*s - pad + kw][ci]
// K-step = one tap x 32 input channels (Cin % 32 == 0).  Block tile = BC output channels
// x BP output pixels (BP, BC in {64, 128}), 4 waves arranged 2 (co) x 2 (px).  Per K-step
// the block stages the weight tile [BC][32] and the gathered input tile [BP][32] into
// LDS (double buffered: the next K-step's global loads are issued before this step's
// MFMAs), rows padded to 40 elements (80 B).
//
// Filling 256 CUs: ResNet-18's deep layers have few output pixels (layer4 at batch 32:
// 1568) and long K (4608), so a plain tiling launches ~50 blocks.  The launch plan
// (conv_gemm_plan) picks the pixel tile and splits K over grid.z; split partials go to an
// fp32 workspace [splits][P][C] and splitk_reduce sums them in fixed split order, then
// does what the epilogue would have done (bf16 store, ReLU mask, BatchNorm statistics).
//
// Epilogue (unsplit): bf16 NHWC store (+ optional bias / ReLU) and, when requested,
// per-block partial per-channel sum and sum-of-squares of the stored values (the
// training BatchNorm that follows needs exactly these; fixed-order reduction in
// bn_finalize).
//
// The data gradient reads the OHWI weight itself: its A operand (rows ci, K = co) is the
// transpose of the stored layout, so the [32 co][BC ci] weight tile is staged as stored
// and the MFMA fragments are read with ds_read_b64_tr_b16 (no transposed weight copy).
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

constexpr int CG_KS = 32;  // K-step (channels of one tap)
#ifndef DDP_AMD_CG_PIPE
#define DDP_AMD_CG_PIPE 1  // 4: slower (512@7 fwd 102 -> 124 us: registers halve the occupancy that hid the latency; profiles/r4_resnet)
#endif
constexpr int CG_PIPE = DDP_AMD_CG_PIPE;  // K-steps of global-load lookahead (forward kernel)
// LDS row stride (elements) of K-contiguous tiles.  40 (20 dwords) shows 4.9-5.3 bank-
// conflict cycles per LDS instruction in the forward (PMC SQ_LDS_BANK_CONFLICT,
// profiles/r1_resnet); the conflict-free 48 (24 dwords, == 8 mod 16) measured no faster
// over the ResNet-18 layers (stem +3 us, the rest within +-1 us): these kernels are not
// LDS-bound, and 40 keeps the LDS footprint smaller.
constexpr int CG_RS = 40;

// K-slot permutation of the transposed (ds_read_b64_tr_b16) fragment read: fragment
// element j of lane group g holds k = 4g + j (j < 4) or 16 + 4g + (j - 4).  The matching
// non-transposed operand is stored to LDS in that order, so it stays one b128 read.
__device__ __forceinline__ int trk_pos(int k4) {  // LDS position of the 4-group starting at k = 4*k4
  return k4 < 4 ? 8 * k4 : 8 * (k4 - 4) + 4;
}

// Stem geometry as constants (SG = 1: ResNet-18's 7x7 / s2 / p3 stem on 224 x 224 inputs,
// 112 x 112 outputs; SG = 0: runtime).  The stem kernels' per-K-step tap / pixel index math
// was ~30 VALU instructions per MFMA with runtime divisors (profiles/r4_resnet/pmc).
template <int SG>
struct StemGeo {
  static constexpr int KW = 0, S = 0, PAD = 0, H = 0, W = 0, OH = 0, OW = 0;
};
template <>
struct StemGeo<1> {
  static constexpr int KW = 7, S = 2, PAD = 3, H = 224, W = 224, OH = 112, OW = 112;
};
inline bool stem_geo_224(const ConvGeom& g) {
  return g.Cin == 4 && g.KH == 7 && g.KW == 7 && g.stride == 2 && g.pad == 3 && g.H == 224 && g.W == 224 &&
         g.OH == 112 && g.OW == 112;
}
#define SG_(f, rt) (StemGeo<SG>::f ? StemGeo<SG>::f : (rt))

// STEM: Cin == 4 (3 real channels + 1 zero pad); a K-step covers 8 taps x 4 channels,
// k = tap*4 + c, so the weight row [KH*KW*4] is still contiguous per K-step.
template <int BP, int BC, bool RELU, bool STATS, bool STEM, bool PART, int SG = 0>
__global__ __launch_bounds__(256) void conv_gemm_fwd_kernel(ConvGeom g, const bf16_t* __restrict__ X,
                                                            const bf16_t* __restrict__ Wt,
                                                            const float* __restrict__ bias,
                                                            bf16_t* __restrict__ Y,
                                                            float* __restrict__ stats,
                                                            float* __restrict__ part, int ks_per) {
  static_assert(!STEM || (BP == 128 && !PART), "stem: 128-pixel tile, unsplit");
  __shared__ __attribute__((aligned(16))) bf16_t sA[2][BC * CG_RS];
  __shared__ __attribute__((aligned(16))) bf16_t sB[2][BP * CG_RS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wco = wave >> 1, wpx = wave & 1;
  constexpr int TCO = BC / 32;  // 16-row tiles per wave (co)
  constexpr int TPX = BP / 32;  // 16-col tiles per wave (px)
  constexpr int TPR = 256 / BP;          // staging threads per pixel row
  constexpr int EPT = CG_KS / TPR;       // elements per thread (16 or 8)
  const int3 bk = xcd_block3();  // XCD-contiguous block order (pixel tiles share an L2)
  const int OWv = SG_(OW, g.OW), OHW = SG_(OH, g.OH) * OWv;
  const int Ptot = g.N * OHW;
  const int p0 = bk.x * BP;
  const int co0 = bk.y * BC;
  const int KWC = g.KH * g.KW * g.Cin;
  const int T = g.KH * g.KW;
  const int nk = STEM ? (T + 7) / 8 : T * (g.Cin / CG_KS);
  const int kb = bk.z * ks_per;
  const int ke = min(nk, kb + ks_per);

  const int bp = tid / TPR, bh = (tid % TPR) * EPT;  // pixel row, element offset
  const int P = p0 + bp;
  const bool pv = P < Ptot;
  int n_ = 0, oh = 0, ow = 0;
  if (pv) {
    n_ = P / OHW;
    const int r = P - n_ * OHW;
    oh = r / OWv;
    ow = r - oh * OWv;
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
          const int KWv = SG_(KW, g.KW), Hv = SG_(H, g.H), Wv = SG_(W, g.W);
          const int kh = tap / KWv, kw = tap - kh * KWv;
          const int ih = oh * SG_(S, g.stride) - SG_(PAD, g.pad) + kh, iw = ow * SG_(S, g.stride) - SG_(PAD, g.pad) + kw;
          const bool ok = pv && tap < T && (unsigned)ih < (unsigned)Hv && (unsigned)iw < (unsigned)Wv;
          two[u] = ok ? *reinterpret_cast<const uint2*>(X + (((long)n_ * Hv + ih) * Wv + iw) * 4)
                      : make_uint2(0u, 0u);
        }
        uint4 q4 = make_uint4(two[0].x, two[0].y, two[1].x, two[1].y);
        rb[h2] = __builtin_bit_cast(bf16x8, q4);
      }
#pragma unroll
      for (int u = 0; u < BC * 4 / 256; ++u) {
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
#pragma unroll
    for (int h = 0; h < EPT / 8; ++h) rb[h] = ok ? ld8(src + 8 * h) : zero8();
    // A: weight rows
#pragma unroll
    for (int u = 0; u < BC * 4 / 256; ++u) {
      const int c = tid + u * 256;
      const int row = c >> 2, off = (c & 3) * 8;
      ra[u] = ld8(Wt + (long)(co0 + row) * KWC + tap * g.Cin + ci0 + off);
    }
  };
  auto store_k = [&](int buf, const bf16x8* ra, const bf16x8* rb) {
#pragma unroll
    for (int h = 0; h < EPT / 8; ++h) *reinterpret_cast<bf16x8*>(&sB[buf][bp * CG_RS + bh + 8 * h]) = rb[h];
#pragma unroll
    for (int u = 0; u < BC * 4 / 256; ++u) {
      const int c = tid + u * 256;
      *reinterpret_cast<bf16x8*>(&sA[buf][(c >> 2) * CG_RS + (c & 3) * 8]) = ra[u];
    }
  };

  f32x4 acc[TCO][TPX];
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int j = 0; j < TPX; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // K loop, software-pipelined CG_PIPE deep: the global loads of K-step ks + CG_PIPE are
  // issued at the start of step ks into register set (ks - kb) % CG_PIPE (free: its step
  // was stored to LDS one step earlier), so each load has CG_PIPE - 1 steps of MFMAs to land
  // before the step that stores it.  With one step of lookahead every step waited out a
  // full L2 / HBM round trip (~1-2 us against ~0.1 us of MFMAs: the ResNet-18 layers ran at
  // 5-15 % of their roofline, profiles/r4_resnet/roofline.md).  LDS stays double-buffered.
  constexpr int NA = BC * 4 / 256 > 0 ? BC * 4 / 256 : 1;
  bf16x8 ra[CG_PIPE][NA], rb[CG_PIPE][2];
#pragma unroll
  for (int u = 0; u < CG_PIPE; ++u)
    if (kb + u < ke) load_k(kb + u, ra[u], rb[u]);
  if (kb < ke) store_k(0, ra[0], rb[0]);
  __syncthreads();
  const int kofs = 8 * (lane >> 4), col = lane & 15;
  for (int base = kb; base < ke; base += CG_PIPE) {
#pragma unroll
    for (int u = 0; u < CG_PIPE; ++u) {
      const int ks = base + u;
      if (ks >= ke) break;  // block-uniform
      const int cur = (ks - kb) & 1;
      if (ks + CG_PIPE < ke) load_k(ks + CG_PIPE, ra[u], rb[u]);  // set u was stored last step
      bf16x8 a[TCO], b[TPX];
#pragma unroll
      for (int i = 0; i < TCO; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(&sA[cur][(wco * (BC / 2) + 16 * i + col) * CG_RS + kofs]);
#pragma unroll
      for (int j = 0; j < TPX; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(&sB[cur][(wpx * (BP / 2) + 16 * j + col) * CG_RS + kofs]);
#pragma unroll
      for (int i = 0; i < TCO; ++i)
#pragma unroll
        for (int j = 0; j < TPX; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
      if (ks + 1 < ke) store_k(cur ^ 1, ra[(u + 1) % CG_PIPE], rb[(u + 1) % CG_PIPE]);
      __syncthreads();
    }
  }

  // ---- epilogue
  if (PART) {  // fp32 split partial [z][P][Cout]: 4 consecutive channels per lane = 16 B
    float* dst = part + (long)bk.z * Ptot * g.Cout;
#pragma unroll
    for (int j = 0; j < TPX; ++j) {
      const int Pj = p0 + wpx * (BP / 2) + 16 * j + col;
      if (Pj >= Ptot) continue;
#pragma unroll
      for (int i = 0; i < TCO; ++i) {
        const int co = co0 + wco * (BC / 2) + 16 * i + 4 * (lane >> 4);
        *reinterpret_cast<float4*>(dst + (long)Pj * g.Cout + co) =
            make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    return;
  }
  float csum[TCO][4], csq[TCO][4];
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) csum[i][r] = csq[i][r] = 0.f;
#pragma unroll
  for (int j = 0; j < TPX; ++j) {
    const int Pj = p0 + wpx * (BP / 2) + 16 * j + col;
    const bool ok = Pj < Ptot;
#pragma unroll
    for (int i = 0; i < TCO; ++i) {
      const int co = co0 + wco * (BC / 2) + 16 * i + 4 * (lane >> 4);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[i][j][r] + (bias ? bias[co + r] : 0.f);
        if (RELU) v[r] = fmaxf(v[r], 0.f);
      }
      const uint2 pk = pack4(v[0], v[1], v[2], v[3]);
      if (ok) *reinterpret_cast<uint2*>(Y + (long)Pj * g.Cout + co) = pk;
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
    __shared__ float s_st[2][2][BC];
#pragma unroll
    for (int i = 0; i < TCO; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = sum16(csum[i][r]), b = sum16(csq[i][r]);
        if (col == 0) {
          const int cl = wco * (BC / 2) + 16 * i + 4 * (lane >> 4) + r;
          s_st[wpx][0][cl] = a;
          s_st[wpx][1][cl] = b;
        }
      }
    __syncthreads();
    // stats slab: [blocks_x][2][Cout]
    for (int c = tid; c < BC; c += 256) {
      float* dst = stats + (long)bk.x * 2 * g.Cout;
      st_wt(dst + co0 + c, s_st[0][0][c] + s_st[1][0][c]);
      st_wt(dst + g.Cout + co0 + c, s_st[0][1][c] + s_st[1][1][c]);
    }
  }
}

// ---------------------------------------------------------------- stem forward, halo form
// The 7x7 / s2 / p3 stem on 224 x 224 x 4 inputs (StemGeo<1>), same block -> pixel map,
// MFMA tiling and epilogue as conv_gemm_fwd_kernel<128, 64, ..., STEM, ..., 1>, but the
// block's input rows are staged into LDS ONCE and its weight fragments are read ONCE into
// registers: the gathered form waited out a global round trip per K-step (7 per block, ~1 us
// each against 8 MFMAs per wave; 47 us per launch at B = 32, profiles/r4_final).
// 128 consecutive output pixels of one image (12544 = 98 x 128: blocks never straddle
// images) lie in at most 3 output rows oh0..oh0+2, i.e. input rows 2*oh0-3 .. 2*oh0+7 (11).
// K-step = one kernel row kh: k = kw * 4 + c for kw = 0..7 (kw = 7: zero weight), so a
// lane's 8 K values are taps 2q, 2q+1 of one input row = 2 adjacent pixels x 4 channels =
// 16 contiguous bytes of the staged row (LDS column j = iw + 3, even for every read).
constexpr int STEM_ROWS = 11, STEM_COLS = 232;  // staged input rows / columns (j = iw + 3)
template <bool RELU, bool STATS>
__global__ __launch_bounds__(256, 2) void conv_stem_halo_fwd_kernel(ConvGeom g, const bf16_t* __restrict__ X,
                                                                 const bf16_t* __restrict__ Wt,
                                                                 const float* __restrict__ bias,
                                                                 bf16_t* __restrict__ Y,
                                                                 float* __restrict__ stats, int ntiles) {
  using SGeo = StemGeo<1>;
  constexpr int BP = 128, BC = 64, TCO = 2, TPX = 4;
  constexpr int OHW = SGeo::OH * SGeo::OW, KWC = 49 * 4, RS = STEM_COLS * 4;  // RS: elements per row
  constexpr int NPAIR = STEM_ROWS * (SGeo::W / 2), XPT = (NPAIR + 255) / 256;  // 16-B pieces per thread
  __shared__ __attribute__((aligned(16))) bf16_t sX[2][STEM_ROWS * RS];
  __shared__ float s_st[2][2][BC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wco = wave >> 1, wpx = wave & 1;
  const int3 bk = xcd_block3();
  const int Ptot = g.N * OHW;
  const int co0 = bk.y * BC;
  const int kofs = 8 * (lane >> 4), col = lane & 15, q = lane >> 4;
  // a contiguous range of 128-pixel tiles per block (neighbouring tiles share input rows;
  // xcd_block3 keeps neighbouring blocks on one XCD): weights once, inputs double-buffered
  const int t_beg = (int)((long)bk.x * ntiles / gridDim.x), t_end = (int)((long)(bk.x + 1) * ntiles / gridDim.x);

  // weight fragments: a[kh][i] = taps 2q, 2q+1 of kernel row kh, output channel
  // co0 + wco*32 + 16i + col
  bf16x8 a[7][TCO];
#pragma unroll
  for (int i = 0; i < TCO; ++i) {
    const bf16_t* wr = Wt + (long)(co0 + wco * 32 + 16 * i + col) * KWC;
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      const uint2 t0 = *reinterpret_cast<const uint2*>(wr + (kh * 7 + 2 * q) * 4);
      const uint2 t1 = q < 3 ? *reinterpret_cast<const uint2*>(wr + (kh * 7 + 2 * q + 1) * 4) : make_uint2(0u, 0u);
      a[kh][i] = __builtin_bit_cast(bf16x8, make_uint4(t0.x, t0.y, t1.x, t1.y));
    }
  }
  // the zero columns of both buffers: j = 0..2 (iw = -3..-1) and j = 227..231 (iw >= 224)
  for (int e = tid; e < 2 * STEM_ROWS * 8; e += 256) {
    const int bf = e / (STEM_ROWS * 8), r = (e >> 3) % STEM_ROWS, k = e & 7;
    const int j = k < 3 ? k : 224 + k;
    *reinterpret_cast<uint2*>(&sX[bf][r * RS + j * 4]) = make_uint2(0u, 0u);
  }
  // input rows of tile t: pairs of input columns (16 B) -> LDS columns j, j + 1 (j odd).
  // Tile t + 1 is requested when tile t starts (a second tile of lookahead, in a second
  // register set, measured no faster: 34.8 vs 34.5 us per launch at B = 32)
  uint4 xr[2][XPT];
  auto load_x = [&](int t, uint4* xs) {
    const int p0 = t * BP, n_ = p0 / OHW, oh0 = (p0 - n_ * OHW) / SGeo::OW;
    const bf16_t* xim = X + (long)n_ * SGeo::H * SGeo::W * 4;
#pragma unroll
    for (int u = 0; u < XPT; ++u) {
      const int e = tid + 256 * u;
      const int r = e / (SGeo::W / 2), c2 = e - r * (SGeo::W / 2);
      const int ih = 2 * oh0 - 3 + r;
      xs[u] = make_uint4(0u, 0u, 0u, 0u);
      if (e < NPAIR && (unsigned)ih < (unsigned)SGeo::H)
        xs[u] = *reinterpret_cast<const uint4*>(xim + ((long)ih * SGeo::W + 2 * c2) * 4);
    }
  };
  auto store_x = [&](int bf, const uint4* xs) {
#pragma unroll
    for (int u = 0; u < XPT; ++u) {
      const int e = tid + 256 * u;
      if (e < NPAIR) {
        const int r = e / (SGeo::W / 2), c2 = e - r * (SGeo::W / 2);
        bf16_t* d = &sX[bf][r * RS + (2 * c2 + 3) * 4];
        *reinterpret_cast<uint2*>(d) = make_uint2(xs[u].x, xs[u].y);
        *reinterpret_cast<uint2*>(d + 4) = make_uint2(xs[u].z, xs[u].w);
      }
    }
  };
  if (t_beg < t_end) {
    load_x(t_beg, xr[0]);
    store_x(0, xr[0]);
  }
  __syncthreads();
  // tile t: LDS buffer and register set cur = (t - t_beg) & 1 (a compile-time constant)
  auto tile = [&](int t, auto CUR) {
    constexpr int cur = decltype(CUR)::value;
    if (t + 1 < t_end) load_x(t + 1, xr[cur ^ 1]);  // lands during this tile's MFMAs and epilogue
    const int p0 = t * BP, n_ = p0 / OHW, oh0 = (p0 - n_ * OHW) / SGeo::OW;
    f32x4 acc[TCO][TPX];
#pragma unroll
    for (int i = 0; i < TCO; ++i)
#pragma unroll
      for (int j = 0; j < TPX; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    int hb[TPX];  // the lane's LDS element offset at kh = 0, per px tile
#pragma unroll
    for (int j = 0; j < TPX; ++j) {
      const int P = p0 + wpx * (BP / 2) + 16 * j + col;
      const int rr = (P < Ptot ? P : p0) - n_ * OHW;
      const int oh = rr / SGeo::OW, ow = rr - oh * SGeo::OW;
      hb[j] = 2 * (oh - oh0) * RS + (2 * ow) * 4 + kofs;
    }
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      bf16x8 b[TPX];
#pragma unroll
      for (int j = 0; j < TPX; ++j) b[j] = *reinterpret_cast<const bf16x8*>(&sX[cur][hb[j] + kh * RS]);
#pragma unroll
      for (int i = 0; i < TCO; ++i)
#pragma unroll
        for (int j = 0; j < TPX; ++j) acc[i][j] = mfma16(a[kh][i], b[j], acc[i][j]);
    }

    // ---- epilogue (conv_gemm_fwd_kernel's, unsplit; stats row = tile)
    float csum[TCO][4], csq[TCO][4];
#pragma unroll
    for (int i = 0; i < TCO; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) csum[i][r] = csq[i][r] = 0.f;
#pragma unroll
    for (int j = 0; j < TPX; ++j) {
      const int Pj = p0 + wpx * (BP / 2) + 16 * j + col;
      const bool ok = Pj < Ptot;
#pragma unroll
      for (int i = 0; i < TCO; ++i) {
        const int co = co0 + wco * (BC / 2) + 16 * i + 4 * (lane >> 4);
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[i][j][r] + (bias ? bias[co + r] : 0.f);
          if (RELU) v[r] = fmaxf(v[r], 0.f);
        }
        const uint2 pk = pack4(v[0], v[1], v[2], v[3]);
        if (ok) *reinterpret_cast<uint2*>(Y + (long)Pj * g.Cout + co) = pk;
        if (STATS) {
          float qv[4];
          unpack4(pk, qv);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = ok ? qv[r] : 0.f;
            csum[i][r] += x;
            csq[i][r] = fmaf(x, x, csq[i][r]);
          }
        }
      }
    }
    if (STATS) {
#pragma unroll
      for (int i = 0; i < TCO; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float sa = sum16(csum[i][r]), sb = sum16(csq[i][r]);
          if (col == 0) {
            const int cl = wco * (BC / 2) + 16 * i + 4 * (lane >> 4) + r;
            s_st[wpx][0][cl] = sa;
            s_st[wpx][1][cl] = sb;
          }
        }
      __syncthreads();
      for (int c = tid; c < BC; c += 256) {
        float* dst = stats + (long)t * 2 * g.Cout;
        st_wt(dst + co0 + c, s_st[0][0][c] + s_st[1][0][c]);
        st_wt(dst + g.Cout + co0 + c, s_st[0][1][c] + s_st[1][1][c]);
      }
    }
    if (t + 1 < t_end) store_x(cur ^ 1, xr[cur ^ 1]);  // tile t + 1 (buffer cur ^ 1 was last read a tile ago)
    __syncthreads();
  };
  for (int t = t_beg; t < t_end; t += 2) {
    tile(t, std::integral_constant<int, 0>{});
    if (t + 1 < t_end) tile(t + 1, std::integral_constant<int, 1>{});
  }
}

// ---------------------------------------------------------------- data gradient
// D[ci][p_in] = sum_{tap, co} W[co][tap][ci] * dY[n][(ih + pad - kh)/s][(iw + pad - kw)/s][co]
// (taps whose offset is not divisible by the stride, or fall outside dY, contribute 0).
// Optional ReLU mask by the layer input's activation (MASK_X) in the epilogue.  Block =
// BC input channels x BP input pixels; K-step = one tap x 32 output channels.  The weight
// tile is [32 co][BC ci] as stored (row stride BC + 16 = an odd multiple of 8 dwords:
// conflict-free transposed reads); dY is stored in the transposed read's K order.
template <int BP, int BC, bool MASK_X, bool PART>
__global__ __launch_bounds__(256) void conv_gemm_dgrad_kernel(ConvGeom g, const bf16_t* __restrict__ dY,
                                                              const bf16_t* __restrict__ W,
                                                              const bf16_t* __restrict__ Xact,
                                                              bf16_t* __restrict__ dX,
                                                              float* __restrict__ part, int ks_per,
                                                              int nsplit, int parity) {
  constexpr int AS = BC + 16;
  __shared__ __attribute__((aligned(16))) bf16_t sA[2][CG_KS * AS];
  __shared__ __attribute__((aligned(16))) bf16_t sB[2][BP * CG_RS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wci = wave >> 1, wpx = wave & 1;
  constexpr int TCI = BC / 32;
  constexpr int TPX = BP / 32;
  constexpr int TPR = 256 / BP;
  constexpr int EPT = CG_KS / TPR;
  constexpr int ACH = CG_KS * BC / 8 / 256;  // 16-B weight chunks per thread
  // Stride-2 parity classes: input pixel (ih, iw) only meets taps with kh = ih + pad
  // (mod 2), kw likewise, so each class (ih % 2, iw % 2) is a dense GEMM over its own
  // 1..4 taps (3x3) instead of all 9 with 3/4 structural zeros.  grid.z = class x split.
  // hardware block order: the XCD remap measured worse here (stride-2 parity classes leave
  // whole blocks idle and contiguous ranges pile them on a few XCDs: 1x1/s2 8.7 -> 14.8 us)
  const int3 bk = make_int3(blockIdx.x, blockIdx.y, blockIdx.z);
  int cls = 0, zs = bk.z;
  if (parity) {
    cls = bk.z / nsplit;
    zs = bk.z - cls * nsplit;
  }
  const int ph = cls >> 1, pw = cls & 1, ts = parity ? 2 : 1;
  const int Hc = (g.H - ph + ts - 1) / ts, Wc = (g.W - pw + ts - 1) / ts;
  const int HWc = Hc * Wc;
  const int Pc = g.N * HWc;  // pixels of this class
  const int p0 = bk.x * BP;
  if (p0 >= Pc) return;  // block-uniform (a smaller class), before any barrier
  const int ci0b = bk.y * BC;
  const int kh0 = parity ? (ph + g.pad) & 1 : 0, kw0 = parity ? (pw + g.pad) & 1 : 0;
  const int nth = (g.KH - kh0 + ts - 1) / ts, ntw = (g.KW - kw0 + ts - 1) / ts;
  const int CK = g.Cout / CG_KS;
  const int nk = nth * ntw * CK;
  const int kper = parity ? (nk + nsplit - 1) / nsplit : ks_per;
  const int kb = zs * kper;
  const int ke = min(nk, kb + kper);
  const int bp = tid / TPR, bh = (tid % TPR) * EPT;
  const int P = p0 + bp;
  const bool pv = P < Pc;
  int n_ = 0, ih = 0, iw = 0;
  if (pv) {
    n_ = P / HWc;
    const int r = P - n_ * HWc;
    const int i = r / Wc;
    ih = ts * i + ph;
    iw = ts * (r - i * Wc) + pw;
  }
  auto load_k = [&](int ks, bf16x8* ra, bf16x8* rb) {
    const int ti = ks / CK;
    const int co0 = (ks - ti * CK) * CG_KS;
    const int thi = ti / ntw;
    const int kh = kh0 + ts * thi, kw = kw0 + ts * (ti - thi * ntw);
    const int tap = kh * g.KW + kw;
    const int th = ih + g.pad - kh, tw = iw + g.pad - kw;
    const int oh = th / g.stride, ow = tw / g.stride;
    const bool ok = pv && th >= 0 && tw >= 0 && th - oh * g.stride == 0 && tw - ow * g.stride == 0 &&
                    oh < g.OH && ow < g.OW;
    const bf16_t* src = dY + (((long)n_ * g.OH + oh) * g.OW + ow) * g.Cout + co0 + bh;
#pragma unroll
    for (int h = 0; h < EPT / 8; ++h) rb[h] = ok ? ld8(src + 8 * h) : zero8();
#pragma unroll
    for (int u = 0; u < ACH; ++u) {
      const int c = tid + u * 256;
      const int row = c / (BC / 8), off = (c % (BC / 8)) * 8;
      ra[u] = ld8(W + ((long)(co0 + row) * (g.KH * g.KW) + tap) * g.Cin + ci0b + off);
    }
  };
  auto store_k = [&](int buf, const bf16x8* ra, const bf16x8* rb) {
    // dY run k = bh .. bh+EPT-1 -> 4-groups at their transposed-read positions
#pragma unroll
    for (int h = 0; h < EPT / 8; ++h) {
      const uint4 q = __builtin_bit_cast(uint4, rb[h]);
      const int k4 = (bh + 8 * h) / 4;
      *reinterpret_cast<uint2*>(&sB[buf][bp * CG_RS + trk_pos(k4)]) = make_uint2(q.x, q.y);
      *reinterpret_cast<uint2*>(&sB[buf][bp * CG_RS + trk_pos(k4 + 1)]) = make_uint2(q.z, q.w);
    }
#pragma unroll
    for (int u = 0; u < ACH; ++u) {
      const int c = tid + u * 256;
      const int row = c / (BC / 8), off = (c % (BC / 8)) * 8;
      *reinterpret_cast<bf16x8*>(&sA[buf][row * AS + off]) = ra[u];
    }
  };
  f32x4 acc[TCI][TPX];
#pragma unroll
  for (int i = 0; i < TCI; ++i)
#pragma unroll
    for (int j = 0; j < TPX; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // K loop pipelined CG_PIPE deep (see conv_gemm_fwd_kernel)
  bf16x8 ra[CG_PIPE][ACH], rb[CG_PIPE][2];
#pragma unroll
  for (int u = 0; u < CG_PIPE; ++u)
    if (kb + u < ke) load_k(kb + u, ra[u], rb[u]);
  if (kb < ke) store_k(0, ra[0], rb[0]);
  __syncthreads();
  const int kofs = 8 * (lane >> 4), col = lane & 15;
  const int gq = lane >> 4, q = col >> 2, pq = col & 3;
  const int rlo = (4 * gq + q) * AS, rhi = (16 + 4 * gq + q) * AS;
  for (int base = kb; base < ke; base += CG_PIPE) {
#pragma unroll
    for (int u = 0; u < CG_PIPE; ++u) {
      const int ks = base + u;
      if (ks >= ke) break;  // block-uniform
      const int cur = (ks - kb) & 1;
      if (ks + CG_PIPE < ke) load_k(ks + CG_PIPE, ra[u], rb[u]);
      bf16x8 a[TCI], b[TPX];
#pragma unroll
      for (int i = 0; i < TCI; ++i) {
        const int m = wci * (BC / 2) + 16 * i + 4 * pq;
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)&sA[cur][rlo + m]);
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)&sA[cur][rhi + m]);
        a[i] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < TPX; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(&sB[cur][(wpx * (BP / 2) + 16 * j + col) * CG_RS + kofs]);
#pragma unroll
      for (int i = 0; i < TCI; ++i)
#pragma unroll
        for (int j = 0; j < TPX; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
      if (ks + 1 < ke) store_k(cur ^ 1, ra[(u + 1) % CG_PIPE], rb[(u + 1) % CG_PIPE]);
      __syncthreads();
    }
  }
  const long Ptot = (long)g.N * g.H * g.W;
#pragma unroll
  for (int j = 0; j < TPX; ++j) {
    const int Pj = p0 + wpx * (BP / 2) + 16 * j + col;
    if (Pj >= Pc) continue;
    long gp = Pj;  // class pixel -> NHWC pixel index
    if (parity) {
      const int n = Pj / HWc;
      const int r = Pj - n * HWc;
      const int i = r / Wc;
      gp = ((long)n * g.H + ts * i + ph) * g.W + ts * (r - i * Wc) + pw;
    }
#pragma unroll
    for (int i = 0; i < TCI; ++i) {
      const int ci = ci0b + wci * (BC / 2) + 16 * i + 4 * (lane >> 4);
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (PART) {
        *reinterpret_cast<float4*>(part + ((long)zs * Ptot + gp) * g.Cin + ci) =
            make_float4(v[0], v[1], v[2], v[3]);
        continue;
      }
      if (MASK_X) {
        float xm[4];
        unpack4(*reinterpret_cast<const uint2*>(Xact + gp * g.Cin + ci), xm);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = xm[r] > 0.f ? v[r] : 0.f;
      }
      *reinterpret_cast<uint2*>(dX + gp * g.Cin + ci) = pack4(v[0], v[1], v[2], v[3]);
    }
  }
}

// ---------------------------------------------------------------- split-K reduction
// part [S][P][C] fp32 -> out bf16 [P][C], summed in split order 0..S-1; optional ReLU mask
// by Xact (> 0) and optional per-block BatchNorm partials [gridDim.x][2][C] (sum, sum of
// squares of the stored bf16 values).  Thread = 8 channels of one pixel; block = C/8
// channel groups x 256/(C/8) pixel lanes over `rpb` pixels.
template <bool MASK, bool STATS>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int S, int P,
                                                            int C, int rpb,
                                                            const bf16_t* __restrict__ Xact,
                                                            bf16_t* __restrict__ out,
                                                            float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) float sred[];  // [pl][2][C]
  const int cg = C / 8, pl = 256 / cg;
  const int tg = threadIdx.x % cg, tp = threadIdx.x / cg;
  const long PC = (long)P * C;
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  const int p0 = blockIdx.x * rpb, p1 = min(P, p0 + rpb);
  for (int p = p0 + tp; p < p1; p += pl) {
    const long off = (long)p * C + tg * 8;
    float v[8];
    {
      const float4 a = *reinterpret_cast<const float4*>(part + off);
      const float4 b = *reinterpret_cast<const float4*>(part + off + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
    for (int z = 1; z < S; ++z) {
      const float4 a = *reinterpret_cast<const float4*>(part + z * PC + off);
      const float4 b = *reinterpret_cast<const float4*>(part + z * PC + off + 4);
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    }
    if (MASK) {
      const uint4 xm = *reinterpret_cast<const uint4*>(Xact + off);
      float x[8];
      unpack4(make_uint2(xm.x, xm.y), x);
      unpack4(make_uint2(xm.z, xm.w), x + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = x[j] > 0.f ? v[j] : 0.f;
    }
    const uint2 lo = pack4(v[0], v[1], v[2], v[3]), hi = pack4(v[4], v[5], v[6], v[7]);
    *reinterpret_cast<uint4*>(out + off) = make_uint4(lo.x, lo.y, hi.x, hi.y);
    if (STATS) {
      float r[8];
      unpack4(lo, r);
      unpack4(hi, r + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += r[j];
        q[j] = fmaf(r[j], r[j], q[j]);
      }
    }
  }
  if (!STATS) return;
  if (tp < pl) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sred[(tp * 2) * C + tg * 8 + j] = s[j];
      sred[(tp * 2 + 1) * C + tg * 8 + j] = q[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int t = 0; t < pl; ++t) {
      a += sred[(t * 2) * C + c];
      b += sred[(t * 2 + 1) * C + c];
    }
    st_wt(stats + (long)blockIdx.x * 2 * C + c, a);
    st_wt(stats + (long)blockIdx.x * 2 * C + C + c, b);
  }
}

// ---------------------------------------------------------------- weight gradient
// D[co][(tap, ci)] = sum_p dY[p][co] * X[p @ tap][ci]; K = output pixels, split over
// blocks (grid.z = pixel chunks).  One chunk: the block writes the gradient itself
// (out = [+ out] + D, `accum` for gradient accumulation); several: an fp32 slab
// [chunks][Cout][KH*KW][Cin] that grad_reduce sums in fixed order.  Block tile: BM co x
// (one tap, BN ci), 4 waves of (BM/2) x (BN/2); per K-step 32 pixels of dY [32][BM] and
// the gathered X [32][BN] go to LDS (row stride BM+16 / BN+16 = an odd multiple of 8
// dwords, so 8 consecutive rows of ds_read_b64_tr_b16 are conflict-free), and the
// K-along-lane MFMA fragments are read with the hardware transpose.
// STEM (Cin == 4 in X, BN = 64): the block's 64 columns are 16 taps x 4 channels (tap
// group blockIdx.y); the output keeps only the 3 real channels: [Cout][T][3].
template <int BM, int BN, bool STEM, int KS, int SG = 0>  // SG: see StemGeo
__global__ __launch_bounds__(256) void conv_gemm_wgrad_kernel(ConvGeom g, const bf16_t* __restrict__ dY,
                                                              const bf16_t* __restrict__ X,
                                                              float* __restrict__ out, int px_per_chunk,
                                                              int accum) {
  static_assert(!STEM || BN == 64, "stem: 16 taps x 4 channels per block");
  constexpr int RD = BM + 16, RX = BN + 16;
  constexpr int DPT = BM * KS / 2048, XPT = BN * KS / 2048;  // 16-B staging chunks per thread
  constexpr int TA = BM / 32, TB = BN / 32;    // 16x16 tiles per wave
  __shared__ __attribute__((aligned(16))) bf16_t sD[2][KS * RD];
  __shared__ __attribute__((aligned(16))) bf16_t sX[2][KS * RX];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // hardware block order: an XCD-contiguous remap (whole pixel chunks per L2) measured
  // +1..+4 us on 6 of 9 layers (scripts/wgrad_tile_sweep.py); the L2 misses are not the bound
  const int3 bk = make_int3(blockIdx.x, blockIdx.y, blockIdx.z);
  const int co0 = bk.x * BM;
  const int T = g.KH * g.KW;
  const int tap = STEM ? 0 : bk.y / (g.Cin / BN);
  const int ci0 = STEM ? 0 : (bk.y - tap * (g.Cin / BN)) * BN;
  const int kh = tap / g.KW, kw = tap - kh * g.KW;
  const int tg0 = STEM ? bk.y * 16 : 0;  // first tap of this block (STEM)
  const int OWv = SG_(OW, g.OW), OHW = SG_(OH, g.OH) * OWv;
  const int Ptot = g.N * OHW;
  const int pbeg = bk.z * px_per_chunk;
  const int pend = min(Ptot, pbeg + px_per_chunk);
  auto load = [&](int pk, bf16x8* vd, bf16x8* vx) {
#pragma unroll
    for (int u = 0; u < DPT; ++u) {
      const int c = tid + 256 * u;
      const int sp = c / (BM / 8), sc = (c % (BM / 8)) * 8;
      const int P = pk + sp;
      vd[u] = P < pend ? ld8(dY + (long)P * g.Cout + co0 + sc) : zero8();
    }
#pragma unroll
    for (int u = 0; u < XPT; ++u) {
      const int c = tid + 256 * u;
      const int sp = c / (BN / 8), sc = (c % (BN / 8)) * 8;
      const int P = pk + sp;
      vx[u] = zero8();
      if (P < pend) {
        const int n_ = P / OHW;
        const int r = P - n_ * OHW;
        const int oh = r / OWv, ow = r - oh * OWv;
        if (STEM) {
          uint2 two[2];
          const int KWv = SG_(KW, g.KW), Hv = SG_(H, g.H), Wv = SG_(W, g.W);
#pragma unroll
          for (int v = 0; v < 2; ++v) {
            const int t = tg0 + sc / 4 + v;
            const int th = t / KWv, tw = t - th * KWv;
            const int ih = oh * SG_(S, g.stride) - SG_(PAD, g.pad) + th, iw = ow * SG_(S, g.stride) - SG_(PAD, g.pad) + tw;
            two[v] = (t < T && (unsigned)ih < (unsigned)Hv && (unsigned)iw < (unsigned)Wv)
                         ? *reinterpret_cast<const uint2*>(X + (((long)n_ * Hv + ih) * Wv + iw) * 4)
                         : make_uint2(0u, 0u);
          }
          vx[u] = __builtin_bit_cast(bf16x8, make_uint4(two[0].x, two[0].y, two[1].x, two[1].y));
        } else {
          const int ih = oh * g.stride - g.pad + kh, iw = ow * g.stride - g.pad + kw;
          if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
            vx[u] = ld8(X + (((long)n_ * g.H + ih) * g.W + iw) * g.Cin + ci0 + sc);
        }
      }
    }
  };
  auto store = [&](int buf, const bf16x8* vd, const bf16x8* vx) {
#pragma unroll
    for (int u = 0; u < DPT; ++u) {
      const int c = tid + 256 * u;
      *reinterpret_cast<bf16x8*>(&sD[buf][(c / (BM / 8)) * RD + (c % (BM / 8)) * 8]) = vd[u];
    }
#pragma unroll
    for (int u = 0; u < XPT; ++u) {
      const int c = tid + 256 * u;
      *reinterpret_cast<bf16x8*>(&sX[buf][(c / (BN / 8)) * RX + (c % (BN / 8)) * 8]) = vx[u];
    }
  };
  // wave w: co half (wave >> 1) x column half (wave & 1)
  const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * (BN / 2);
  const int gq = lane >> 4, i16 = lane & 15, q = i16 >> 2, pq = i16 & 3;
  f32x4 acc[TA][TB];
#pragma unroll
  for (int a = 0; a < TA; ++a)
#pragma unroll
    for (int b = 0; b < TB; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 vd[DPT], vx[XPT];
  load(pbeg, vd, vx);
  store(0, vd, vx);
  __syncthreads();
  int cur = 0;
  const int kA = 4 * gq + q, kB = 16 + 4 * gq + q;
  for (int pk = pbeg; pk < pend; pk += KS) {
    const bool more = pk + KS < pend;
    if (more) load(pk + KS, vd, vx);
#pragma unroll
    for (int kk = 0; kk < KS / 32; ++kk) {  // KS/32 MFMA K-steps per barrier
      bf16x8 fa[TA], fb[TB];
#pragma unroll
      for (int a = 0; a < TA; ++a) {
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)&sD[cur][(32 * kk + kA) * RD + wm + 16 * a + 4 * pq]);
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)&sD[cur][(32 * kk + kB) * RD + wm + 16 * a + 4 * pq]);
        fa[a] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int b = 0; b < TB; ++b) {
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)&sX[cur][(32 * kk + kA) * RX + wn + 16 * b + 4 * pq]);
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)&sX[cur][(32 * kk + kB) * RX + wn + 16 * b + 4 * pq]);
        fb[b] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int a = 0; a < TA; ++a)
#pragma unroll
        for (int b = 0; b < TB; ++b) acc[a][b] = mfma16(fa[a], fb[b], acc[a][b]);
    }
    if (more) store(cur ^ 1, vd, vx);
    __syncthreads();
    cur ^= 1;
  }
  const int ocin = STEM ? 3 : g.Cin;
  float* o = out + (long)bk.z * g.Cout * T * ocin;
  // output index of accumulator element (a, b, r); -1 = a padding column of the stem
  auto out_idx = [&](int a, int b, int r) -> long {
    const int co = co0 + wm + 16 * a + 4 * gq + r;
    if (STEM) {
      const int j = wn + 16 * b + i16;  // column = tap offset * 4 + channel
      const int t = tg0 + j / 4;
      if (t >= T || (j & 3) == 3) return -1;
      return ((long)co * T + t) * 3 + (j & 3);
    }
    return ((long)co * T + tap) * g.Cin + ci0 + wn + 16 * b + i16;
  };
  if (accum) {  // all old values in flight at once, then the stores
    float old[TA][TB][4];
#pragma unroll
    for (int a = 0; a < TA; ++a)
#pragma unroll
      for (int b = 0; b < TB; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long idx = out_idx(a, b, r);
          old[a][b][r] = idx >= 0 ? o[idx] : 0.f;
        }
#pragma unroll
    for (int a = 0; a < TA; ++a)
#pragma unroll
      for (int b = 0; b < TB; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long idx = out_idx(a, b, r);
          if (idx >= 0) o[idx] = old[a][b][r] + acc[a][b][r];
        }
  } else {
#pragma unroll
    for (int a = 0; a < TA; ++a)
#pragma unroll
      for (int b = 0; b < TB; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long idx = out_idx(a, b, r);
          if (idx >= 0) o[idx] = acc[a][b][r];
        }
  }
}

// ---------------------------------------------------------------- host side
// Launch plan: pixel tile, channel tile and K splits.  Tuned on MI355X with
// scripts/resnet_conv_sweep.py over ResNet-18 at batch 32 (profiles/r1_resnet):
//  * K splits pay only for long K (>= 72 K-steps: 3x3 over >= 256 channels), where the
//    grid is small and every split still runs >= 18 K-steps; below that the fp32
//    partial round trip costs more than the idle CUs;
//  * the forward takes 64-pixel tiles when 128-pixel ones give < 512 blocks, and
//    64x64 tiles for 1x1 convolutions (2-8 K-steps: more blocks beat reuse);
//  * the data gradient keeps 128-pixel tiles (its gather is the costlier operand).
ConvPlan conv_gemm_plan(const ConvGeom& g, bool dgrad, int bp, int bc, int splits, int parity,
                        int halo) {
  ConvPlan pl{};
  // stride-1 3x3 forward through the LDS halo tile: R full rows of one image (a 128-
  // or, for narrow layers, 64-pixel tile) and 64 output channels per block.
  // Auto-picked only when that grid fills the GPU without K splits; with splits the fp32
  // partial round trip cost more than the halo saved.  ResNet-18 (conv_sweep.jsonl):
  // layer1 24.4 -> 21.5 us, layer2 26.3 -> 17.2 us.  halo = 1 forces it.
  // The stride-1 3x3 data gradient is the same halo GEMM over dY (conv_halo.hip).
  const int hrows = dgrad ? g.Cin : g.Cout, hk = dgrad ? g.Cout : g.Cin;
  int hbp = 0;
  long hgrid = 0;
  for (int cand : {128, 64}) {
    if (bp && bp != cand) continue;
    if (!conv_halo_fits(g, cand) || hk % CG_KS != 0) continue;
    const int r = conv_halo_rows(g, cand);
    hbp = cand;
    hgrid = (long)g.N * ((g.H + r - 1) / r) * (hrows / 64);
    if (hgrid >= 384) break;
  }
  if (hbp && !(bp && halo != 1) && (halo == 1 || (halo < 0 && hgrid >= 384 && splits <= 1))) {
    pl.halo = 1;
    pl.bp = hbp;
    pl.bc = bc ? bc : 64;
    const int R = conv_halo_rows(g, hbp), RG = (g.H + R - 1) / R, nch = hk / CG_KS;
    pl.grid_x = g.N * RG;
    pl.grid_y = hrows / pl.bc;
    const long base = (long)pl.grid_x * pl.grid_y;
    int s = splits;
    if (s <= 0) {
      s = base >= 384 ? 1 : (int)((768 + base - 1) / base);
      if (s > nch / 2) s = nch / 2;
    }
    if (s < 1) s = 1;
    if (s > nch) s = nch;
    const int cps = (nch + s - 1) / s;
    pl.splits = (nch + cps - 1) / cps;
    pl.ks_per = cps * 9;
    pl.grid_z = pl.splits;
    return pl;
  }
  const int C = dgrad ? g.Cin : g.Cout;     // GEMM rows
  const int T = g.KH * g.KW;
  const bool stem = !dgrad && g.Cin == 4;
  pl.parity = (dgrad && g.stride == 2 && parity != 0) ? 1 : 0;
  // pixels per GEMM (the largest parity class) and K-steps (the class with most taps)
  const long P = !dgrad ? (long)g.N * g.OH * g.OW
                        : pl.parity ? (long)g.N * ((g.H + 1) / 2) * ((g.W + 1) / 2) : (long)g.N * g.H * g.W;
  const int taps = pl.parity ? ((g.KH + 1) / 2) * ((g.KW + 1) / 2) : T;
  const int nk = stem ? (T + 7) / 8 : taps * ((dgrad ? g.Cout : g.Cin) / CG_KS);
  const int classes = pl.parity ? 4 : 1;
  const bool pointwise = T == 1;
  int c = bc ? bc : (C % 128 == 0 ? 128 : 64);
  if (!bc && !dgrad && pointwise) c = 64;
  if (stem) c = 64;
  pl.bc = c;
  auto blocks = [&](int bpx) { return classes * ((P + bpx - 1) / bpx) * (long)(C / pl.bc); };
  // parity classes: the 1x1 downsample has one live class (64 x 64 tiles), a 3x3 takes
  // the narrower channel tile when the grid is small (more blocks beat K splits)
  if (pl.parity && !bc && (pointwise || blocks(128) < 256)) pl.bc = c = 64;
  if (bp) pl.bp = bp;
  else if (pl.parity && pointwise) pl.bp = 64;
  else if (dgrad || stem) pl.bp = 128;
  else pl.bp = (!pointwise && blocks(128) >= 512) ? 128 : 64;
  if (stem) pl.bp = 128;
  int s = splits;
  if (s <= 0) {
    if (pl.parity) {  // short per-class K: split only a small grid, >= 8 K-steps per split
      const long base = blocks(pl.bp);
      s = (pointwise || base >= 256) ? 1 : (int)((768 + base - 1) / base);
      if (s > 4) s = 4;
      if (s > nk / 8) s = nk / 8;
    } else {
      s = nk >= 72 ? nk / 18 : 1;
    }
  }
  if (s > 8) s = 8;
  if (stem || s < 1) s = 1;
  if (s > nk) s = nk;
  pl.ks_per = (nk + s - 1) / s;
  pl.splits = pl.parity ? s : (nk + pl.ks_per - 1) / pl.ks_per;  // parity: every class splits its own K
  pl.grid_x = (int)((P + pl.bp - 1) / pl.bp);
  pl.grid_y = C / pl.bc;
  pl.grid_z = classes * pl.splits;
  return pl;
}

static int splitk_rows(long P, int C, int* rpb) {
  const int pl = 256 / (C / 8);
  long nb = (P + pl - 1) / pl;
  if (nb > 512) nb = 512;
  long r = (P + nb - 1) / nb;
  r = (r + pl - 1) / pl * pl;
  *rpb = (int)r;
  return (int)((P + r - 1) / r);
}

int conv_gemm_stat_rows(const ConvGeom& g, const ConvPlan& pl) {
  if (pl.splits <= 1) return pl.grid_x;
  int rpb;
  return splitk_rows((long)g.N * g.OH * g.OW, g.Cout, &rpb);
}

static void splitk_reduce(const float* part, int S, long P, int C, const bf16_t* Xact, bf16_t* out,
                          float* stats, hipStream_t s) {
  int rpb;
  const int nb = splitk_rows(P, C, &rpb);
  const size_t lds = stats ? sizeof(float) * (256 / (C / 8)) * 2 * C : 0;
#define SKR(M, ST) hipLaunchKernelGGL((splitk_reduce_kernel<M, ST>), dim3(nb), dim3(256), lds, s, part, S, (int)P, C, rpb, Xact, out, stats)
  if (Xact) { if (stats) SKR(true, true); else SKR(true, false); }
  else { if (stats) SKR(false, true); else SKR(false, false); }
#undef SKR
}

void conv_gemm_fwd(const ConvGeom& g, const ConvPlan& pl, const bf16_t* X, const bf16_t* Wt,
                   const float* bias, bf16_t* Y, bool relu, float* stats, float* part, hipStream_t s,
                   const BnAffine* aff) {
  if (aff && aff->mean && !pl.halo)
    throw std::runtime_error("conv_gemm_fwd: an input BatchNorm affine needs the halo plan");
  if (pl.halo) {  // no bias / ReLU epilogue on this path (the host plans it off then)
    conv_halo_fwd(g, pl.bp, pl.bc, pl.splits, X, Wt, Y, stats, part, s, aff);
    if (pl.splits > 1) splitk_reduce(part, pl.splits, (long)g.N * g.OH * g.OW, g.Cout, nullptr, Y, stats, s);
    return;
  }
  const dim3 grid(pl.grid_x, pl.grid_y, pl.splits);
  const int kp = pl.ks_per;
  if (g.Cin == 4) {  // stem: 8 taps x 4 channels per K-step (host enforces Cout % 64)
    const bool s224 = stem_geo_224(g);
    // the 224 x 224 stem: staged-halo kernel (DDP_AMD_STEM_HALO=0: the gathered K loop)
    static const int stem_halo = [] { const char* e = getenv("DDP_AMD_STEM_HALO"); return e ? atoi(e) : 1; }();
    if (s224 && stem_halo && pl.splits <= 1 && grid.x * 128 >= (unsigned)(g.N * 112 * 112)) {
      // persistent: two blocks per CU, each over a contiguous range of the 128-pixel tiles
      static const int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 256;
        return n > 0 ? n : 256;
      }();
      const int ntiles = (int)grid.x;
      const dim3 sg(std::min(ntiles, 2 * cus), grid.y, 1);
#define CSH(RL, ST) hipLaunchKernelGGL((conv_stem_halo_fwd_kernel<RL, ST>), sg, dim3(256), 0, s, g, X, Wt, bias, Y, stats, ntiles)
      if (stats) CSH(false, true);
      else if (relu) CSH(true, false);
      else CSH(false, false);
#undef CSH
      return;
    }
#define CGS(RL, ST)                                                                                                  \
  do {                                                                                                               \
    if (s224) hipLaunchKernelGGL((conv_gemm_fwd_kernel<128, 64, RL, ST, true, false, 1>), grid, dim3(256), 0, s, g, X, Wt, bias, Y, stats, part, kp); \
    else hipLaunchKernelGGL((conv_gemm_fwd_kernel<128, 64, RL, ST, true, false, 0>), grid, dim3(256), 0, s, g, X, Wt, bias, Y, stats, part, kp); \
  } while (0)
    if (stats) CGS(false, true);
    else if (relu) CGS(true, false);
    else CGS(false, false);
#undef CGS
    return;
  }
#define CGF(BP, BC, RL, ST, PT) hipLaunchKernelGGL((conv_gemm_fwd_kernel<BP, BC, RL, ST, false, PT>), grid, dim3(256), 0, s, g, X, Wt, bias, Y, stats, part, kp)
#define CGF_BP(BP, BC)                                                           \
  if (pl.splits > 1) CGF(BP, BC, false, false, true);                            \
  else if (stats) { if (relu) CGF(BP, BC, true, true, false); else CGF(BP, BC, false, true, false); } \
  else { if (relu) CGF(BP, BC, true, false, false); else CGF(BP, BC, false, false, false); }
  if (pl.bp == 128) { if (pl.bc == 128) { CGF_BP(128, 128) } else { CGF_BP(128, 64) } }
  else { if (pl.bc == 128) { CGF_BP(64, 128) } else { CGF_BP(64, 64) } }
#undef CGF_BP
#undef CGF
  if (pl.splits > 1) {
    // bias / ReLU of the split path: only the BatchNorm use (no bias, no ReLU) is split
    splitk_reduce(part, pl.splits, (long)g.N * g.OH * g.OW, g.Cout, nullptr, Y, stats, s);
  }
}

void conv_gemm_dgrad(const ConvGeom& g, const ConvPlan& pl, const bf16_t* dY, const bf16_t* W,
                     const bf16_t* Xact, bf16_t* dX, float* part, hipStream_t s) {
  if (pl.halo) {
    conv_halo_dgrad(g, pl.bp, pl.bc, pl.splits, dY, W, pl.splits > 1 ? nullptr : Xact, dX, part, s);
    if (pl.splits > 1) splitk_reduce(part, pl.splits, (long)g.N * g.H * g.W, g.Cin, Xact, dX, nullptr, s);
    return;
  }
  const dim3 grid(pl.grid_x, pl.grid_y, pl.grid_z);
  const int kp = pl.ks_per, ns = pl.splits, par = pl.parity;
#define CGD(BP, BC, MX, PT) hipLaunchKernelGGL((conv_gemm_dgrad_kernel<BP, BC, MX, PT>), grid, dim3(256), 0, s, g, dY, W, Xact, dX, part, kp, ns, par)
#define CGD_BP(BP, BC)                     \
  if (pl.splits > 1) CGD(BP, BC, false, true); \
  else if (Xact) CGD(BP, BC, true, false); \
  else CGD(BP, BC, false, false);
  if (pl.bp == 128) { if (pl.bc == 128) { CGD_BP(128, 128) } else { CGD_BP(128, 64) } }
  else { if (pl.bc == 128) { CGD_BP(64, 128) } else { CGD_BP(64, 64) } }
#undef CGD_BP
#undef CGD
  if (pl.splits > 1) splitk_reduce(part, pl.splits, (long)g.N * g.H * g.W, g.Cin, Xact, dX, nullptr, s);
}

int conv_gemm_wgrad_chunks(const ConvGeom& g, int px_per_chunk) {
  const long P = (long)g.N * g.OH * g.OW;
  return (int)((P + px_per_chunk - 1) / px_per_chunk);
}

// Block tile of the weight gradient (scripts/resnet_conv_sweep.py, wgrad_tile_sweep.py,
// profiles/r1_resnet):
// 128-wide tiles only while the 128-tile grid is small (< 64 tiles: those layers are
// chunked over pixels anyway and the wider tile halves the slab traffic); otherwise
// 64 x 64, whose 4x larger grid fills the CUs without chunking.
static int g_wgrad_force_bm = 0, g_wgrad_force_bn = 0;  // sweep override (0 = auto)
void conv_gemm_wgrad_force_tile(int bm, int bn) {
  g_wgrad_force_bm = (bm == 64 || bm == 128) ? bm : 0;
  g_wgrad_force_bn = (bn == 64 || bn == 128) ? bn : 0;
}

static void wgrad_tile(const ConvGeom& g, int* bm, int* bn) {
  const int T = g.KH * g.KW;
  *bm = 64;
  *bn = 64;
  if (g.Cin == 4 || T == 1) return;
  if (g_wgrad_force_bm && g.Cout % g_wgrad_force_bm == 0 && g.Cin % g_wgrad_force_bn == 0) {
    *bm = g_wgrad_force_bm;
    *bn = g_wgrad_force_bn;
    return;
  }
  // stride 2: the narrower X tile (l3 3x3/s2: 27.7 -> 22.8 us, scripts/wgrad_tile_sweep.py)
  const int bm2 = g.Cout % 128 == 0 ? 128 : 64, bn2 = (g.Cin % 128 == 0 && g.stride == 1) ? 128 : 64;
  if ((long)(g.Cout / bm2) * T * (g.Cin / bn2) < 64) {
    *bm = bm2;
    *bn = bn2;
  }
}

// tap-fused halo weight gradient (conv_halo.hip) for stride-1 3x3 layers: plan = chunks of
// whole output rows so that the launch has ~g_wgrad_halo_target blocks of 64 co x 32 ci
static int g_wgrad_halo = 1, g_wgrad_halo_target = 256;  // halo: 0 off, 1 auto, 2 wherever eligible
static int g_wgrad_halo_cit = 0;                             // input channels per block (0 = auto)
void conv_gemm_wgrad_set_halo(int halo, int target, int cit) {
  g_wgrad_halo = halo < 0 ? 0 : (halo > 2 ? 2 : halo);
  g_wgrad_halo_target = target > 0 ? target : 256;
  g_wgrad_halo_cit = (cit == 16 || cit == 32) ? cit : 0;
}
static int wgrad_halo_cit(const ConvGeom& g) { return g_wgrad_halo_cit ? g_wgrad_halo_cit : 32; }
// auto (1): every eligible layer.  Per launch the halo kernel beats the per-tap GEMM's
// 64 x 64 tile (ResNet-18/224 layer1: 32.7 -> 23.6 us, layer4: 37.3 -> 23.6 us) and loses a
// little to its 128 x 128 tile (layer2 / layer3: 22.2 / 20.9 vs 23.6 us), but its smaller
// slabs make the whole step faster on every layer (14.29-14.31k -> 14.36-14.40k img/s over
// "64 x 64 layers only", profiles/r2_halo_wgrad); 2 = the same, kept for the sweeps
static bool wgrad_use_halo(const ConvGeom& g) {
  if (!g_wgrad_halo || !conv_halo_wgrad_ok(g)) return false;
  return true;
}
static int wgrad_halo_ppc(const ConvGeom& g) {
  const int bpc = (g.Cout / 64) * (g.Cin / wgrad_halo_cit(g));
  int chunks = g_wgrad_halo_target / bpc;
  if (chunks < 1) chunks = 1;
  const int rows = g.N * g.H;
  int rpc = (rows + chunks - 1) / chunks;
  const int q = conv_halo_wgrad_row_quantum(g);  // whole images when groups stack images
  rpc = (rpc + q - 1) / q * q;
  return rpc * g.W;
}

int conv_gemm_wgrad_tiles(const ConvGeom& g) {
  int bm, bn;
  wgrad_tile(g, &bm, &bn);
  const int gy = g.Cin == 4 ? (g.KH * g.KW + 15) / 16 : g.KH * g.KW * (g.Cin / bn);
  return (g.Cout / bm) * gy;
}

// pixels per chunk: split K until the grid has ~target blocks (1x1: 256 - a tiny GEMM
// whose slab reduction dominates; 128-wide tiles: 512; 64 x 64: 1024)
bool conv_gemm_wgrad_ppc_ok(const ConvGeom& g, int ppc) {
  if (ppc <= 0) return false;
  if (ppc % 32 == 0) return true;
  return wgrad_use_halo(g) && ppc % (g.W * conv_halo_wgrad_row_quantum(g)) == 0;
}

int conv_gemm_wgrad_ppc(const ConvGeom& g) {
  if (wgrad_use_halo(g)) return wgrad_halo_ppc(g);
  int bm, bn;
  wgrad_tile(g, &bm, &bn);
  const int T = g.KH * g.KW;
  const long target = T == 1 ? 256 : ((bm == 128 || bn == 128) ? 512 : 1024);
  const long tiles = conv_gemm_wgrad_tiles(g);
  long chunks = target / tiles;
  if (chunks < 1) chunks = 1;
  const long P = (long)g.N * g.OH * g.OW;
  long ppc = (P + chunks - 1) / chunks;
  ppc = (ppc + 31) / 32 * 32;
  return (int)(ppc < 32 ? 32 : ppc);
}

// ks: pixels staged per barrier (32 or 64; 0 = 32).  Staging 64 pixels halves the
// barriers per MFMA but measured neutral on every ResNet-18 layer (conv_sweep.jsonl,
// "auto/ks32" vs "auto/ks64"): the 64 x 64 tiles are bound by L2 traffic - dY and the
// gathered X are re-read once per tap block - not by the barrier.
bool conv_gemm_wgrad_uses_halo(const ConvGeom& g, int px_per_chunk) {
  return wgrad_use_halo(g) && px_per_chunk % (g.W * conv_halo_wgrad_row_quantum(g)) == 0;  // whole rows
}

void conv_gemm_wgrad(const ConvGeom& g, const bf16_t* dY, const bf16_t* X, float* out,
                     int px_per_chunk, bool accum, hipStream_t s, int ks, const BnAffine* aff) {
  const int ch = conv_gemm_wgrad_chunks(g, px_per_chunk);
  const int acc = (accum && ch == 1) ? 1 : 0;
  if (conv_gemm_wgrad_uses_halo(g, px_per_chunk)) {
    conv_halo_wgrad(g, dY, X, out, px_per_chunk / g.W, acc != 0, s, wgrad_halo_cit(g), aff);
    return;
  }
  if (aff && aff->mean)
    throw std::runtime_error("conv_gemm_wgrad: an input BatchNorm affine needs the halo weight gradient");
  int bm, bn;
  wgrad_tile(g, &bm, &bn);
  if (ks != 32 && ks != 64) ks = 32;
  if (g.Cin == 4) {
    const dim3 grid(g.Cout / bm, (g.KH * g.KW + 15) / 16, ch);
    const bool s224 = stem_geo_224(g);
#define CGWS(M, K)                                                                                                   \
  do {                                                                                                               \
    if (s224) hipLaunchKernelGGL((conv_gemm_wgrad_kernel<M, 64, true, K, 1>), grid, dim3(256), 0, s, g, dY, X, out, px_per_chunk, acc); \
    else hipLaunchKernelGGL((conv_gemm_wgrad_kernel<M, 64, true, K, 0>), grid, dim3(256), 0, s, g, dY, X, out, px_per_chunk, acc); \
  } while (0)
    if (bm == 128) { if (ks == 64) CGWS(128, 64); else CGWS(128, 32); }
    else { if (ks == 64) CGWS(64, 64); else CGWS(64, 32); }
#undef CGWS
    return;
  }
  const dim3 grid(g.Cout / bm, g.KH * g.KW * (g.Cin / bn), ch);
#define CGW(M, N, K) hipLaunchKernelGGL((conv_gemm_wgrad_kernel<M, N, false, K>), grid, dim3(256), 0, s, g, dY, X, out, px_per_chunk, acc)
  if (ks == 64) {
    if (bm == 128) { if (bn == 128) CGW(128, 128, 64); else CGW(128, 64, 64); }
    else { if (bn == 128) CGW(64, 128, 64); else CGW(64, 64, 64); }
  } else {
    if (bm == 128) { if (bn == 128) CGW(128, 128, 32); else CGW(128, 64, 32); }
    else { if (bn == 128) CGW(64, 128, 32); else CGW(64, 64, 32); }
  }
#undef CGW
}

}  // namespace ddp_amd
